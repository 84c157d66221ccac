#!/bin/bash
# -fa 0 decode at depth 0: llama-bench tg128 (fa 0 / fa 1, same box) and the fa 0 kernel stats; op tests of the nofa chain (threshold 512)
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_ops_gpu.py -k "nofa" -x -q -s --timeout 300 --timeout-method thread > gpurun_out/r5_c23_ops.log 2>&1
rc=$?; echo "ops rc=$rc"; tail -2 gpurun_out/r5_c23_ops.log; [ $rc -ne 0 ] && exit $rc
G8=$(python -c "import bench; print(bench.bench_gguf('llama3_8b', 'q4_k_m'))") || exit 1
export GGML_BACKEND_PATH=$PWD/llama-mi50.cpp_amd/lib/libggml-mi355x.so
for fa in 0 1 0 1; do
  timeout -k 10 600 oracle/_ref/llama-bench -m $G8 -t 8 -ngl 99 -fa $fa -p 0 -n 128 -r 3 -o jsonl > gpurun_out/tg_fa$fa.log 2>&1 || exit 1
  echo "fa=$fa: $(grep -o '"samples_ts": \[[^]]*\]' gpurun_out/tg_fa$fa.log)"
done
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_fa0 -o run --output-format csv -- \
    oracle/_ref/llama-bench -m $G8 -t 8 -ngl 99 -fa 0 -p 0 -n 128 -r 1 -o jsonl > gpurun_out/prof_fa0.log 2>&1 || exit 1
cut -d, -f1-4 gpurun_out/prof_fa0/run_kernel_stats.csv | head -16
