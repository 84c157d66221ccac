#!/bin/bash
# long-cache -fa 0 decode chain (k_nofa_scores / k_nofa_pv / k_nofa_sum): op tests, drop-in -fa 0 at depth
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_ops_gpu.py -k "nofa" -x -q -s --timeout 300 --timeout-method thread > gpurun_out/r5_c21_ops.log 2>&1
rc=$?; echo "ops rc=$rc"; tail -3 gpurun_out/r5_c21_ops.log; grep -E "^FAILED|Error|assert" gpurun_out/r5_c21_ops.log | head -10
[ $rc -ne 0 ] && exit $rc
G8=$(python -c "import bench; print(bench.bench_gguf('llama3_8b', 'q4_k_m'))") || exit 1
export GGML_BACKEND_PATH=$PWD/llama-mi50.cpp_amd/lib/libggml-mi355x.so
for d in 512 256; do for mn in 512 100000; do
  GGML_MI355X_NOFA_LONG_MIN=$mn timeout -k 10 600 oracle/_ref/llama-bench -m $G8 -t 8 -ngl 99 -fa 0 -p 0 -n 128 -d $d -r 3 -o jsonl > gpurun_out/nl_$d.log 2>&1 || exit 1
  echo "fa0 d=$d long_min=$mn: $(grep -o '"samples_ts": \[[^]]*\]' gpurun_out/nl_$d.log)"
done; done
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_nl -o run --output-format csv -- \
    oracle/_ref/llama-bench -m $G8 -t 8 -ngl 99 -fa 0 -p 0 -n 64 -d 16384 -r 1 -o jsonl > gpurun_out/prof_nl.log 2>&1 || exit 1
grep -E "nofa|gemv2|fa_mma" gpurun_out/prof_nl/run_kernel_stats.csv | cut -d, -f1-4 | head -12
