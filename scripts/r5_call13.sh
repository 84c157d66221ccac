#!/bin/bash
# streaming long-cache decode attention (k_fattn_dec3): op tests, then drop-in tg128 at depth 16384 A/B
# (GGML_MI355X_FA_STREAM=0 = the LONG geometry + combine) and a kernel-stats profile
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_ops_gpu.py -k "flash_attn" -x -q -s --timeout 300 --timeout-method thread > gpurun_out/r5_c13_ops.log 2>&1
rc=$?; echo "ops rc=$rc"; tail -3 gpurun_out/r5_c13_ops.log; grep -E "^FAILED|Error|assert" gpurun_out/r5_c13_ops.log | head -10
[ $rc -ne 0 ] && exit $rc
G8=$(python -c "import bench; print(bench.bench_gguf('llama3_8b', 'q4_k_m'))") || exit 1
export GGML_BACKEND_PATH=$PWD/llama-mi50.cpp_amd/lib/libggml-mi355x.so
for pass in 1 2; do for arm in 1 0; do
  GGML_MI355X_FA_STREAM=$arm timeout -k 10 600 oracle/_ref/llama-bench -m $G8 -t 8 -ngl 99 -fa 1 -p 0 -n 128 -d 16384 -r 3 -o jsonl > gpurun_out/d16k_$arm.log 2>&1 || exit 1
  echo "pass $pass stream=$arm d16k: $(grep -o '"samples_ts": \[[^]]*\]' gpurun_out/d16k_$arm.log)"
done; done
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_d16k_s -o run --output-format csv -- \
    oracle/_ref/llama-bench -m $G8 -t 8 -ngl 99 -fa 1 -p 0 -n 128 -d 16384 -r 1 -o jsonl > gpurun_out/prof_d16k_s.log 2>&1 || exit 1
head -16 gpurun_out/prof_d16k_s/run_kernel_stats.csv | cut -c1-140
