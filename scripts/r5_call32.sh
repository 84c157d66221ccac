#!/bin/bash
# threshold 8192: FA tests, depth test, d8192 A/B
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_ops_gpu.py tests/test_dropin_shapes_gpu.py -k "flash_attn or at_depth" -x -q --timeout 600 --timeout-method thread > gpurun_out/r5_c32.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r5_c32.log; grep -E "^E  .*(Assert|assert)" gpurun_out/r5_c32.log | head -6
[ $rc -ne 0 ] && exit $rc
G8=$(python -c "import bench; print(bench.bench_gguf('llama3_8b', 'q4_k_m'))") || exit 1
export GGML_BACKEND_PATH=$PWD/llama-mi50.cpp_amd/lib/libggml-mi355x.so
for pass in 1 2; do for arm in 1 0; do
  GGML_MI355X_FA_STREAM=$arm timeout -k 10 600 oracle/_ref/llama-bench -m $G8 -t 8 -ngl 99 -fa 1 -p 0 -n 128 -d 8192 -r 3 -o jsonl > gpurun_out/fs_$arm.log 2>&1 || exit 1
  echo "pass $pass d=8192 stream=$arm: $(grep -o '"samples_ts": \[[^]]*\]' gpurun_out/fs_$arm.log)"
done; done
