#!/bin/bash
# k_fattn_dec3 (relaxed count, q behind the DMA): isolation trace, op tests, drop-in tg128 @ d16384 A/B
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python tools/opbench.py --only fa_16384 --trace --trace-blocks > gpurun_out/r5_c15_trace.log 2>&1 || { tail -20 gpurun_out/r5_c15_trace.log; exit 1; }
grep -E "trace|blocks" gpurun_out/r5_c15_trace.log | head -30
timeout -k 10 300 python tools/opbench.py --only fa_4096 fa_16384 fa_32768 --ab 34=0 34=1 > gpurun_out/r5_c15_ab.log 2>&1 || { tail -20 gpurun_out/r5_c15_ab.log; exit 1; }
grep -v "^#" gpurun_out/r5_c15_ab.log | tail -8
timeout -k 10 600 python -u -m pytest tests/test_ops_gpu.py -k "flash_attn" -x -q -s --timeout 300 --timeout-method thread > gpurun_out/r5_c15_ops.log 2>&1
rc=$?; echo "ops rc=$rc"; tail -2 gpurun_out/r5_c15_ops.log; [ $rc -ne 0 ] && exit $rc
G8=$(python -c "import bench; print(bench.bench_gguf('llama3_8b', 'q4_k_m'))") || exit 1
export GGML_BACKEND_PATH=$PWD/llama-mi50.cpp_amd/lib/libggml-mi355x.so
for pass in 1 2; do for arm in 1 0; do
  GGML_MI355X_FA_STREAM=$arm timeout -k 10 600 oracle/_ref/llama-bench -m $G8 -t 8 -ngl 99 -fa 1 -p 0 -n 128 -d 16384 -r 3 -o jsonl > gpurun_out/d16k_$arm.log 2>&1 || exit 1
  echo "pass $pass stream=$arm d16k: $(grep -o '"samples_ts": \[[^]]*\]' gpurun_out/d16k_$arm.log)"
done; done
