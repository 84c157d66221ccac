#!/bin/bash
# k_fattn_dec3 geometry A/B: 4 waves x 4 stages vs 8 waves x 2 stages (g_tune[37]); tests; drop-in d16384
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python tools/opbench.py --only fa_4096 fa_16384 fa_32768 --ab 37=0 37=1 37=0 37=1 > gpurun_out/r5_c29_ab.log 2>&1 || { tail -20 gpurun_out/r5_c29_ab.log; exit 1; }
grep -v "^#" gpurun_out/r5_c29_ab.log | tail -14
GGML_MI355X_FA_STREAM_GEOM=1 timeout -k 10 600 python -u -m pytest tests/test_ops_gpu.py -k "flash_attn_stream" -x -q -s --timeout 300 --timeout-method thread > gpurun_out/r5_c29_ops.log 2>&1
rc=$?; echo "ops(geom 1) rc=$rc"; tail -2 gpurun_out/r5_c29_ops.log; [ $rc -ne 0 ] && exit $rc
G8=$(python -c "import bench; print(bench.bench_gguf('llama3_8b', 'q4_k_m'))") || exit 1
export GGML_BACKEND_PATH=$PWD/llama-mi50.cpp_amd/lib/libggml-mi355x.so
for pass in 1 2; do for geom in 0 1; do
  GGML_MI355X_FA_STREAM_GEOM=$geom timeout -k 10 600 oracle/_ref/llama-bench -m $G8 -t 8 -ngl 99 -fa 1 -p 0 -n 128 -d 16384 -r 3 -o jsonl > gpurun_out/g_$geom.log 2>&1 || exit 1
  echo "pass $pass geom=$geom d16k: $(grep -o '"samples_ts": \[[^]]*\]' gpurun_out/g_$geom.log)"
done; done
