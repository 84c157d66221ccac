#!/bin/bash
# QKV with its norm source staged by LDS-DMA (g_tune[41] = 1): decode parity with it on, then
# tg128 A/B (fa 1 and fa 0), three interleaved passes
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
GGML_MI355X_TUNE=41=1 timeout -k 10 600 python -u -m pytest tests/test_dropin_gpu.py tests/test_dropin_shapes_gpu.py tests/test_ops_gpu.py \
  -k "incremental_decode or test_llama3_8b_width_decode or qkv" -x -q --timeout 300 --timeout-method thread > gpurun_out/r5_c45_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r5_c45_tests.log; [ $rc -ne 0 ] && exit $rc
PASSES=3 AB="- GGML_MI355X_TUNE=41=1" timeout -k 10 600 bash scripts/r5_ab_env.sh > gpurun_out/r5_c45_fa1.txt 2>&1
rc=$?; cut -c1-140 gpurun_out/r5_c45_fa1.txt; [ $rc -ne 0 ] && exit $rc
FA=0 PASSES=2 AB="- GGML_MI355X_TUNE=41=1" timeout -k 10 600 bash scripts/r5_ab_env.sh > gpurun_out/r5_c45_fa0.txt 2>&1
rc=$?; cut -c1-140 gpurun_out/r5_c45_fa0.txt; exit $rc
