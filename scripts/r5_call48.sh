#!/bin/bash
# XStage::postscale on the register-staged norm source only (the QKV block): decode parity, then a
# tg128 A/B against scale-first (g_tune[42] = 1), four interleaved passes at fa 1, two at fa 0
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_ops_gpu.py tests/test_dropin_gpu.py tests/test_dropin_shapes_gpu.py \
  -k "gemv or qkv or norm or glu or incremental_decode or decode or row_split or layer_split" -x -q --timeout 300 --timeout-method thread > gpurun_out/r5_c48_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r5_c48_tests.log; [ $rc -ne 0 ] && exit $rc
PASSES=4 AB="- GGML_MI355X_TUNE=42=1" timeout -k 10 600 bash scripts/r5_ab_env.sh > gpurun_out/r5_c48_fa1.txt 2>&1
rc=$?; cut -c1-140 gpurun_out/r5_c48_fa1.txt; [ $rc -ne 0 ] && exit $rc
FA=0 PASSES=2 AB="- GGML_MI355X_TUNE=42=1" timeout -k 10 600 bash scripts/r5_ab_env.sh > gpurun_out/r5_c48_fa0.txt 2>&1
rc=$?; cut -c1-140 gpurun_out/r5_c48_fa0.txt; exit $rc
