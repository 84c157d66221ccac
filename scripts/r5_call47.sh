#!/bin/bash
# RMS scale applied after the dots for register-staged norm sources (XStage::postscale): op and
# decode parity, then tg128 A/B against the scale-first path (g_tune[42] = 1), same binary
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_ops_gpu.py tests/test_dropin_gpu.py tests/test_dropin_shapes_gpu.py \
  -k "gemv or qkv or norm or glu or incremental_decode or decode or row_split or layer_split" -x -q --timeout 300 --timeout-method thread > gpurun_out/r5_c47_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r5_c47_tests.log; grep -E "^FAILED|Error|assert" gpurun_out/r5_c47_tests.log | head -5; [ $rc -ne 0 ] && exit $rc
PASSES=3 AB="- GGML_MI355X_TUNE=42=1" timeout -k 10 600 bash scripts/r5_ab_env.sh > gpurun_out/r5_c47_fa1.txt 2>&1
rc=$?; cut -c1-140 gpurun_out/r5_c47_fa1.txt; [ $rc -ne 0 ] && exit $rc
FA=0 PASSES=2 AB="- GGML_MI355X_TUNE=42=1" timeout -k 10 600 bash scripts/r5_ab_env.sh > gpurun_out/r5_c47_fa0.txt 2>&1
rc=$?; cut -c1-140 gpurun_out/r5_c47_fa0.txt; exit $rc
