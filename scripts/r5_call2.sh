#!/bin/bash
# round 5: FA split partials merged in the O projection's prologue — op tests, drop-in A/B, profile
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_ops_gpu.py -k "attn_split_oproj or flash_attn or fused_mul_mat_add or attn_oproj" -x -q -s \
    --timeout 300 --timeout-method thread > gpurun_out/r5_c2_tests.log 2>&1
rc=$?; echo "ops tests rc=$rc"; tail -5 gpurun_out/r5_c2_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest tests/test_dropin_shapes_gpu.py -k "8b_width_decode or launch_mix" -x -q -s \
    --timeout 400 --timeout-method thread > gpurun_out/r5_c2_dropin_tests.log 2>&1
rc=$?; echo "dropin tests rc=$rc"; tail -5 gpurun_out/r5_c2_dropin_tests.log; [ $rc -ge 124 ] && exit $rc
PASSES=2 AB="GGML_MI355X_TUNE=32=1 - GGML_MI355X_TUNE=33=2" timeout -k 10 900 bash scripts/r5_ab_env.sh > gpurun_out/r5_fasplit_ab.txt 2>&1
rc=$?; cut -c1-200 gpurun_out/r5_fasplit_ab.txt; [ $rc -ne 0 ] && exit $rc
OUT=gpurun_out/prof_r5_dropin timeout -k 10 400 bash scripts/prof_dropin.sh | head -24
