#!/bin/bash
# the tests that counted klog lines twice (eager pass + the capture behind it)
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_dropin_shapes_gpu.py tests/test_shapes_gpu.py -k "pp512 or pp2048 or launch_mix or ffn_block" -q --timeout 600 --timeout-method thread > gpurun_out/r5_c25.log 2>&1
rc=$?; echo "rc=$rc"; tail -3 gpurun_out/r5_c25.log; grep -E "^E  .*(Assert|assert)" gpurun_out/r5_c25.log | head -10
