#!/bin/bash
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -k "attn_split_oproj" -x -q -s \
    --timeout 200 --timeout-method thread > gpurun_out/r5_c3_tests.log 2>&1
rc=$?; echo "ops tests rc=$rc"; grep -v "^  File" gpurun_out/r5_c3_tests.log | head -30
