#!/bin/bash
# row split tests incl. the local-slice fused path (klog glu_split / mm_split_add), logits vs the reference CPU run
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_dropin_gpu.py -k "row_split" > gpurun_out/r4_rowsplit_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/r4_rowsplit_tests.log | tail -8
