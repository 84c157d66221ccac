#!/bin/bash
# k_mmq5 (256-token glu) parity + A/B against k_mmq4 (g_tune[3]=8)
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_mmq4_gpu.py > gpurun_out/r4_mmq5_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r4_mmq5_tests.log
[ $rc -eq 0 ] || exit 1
OUT=gpurun_out/mm5 timeout -k 10 500 bash scripts/opbench.sh --only pp_glu_q4k pp_glu_q4k_2048 --ab 0=0 3=8 0=0 3=8 > gpurun_out/r4_mm5.txt 2>&1; echo "ab rc=$?"; grep -E "==|k_mmq" gpurun_out/mm5/report.txt
