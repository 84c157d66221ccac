#!/bin/bash
# k_mmq5 interleaved issue: parity + A/B (0 interleaved, 3=16 burst, 3=8 k_mmq4)
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_mmq4_gpu.py -k "glu" > gpurun_out/r4_mmq5b_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r4_mmq5b_tests.log
[ $rc -eq 0 ] || exit 1
OUT=gpurun_out/mm5b timeout -k 10 500 bash scripts/opbench.sh --only pp_glu_q4k pp_glu_q4k_2048 --ab 0=0 0=0 3=16 3=8 0=0 3=16 3=8 > gpurun_out/r4_mm5b.txt 2>&1; echo "ab rc=$?"; grep -E "==|k_mmq" gpurun_out/mm5b/report.txt
