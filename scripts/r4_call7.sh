#!/bin/bash
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
GGML_MI355X_TUNE="3=3" timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_mmq4_gpu.py > gpurun_out/r4_mmq4_x64_tests.log 2>&1; echo "x64 tests rc=$?"; tail -2 gpurun_out/r4_mmq4_x64_tests.log
OUT=gpurun_out/mm5s timeout -k 10 500 bash scripts/opbench.sh --only pp_glu_q4k pp_down_q4k pp_down_q6k pp_qkv --ab 0=0 3=3 0=0 3=3 > gpurun_out/r4_mm5s.txt 2>&1; echo "ab rc=$?"; grep -E "==|k_mmq4<" gpurun_out/mm5s/report.txt
