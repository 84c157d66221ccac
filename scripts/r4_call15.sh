#!/bin/bash
# k_mmq5: swapped-operand epilogue (g_tune[3]=32) parity + A/B; phase cycle sums (variant lib)
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
GGML_MI355X_TUNE="3=32" timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_mmq4_gpu.py -k "glu" > gpurun_out/r4_mmq5c_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r4_mmq5c_tests.log
[ $rc -eq 0 ] || exit 1
OUT=gpurun_out/mm5c timeout -k 10 400 bash scripts/opbench.sh --only pp_glu_q4k pp_glu_q4k_2048 --ab 0=0 0=0 3=32 0=0 3=32 > gpurun_out/r4_mm5c.txt 2>&1; echo "ab rc=$?"; grep -E "==|k_mmq" gpurun_out/mm5c/report.txt
for tn in 0 32; do
GGML_MI355X_TUNE="3=$tn" GGML_MI355X_LIB=$PWD/llama-mi50.cpp_amd/lib_m5x/libggml-mi355x.so GGML_MI355X_DISABLE_GRAPHS=1 timeout -k 10 200 python3 tools/opbench.py --only pp_glu_q4k --iters 5 --trace > gpurun_out/r4_m5trace_$tn.txt 2>&1; echo "trace $tn rc=$?"; grep trace gpurun_out/r4_m5trace_$tn.txt | head -4
done
