#!/bin/bash
# FA prefill key split (default; g_tune[0]=1 off) parity + A/B; k_mmq5 swapped epilogue (3=32) parity + A/B; k_mmq5 phase sums
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_ops_gpu.py -k "fa or flash or attn" > gpurun_out/r4_faks_tests.log 2>&1; rc=$?; echo "fa tests rc=$rc"; tail -2 gpurun_out/r4_faks_tests.log
[ $rc -eq 0 ] || exit 1
GGML_MI355X_TUNE="3=32" timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_mmq4_gpu.py -k "glu" > gpurun_out/r4_mmq5c_tests.log 2>&1; rc=$?; echo "mmq5 3=32 tests rc=$rc"; tail -2 gpurun_out/r4_mmq5c_tests.log
[ $rc -eq 0 ] || exit 1
OUT=gpurun_out/ab16 timeout -k 10 400 bash scripts/opbench.sh --only fa_pp512 fa_pp2048 pp_glu_q4k --ab 0=0 0=0 0=1 3=32 0=0 0=1 3=32 > gpurun_out/r4_ab16.txt 2>&1; echo "ab rc=$?"; grep -E "==|k_mmq|k_fa" gpurun_out/ab16/report.txt
for tn in 0 32; do
GGML_MI355X_TUNE="3=$tn" GGML_MI355X_LIB=$PWD/llama-mi50.cpp_amd/lib_m5x/libggml-mi355x.so GGML_MI355X_DISABLE_GRAPHS=1 timeout -k 10 200 python3 tools/opbench.py --only pp_glu_q4k --iters 5 --trace > gpurun_out/r4_m5trace_$tn.txt 2>&1; echo "trace $tn rc=$?"; grep trace gpurun_out/r4_m5trace_$tn.txt | head -4
done
timeout -k 10 300 python3 tools/probe_f16_gemm.py > gpurun_out/r4_f16gemm.txt 2>&1; echo "f16 probe rc=$?"; tail -8 gpurun_out/r4_f16gemm.txt
