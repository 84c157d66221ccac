#!/bin/bash
# k_mmq5 per-wave cycle sums of workgroup 0 (prologue, chunk-head wait+barrier, compute, epilogue)
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
GGML_MI355X_LIB=$PWD/llama-mi50.cpp_amd/lib_m5x/libggml-mi355x.so GGML_MI355X_DISABLE_GRAPHS=1 timeout -k 10 300 python3 tools/opbench.py --only pp_glu_q4k pp_glu_q4k_2048 --iters 5 --trace > gpurun_out/r4_m5trace.txt 2>&1; echo "rc=$?"; grep trace gpurun_out/r4_m5trace.txt | head -20
