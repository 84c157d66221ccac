#!/bin/bash
# k_mmq5 decomposition (variant build lib_m5x): 31=1 no wait+barrier, 31=2 no dequant,
# 19=4 no activation DMA, 19=8 weights of chunk 0
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
GGML_MI355X_LIB=$PWD/llama-mi50.cpp_amd/lib_m5x/libggml-mi355x.so OUT=gpurun_out/m5d timeout -k 10 500 bash scripts/opbench.sh --only pp_glu_q4k \
  --ab 0=0 0=0 31=1 31=2 31=3 19=4 19=8 19=12 19=12,31=1 19=12,31=3 3=8 > gpurun_out/r4_m5d.txt 2>&1; echo "ab rc=$?"; grep -E "==|k_mmq" gpurun_out/m5d/report.txt
