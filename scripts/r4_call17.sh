#!/bin/bash
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python3 tools/probe_f16_gemm.py > gpurun_out/r4_f16gemm.txt 2>&1; echo "rc=$?"; cat gpurun_out/r4_f16gemm.txt | tail -8
