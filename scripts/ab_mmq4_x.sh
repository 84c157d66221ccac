#!/bin/bash
# k_mmq4 variants (g_tune[31] = X bits, see ops_mmq4.hip) on the prefill GEMM cases, one build
cd "$(dirname "$0")/.."
OUT=gpurun_out/mmx bash scripts/opbench.sh --only ${CASES:-pp_glu_q4k pp_down_q6k pp_down_q4k} --ab ${AB:-0=0 31=16 31=8 31=24 19=12,31=16} > gpurun_out/mmx.txt 2>&1
rc=$?; grep -E '==|k_mmq4<' gpurun_out/mmx/report.txt | paste - - | awk '{print $2, $3}'; exit $rc
