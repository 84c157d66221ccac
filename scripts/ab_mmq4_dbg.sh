#!/bin/bash
# Prefill GEMM skeleton decomposition (one build): the glu / down cases under the k_mmq4
# experiment variants of g_tune[31] (1 no per-chunk wait+barrier, 2 no dequantisation,
# 4 LDS fragments once per chunk, 7 all three, 8 short Q6_K dequant) and g_tune[19] = 12
# (no activation DMA, weights of chunk 0 only). Variants 1/2/4/7 compute wrong results by
# construction (timing only).
cd "$(dirname "$0")/.."
OUT=gpurun_out/mmd bash scripts/opbench.sh --only pp_glu_q4k pp_down_q6k pp_down_q4k \
  --ab 0=0 31=1 31=2 31=4 31=7 31=8 19=12 19=12,31=1 19=12,31=2 19=12,31=4 19=12,31=7 > gpurun_out/mmd.txt 2>&1
rc=$?; cat gpurun_out/mmd/report.txt; exit $rc
