#!/bin/bash
# SQ counters of k_mmq5 vs k_mmq4 on the pp512 glu (opbench, one pass)
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
OUT=gpurun_out/pmc_m5 COUNTERS="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE" KFILTER="k_mmq" \
  bash scripts/pmc_sq.sh python3 tools/opbench.py --only pp_glu_q4k --iters 10 --ab 0=0 3=8
echo "rc=$?"
