#!/bin/bash
# L2 counters of k_mmq5 vs k_mmq4 on the pp512 glu
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
OUT=gpurun_out/pmc_m5_tcc COUNTERS="TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum GRBM_GUI_ACTIVE" KFILTER="k_mmq" \
  bash scripts/pmc_sq.sh python3 tools/opbench.py --only pp_glu_q4k --iters 10 --ab 0=0 3=8
echo "rc=$?"
OUT=gpurun_out/pmc_m5_tcp COUNTERS="TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TA_BUSY_avr TD_BUSY_avr GRBM_GUI_ACTIVE" KFILTER="k_mmq" \
  bash scripts/pmc_sq.sh python3 tools/opbench.py --only pp_glu_q4k --iters 10 --ab 0=0 3=8
echo "rc=$?"
