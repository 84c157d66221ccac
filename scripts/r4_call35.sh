#!/bin/bash
# decode kernel counters (runner tg, graphs off under --pmc): SQ wait/issue shares and FETCH bytes per kernel
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
CMD="python3 bench.py --mode single --steps 1 --warmup 0 --tg 32 --no-cpu-baseline --no-dropin --skip-roofline --no-pp2048"
OUT=gpurun_out/pmc_dec_sq COUNTERS="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE" KFILTER="k_gemv2|k_fattn|k_qkv|k_attn" TMO=400 bash scripts/pmc_sq.sh $CMD; echo "sq rc=$?"
OUT=gpurun_out/pmc_dec_fetch COUNTERS="FETCH_SIZE GRBM_GUI_ACTIVE" KFILTER="k_gemv2|k_fattn|k_qkv|k_attn" TMO=400 bash scripts/pmc_sq.sh $CMD; echo "fetch rc=$?"
