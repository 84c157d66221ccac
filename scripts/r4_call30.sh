#!/bin/bash
# drop-in tg128 kernel stats, graphs on: -fa 0 vs -fa 1
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
OUT=gpurun_out/prof_tg_fa0 FA=0 TMO=300 bash scripts/prof_dropin.sh > gpurun_out/r4_prof_tg_fa0.txt 2>&1; echo "fa0 rc=$?"
OUT=gpurun_out/prof_tg_fa1 FA=1 TMO=300 bash scripts/prof_dropin.sh > gpurun_out/r4_prof_tg_fa1.txt 2>&1; echo "fa1 rc=$?"
