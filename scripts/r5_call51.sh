#!/bin/bash
# Mixtral-8x7B Q5_K_M leg at HEAD (bench.py --moe-only): drop-in tg128 / pp512 through llama-bench
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 1100 python bench.py --moe-only --dropin-reps 3 > gpurun_out/r5_moe_final.json 2> gpurun_out/r5_moe_final.err
rc=$?; echo "moe leg rc=$rc"; grep '^{' gpurun_out/r5_moe_final.json | tail -1 | cut -c1-1500; exit $rc
