#!/bin/bash
# final default bench.py run (+ the Mixtral leg)
cd "$(dirname "$0")/../../.."
mkdir -p gpurun_out/r6
BTMO=1500 bash scripts/r6.sh "bench --steps 5 --warmup 1 --moe-leg"
