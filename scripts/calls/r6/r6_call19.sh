#!/bin/bash
# depth-16384 decode kernel stats: f16 vs q8_0 KV
cd "$(dirname "$0")/../../.."
mkdir -p gpurun_out/r6
bash scripts/r6.sh "prof prof_d16k_q8 -fa 1 -p 0 -n 32 -d 16384 -r 1 -ctk 8"
