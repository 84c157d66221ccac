#!/bin/bash
# staged-write/free test; pp2048 -fa 0 vs -fa 1 kernel stats
cd "$(dirname "$0")/../../.."
mkdir -p gpurun_out/r6
bash scripts/r6.sh "tests tests/test_ops_gpu.py -k staged_write" && \
bash scripts/r6.sh "prof prof_pp2048_fa0 -fa 0 -p 2048 -n 0 -r 1" "prof prof_pp2048_fa1 -fa 1 -p 2048 -n 0 -r 1"
