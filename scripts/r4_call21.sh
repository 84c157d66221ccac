#!/bin/bash
# in-model prefill kernel stats: drop-in pp512 (fa1) and the runner pp512
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
OUT=gpurun_out/prof_dpp RUN="-p 512 -n 0 -c 512" TMO=300 bash scripts/prof_dropin.sh > gpurun_out/r4_prof_dpp.txt 2>&1; echo "dropin pp rc=$?"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_rpp -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --tg 8 --no-cpu-baseline --no-dropin --skip-roofline --no-pp2048 > gpurun_out/prof_rpp.log 2>&1; echo "runner pp rc=$?"
