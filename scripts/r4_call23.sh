#!/bin/bash
# round-4 roofline evidence: PMC HBM traffic of the roofline kernel + its rocprofv3 --stats summary
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
OUT=gpurun_out/pmc4 bash scripts/pmc_roofline.sh > gpurun_out/r4_pmc.txt 2>&1; echo "pmc rc=$?"; tail -5 gpurun_out/r4_pmc.txt
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_roof -o run --output-format csv -- python3 bench.py --roofline-only > gpurun_out/prof_roof.log 2>&1; echo "roof stats rc=$?"; grep '^{' gpurun_out/prof_roof.log | tail -1 | cut -c1-400
