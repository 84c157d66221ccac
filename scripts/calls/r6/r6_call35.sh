#!/bin/bash
# round-6 roofline evidence: PMC HBM traffic of bench.py's roofline launch, its rocprofv3 stats,
# and the drop-in decode / prefill kernel stats at HEAD
cd "$(dirname "$0")/../../.."
mkdir -p gpurun_out/r6
OUT=gpurun_out/r6/pmc_roof TMO=500 bash scripts/pmc_roofline.sh || exit 1
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/r6/roof_stats -o run --output-format csv -- python3 bench.py --roofline-only > gpurun_out/r6/roof_stats.log 2>&1 || exit 1
bash scripts/r6.sh "prof prof_tg_final -fa 1 -p 0 -n 128 -r 1" "prof prof_pp_final -fa 1 -p 512 -n 0 -r 3"
