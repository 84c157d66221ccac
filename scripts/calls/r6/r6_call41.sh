#!/bin/bash
# closing check at the round's last commit: smoke() and the default bench.py line
cd "$(dirname "$0")/../../.."
mkdir -p gpurun_out/r6
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6/smoke_head.log 2>&1 || exit 1
BTMO=1200 bash scripts/r6.sh "bench --steps 5 --warmup 1"
