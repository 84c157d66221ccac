#!/bin/bash
# full -m gpu suite + smoke + bench (defaults: k_mmq5 glu, FA key split)
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 840 python -u -m pytest tests -m gpu -q --timeout 600 --timeout-method thread > gpurun_out/r4_full_tests6.log 2>&1
rc=$?; echo "suite rc=$rc"; tail -4 gpurun_out/r4_full_tests6.log; grep -E "^FAILED|^ERROR" gpurun_out/r4_full_tests2.log | head -20
[ $rc -ge 124 ] && exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4_smoke6.log 2>&1; echo "smoke rc=$?"; tail -2 gpurun_out/r4_smoke2.log
timeout -k 10 600 python bench.py > gpurun_out/r4_bench_v6.json 2> gpurun_out/r4_bench_v6.err; echo "bench rc=$?"; grep '^{' gpurun_out/r4_bench_v6.json | tail -1 | cut -c1-1500
