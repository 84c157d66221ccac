#!/bin/bash
# round-5 end state: smoke, the full -m gpu suite, then the default bench.py (headline through
# the reference's llama-bench, roofline + PMC lookup, CPU baseline)
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5_final2_smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/r5_final2_smoke.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 1500 python -u -m pytest tests -m gpu -q --timeout 600 --timeout-method thread > gpurun_out/r5_final2_tests.log 2>&1
rc=$?; echo "suite rc=$rc"; tail -4 gpurun_out/r5_final2_tests.log; grep -E "^FAILED|^ERROR" gpurun_out/r5_final2_tests.log | head -20
[ $rc -ge 124 ] && exit $rc
timeout -k 10 900 python bench.py > gpurun_out/r5_bench_final2.json 2> gpurun_out/r5_bench_final2.err; echo "bench rc=$?"; grep '^{' gpurun_out/r5_bench_final2.json | tail -1 | cut -c1-3000
