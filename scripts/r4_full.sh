#!/bin/bash
# full -m gpu suite + smoke + default bench (the round-end driver's three steps)
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 840 python -u -m pytest tests -m gpu -q --timeout 600 --timeout-method thread > gpurun_out/r4_full_tests.log 2>&1
rc=$?; echo "suite rc=$rc"; tail -4 gpurun_out/r4_full_tests.log; grep -E "^FAILED|^ERROR" gpurun_out/r4_full_tests.log | head -20
[ $rc -ge 124 ] && exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4_smoke.log 2>&1; echo "smoke rc=$?"; tail -2 gpurun_out/r4_smoke.log
