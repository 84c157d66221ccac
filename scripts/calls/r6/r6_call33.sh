#!/bin/bash
# shipped library: smoke + decode/prefill drop-in subset
cd "$(dirname "$0")/../../.."
mkdir -p gpurun_out/r6
timeout -k 10 600 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r6/smoke.log 2>&1; rc=$?; tail -3 gpurun_out/r6/smoke.log; [ $rc -eq 0 ] || exit $rc
bash scripts/r6.sh "tests tests/test_dropin_gpu.py -k prefill+or+incremental" "lb tg_final -fa 1 -p 0 -n 128 -r 3"
