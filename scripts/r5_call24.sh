#!/bin/bash
# full -m gpu suite + bench (real llama-bench headline, FA split path)
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 600 --timeout-method thread > gpurun_out/r5_full_tests2.log 2>&1
rc=$?; echo "suite rc=$rc"; tail -4 gpurun_out/r5_full_tests2.log; grep -E "^FAILED|^ERROR" gpurun_out/r5_full_tests2.log | head -20
[ $rc -ge 124 ] && exit $rc
timeout -k 10 600 python bench.py > gpurun_out/r5_bench_v2.json 2> gpurun_out/r5_bench_v2.err; echo "bench rc=$?"; grep '^{' gpurun_out/r5_bench_v2.json | tail -1 | cut -c1-2500
