#!/bin/bash
# rocprofv3 kernel trace of the bench decode (HIP graphs off: rocprofv3 + hipGraph
# instantiate crashes in this ROCm; kernel durations are unaffected).
cd "$(dirname "$0")/.."
OUT=${OUT:-gpurun_out/prof}
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
GGML_MI355X_DISABLE_GRAPHS=1 timeout -k 10 ${TMO:-600} rocprofv3 --kernel-trace --stats -d $OUT -o run --output-format csv -- \
  python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline ${PROF_ARGS:---pp 0} > $OUT.log 2>&1
rc=$?
echo "prof rc=$rc"; head -25 $OUT/run_kernel_stats.csv
exit $rc
