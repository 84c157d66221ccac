#!/bin/bash
# rocprofv3 kernel trace of the bench decode, HIP graphs on (the production path). Under
# rocprofv3 the CLR's graph packet capture is turned off (DEBUG_CLR_GRAPH_PACKET_CAPTURE=0):
# with it on, rocprofiler-sdk faults in hipGraphLaunch. GRAPHS=0: eager.
cd "$(dirname "$0")/.."
OUT=${OUT:-gpurun_out/prof}
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
[ "${GRAPHS:-1}" = 0 ] && export GGML_MI355X_DISABLE_GRAPHS=1
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -k 10 ${TMO:-600} rocprofv3 --kernel-trace --stats -d $OUT -o run --output-format csv -- \
  python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline ${PROF_ARGS:---pp 0} > $OUT.log 2>&1
rc=$?
echo "prof rc=$rc"; head -25 $OUT/run_kernel_stats.csv
exit $rc
