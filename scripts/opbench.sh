#!/bin/bash
# Per-op decode micro-benchmark under rocprofv3 (see tools/opbench.py).
cd "$(dirname "$0")/.."
OUT=${OUT:-gpurun_out/ob}
mkdir -p $OUT
ROOTDIR=$PWD
cd /tmp && export TMPDIR=/tmp && cd "$ROOTDIR"
export OPBENCH_CASES=$OUT/cases.txt
GGML_MI355X_DISABLE_GRAPHS=1 timeout -k 10 ${TMO:-400} rocprofv3 --kernel-trace -d $OUT -o ob --output-format csv -- \
  python3 tools/opbench.py "$@" > $OUT/log.txt 2>&1
rc=$?
echo "opbench rc=$rc"
[ $rc -ne 0 ] && { tail -20 $OUT/log.txt; exit $rc; }
python3 tools/opbench_report.py $OUT/ob_kernel_trace.csv $OUT/cases.txt | tee $OUT/report.txt
