#!/bin/bash
# rocprofv3 kernel trace of the bench's pp512 prefill (HIP graphs off, see prof_decode.sh).
cd "$(dirname "$0")/.."
OUT=${OUT:-gpurun_out/profpp}
ROOTDIR=$PWD
cd /tmp && export TMPDIR=/tmp && cd "$ROOTDIR"
GGML_MI355X_DISABLE_GRAPHS=1 timeout -k 10 ${TMO:-600} rocprofv3 --kernel-trace --stats -d $OUT -o run --output-format csv -- \
  python3 bench.py --steps 1 --warmup 0 --tg 1 --pp 512 --no-cpu-baseline --skip-roofline > $OUT.log 2>&1
rc=$?
echo "profpp rc=$rc"; head -25 $OUT/run_kernel_stats.csv | cut -c1-160
exit $rc
