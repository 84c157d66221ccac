#!/bin/bash
# rocprofv3 kernel stats of the bench's pp512 prefill (graphs off) under two tuning
# settings: per-kernel totals for an A/B of a prefill fusion. Usage: prof_pp_ab.sh A B
cd "$(dirname "$0")/.."
ROOTDIR=$PWD
cd /tmp && export TMPDIR=/tmp && cd "$ROOTDIR"
for t in "$@"; do
  OUT=gpurun_out/ppab_${t//[=,]/_}
  GGML_MI355X_DISABLE_GRAPHS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT -o run --output-format csv -- \
    python3 bench.py --steps 1 --warmup 0 --tg 1 --pp 512 --no-pp2048 --no-cpu-baseline --skip-roofline --no-dropin --tune $t > $OUT.log 2>&1 || exit $?
  echo "== tune $t"; head -14 $OUT/run_kernel_stats.csv | cut -d, -f1-4
done
