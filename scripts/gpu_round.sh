#!/bin/bash
# One GPU session: smoke, gpu tests, bench, rocprof. Stops at the first crash/timeout
# (exit >= 124 or signal) so a faulting kernel is never re-run; plain test failures
# (rc 1) do not stop the later measurement steps.
cd "$(dirname "$0")/.."
OUT=${OUT:-gpurun_out}
mkdir -p $OUT
step() {  # name timeout cmd...
  local name=$1 tmo=$2; shift 2
  echo "== $name"
  timeout -k 10 $tmo "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -n ${TAILN:-15} $OUT/$name.log
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "stopping: $name rc=$rc"; exit $rc; fi
  return 0
}
for s in ${STEPS:-smoke tests bench prof}; do
  case $s in
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    tests) step tests 900 python -m pytest tests -m gpu -x -q ${PYTEST_ARGS:-} ;;
    refops) step refops 1200 env OUT=$OUT/refops bash scripts/gpu_ref_ops.sh ;;
    opbench) step opbench 900 bash scripts/opbench.sh ${OPBENCH_ARGS:-} ;;
    bench) step bench 900 python bench.py ${BENCH_ARGS:---steps 3 --warmup 1} ;;
    prof) cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
          step prof 900 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline ${PROF_ARGS:-} ;;
  esac
done
