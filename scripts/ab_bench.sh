#!/bin/bash
# decode bench (tg128 only) under alternative tuning knobs: AB="14=0 14=1" (one arm per word;
# commas join knobs within an arm)
cd "$(dirname "$0")/.."
for arm in ${AB:-0=0}; do
  timeout -k 10 300 python bench.py --steps ${STEPS_N:-3} --warmup 1 --no-cpu-baseline --skip-roofline --pp 0 --tune ${arm//,/ } > gpurun_out/ab_$arm.log 2>&1 || exit $?
  echo "arm=$arm $(grep -o '"value": [0-9.]*' gpurun_out/ab_$arm.log)"
done
