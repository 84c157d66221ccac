#!/bin/bash
cd "$(dirname "$0")/../../.."
mkdir -p gpurun_out/r6; timeout -k 10 900 bash scripts/asan_dropin.sh > gpurun_out/r6/asan.txt 2>&1; rc=$?; tail -14 gpurun_out/r6/asan.txt
[ $rc -ge 124 ] && exit $rc
bash scripts/r6.sh "lb d16k_f16 -fa 1 -p 0 -n 128 -d 16384 -r 3" "lb d16k_q8kv -fa 1 -p 0 -n 128 -d 16384 -r 3 -ctk q8_0 -ctv q8_0" "lb d16k_q8kf16v -fa 1 -p 0 -n 128 -d 16384 -r 3 -ctk q8_0 -ctv f16" && \
BTMO=1500 bash scripts/r6.sh "bench --steps 5 --warmup 1"
