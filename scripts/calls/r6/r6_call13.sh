#!/bin/bash
cd "$(dirname "$0")/../../.."
mkdir -p gpurun_out/r6; timeout -k 10 900 bash scripts/asan_dropin.sh > gpurun_out/r6/asan.txt 2>&1; rc=$?; tail -14 gpurun_out/r6/asan.txt
[ $rc -ge 124 ] && exit $rc
bash scripts/r6.sh "tests tests/test_dropin_gpu.py -k q8+or+mixed+or+incremental"
