#!/bin/bash
# host ASan drop-in runs at HEAD
cd "$(dirname "$0")/../../.."
mkdir -p gpurun_out/r6
timeout -k 10 900 bash scripts/asan_dropin.sh > gpurun_out/r6/asan_final.txt 2>&1; rc=$?; tail -14 gpurun_out/r6/asan_final.txt; exit $rc
