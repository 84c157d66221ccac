#!/bin/bash
cd "$(dirname "$0")/../../.."
mkdir -p gpurun_out/r6
P="type_a=(q4_0|q8_0|q4_K|q5_K|q6_K),type_b=f32,m=4096,n=(1|2|3|4|5|6|7|8),k=14336"
bash scripts/r6.sh "tests tests/test_ops_gpu.py -k mul_mat_multicolumn+or+mul_mat_quant" && \
bash scripts/r6.sh "tbo perf_mm_nc perf -b MI355X0 -o MUL_MAT -p $P" && \
GGML_MI355X_GEMV_NC_OFF=1 bash scripts/r6.sh "tbo perf_mm_nc_off perf -b MI355X0 -o MUL_MAT -p $P" && \
bash scripts/r6.sh "tbo mm_test test -b MI355X0 -o MUL_MAT"
timeout -k 10 900 bash scripts/asan_dropin.sh > gpurun_out/r6/asan.txt 2>&1; rc=$?; tail -14 gpurun_out/r6/asan.txt
exit $rc
