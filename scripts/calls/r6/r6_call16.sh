#!/bin/bash
# multi-column GEMV with two register stages: parity + test-backend-ops perf table
cd "$(dirname "$0")/../../.."
mkdir -p gpurun_out/r6
P="type_a=(q4_0|q8_0|q4_K|q5_K|q6_K),type_b=f32,m=4096,n=(1|2|3|4|5|6|7|8),k=14336"
bash scripts/r6.sh "tests tests/test_ops_gpu.py -k mul_mat_multicolumn+or+mul_mat_quant" && \
bash scripts/r6.sh "tbo perf_mm_nc2 perf -b MI355X0 -o MUL_MAT -p $P" && \
bash scripts/r6.sh "tbo mm_test2 test -b MI355X0 -o MUL_MAT" && \
bash scripts/r6.sh "lb tg_check -fa 1 -p 0 -n 128 -r 3"
