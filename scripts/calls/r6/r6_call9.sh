#!/bin/bash
cd "$(dirname "$0")/../../.."
bash scripts/r6.sh "tests tests/test_ops_gpu.py tests/test_refops_gpu.py tests/test_shapes_gpu.py -k mul_mat+or+MUL_MAT+or+glu+or+ffn" && \
bash scripts/r6.sh "tbo perf_mulmat_v2 perf -b MI355X0 -o MUL_MAT -p type_a=(q4_0|q8_0|q4_K|q5_K|q6_K),type_b=f32,m=4096,n=(1|2|3|4|5|8),k=14336" && \
MODEL=llama3_70b LTMO=900 bash scripts/r6.sh "lb b70 -fa 1 -p 512 -n 128 -r 3"
