#!/bin/bash
cd "$(dirname "$0")/../../.."
P="type_a=(q4_0|q8_0|q4_K|q6_K),type_b=f32,m=4096,n=(1|2|3|4),k=14336"
bash scripts/r6.sh "tests tests/test_dropin_gpu.py tests/test_dropin_shapes_gpu.py tests/test_ops_gpu.py -k row_split+or+mul_mat" && \
bash scripts/r6.sh "tbo perf_mm_v4 perf -b MI355X0 -o MUL_MAT -p $P" && \
bash scripts/r6.sh "lb rs_none -fa 1 -p 0 -n 128 -r 3" && \
GGML_MI355X_VIRTUAL_DEVICES=2 GGML_MI355X_FORCE_PEER=1 bash scripts/r6.sh "lb rs_2 -fa 1 -p 0 -n 128 -r 3 -sm row -ts 1/1" && \
GGML_MI355X_VIRTUAL_DEVICES=4 GGML_MI355X_FORCE_PEER=1 bash scripts/r6.sh "lb rs_4 -fa 1 -p 0 -n 128 -r 3 -sm row -ts 1/1/1/1" && \
GGML_MI355X_VIRTUAL_DEVICES=2 GGML_MI355X_FORCE_PEER=1 GGML_MI355X_SPLIT_FAP=1 bash scripts/r6.sh "lb rs_2_fap -fa 1 -p 0 -n 128 -r 3 -sm row -ts 1/1"
