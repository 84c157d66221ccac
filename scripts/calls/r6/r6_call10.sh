#!/bin/bash
cd "$(dirname "$0")/../../.."
P="type_a=(q4_0|q8_0|q4_K|q6_K),type_b=f32,m=4096,n=(1|2|3|4|5|8),k=14336"
bash scripts/r6.sh "tests tests/test_ops_gpu.py tests/test_dropin_shapes_gpu.py -k mul_mat+or+mixtral" && \
bash scripts/r6.sh "tbo perf_mm_v3 perf -b MI355X0 -o MUL_MAT -p $P" && \
GGML_MI355X_TUNE=41=32 bash scripts/r6.sh "tbo perf_mm_v3_l32 perf -b MI355X0 -o MUL_MAT -p $P" && \
GGML_MI355X_TUNE=43=4 bash scripts/r6.sh "tbo perf_mm_v3_u4 perf -b MI355X0 -o MUL_MAT -p $P" && \
GGML_MI355X_TUNE=44=1 bash scripts/r6.sh "tbo perf_mm_v3_old perf -b MI355X0 -o MUL_MAT -p $P" && \
MODEL=mixtral_2l RECIPE=q5_k_m bash scripts/r6.sh "prof prof_mx2l_tg -fa 1 -p 0 -n 64 -c 256 -r 1" && \
MODEL=mixtral_2l RECIPE=q5_k_m GGML_MI355X_TUNE=45=1 bash scripts/r6.sh "prof prof_mx2l_tg_acqrel -fa 1 -p 0 -n 64 -c 256 -r 1"
