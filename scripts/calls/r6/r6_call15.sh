#!/bin/bash
# LDS activation-chunk permutation (act_swz) A/B + down-projection geometry sweep
cd "$(dirname "$0")/../../.."
mkdir -p gpurun_out/r6
NS=$PWD/llama-mi50.cpp_amd/lib/noswz/libggml-mi355x.so
P="type_a=(q4_0|q8_0|q4_K|q5_K|q6_K),type_b=f32,m=4096,n=(1|2|3|4|5|6|7|8),k=14336"
bash scripts/r6.sh "tests tests/test_ops_gpu.py -k mul_mat+or+fused+or+norm_absorbed+or+gemv+or+oproj+or+moe+or+grouped" \
  "tests tests/test_dropin_gpu.py -k incremental+or+prefill+or+mixed" \
  "tests tests/test_dropin_shapes_gpu.py -k llama3_8b_width" && \
bash scripts/r6.sh "lb ab_swz1 -fa 1 -p 0 -n 128 -r 5" && \
MXLIB=$NS bash scripts/r6.sh "lb ab_swz0 -fa 1 -p 0 -n 128 -r 5" && \
bash scripts/r6.sh "lb ab_swz1b -fa 1 -p 0 -n 128 -r 5" && \
MXLIB=$NS bash scripts/r6.sh "lb ab_swz0b -fa 1 -p 0 -n 128 -r 5" && \
bash scripts/r6.sh "tbo perf_mm_nc_swz perf -b MI355X0 -o MUL_MAT -p $P" && \
bash scripts/r6.sh "envlb dn_32x8 GGML_MI355X_TUNE=44=32,45=8 -- -fa 1 -p 0 -n 128 -r 5" \
  "envlb dn_64x4 GGML_MI355X_TUNE=44=64,45=4 -- -fa 1 -p 0 -n 128 -r 5" \
  "envlb dn_64x2 GGML_MI355X_TUNE=44=64,45=2 -- -fa 1 -p 0 -n 128 -r 5" \
  "envlb dn_16x4 GGML_MI355X_TUNE=44=16,45=4 -- -fa 1 -p 0 -n 128 -r 5" \
  "envlb dn_32x4 GGML_MI355X_TUNE=44=32,45=4 -- -fa 1 -p 0 -n 128 -r 5" \
  "lb dn_default -fa 1 -p 0 -n 128 -r 5"
