#!/bin/bash
# multi-column GEMV: 8-row workgroups (g_tune[47] = 32) vs 16 — parity + test-backend-ops perf
cd "$(dirname "$0")/../../.."
mkdir -p gpurun_out/r6
P="type_a=(q4_0|q8_0|q4_K|q5_K|q6_K),type_b=f32,m=4096,n=(2|3|4|5|8),k=14336"
GGML_MI355X_TUNE=47=32 bash scripts/r6.sh "tests tests/test_ops_gpu.py -k mul_mat_multicolumn" || exit 1
for pass in a b; do
  bash scripts/r6.sh "tbo gnc16_$pass perf -b MI355X0 -o MUL_MAT -p $P" && \
  GGML_MI355X_TUNE=47=32 bash scripts/r6.sh "tbo gnc32_$pass perf -b MI355X0 -o MUL_MAT -p $P" || exit 1
done
