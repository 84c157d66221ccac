#!/bin/bash
# Mixtral decode: QKV geometry (g_tune[12]) — the Q8_0 k rows take 4 batches at cfg 5
cd "$(dirname "$0")/../../.."
mkdir -p gpurun_out/r6
for pass in a b; do
  MODEL=mixtral_8x7b RECIPE=q5_k_m bash scripts/r6.sh "lb mxq_def_$pass -fa 1 -p 0 -n 128 -r 3" \
    "envlb mxq_c3_$pass GGML_MI355X_TUNE=12=4 -- -fa 1 -p 0 -n 128 -r 3" \
    "envlb mxq_c0_$pass GGML_MI355X_TUNE=12=1 -- -fa 1 -p 0 -n 128 -r 3" || exit 1
done
