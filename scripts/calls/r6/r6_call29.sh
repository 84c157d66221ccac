#!/bin/bash
# prefill Q6_K dequantisation as one packed FMA per pair — parity + same-box A/B + profile
cd "$(dirname "$0")/../../.."
mkdir -p gpurun_out/r6
B=$PWD/llama-mi50.cpp_amd/lib/base/libggml-mi355x.so
bash scripts/r6.sh "tests tests/test_mmq4_gpu.py" "tests tests/test_ops_gpu.py -k mul_mat_quant_prefill+or+grouped+or+mul_mat_quant" \
  "tests tests/test_dropin_gpu.py -k prefill" "tests tests/test_dropin_shapes_gpu.py -k pp512+or+prefill" || exit 1
bash scripts/r6.sh "prof prof_pp512_q6fma -fa 1 -p 512 -n 0 -r 3" || exit 1
for pass in a b; do
  bash scripts/r6.sh "lb pp_q6fma_$pass -fa 1 -p 512,2048 -n 0 -r 3" && \
  MXLIB=$B bash scripts/r6.sh "lb pp_base_$pass -fa 1 -p 512,2048 -n 0 -r 3" || exit 1
done
