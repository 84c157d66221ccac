#!/bin/bash
# q8_0 decode attention: new-row quantisation only where needed, V scale folded — parity + same-box A/B
cd "$(dirname "$0")/../../.."
mkdir -p gpurun_out/r6
B=$PWD/llama-mi50.cpp_amd/lib/base/libggml-mi355x.so
bash scripts/r6.sh "tests tests/test_ops_gpu.py -k flash_attn" "tests tests/test_dropin_gpu.py -k q8+or+mixed+or+incremental+or+kv_state" \
  "tests tests/test_dropin_shapes_gpu.py -k depth" || exit 1
for pass in a b; do
  bash scripts/r6.sh "lb q8d0_new_$pass -fa 1 -p 0 -n 128 -r 3 -ctk q8_0 -ctv q8_0" && \
  MXLIB=$B bash scripts/r6.sh "lb q8d0_base_$pass -fa 1 -p 0 -n 128 -r 3 -ctk q8_0 -ctv q8_0" && \
  bash scripts/r6.sh "lb q8d8k_new_$pass -fa 1 -p 0 -n 64 -d 8192 -r 2 -ctk q8_0 -ctv q8_0" && \
  MXLIB=$B bash scripts/r6.sh "lb q8d8k_base_$pass -fa 1 -p 0 -n 64 -d 8192 -r 2 -ctk q8_0 -ctv q8_0" && \
  bash scripts/r6.sh "lb q8kf16v_new_$pass -fa 1 -p 0 -n 128 -r 3 -ctk q8_0 -ctv f16" && \
  MXLIB=$B bash scripts/r6.sh "lb q8kf16v_base_$pass -fa 1 -p 0 -n 128 -r 3 -ctk q8_0 -ctv f16" || exit 1
done
