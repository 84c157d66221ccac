#!/bin/bash
# q8_0 LONG decode attention: four heads per workgroup, new-row selects only where the row is
cd "$(dirname "$0")/../../.."
mkdir -p gpurun_out/r6
B=$PWD/llama-mi50.cpp_amd/lib/base/libggml-mi355x.so
bash scripts/r6.sh "tests tests/test_ops_gpu.py -k flash_attn" "tests tests/test_dropin_gpu.py -k q8+or+mixed+or+kv_state" \
  "tests tests/test_dropin_shapes_gpu.py -k depth" || exit 1
for pass in a b; do
  for d in 4096 16384; do
    bash scripts/r6.sh "lb q8_d${d}_new_$pass -fa 1 -p 0 -n 64 -d $d -r 2 -ctk q8_0 -ctv q8_0" && \
    MXLIB=$B bash scripts/r6.sh "lb q8_d${d}_base_$pass -fa 1 -p 0 -n 64 -d $d -r 2 -ctk q8_0 -ctv q8_0" || exit 1
  done
  bash scripts/r6.sh "lb q8kf16v_d16384_new_$pass -fa 1 -p 0 -n 64 -d 16384 -r 2 -ctk q8_0 -ctv f16" && \
  MXLIB=$B bash scripts/r6.sh "lb q8kf16v_d16384_base_$pass -fa 1 -p 0 -n 64 -d 16384 -r 2 -ctk q8_0 -ctv f16" || exit 1
done
