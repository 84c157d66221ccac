#!/bin/bash
# MoE router in one 1024-thread workgroup: parity, Mixtral tg128 A/B, profile
cd "$(dirname "$0")/../../.."
mkdir -p gpurun_out/r6
bash scripts/r6.sh "tests tests/test_ops_gpu.py -k moe" "tests tests/test_dropin_gpu.py -k tiny_moe" "tests tests/test_dropin_shapes_gpu.py -k mixtral" && \
MODEL=mixtral_2l RECIPE=q5_k_m bash scripts/r6.sh "prof prof_mx2l_tg_r1 -fa 1 -p 0 -n 64 -c 256 -r 1" && \
MODEL=mixtral_8x7b RECIPE=q5_k_m bash scripts/r6.sh "lb mx_tg_r1 -fa 1 -p 0 -n 128 -r 3" \
  "envlb mx_tg_r8 GGML_MI355X_MOE_ROUTER_WG=1 -- -fa 1 -p 0 -n 128 -r 3" \
  "lb mx_tg_r1b -fa 1 -p 0 -n 128 -r 3" \
  "envlb mx_tg_r8b GGML_MI355X_MOE_ROUTER_WG=1 -- -fa 1 -p 0 -n 128 -r 3" \
  "lb mx_pp -fa 1 -p 512 -n 0 -r 3"
