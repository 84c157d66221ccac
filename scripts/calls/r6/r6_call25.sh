#!/bin/bash
# MoE prefill: partial last token tiles on a 64-token launch — parity, Mixtral pp512 A/B, profile
cd "$(dirname "$0")/../../.."
mkdir -p gpurun_out/r6
bash scripts/r6.sh "tests tests/test_mmq4_gpu.py -k moe" "tests tests/test_dropin_gpu.py -k tiny_moe" "tests tests/test_dropin_shapes_gpu.py -k mixtral" && \
MODEL=mixtral_2l RECIPE=q5_k_m bash scripts/r6.sh "prof prof_mx2l_pp_tail -fa 1 -p 512 -n 0 -r 3" && \
MODEL=mixtral_8x7b RECIPE=q5_k_m bash scripts/r6.sh "lb mxpp_tail -fa 1 -p 512 -n 0 -r 3" \
  "envlb mxpp_notail GGML_MI355X_MOE_TAIL_OFF=1 -- -fa 1 -p 512 -n 0 -r 3" \
  "lb mxpp_tail2 -fa 1 -p 512 -n 0 -r 3" \
  "envlb mxpp_notail2 GGML_MI355X_MOE_TAIL_OFF=1 -- -fa 1 -p 512 -n 0 -r 3"
