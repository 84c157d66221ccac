#!/bin/bash
# second-box confirmation of round 6's adopted decode changes (interleaved A/B, env switches)
cd "$(dirname "$0")/../../.."
mkdir -p gpurun_out/r6
for pass in a b; do
  MODEL=mixtral_8x7b RECIPE=q5_k_m bash scripts/r6.sh "lb c_mx_on_$pass -fa 1 -p 0 -n 128 -r 3" \
    "envlb c_mx_nodc_$pass GGML_MI355X_NO_MOE_DOWN_COMBINE=1 -- -fa 1 -p 0 -n 128 -r 3" \
    "envlb c_mx_r8_$pass GGML_MI355X_MOE_ROUTER_WG=1 -- -fa 1 -p 0 -n 128 -r 3" || exit 1
  bash scripts/r6.sh "lb c_q8_on_$pass -fa 1 -p 0 -n 128 -r 3 -ctk q8_0 -ctv q8_0" \
    "envlb c_q8_nodefer_$pass GGML_MI355X_NO_KV_DEFER=1 -- -fa 1 -p 0 -n 128 -r 3 -ctk q8_0 -ctv q8_0" \
    "lb c_fa0pp_on_$pass -fa 0 -p 2048 -n 0 -r 3" \
    "envlb c_fa0pp_nocache_$pass GGML_MI355X_NO_MASK_CACHE=1 -- -fa 0 -p 2048 -n 0 -r 3" || exit 1
done
