#!/bin/bash
# Mixtral prefill kernel stats (mixtral_2l, pp512)
cd "$(dirname "$0")/../../.."
mkdir -p gpurun_out/r6
MODEL=mixtral_2l RECIPE=q5_k_m bash scripts/r6.sh "prof prof_mx2l_pp -fa 1 -p 512 -n 0 -r 3"
