#!/bin/bash
# -fa 0 prefill: the f16 mask converted once per graph pass — parity + same-box A/B
cd "$(dirname "$0")/../../.."
mkdir -p gpurun_out/r6
bash scripts/r6.sh "tests tests/test_ops_gpu.py -k nofa+or+staged" "tests tests/test_dropin_gpu.py -k prefill+or+incremental+or+layer_split" \
  "tests tests/test_dropin_shapes_gpu.py -k pp512+or+pp2048+or+prefill" || exit 1
for pass in a b; do
  bash scripts/r6.sh "lb fa0pp_new_$pass -fa 0 -p 512,2048 -n 0 -r 3" && \
  bash scripts/r6.sh "envlb fa0pp_old_$pass GGML_MI355X_NO_MASK_CACHE=1 -- -fa 0 -p 512,2048 -n 0 -r 3" || exit 1
done
