#!/bin/bash
# second A/B of GGML_MI355X_GRAPH_UPLOAD=1 (tg128 and pp2048, interleaved, three pairs / two pairs)
cd "$(dirname "$0")/../../.."
mkdir -p gpurun_out/r6
bash scripts/r6.sh "envlb up2_on_t1 GGML_MI355X_GRAPH_UPLOAD=1 -- -p 0 -n 128 -fa 1 -r 5" "lb up2_base_t1 -p 0 -n 128 -fa 1 -r 5" \
  "envlb up2_on_t2 GGML_MI355X_GRAPH_UPLOAD=1 -- -p 0 -n 128 -fa 1 -r 5" "lb up2_base_t2 -p 0 -n 128 -fa 1 -r 5" \
  "lb up2_base_t3 -p 0 -n 128 -fa 1 -r 5" "envlb up2_on_t3 GGML_MI355X_GRAPH_UPLOAD=1 -- -p 0 -n 128 -fa 1 -r 5" \
  "envlb up2_on_p1 GGML_MI355X_GRAPH_UPLOAD=1 -- -p 2048 -n 0 -fa 1 -r 5" "lb up2_base_p1 -p 2048 -n 0 -fa 1 -r 5" \
  "lb up2_base_p2 -p 2048 -n 0 -fa 1 -r 5" "envlb up2_on_p2 GGML_MI355X_GRAPH_UPLOAD=1 -- -p 2048 -n 0 -fa 1 -r 5"
