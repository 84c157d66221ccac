#!/bin/bash
# A/B: hipGraphUpload right behind the first-sighting instantiate (GGML_MI355X_GRAPH_UPLOAD=1)
# against the default, interleaved: llama-bench's first timed repetition of pp512 / pp2048
cd "$(dirname "$0")/../../.."
mkdir -p gpurun_out/r6
bash scripts/r6.sh "lb up_base_a -p 512 -n 0 -fa 1 -r 5" "envlb up_on_a GGML_MI355X_GRAPH_UPLOAD=1 -- -p 512 -n 0 -fa 1 -r 5" \
  "lb up_base_b -p 512 -n 0 -fa 1 -r 5" "envlb up_on_b GGML_MI355X_GRAPH_UPLOAD=1 -- -p 512 -n 0 -fa 1 -r 5" \
  "lb up_base_c -p 2048 -n 0 -fa 1 -r 5" "envlb up_on_c GGML_MI355X_GRAPH_UPLOAD=1 -- -p 2048 -n 0 -fa 1 -r 5" \
  "lb up_base_d -p 0 -n 128 -fa 1 -r 5" "envlb up_on_d GGML_MI355X_GRAPH_UPLOAD=1 -- -p 0 -n 128 -fa 1 -r 5"
