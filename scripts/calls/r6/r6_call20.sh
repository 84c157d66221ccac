#!/bin/bash
# q8_0 KV at depth 16384: LONG-geometry heads per workgroup (g_tune[29]) / keys per lane (g_tune[28])
cd "$(dirname "$0")/../../.."
mkdir -p gpurun_out/r6
A="-fa 1 -p 0 -n 64 -d 16384 -r 2 -ctk q8_0 -ctv q8_0"
bash scripts/r6.sh "lb dq_def $A" "envlb dq_g4 GGML_MI355X_TUNE=29=4 -- $A" "envlb dq_g1 GGML_MI355X_TUNE=29=1 -- $A" \
  "envlb dq_ni16 GGML_MI355X_TUNE=28=16 -- $A" "envlb dq_ni4 GGML_MI355X_TUNE=28=4 -- $A" "envlb dq_g4ni16 GGML_MI355X_TUNE=29=4,28=16 -- $A" \
  "lb dq_def2 $A"
