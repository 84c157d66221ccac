#!/bin/bash
# launch-geometry knobs re-swept at the round-5 end state (drop-in tg128 -fa 1, two passes):
# QKV geometry (g_tune[12]), SwiGLU 16-wave register staging (4=3), staging mode (9), XCD order (15)
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
PASSES=2 R=3 AB="- GGML_MI355X_TUNE=12=1 GGML_MI355X_TUNE=12=4 GGML_MI355X_TUNE=12=5 GGML_MI355X_TUNE=4=3 GGML_MI355X_TUNE=9=1 GGML_MI355X_TUNE=9=2 GGML_MI355X_TUNE=15=1" \
  timeout -k 10 900 bash scripts/r5_ab_env.sh > gpurun_out/r5_c44.txt 2>&1
rc=$?; cut -c1-140 gpurun_out/r5_c44.txt; exit $rc
