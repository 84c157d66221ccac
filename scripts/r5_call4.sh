#!/bin/bash
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
PASSES=2 AB="- GGML_MI355X_TUNE=33=8 GGML_MI355X_FA_PREFETCH_MB=8 GGML_MI355X_FA_PREFETCH_MB=24 GGML_MI355X_FA_PREFETCH_MB=0" \
  timeout -k 10 900 bash scripts/r5_ab_env.sh > gpurun_out/r5_c4_ab.txt 2>&1
rc=$?; cut -c1-200 gpurun_out/r5_c4_ab.txt; exit $rc
