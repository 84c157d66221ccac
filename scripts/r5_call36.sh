#!/bin/bash
# Second-box confirmation of the round-5 decode A/Bs under 3 %:
# fa 1: default vs split-O off (g_tune[32] = 1) vs the 16 MB weight prefetch under the attention;
# fa 0: default vs the split-O -fa 0 path off. Three interleaved passes each.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
PASSES=3 AB="- GGML_MI355X_TUNE=32=1 GGML_MI355X_FA_PREFETCH_MB=16" timeout -k 10 600 bash scripts/r5_ab_env.sh > gpurun_out/r5_c36_fa1.txt 2>&1
rc=$?; cut -c1-150 gpurun_out/r5_c36_fa1.txt; [ $rc -ne 0 ] && exit $rc
FA=0 PASSES=3 AB="- GGML_MI355X_NO_NOFA_SPLIT_O=1" timeout -k 10 600 bash scripts/r5_ab_env.sh > gpurun_out/r5_c36_fa0.txt 2>&1
rc=$?; cut -c1-150 gpurun_out/r5_c36_fa0.txt; exit $rc
