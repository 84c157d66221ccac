#!/bin/bash
# QKV geometry cfg 3 (Q/K 32 lanes x 2 units, V 32 x 2: g_tune[12] = 4) against the default cfg 5,
# four interleaved passes at fa 1 (the end-state sweep put it at +0.3 %)
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
PASSES=4 AB="- GGML_MI355X_TUNE=12=4" timeout -k 10 600 bash scripts/r5_ab_env.sh > gpurun_out/r5_c49_fa1.txt 2>&1
rc=$?; cut -c1-140 gpurun_out/r5_c49_fa1.txt; exit $rc
