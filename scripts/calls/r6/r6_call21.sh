#!/bin/bash
# LONG-geometry keys per lane (g_tune[28] = 16 vs the default) across depths and cache types
cd "$(dirname "$0")/../../.."
mkdir -p gpurun_out/r6
steps=()
for d in 4096 8192 16384; do
  for ct in "f16:" "q8kv:-ctk q8_0 -ctv q8_0" "q8kf16v:-ctk q8_0 -ctv f16"; do
    n=${ct%%:*}; f=${ct#*:}
    steps+=("lb s_${n}_d${d}_def -fa 1 -p 0 -n 64 -d $d -r 2 $f")
    steps+=("envlb s_${n}_d${d}_ni16 GGML_MI355X_TUNE=28=16 -- -fa 1 -p 0 -n 64 -d $d -r 2 $f")
  done
done
steps+=("lb s_q8kv_d0_def -fa 1 -p 0 -n 128 -r 3 -ctk q8_0 -ctv q8_0" "envlb s_q8kv_d0_ni16 GGML_MI355X_TUNE=28=16 -- -fa 1 -p 0 -n 128 -r 3 -ctk q8_0 -ctv q8_0")
steps+=("lb s_f16_d0_def -fa 1 -p 0 -n 128 -r 3" "envlb s_f16_d0_ni16 GGML_MI355X_TUNE=28=16 -- -fa 1 -p 0 -n 128 -r 3")
bash scripts/r6.sh "${steps[@]}"
