#!/bin/bash
# Same-box A/B of GEMV build variants (lib_<name>/ built with EXTRA defines, see
# scripts/build_variants.sh): the isolated decode SwiGLU launch (bench.py --roofline-only)
# and the runner tg128, interleaved twice. VARIANTS="head one0 ext0 both" by default.
cd "$(dirname "$0")/.."
O=$PWD/gpurun_out/abv
mkdir -p $O
B="--steps 3 --warmup 1 --no-cpu-baseline --no-dropin --skip-roofline --pp 0"
for i in 1 2; do
  for v in ${VARIANTS:-head one0 ext0 both}; do
    L=""; [ "$v" != head ] && L=$PWD/llama-mi50.cpp_amd/lib_$v/libggml-mi355x.so
    GGML_MI355X_LIB=$L timeout -k 10 240 python3 bench.py --roofline-only > $O/roof_${v}_$i.log 2>&1 || { echo "$v roof failed"; exit 1; }
    GGML_MI355X_LIB=$L timeout -k 10 300 python3 bench.py $B > $O/tg_${v}_$i.log 2>&1 || { echo "$v tg failed"; exit 2; }
    echo "$i $v $(grep -o '"avg_launch_us": [0-9.]*' $O/roof_${v}_$i.log) tg $(grep -o '"value": [0-9.]*' $O/tg_${v}_$i.log)"
  done
done
