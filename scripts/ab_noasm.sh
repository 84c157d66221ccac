#!/bin/bash
# Same-box A/B of HEAD against its MX_PROLOGUE_ASM=0 build (lib_noasm/): the SwiGLU case of
# tools/opbench.py under the GEMV dbg masks (0 full, 1 no prologue, 2 no dots, 3 neither)
# and the runner tg128, interleaved twice.
cd "$(dirname "$0")/.."
O=$PWD/gpurun_out/noasm
mkdir -p $O
NOASM=$PWD/llama-mi50.cpp_amd/lib_noasm/libggml-mi355x.so
OUT=$O/ob_asm bash scripts/opbench.sh --only ffn_block glu_q4k --dbg 0 1 2 3 > $O/ob_asm.txt 2>&1 || exit 1
GGML_MI355X_LIB=$NOASM OUT=$O/ob_noasm bash scripts/opbench.sh --only ffn_block glu_q4k --dbg 0 1 2 3 > $O/ob_noasm.txt 2>&1 || exit 2
B="--steps 3 --warmup 1 --no-cpu-baseline --no-dropin --skip-roofline --pp 0"
for i in 1 2; do
  timeout -k 10 300 python3 bench.py $B > $O/tg_asm_$i.log 2>&1 || exit 3
  GGML_MI355X_LIB=$NOASM timeout -k 10 300 python3 bench.py $B > $O/tg_noasm_$i.log 2>&1 || exit 4
  echo "$i asm $(grep -o '"value": [0-9.]*' $O/tg_asm_$i.log) noasm $(grep -o '"value": [0-9.]*' $O/tg_noasm_$i.log)"
done
