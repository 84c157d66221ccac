#!/bin/bash
# row split (-sm row -ts 1,1) over two virtual devices of one MI355X vs unsplit: tg128 and
# pp512 through the reference libllama; then the split tests
cd "$(dirname "$0")/.."
G=${TMPDIR:-/tmp}/mx_bench_llama3_8b_q4_k_m.gguf
[ -f $G ] || timeout -k 10 600 python tools/gguf_synth.py --shape llama3_8b --recipe q4_k_m --out $G > /dev/null || exit 1
L=$PWD/llama-mi50.cpp_amd/lib/libggml-mi355x.so
for arm in "unsplit|" "row2|-sm row -ts 1,1" "row2_peer|-sm row -ts 1,1|GGML_MI355X_FORCE_PEER=1" "row2_nocapture|-sm row -ts 1,1|GGML_MI355X_SPLIT_GRAPHS=0" "row4|-sm row -ts 1,1,1,1|GGML_MI355X_VIRTUAL_DEVICES=4"; do
  name=${arm%%|*}; rest=${arm#*|}; flags=${rest%%|*}; envx=""; [ "$rest" != "$flags" ] && envx=${rest#*|}
  r=$(env GGML_MI355X_VIRTUAL_DEVICES=2 GGML_MI355X_STATS=1 $envx GGML_BACKEND_PATH=$L timeout -k 10 300 oracle/_ref/ref-llama-bench -m $G -t 8 -ngl 99 -fa 1 -p 512 -n 128 -r 3 $flags 2> gpurun_out/rowsplit_$name.err | grep '^{')
  echo "$name: $(echo $r | grep -o '"pp_tok_s": [0-9.]*') $(echo $r | grep -o '"tg_tok_s": [0-9.]*')"
done
