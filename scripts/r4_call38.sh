#!/bin/bash
# row split: captured split graphs (default on one GPU) vs eager (GGML_MI355X_SPLIT_GRAPHS=0), with the per-slice fusions
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
G=${TMPDIR:-/tmp}/mx_bench_llama3_8b_q4_k_m.gguf
[ -f $G ] || timeout -k 10 600 python tools/gguf_synth.py --shape llama3_8b --recipe q4_k_m --out $G > /dev/null || exit 1
for pass in 1 2; do
  for arm in 1 0; do
    r=$(GGML_MI355X_SPLIT_GRAPHS=$arm GGML_MI355X_VIRTUAL_DEVICES=2 GGML_BACKEND_PATH=$PWD/llama-mi50.cpp_amd/lib/libggml-mi355x.so timeout -k 10 300 \
        oracle/_ref/ref-llama-bench -m $G -t 8 -ngl 99 -fa 1 -p 512 -n 128 -r 3 -sm row -ts 1,1 2>/dev/null | grep '^{')
    echo "pass=$pass split_graphs=$arm $(echo $r | grep -o '"pp_tok_s": [0-9.]*') $(echo $r | grep -o '"tg_tok_s": [0-9.]*') $(echo $r | grep -o '"tg_samples": \[[^]]*\]')"
  done
done
r=$(GGML_BACKEND_PATH=$PWD/llama-mi50.cpp_amd/lib/libggml-mi355x.so timeout -k 10 300 oracle/_ref/ref-llama-bench -m $G -t 8 -ngl 99 -fa 1 -p 512 -n 128 -r 3 2>/dev/null | grep '^{')
echo "unsplit $(echo $r | grep -o '"pp_tok_s": [0-9.]*') $(echo $r | grep -o '"tg_tok_s": [0-9.]*')"
