#!/bin/bash
# drop-in prefill: prefill-sized graphs eager (default now) vs captured (GGML_MI355X_PP_GRAPHS=1)
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
G=${TMPDIR:-/tmp}/mx_bench_llama3_8b_q4_k_m.gguf
[ -f $G ] || timeout -k 10 600 python tools/gguf_synth.py --shape llama3_8b --recipe q4_k_m --out $G > /dev/null || exit 1
for pass in 1 2; do
  for arm in eager capture; do
    for P in 512 2048; do
      if [ $arm = capture ]; then export GGML_MI355X_PP_GRAPHS=1; else unset GGML_MI355X_PP_GRAPHS; fi
      r=$(GGML_BACKEND_PATH=$PWD/llama-mi50.cpp_amd/lib/libggml-mi355x.so timeout -k 10 300 \
          oracle/_ref/ref-llama-bench -m $G -t 8 -ngl 99 -fa 1 -p $P -n 0 -r 5 2>/dev/null | grep '^{')
      echo "pass=$pass arm=$arm pp$P $(echo $r | grep -o '"pp_tok_s": [0-9.]*') $(echo $r | grep -o '"pp_samples": \[[^]]*\]')"
    done
  done
done
unset GGML_MI355X_PP_GRAPHS
