#!/bin/bash
# eager code-object loading (library constructor; GGML_MI355X_KEEP_DEFERRED_LOADING=1 = old behaviour):
# the bench's drop-in legs, pp512 / pp2048 / tg128 separately, interleaved
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
G=${TMPDIR:-/tmp}/mx_bench_llama3_8b_q4_k_m.gguf
[ -f $G ] || timeout -k 10 600 python tools/gguf_synth.py --shape llama3_8b --recipe q4_k_m --out $G > /dev/null || exit 1
for pass in 1 2; do
  for arm in new old; do
    if [ $arm = old ]; then export GGML_MI355X_KEEP_DEFERRED_LOADING=1; else unset GGML_MI355X_KEEP_DEFERRED_LOADING; fi
    for RUN in "-p 512 -n 0" "-p 2048 -n 0" "-p 0 -n 128"; do
      r=$(GGML_BACKEND_PATH=$PWD/llama-mi50.cpp_amd/lib/libggml-mi355x.so timeout -k 10 300 \
          oracle/_ref/ref-llama-bench -m $G -t 8 -ngl 99 -fa 1 $RUN -r 5 2>/dev/null | grep '^{')
      echo "pass=$pass $arm [$RUN] $(echo $r | grep -o '"pp_tok_s": [0-9.]*') $(echo $r | grep -o '"tg_tok_s": [0-9.]*') $(echo $r | grep -o '"pp_samples": \[[^]]*\]') $(echo $r | grep -o '"tg_samples": \[[^]]*\]')"
    done
  done
done
unset GGML_MI355X_KEEP_DEFERRED_LOADING
