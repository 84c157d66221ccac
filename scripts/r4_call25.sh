#!/bin/bash
# drop-in first-repetition cost: per-module lazy code-object loading? (HIP_ENABLE_DEFERRED_LOADING=0 arm)
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
G=${TMPDIR:-/tmp}/mx_bench_llama3_8b_q4_k_m.gguf
[ -f $G ] || timeout -k 10 600 python tools/gguf_synth.py --shape llama3_8b --recipe q4_k_m --out $G > /dev/null || exit 1
for pass in 1 2; do
  for arm in 1 0; do
    r=$(HIP_ENABLE_DEFERRED_LOADING=$arm GGML_BACKEND_PATH=$PWD/llama-mi50.cpp_amd/lib/libggml-mi355x.so timeout -k 10 300 \
        oracle/_ref/ref-llama-bench -m $G -t 8 -ngl 99 -fa 1 -p 512 -n 128 -r 5 2>/dev/null | grep '^{')
    echo "pass=$pass deferred=$arm $(echo $r | grep -o '"pp_samples": \[[^]]*\]') $(echo $r | grep -o '"tg_samples": \[[^]]*\]')"
  done
done
