#!/bin/bash
# drop-in decode A/B: the reference libllama (ref-llama-bench tg128, -r R) under knob sets
# passed through GGML_MI355X_TUNE; AB="0=0 1=4" (one arm per word), interleaved PASSES times
cd "$(dirname "$0")/.."
G=${TMPDIR:-/tmp}/mx_bench_llama3_8b_q4_k_m.gguf
[ -f $G ] || timeout -k 10 600 python tools/gguf_synth.py --shape llama3_8b --recipe q4_k_m --out $G > /dev/null || exit 1
for pass in $(seq ${PASSES:-2}); do
  for arm in ${AB:-0=0}; do
    r=$(GGML_MI355X_TUNE=$arm GGML_BACKEND_PATH=$PWD/llama-mi50.cpp_amd/lib/libggml-mi355x.so timeout -k 10 300 \
        oracle/_ref/ref-llama-bench -m $G -t 8 -ngl 99 -fa ${FA:-1} -p 0 -n 128 -c 256 -r ${R:-5} ${EXTRA:-} 2>/dev/null | grep '^{')
    echo "pass=$pass arm=$arm $(echo $r | grep -o '"tg_tok_s": [0-9.]*') $(echo $r | grep -o '"tg_samples": \[[^]]*\]')"
  done
done
