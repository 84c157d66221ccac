#!/bin/bash
# drop-in A/B over environment arms: AB="A=1 B=0,C=1" (one arm per word, commas separate
# several assignments of one arm; "-" = no extra env), interleaved PASSES times.
# ref-llama-bench tg128 (-r R) through the reference libllama on this backend.
cd "$(dirname "$0")/.."
G=${TMPDIR:-/tmp}/mx_bench_llama3_8b_q4_k_m.gguf
[ -f $G ] || timeout -k 10 600 python tools/gguf_synth.py --shape llama3_8b --recipe q4_k_m --out $G > /dev/null || exit 1
for pass in $(seq ${PASSES:-2}); do
  for arm in ${AB:--}; do
    envs=""; [ "$arm" != "-" ] && envs=$(echo $arm | tr ',' ' ')
    r=$(env $envs GGML_MI355X_STATS=1 GGML_BACKEND_PATH=$PWD/llama-mi50.cpp_amd/lib/libggml-mi355x.so timeout -k 10 300 \
        oracle/_ref/ref-llama-bench -m $G -t 8 -ngl 99 -fa ${FA:-1} -p ${PP:-0} -n ${NG:-128} -c ${CTX:-256} -r ${R:-5} ${EXTRA:-} 2>/tmp/ab_err.txt | grep '^{')
    rc=$?
    st=$(grep -o '"host_us": {[^}]*}, "n_set[^}]*}' /tmp/ab_err.txt | tail -1)
    echo "pass=$pass arm=$arm $(echo $r | grep -o '"tg_tok_s": [0-9.]*') $(echo $r | grep -o '"pp_tok_s": [0-9.]*') $(echo $r | grep -o '"tg_samples": \[[^]]*\]') stats=$st"
  done
done
