#!/bin/bash
# (1) row split ratio with the round's final code; (2) decode weight-prefetch budget A/B (GGML_MI355X_FA_PREFETCH_MB)
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 900 bash scripts/r4_rowsplit.sh > gpurun_out/r4_rowsplit_v2.txt 2>&1; echo "rowsplit rc=$?"; grep -E "tok_s" gpurun_out/r4_rowsplit_v2.txt | head -8
G=${TMPDIR:-/tmp}/mx_bench_llama3_8b_q4_k_m.gguf
for pass in 1 2; do
  for mb in 16 8 24 0; do
    r=$(GGML_MI355X_FA_PREFETCH_MB=$mb GGML_BACKEND_PATH=$PWD/llama-mi50.cpp_amd/lib/libggml-mi355x.so timeout -k 10 300 \
        oracle/_ref/ref-llama-bench -m $G -t 8 -ngl 99 -fa 1 -p 0 -n 128 -r 5 2>/dev/null | grep '^{')
    echo "pass=$pass pf_mb=$mb $(echo $r | grep -o '"tg_tok_s": [0-9.]*') $(echo $r | grep -o '"tg_samples": \[[^]]*\]')"
  done
done
