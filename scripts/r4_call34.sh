#!/bin/bash
# one-round-trip split merge (k_fattn_dec2_combine2): parity, opbench A/B (g_tune[2]=11: round-3 merge), drop-in depth A/B
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_ops_gpu.py -k "fa or flash or attn" > gpurun_out/r4_comb_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r4_comb_tests.log
[ $rc -eq 0 ] || exit 1
OUT=gpurun_out/comb timeout -k 10 400 bash scripts/opbench.sh --only fa_4096 fa_16384 fa_32768 --ab 0=0 0=0 2=11 0=0 2=11 > gpurun_out/r4_comb.txt 2>&1; echo "ab rc=$?"; grep -E "==|fattn" gpurun_out/comb/report.txt
G=${TMPDIR:-/tmp}/mx_bench_llama3_8b_q4_k_m.gguf
[ -f $G ] || timeout -k 10 600 python tools/gguf_synth.py --shape llama3_8b --recipe q4_k_m --out $G > /dev/null || exit 1
for pass in 1 2; do
  for arm in 0=0 2=11; do
    for d in 4096 16384; do
      r=$(GGML_MI355X_TUNE=$arm GGML_BACKEND_PATH=$PWD/llama-mi50.cpp_amd/lib/libggml-mi355x.so timeout -k 10 300 \
          oracle/_ref/ref-llama-bench -m $G -t 8 -ngl 99 -fa 1 -p 0 -n 128 -d $d -r 3 2>/dev/null | grep '^{')
      echo "pass=$pass arm=$arm d=$d $(echo $r | grep -o '"tg_tok_s": [0-9.]*') $(echo $r | grep -o '"tg_samples": \[[^]]*\]')"
    done
  done
done
