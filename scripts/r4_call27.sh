#!/bin/bash
# multi-slot graph cache: graph-sensitive GPU tests, then drop-in A/B (GGML_MI355X_GRAPH_SLOTS=1 = one capture)
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_dropin_gpu.py tests/test_llama_gpu.py > gpurun_out/r4_slots_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r4_slots_tests.log
[ $rc -eq 0 ] || exit 1
G=${TMPDIR:-/tmp}/mx_bench_llama3_8b_q4_k_m.gguf
[ -f $G ] || timeout -k 10 600 python tools/gguf_synth.py --shape llama3_8b --recipe q4_k_m --out $G > /dev/null || exit 1
for pass in 1 2; do
  for arm in 8 1; do
    for RUN in "-p 512 -n 0" "-p 2048 -n 0" "-p 0 -n 128" "-p 512 -n 128"; do
      r=$(GGML_MI355X_GRAPH_SLOTS=$arm GGML_BACKEND_PATH=$PWD/llama-mi50.cpp_amd/lib/libggml-mi355x.so timeout -k 10 300 \
          oracle/_ref/ref-llama-bench -m $G -t 8 -ngl 99 -fa 1 $RUN -r 5 2>/dev/null | grep '^{')
      echo "pass=$pass slots=$arm [$RUN] $(echo $r | grep -o '"pp_tok_s": [0-9.]*') $(echo $r | grep -o '"tg_tok_s": [0-9.]*') $(echo $r | grep -o '"pp_samples": \[[^]]*\]') $(echo $r | grep -o '"tg_samples": \[[^]]*\]')"
    done
  done
done
