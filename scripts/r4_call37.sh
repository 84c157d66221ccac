#!/bin/bash
# per-slice fused SwiGLU + residual GEMVs for local row splits: split tests, then -sm row A/B (GGML_MI355X_NO_SPLIT_FUSION=1 = before)
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_dropin_gpu.py tests/test_dropin_shapes_gpu.py -k "split or row" > gpurun_out/r4_splitfuse_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r4_splitfuse_tests.log
[ $rc -eq 0 ] || exit 1
G=${TMPDIR:-/tmp}/mx_bench_llama3_8b_q4_k_m.gguf
[ -f $G ] || timeout -k 10 600 python tools/gguf_synth.py --shape llama3_8b --recipe q4_k_m --out $G > /dev/null || exit 1
for pass in 1 2; do
  for arm in new old; do
    if [ $arm = old ]; then export GGML_MI355X_NO_SPLIT_FUSION=1; else unset GGML_MI355X_NO_SPLIT_FUSION; fi
    r=$(GGML_MI355X_VIRTUAL_DEVICES=2 GGML_BACKEND_PATH=$PWD/llama-mi50.cpp_amd/lib/libggml-mi355x.so timeout -k 10 300 \
        oracle/_ref/ref-llama-bench -m $G -t 8 -ngl 99 -fa 1 -p 0 -n 128 -r 3 -sm row -ts 1,1 2>/dev/null | grep '^{')
    echo "pass=$pass $arm row2 $(echo $r | grep -o '"tg_tok_s": [0-9.]*') $(echo $r | grep -o '"tg_samples": \[[^]]*\]')"
  done
done
unset GGML_MI355X_NO_SPLIT_FUSION
