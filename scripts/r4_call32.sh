#!/bin/bash
# compact graph signature: graph/drop-in GPU tests, then drop-in tg128 A/B against the previous library (lib_sigold)
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_llama_gpu.py tests/test_dropin_gpu.py > gpurun_out/r4_sig_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r4_sig_tests.log
[ $rc -eq 0 ] || exit 1
G=${TMPDIR:-/tmp}/mx_bench_llama3_8b_q4_k_m.gguf
[ -f $G ] || timeout -k 10 600 python tools/gguf_synth.py --shape llama3_8b --recipe q4_k_m --out $G > /dev/null || exit 1
for pass in 1 2 3; do
  for lib in lib lib_sigold; do
    r=$(GGML_MI355X_STATS=1 GGML_BACKEND_PATH=$PWD/llama-mi50.cpp_amd/$lib/libggml-mi355x.so timeout -k 10 300 \
        oracle/_ref/ref-llama-bench -m $G -t 8 -ngl 99 -fa 1 -p 0 -n 128 -r 5 2>gpurun_out/sig_$lib.err | grep '^{')
    echo "pass=$pass $lib $(echo $r | grep -o '"tg_tok_s": [0-9.]*') $(echo $r | grep -o '"tg_samples": \[[^]]*\]') $(grep -o '"signature": [0-9.]*' gpurun_out/sig_$lib.err | head -1)"
  done
done
