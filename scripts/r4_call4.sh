#!/bin/bash
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
T="python -u -m pytest -v --timeout 600 --timeout-method thread -m gpu"
timeout -k 10 900 $T tests/test_dropin_shapes_gpu.py tests/test_dropin_gpu.py -k "launch_mix or 8b_width_decode or 70b_width_decode" > gpurun_out/r4_c4_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "PASSED|FAILED|^E " gpurun_out/r4_c4_tests.log | head -30
[ $rc -ge 124 ] && exit $rc
G=${TMPDIR:-/tmp}/mx_bench_llama3_8b_q4_k_m.gguf
[ -f $G ] || timeout -k 10 600 python tools/gguf_synth.py --shape llama3_8b --recipe q4_k_m --out $G > /dev/null
L=$PWD/llama-mi50.cpp_amd/lib/libggml-mi355x.so
for arm in "" "GGML_MI355X_DISABLE_GRAPHS=1"; do
  r=$(env $arm GGML_BACKEND_PATH=$L timeout -k 10 300 oracle/_ref/ref-llama-bench -m $G -t 8 -ngl 99 -fa 1 -p 512 -n 0 -r 8 2>/dev/null | grep '^{')
  echo "pp512 r8 [$arm] $(echo $r | grep -o '"pp_samples": \[[^]]*\]')"
done
for pass in 1 2; do
  r=$(GGML_BACKEND_PATH=$L timeout -k 10 300 oracle/_ref/ref-llama-bench -m $G -t 8 -ngl 99 -fa 1 -p 0 -n 128 -r 5 2>/dev/null | grep '^{')
  echo "tg128 $(echo $r | grep -o '"tg_tok_s": [0-9.]*')"
  r=$(GGML_BACKEND_PATH=$L timeout -k 10 300 oracle/_ref/ref-llama-bench -m $G -t 8 -ngl 99 -fa 0 -p 0 -n 128 -r 5 2>/dev/null | grep '^{')
  echo "tg128 fa0 $(echo $r | grep -o '"tg_tok_s": [0-9.]*')"
done
