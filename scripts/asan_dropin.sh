#!/bin/bash
# Host-side AddressSanitizer run: the reference libllama (oracle/_ref) drives
# lib/asan/libggml-mi355x.so — the backend's host code instrumented (make -C
# llama-mi50.cpp_amd asan), device code not — through prefill and incremental decode at
# -fa 1 / -fa 0 and with q8_0 / mixed KV caches, graph capture and replay on, plus a row
# split over two logical devices and a KV-state save / restore. Any ASan report fails it.
cd "$(dirname "$0")/.."
OUT=${OUT:-gpurun_out/asan}
mkdir -p $OUT
RT=$(gcc -print-file-name=libasan.so)   # GCC's runtime (Makefile: clang's intercepts HSA allocations)
LIB=$PWD/llama-mi50.cpp_amd/lib/asan/libggml-mi355x.so
G=$OUT/small.gguf
[ -f $G ] || python tools/gguf_synth.py --shape small --recipe q4_k_m --out $G > /dev/null || exit 1
python -c "import numpy as np; np.random.default_rng(3).integers(0, 1000, 40).astype(np.int32).tofile('$OUT/t.i32')"
export ASAN_OPTIONS=detect_leaks=0:abort_on_error=0:halt_on_error=1:exitcode=66
fail=0
run() {  # name args...
  local name=$1; shift
  env LD_PRELOAD=$RT GGML_BACKEND_PATH=$LIB "$@" > $OUT/$name.log 2>&1
  local rc=$?
  local nrep=$(grep -c "ERROR: AddressSanitizer" $OUT/$name.log)
  echo "$name rc=$rc asan_reports=$nrep"
  if [ $rc -ne 0 ] || [ $nrep -ne 0 ]; then fail=1; grep -A 12 "ERROR: AddressSanitizer" $OUT/$name.log | head -40; fi
  if [ $rc -ge 124 ] && [ $rc -ne 66 ]; then echo "stopping: $name rc=$rc"; exit $rc; fi
}
R=oracle/_ref/ref-llama-bench
for fa in 1 0; do
  run pre_fa$fa timeout -k 10 300 $R -m $G -t 8 -ngl 99 -fa $fa --logits $OUT/t.i32 $OUT/o.f32
  run inc_fa$fa timeout -k 10 300 $R -m $G -t 8 -ngl 99 -fa $fa --logits $OUT/t.i32 $OUT/o.f32 --incremental
done
run inc_q8kv timeout -k 10 300 $R -m $G -t 8 -ngl 99 -fa 1 -ctk 8 --logits $OUT/t.i32 $OUT/o.f32 --incremental
run inc_q8k_f16v timeout -k 10 300 $R -m $G -t 8 -ngl 99 -fa 1 -ctk 8 -ctv 1 --logits $OUT/t.i32 $OUT/o.f32 --incremental
run bench_tg timeout -k 10 300 $R -m $G -t 8 -ngl 99 -fa 1 -p 64 -n 32 -r 2
run row_split env GGML_MI355X_VIRTUAL_DEVICES=2 GGML_MI355X_FORCE_PEER=1 timeout -k 10 300 $R -m $G -t 8 -ngl 99 -fa 1 \
    -sm row -ts 1,1 --logits $OUT/t.i32 $OUT/o.f32 --incremental
run layer_split env GGML_MI355X_VIRTUAL_DEVICES=2 GGML_MI355X_FORCE_PEER=1 timeout -k 10 300 $R -m $G -t 8 -ngl 99 -fa 1 \
    -sm layer -ts 1,1 --logits $OUT/t.i32 $OUT/o.f32
python -c "import numpy as np; r=np.random.default_rng(4); r.integers(0,1000,37).astype(np.int32).tofile('$OUT/p.i32'); r.integers(0,1000,6).astype(np.int32).tofile('$OUT/g.i32')"
run kv_state timeout -k 10 300 oracle/_ref/state-probe -m $G -fa 1 --prompt $OUT/p.i32 --gen $OUT/g.i32 --out $OUT
echo "asan_dropin fail=$fail"
exit $fail
