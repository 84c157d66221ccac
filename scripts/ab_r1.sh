#!/bin/bash
# Same-box A/B of the round-1 build (ab_r1/: `git archive 3bdaf0b`, built in place) against
# HEAD: runner tg128, the isolated SwiGLU roofline launch, the drop-in tg128 through the
# reference libllama (GGML_BACKEND_PATH = either library), interleaved twice.
# Stops at the first failing step.
cd "$(dirname "$0")/.."
O=gpurun_out/ab
mkdir -p $O
B="--steps 3 --warmup 1 --no-cpu-baseline --skip-roofline --pp 0"
GGUF=$(python3 -c "import bench; print(bench.bench_gguf())") || exit 1
for i in 1 2; do
  (cd ab_r1 && timeout -k 10 300 python3 bench.py $B > ../$O/r1_tg_$i.log 2>&1) || exit 11
  timeout -k 10 300 python3 bench.py $B --no-dropin > $O/head_tg_$i.log 2>&1 || exit 12
  (cd ab_r1 && timeout -k 10 300 python3 bench.py --roofline-only > ../$O/r1_roof_$i.log 2>&1) || exit 13
  timeout -k 10 300 python3 bench.py --roofline-only > $O/head_roof_$i.log 2>&1 || exit 14
  for v in r1 head; do
    lib=llama-mi50.cpp_amd/lib/libggml-mi355x.so; [ $v = r1 ] && lib=ab_r1/$lib
    GGML_BACKEND_PATH=$PWD/$lib timeout -k 10 300 oracle/_ref/ref-llama-bench -m $GGUF -t 8 -ngl 99 -fa 1 -p 0 -n 128 -r 5 -c 256 \
      > $O/${v}_dropin_$i.log 2>&1 || exit 15
  done
  echo "round $i"
  for v in r1 head; do
    echo "$v tg $(grep -o '"value": [0-9.]*' $O/${v}_tg_$i.log) roof $(grep -o '"avg_launch_us": [0-9.]*' $O/${v}_roof_$i.log) dropin $(grep -o '"tg_tok_s": [0-9.]*' $O/${v}_dropin_$i.log)"
  done
done
