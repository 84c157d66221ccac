#!/bin/bash
# second-box A/B: k_fattn_dec3 (default) vs the LONG kernel + combine (GGML_MI355X_FA_STREAM=0), tg128 at depth 4096 / 16384
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
G8=$(python -c "import bench; print(bench.bench_gguf('llama3_8b', 'q4_k_m'))") || exit 1
export GGML_BACKEND_PATH=$PWD/llama-mi50.cpp_amd/lib/libggml-mi355x.so
for pass in 1 2 3; do for d in 4096 16384; do for arm in 1 0; do
  GGML_MI355X_FA_STREAM=$arm timeout -k 10 600 oracle/_ref/llama-bench -m $G8 -t 8 -ngl 99 -fa 1 -p 0 -n 128 -d $d -r 3 -o jsonl > gpurun_out/fs_$arm.log 2>&1 || exit 1
  echo "pass $pass d=$d stream=$arm: $(grep -o '"samples_ts": \[[^]]*\]' gpurun_out/fs_$arm.log)"
done; done; done
