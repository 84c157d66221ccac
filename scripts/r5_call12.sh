#!/bin/bash
# (1) Mixtral pp512 MoE GEMMs at 64-token tiles (GGML_MI355X_TUNE=18=2) vs default, kernel stats
# (2) 8B drop-in tg128 at depth 16384: llama-bench + kernel stats (FA per layer at 16k)
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
G=$(python -c "import bench; print(bench.bench_gguf('mixtral_8x7b', 'q5_k_m'))") || exit 1
export GGML_BACKEND_PATH=$PWD/llama-mi50.cpp_amd/lib/libggml-mi355x.so DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
for arm in 18=2 0=0; do
  GGML_MI355X_TUNE=$arm timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_moe5_$arm -o run --output-format csv -- \
    oracle/_ref/llama-bench -m $G -t 8 -ngl 99 -fa 1 -p 512 -n 0 -r 3 -o jsonl > gpurun_out/prof_moe5_$arm.log 2>&1 || exit 1
  echo "arm $arm: $(grep -o '"samples_ts": \[[^]]*\]' gpurun_out/prof_moe5_$arm.log)"
  head -6 gpurun_out/prof_moe5_$arm/run_kernel_stats.csv | cut -c1-120
done
G8=$(python -c "import bench; print(bench.bench_gguf('llama3_8b', 'q4_k_m'))") || exit 1
timeout -k 10 600 oracle/_ref/llama-bench -m $G8 -t 8 -ngl 99 -fa 1 -p 0 -n 128 -d 16384 -r 3 -o jsonl > gpurun_out/d16k_tg.log 2>&1 || exit 1
echo "d16k: $(grep -o '"samples_ts": \[[^]]*\]' gpurun_out/d16k_tg.log)"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_d16k -o run --output-format csv -- \
    oracle/_ref/llama-bench -m $G8 -t 8 -ngl 99 -fa 1 -p 0 -n 128 -d 16384 -r 1 -o jsonl > gpurun_out/prof_d16k.log 2>&1 || exit 1
head -16 gpurun_out/prof_d16k/run_kernel_stats.csv | cut -c1-140
