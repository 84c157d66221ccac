#!/bin/bash
# kernel-choice logs of the drop-in decode at depth 0 and depth 16384 (why the decode fusions drop at depth)
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
G8=$(python -c "import bench; print(bench.bench_gguf('llama3_8b', 'q4_k_m'))") || exit 1
export GGML_BACKEND_PATH=$PWD/llama-mi50.cpp_amd/lib/libggml-mi355x.so
for d in 0 16384; do
  GGML_MI355X_STATS=1 GGML_MI355X_KLOG=gpurun_out/klog_d$d.txt timeout -k 10 600 oracle/_ref/llama-bench -m $G8 -t 8 -ngl 99 -fa 1 -p 0 -n 4 -d $d -r 1 -o jsonl > gpurun_out/klog_d$d.log 2>&1 || exit 1
  wc -l gpurun_out/klog_d$d.txt; grep stats gpurun_out/klog_d$d.log | cut -c1-300
done
