#!/bin/bash
# host-side time of the drop-in pp512 (executor stats: set_async bytes / time, graph_compute, synchronize)
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
G8=$(python -c "import bench; print(bench.bench_gguf('llama3_8b', 'q4_k_m'))") || exit 1
export GGML_BACKEND_PATH=$PWD/llama-mi50.cpp_amd/lib/libggml-mi355x.so
GGML_MI355X_STATS=1 timeout -k 10 600 oracle/_ref/llama-bench -m $G8 -t 8 -ngl 99 -fa 1 -p 512 -n 0 -r 10 -o jsonl > gpurun_out/pp_stats.log 2>&1 || exit 1
grep -o '"samples_ts": \[[^]]*\]' gpurun_out/pp_stats.log; grep "mi355x\] stats" gpurun_out/pp_stats.log | cut -c1-700
