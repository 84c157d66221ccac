#!/bin/bash
# Current drop-in decode profiles (graphs on): tg128 -fa 1 and -fa 0, kernel stats
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
G=$(python -c "import bench; print(bench.bench_gguf('llama3_8b', 'q4_k_m'))") || exit 1
ROOTDIR=$PWD; cd /tmp && export TMPDIR=/tmp && cd "$ROOTDIR"
export GGML_BACKEND_PATH=$PWD/llama-mi50.cpp_amd/lib/libggml-mi355x.so DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
for fa in 1 0; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_tg_fa$fa -o run --output-format csv -- \
    oracle/_ref/llama-bench -m $G -t 8 -ngl 99 -fa $fa -p 0 -n 128 -r 1 -o jsonl > gpurun_out/prof_tg_fa$fa.log 2>&1
  rc=$?; echo "fa$fa rc=$rc"; [ $rc -ne 0 ] && exit $rc
  head -16 gpurun_out/prof_tg_fa$fa/run_kernel_stats.csv | cut -c1-160
done
