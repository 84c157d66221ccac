#!/bin/bash
# row split under FORCE_PEER: captured vs eager (SPLIT_GRAPHS=0), and a kernel trace of the captured -ts 1/1 decode
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
G8=$(python -c "import bench; print(bench.bench_gguf('llama3_8b', 'q4_k_m'))") || exit 1
export GGML_BACKEND_PATH=$PWD/llama-mi50.cpp_amd/lib/libggml-mi355x.so
for sg in 1 0; do
  GGML_MI355X_SPLIT_GRAPHS=$sg GGML_MI355X_VIRTUAL_DEVICES=2 GGML_MI355X_FORCE_PEER=1 timeout -k 10 600 oracle/_ref/llama-bench -m $G8 -t 8 -ngl 99 -fa 1 -p 0 -n 128 -sm row -ts 1/1 -r 3 -o jsonl > gpurun_out/rs_sg$sg.log 2>&1 || exit 1
  echo "split_graphs=$sg: $(grep -o '"samples_ts": \[[^]]*\]' gpurun_out/rs_sg$sg.log)"
done
GGML_MI355X_VIRTUAL_DEVICES=2 GGML_MI355X_FORCE_PEER=1 DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -k 10 600 rocprofv3 --kernel-trace -d gpurun_out/prof_rs -o run --output-format csv -- \
  oracle/_ref/llama-bench -m $G8 -t 8 -ngl 99 -fa 1 -p 0 -n 32 -sm row -ts 1/1 -r 1 -o jsonl > gpurun_out/prof_rs.log 2>&1 || exit 1
python tools/trace_gaps.py gpurun_out/prof_rs/run_kernel_trace.csv --gap-us 20 | head -40
