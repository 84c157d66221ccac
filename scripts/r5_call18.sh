#!/bin/bash
# row split under FORCE_PEER through llama-bench (-ts a/b: llama-bench splits values with '/'), and the -fa 0 depth-16384 decode klog
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
G8=$(python -c "import bench; print(bench.bench_gguf('llama3_8b', 'q4_k_m'))") || exit 1
export GGML_BACKEND_PATH=$PWD/llama-mi50.cpp_amd/lib/libggml-mi355x.so
for pass in 1 2; do
for arm in "none 1 0" "row 1/1 1" "row 1/1/1/1 1" "row 1/1 0"; do
  set -- $arm
  n=$(echo $2 | tr '/' '\n' | wc -l)
  GGML_MI355X_VIRTUAL_DEVICES=$n GGML_MI355X_FORCE_PEER=$3 timeout -k 10 600 oracle/_ref/llama-bench -m $G8 -t 8 -ngl 99 -fa 1 -p 0 -n 128 -sm $1 -ts $2 -r 3 -o jsonl > gpurun_out/rs_$n.log 2>&1 || exit 1
  echo "pass $pass sm=$1 ts=$2 force_peer=$3: $(grep -o '"samples_ts": \[[^]]*\]' gpurun_out/rs_$n.log)"
done; done
GGML_MI355X_KLOG=gpurun_out/klog18_fa0_d16384.txt timeout -k 10 600 oracle/_ref/llama-bench -m $G8 -t 8 -ngl 99 -fa 0 -p 0 -n 2 -d 16384 -r 1 -o jsonl > /dev/null 2>&1 || exit 1
tail -12 gpurun_out/klog18_fa0_d16384.txt
