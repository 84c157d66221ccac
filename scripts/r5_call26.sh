#!/bin/bash
# pp512 ramp: llama-bench -r 15 (does the drop-in plateau at the runner's rate?), and the same after a warm tg run
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
G8=$(python -c "import bench; print(bench.bench_gguf('llama3_8b', 'q4_k_m'))") || exit 1
export GGML_BACKEND_PATH=$PWD/llama-mi50.cpp_amd/lib/libggml-mi355x.so
timeout -k 10 600 oracle/_ref/llama-bench -m $G8 -t 8 -ngl 99 -fa 1 -p 512 -n 0 -r 15 -o jsonl > gpurun_out/pp_r15.log 2>&1 || exit 1
echo "pp512 -r 15: $(grep -o '"samples_ts": \[[^]]*\]' gpurun_out/pp_r15.log)"
timeout -k 10 600 oracle/_ref/llama-bench -m $G8 -t 8 -ngl 99 -fa 1 -p 2048 -n 0 -r 10 -o jsonl > gpurun_out/pp2k_r10.log 2>&1 || exit 1
echo "pp2048 -r 10: $(grep -o '"samples_ts": \[[^]]*\]' gpurun_out/pp2k_r10.log)"
timeout -k 10 600 python bench.py --mode single --no-dropin --no-cpu-baseline --skip-roofline --steps 3 > gpurun_out/runner_only.json 2>/dev/null; echo "runner rc=$?"; grep -o "\"runner\": {[^}]*}" gpurun_out/runner_only.json | cut -c1-400
