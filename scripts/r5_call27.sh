#!/bin/bash
# pp512 drop-in vs runner: kernel traces (busy / idle per ubatch, per-kernel totals)
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
G8=$(python -c "import bench; print(bench.bench_gguf('llama3_8b', 'q4_k_m'))") || exit 1
export DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
GGML_BACKEND_PATH=$PWD/llama-mi50.cpp_amd/lib/libggml-mi355x.so timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_pp_dropin -o run --output-format csv -- \
  oracle/_ref/llama-bench -m $G8 -t 8 -ngl 99 -fa 1 -p 512 -n 0 -r 5 -o jsonl > gpurun_out/prof_pp_dropin.log 2>&1 || exit 1
python tools/trace_gaps.py gpurun_out/prof_pp_dropin/run_kernel_trace.csv --gap-us 30 --segment-us 1000 | head -30
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_pp_runner -o run --output-format csv -- \
  python bench.py --mode single --no-dropin --no-cpu-baseline --skip-roofline --steps 1 --no-pp2048 > gpurun_out/prof_pp_runner.log 2>&1 || exit 1
python tools/trace_gaps.py gpurun_out/prof_pp_runner/run_kernel_trace.csv --gap-us 30 --segment-us 1000 | tail -25
