#!/bin/bash
# PMC passes for the remaining round-5 kernels: k_nofa_part (-fa 0 decode), k_moe_router + the MoE expert GEMVs
# (Mixtral tg), k_mmq4 EPI 3 (Mixtral pp512); SQ set + FETCH_SIZE each
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
G8=$(python -c "import bench; print(bench.bench_gguf('llama3_8b', 'q4_k_m'))") || exit 1
GM=$(python -c "import bench; print(bench.bench_gguf('mixtral_8x7b', 'q5_k_m'))") || exit 1
export GGML_BACKEND_PATH=$PWD/llama-mi50.cpp_amd/lib/libggml-mi355x.so
OUT=gpurun_out/pmc_fa0_sq KFILTER="k_nofa_part|k_gemv2" TMO=240 bash scripts/pmc_sq.sh oracle/_ref/llama-bench -m $G8 -t 8 -ngl 99 -fa 0 -p 0 -n 16 -r 1 -o jsonl && \
OUT=gpurun_out/pmc_fa0_fetch KFILTER="k_nofa_part|k_gemv2" TMO=240 COUNTERS="FETCH_SIZE GRBM_GUI_ACTIVE" bash scripts/pmc_sq.sh oracle/_ref/llama-bench -m $G8 -t 8 -ngl 99 -fa 0 -p 0 -n 16 -r 1 -o jsonl && \
OUT=gpurun_out/pmc_moe_tg_sq KFILTER="k_moe|k_gemv2" TMO=300 bash scripts/pmc_sq.sh oracle/_ref/llama-bench -m $GM -t 8 -ngl 99 -fa 1 -p 0 -n 8 -r 1 -o jsonl && \
OUT=gpurun_out/pmc_moe_tg_fetch KFILTER="k_moe|k_gemv2" TMO=300 COUNTERS="FETCH_SIZE GRBM_GUI_ACTIVE" bash scripts/pmc_sq.sh oracle/_ref/llama-bench -m $GM -t 8 -ngl 99 -fa 1 -p 0 -n 8 -r 1 -o jsonl && \
OUT=gpurun_out/pmc_moe_pp_sq KFILTER="k_mmq4|k_moe" TMO=300 bash scripts/pmc_sq.sh oracle/_ref/llama-bench -m $GM -t 8 -ngl 99 -fa 1 -p 512 -n 0 -r 1 -o jsonl
