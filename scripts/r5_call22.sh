#!/bin/bash
# PMC passes (separate runs, no trace domains): roofline HBM traffic, prefill GEMM SQ counters
# (k_mmq5_glu / k_mmq4 — the int8-or-not question), and the round-5 decode kernels
# (k_fattn_dec3, k_nofa_*, k_moe_router are covered by their own launches below)
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
G8=$(python -c "import bench; print(bench.bench_gguf('llama3_8b', 'q4_k_m'))") || exit 1
export GGML_BACKEND_PATH=$PWD/llama-mi50.cpp_amd/lib/libggml-mi355x.so
OUT=gpurun_out/pmc_r5 TMO=300 bash scripts/pmc_roofline.sh && cat gpurun_out/pmc_r5/pmc_glu.json | head -20 && \
OUT=gpurun_out/pmc_pp_sq KFILTER="k_mmq5|k_mmq4|k_fa_mma2" TMO=240 bash scripts/pmc_sq.sh oracle/_ref/llama-bench -m $G8 -t 8 -ngl 99 -fa 1 -p 512 -n 0 -r 1 -o jsonl && \
OUT=gpurun_out/pmc_pp_inst KFILTER="k_mmq5|k_mmq4" TMO=240 COUNTERS="SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_LDS GRBM_GUI_ACTIVE" bash scripts/pmc_sq.sh oracle/_ref/llama-bench -m $G8 -t 8 -ngl 99 -fa 1 -p 512 -n 0 -r 1 -o jsonl && \
OUT=gpurun_out/pmc_d16k_sq KFILTER="k_fattn_dec3|k_nofa|k_gemv2" TMO=300 bash scripts/pmc_sq.sh oracle/_ref/llama-bench -m $G8 -t 8 -ngl 99 -fa 1 -p 0 -n 8 -d 16384 -r 1 -o jsonl && \
OUT=gpurun_out/pmc_d16k_fetch KFILTER="k_fattn_dec3|k_nofa" TMO=300 COUNTERS="FETCH_SIZE GRBM_GUI_ACTIVE" bash scripts/pmc_sq.sh oracle/_ref/llama-bench -m $G8 -t 8 -ngl 99 -fa 1 -p 0 -n 8 -d 16384 -r 1 -o jsonl && \
OUT=gpurun_out/pmc_d16k_fa0_fetch KFILTER="k_nofa" TMO=300 COUNTERS="FETCH_SIZE GRBM_GUI_ACTIVE" bash scripts/pmc_sq.sh oracle/_ref/llama-bench -m $G8 -t 8 -ngl 99 -fa 0 -p 0 -n 8 -d 16384 -r 1 -o jsonl
