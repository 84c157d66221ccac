#!/bin/bash
# SQ / HBM counters of round 6's new decode kernels: k_moe_down_comb, k_moe_router1 (mixtral_2l tg),
# k_gemv_nc (test-backend-ops perf, 4096 x bs x 14336)
cd "$(dirname "$0")/../../.."
mkdir -p gpurun_out/r6
G=$(python -c "import bench; print(bench.bench_gguf('mixtral_2l', 'q5_k_m'))") || exit 1
export GGML_BACKEND_PATH=$PWD/llama-mi50.cpp_amd/lib/libggml-mi355x.so
C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_WAVES"
OUT=gpurun_out/r6/pmc_moe_sq COUNTERS="$C" KFILTER="k_moe_down_comb|k_moe_router1|k_gemv2" TMO=200 bash scripts/pmc_sq.sh oracle/_ref/ref-llama-bench -m $G -t 8 -ngl 99 -fa 1 -p 0 -n 16 -r 1 && \
OUT=gpurun_out/r6/pmc_moe_fetch COUNTERS="FETCH_SIZE" KFILTER="k_moe_down_comb|k_moe_router1|k_gemv2" TMO=200 bash scripts/pmc_sq.sh oracle/_ref/ref-llama-bench -m $G -t 8 -ngl 99 -fa 1 -p 0 -n 16 -r 1 && \
OUT=gpurun_out/r6/pmc_gnc_sq COUNTERS="$C" KFILTER="k_gemv_nc" TMO=200 bash scripts/pmc_sq.sh oracle/_ref/test-backend-ops perf -b MI355X0 -o MUL_MAT -p "type_a=q4_K,type_b=f32,m=4096,n=(2|4|8),k=14336"
