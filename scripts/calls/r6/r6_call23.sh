#!/bin/bash
# SQ counters of the decode attention at depth 8192 (LONG geometry): f16 vs q8_0 caches
cd "$(dirname "$0")/../../.."
mkdir -p gpurun_out/r6
G=$(python -c "import bench; print(bench.bench_gguf())") || exit 1
export GGML_BACKEND_PATH=$PWD/llama-mi50.cpp_amd/lib/libggml-mi355x.so
C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_WAVES"
OUT=gpurun_out/r6/pmc_d8k_f16 COUNTERS="$C" KFILTER="k_fattn_dec2" TMO=200 bash scripts/pmc_sq.sh oracle/_ref/ref-llama-bench -m $G -t 8 -ngl 99 -fa 1 -p 0 -n 4 -d 8192 -r 1 && \
OUT=gpurun_out/r6/pmc_d8k_q8 COUNTERS="$C" KFILTER="k_fattn_dec2" TMO=200 bash scripts/pmc_sq.sh oracle/_ref/ref-llama-bench -m $G -t 8 -ngl 99 -fa 1 -p 0 -n 4 -d 8192 -r 1 -ctk 8
cat gpurun_out/r6/pmc_d8k_f16/summary.json gpurun_out/r6/pmc_d8k_q8/summary.json
