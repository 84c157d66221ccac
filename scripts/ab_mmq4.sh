#!/bin/bash
# Same-box A/B of the prefill GEMM (k_mmq4): the in-tree build against lib_<v>/ builds
# (opbench pp cases under rocprofv3 kernel trace), VARIANTS="both lda2 andor"
cd "$(dirname "$0")/.."
C="--only pp_glu_q4k pp_down_q6k pp_down_q4k pp_q_q4k"
OUT=gpurun_out/mm_head bash scripts/opbench.sh $C > gpurun_out/mm_head.txt 2>&1 || exit 1
for V in ${VARIANTS:-both lda2 andor}; do
  GGML_MI355X_LIB=$PWD/llama-mi50.cpp_amd/lib_$V/libggml-mi355x.so OUT=gpurun_out/mm_$V bash scripts/opbench.sh $C > gpurun_out/mm_$V.txt 2>&1 || exit 2
done
for V in head ${VARIANTS:-both lda2 andor}; do echo "== $V"; grep -E 'us|==' gpurun_out/mm_$V/report.txt; done
