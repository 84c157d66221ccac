#!/bin/bash
# Decode GEMV cost decomposition (tools/opbench.py dbg masks: 1 no prologue, 2 no dot
# products, 3 neither) next to the pure streaming floors (tools/stream_probe), and the
# drop-in -fa 0 pp512 kernel profile with its kernel-choice log.
cd "$(dirname "$0")/.."
O=gpurun_out/decomp
mkdir -p $O
timeout -k 10 120 ./tools/stream_probe > $O/stream_probe.txt 2>&1 || exit 1
OUT=$O/ob bash scripts/opbench.sh --only attn_in o_q4k_add glu_q4k ffn_block down_q4k_add down_q6k_add lm_head_q6k \
  --dbg 0 1 2 3 > $O/ob.txt 2>&1 || exit 2
G=$(python3 -c "import bench; print(bench.bench_gguf())") || exit 3
GGML_BACKEND_PATH=$PWD/llama-mi50.cpp_amd/lib/libggml-mi355x.so GGML_MI355X_KLOG=$PWD/$O/klog_pp_fa0.txt \
  timeout -k 10 300 oracle/_ref/ref-llama-bench -m $G -t 8 -ngl 99 -fa 0 -p 512 -n 0 -r 3 -c 512 > $O/pp_fa0.log 2>&1 || exit 4
FA=0 RUN="-p 512 -n 0 -c 512" OUT=$O/prof_pp_fa0 bash scripts/prof_dropin.sh > /dev/null 2>&1 || exit 5
FA=1 RUN="-p 512 -n 0 -c 512" OUT=$O/prof_pp_fa1 bash scripts/prof_dropin.sh > /dev/null 2>&1 || exit 6
echo ok
