#!/bin/bash
# A/B of the streaming GEMV form (g_tune[27]): opbench per-kernel times and tg128, plus the
# -fa 0 prefill after the one-element SET_ROWS kernel.
cd "$(dirname "$0")/.."
O=gpurun_out/pipe
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_ops_gpu.py -k "set_rows or gemv or mul_mat_quant" > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -2 $O/tests.log
OUT=$O/ob bash scripts/opbench.sh --only attn_in o_q4k_add ffn_block ffn_q4k_q6k down_q4k_add down_q6k_add lm_head_q6k \
  --ab 27=0 27=1 > $O/ob.txt 2>&1 || exit 2
STEPS_N=3 AB="27=0 27=1 27=2 27=3 27=0 27=1" bash scripts/ab_bench.sh || exit 3
G=$(python3 -c "import bench; print(bench.bench_gguf())") || exit 4
for fa in 0 1; do
  GGML_BACKEND_PATH=$PWD/llama-mi50.cpp_amd/lib/libggml-mi355x.so timeout -k 10 300 oracle/_ref/ref-llama-bench -m $G -t 8 -ngl 99 \
    -fa $fa -p 512 -n 0 -r 3 -c 512 > $O/pp_fa$fa.log 2>&1 || exit 5
  echo "pp512 fa$fa $(grep -o '"pp_tok_s": [0-9.]*' $O/pp_fa$fa.log)"
done
