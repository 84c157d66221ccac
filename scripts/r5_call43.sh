#!/bin/bash
# swizzled LDS q8 activation image: GEMV / QKV / MoE op tests and decode drop-in parity, then
# tg128 A/B against the HEAD build (ab_base/), same box, interleaved
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_ops_gpu.py tests/test_mmq4_gpu.py tests/test_dropin_shapes_gpu.py -k "gemv or qkv or moe or router or split_o or decode or attn" -x -q \
  --timeout 300 --timeout-method thread > gpurun_out/r5_c43_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r5_c43_tests.log; grep -E "^FAILED|Error" gpurun_out/r5_c43_tests.log | head; [ $rc -ne 0 ] && exit $rc
G=$(python -c "import bench; print(bench.bench_gguf('llama3_8b', 'q4_k_m'))") || exit 1
O=gpurun_out/r5_c43_ab.txt; : > $O
for fa in 1 0; do
for pass in 1 2 3; do
  for arm in ab_base/libggml-mi355x.so llama-mi50.cpp_amd/lib/libggml-mi355x.so; do
    GGML_BACKEND_PATH=$PWD/$arm timeout -k 10 300 oracle/_ref/llama-bench -m $G -t 8 -ngl 99 -fa $fa -p 0 -n 128 -r 3 -o jsonl > gpurun_out/r5_c43.jsonl 2> gpurun_out/r5_c43.err
    rc=$?; [ $rc -ne 0 ] && { echo "rc=$rc $arm"; tail -5 gpurun_out/r5_c43.err; exit $rc; }
    echo "fa=$fa pass=$pass lib=$arm $(grep -o '"avg_ts": [0-9.]*' gpurun_out/r5_c43.jsonl) $(grep -o '"samples_ts": \[[^]]*\]' gpurun_out/r5_c43.jsonl)" >> $O
  done
done
done
cat $O
