#!/bin/bash
# -fa 0 decode with split partials into the O projection (attn_nofa_part): tests + same-box A/B
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_dropin_shapes_gpu.py tests/test_dropin_gpu.py tests/test_ops_gpu.py -k "llama3_8b_width_decode or nofa or dropin_logits or fa0 or incremental" -x -q --timeout 600 --timeout-method thread > gpurun_out/r5_c30.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r5_c30.log; grep -E "^E  .*(Assert|assert)" gpurun_out/r5_c30.log | head -6
[ $rc -ne 0 ] && exit $rc
G8=$(python -c "import bench; print(bench.bench_gguf('llama3_8b', 'q4_k_m'))") || exit 1
export GGML_BACKEND_PATH=$PWD/llama-mi50.cpp_amd/lib/libggml-mi355x.so
for pass in 1 2; do for arm in 0 1; do
  GGML_MI355X_TUNE=38=$arm timeout -k 10 600 oracle/_ref/llama-bench -m $G8 -t 8 -ngl 99 -fa 0 -p 0 -n 128 -r 3 -o jsonl > gpurun_out/nso_$arm.log 2>&1 || exit 1
  echo "pass $pass tune38=$arm fa0 tg128: $(grep -o '"samples_ts": \[[^]]*\]' gpurun_out/nso_$arm.log)"
done; done
