#!/bin/bash
# row split: one fork/join per group, main slice local under FORCE_PEER; tests + llama-bench A/B
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_dropin_gpu.py -k "row_split or layer_split" -x -q -s --timeout 800 --timeout-method thread > gpurun_out/r5_c19_rowsplit.log 2>&1
rc=$?; echo "split tests rc=$rc"; tail -3 gpurun_out/r5_c19_rowsplit.log; grep -E "^FAILED|Error|assert" gpurun_out/r5_c19_rowsplit.log | head -10
[ $rc -ne 0 ] && exit $rc
G8=$(python -c "import bench; print(bench.bench_gguf('llama3_8b', 'q4_k_m'))") || exit 1
export GGML_BACKEND_PATH=$PWD/llama-mi50.cpp_amd/lib/libggml-mi355x.so
for pass in 1 2; do
for arm in "none 1 0" "row 1/1 1" "row 1/1/1/1 1" "row 1/1 0"; do
  set -- $arm
  n=$(echo $2 | tr '/' '\n' | wc -l)
  GGML_MI355X_VIRTUAL_DEVICES=$n GGML_MI355X_FORCE_PEER=$3 timeout -k 10 600 oracle/_ref/llama-bench -m $G8 -t 8 -ngl 99 -fa 1 -p 0 -n 128 -sm $1 -ts $2 -r 3 -o jsonl > gpurun_out/rs_$n.log 2>&1 || exit 1
  echo "pass $pass sm=$1 ts=$2 force_peer=$3: $(grep -o '"samples_ts": \[[^]]*\]' gpurun_out/rs_$n.log)"
done; done
