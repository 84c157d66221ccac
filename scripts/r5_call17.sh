#!/bin/bash
# decode fusions at depth (absorbed deferred norm): depth test, 8B decode tests, d16k / d4096 / d0 tg128 + klog
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_dropin_shapes_gpu.py -k "llama3_8b_width_decode" -x -q -s --timeout 800 --timeout-method thread > gpurun_out/r5_c17_test.log 2>&1
rc=$?; echo "test rc=$rc"; tail -3 gpurun_out/r5_c17_test.log; grep -E "^FAILED|Error|assert" gpurun_out/r5_c17_test.log | head -10
[ $rc -ne 0 ] && exit $rc
G8=$(python -c "import bench; print(bench.bench_gguf('llama3_8b', 'q4_k_m'))") || exit 1
export GGML_BACKEND_PATH=$PWD/llama-mi50.cpp_amd/lib/libggml-mi355x.so
GGML_MI355X_KLOG=gpurun_out/klog17_d16384.txt timeout -k 10 600 oracle/_ref/llama-bench -m $G8 -t 8 -ngl 99 -fa 1 -p 0 -n 4 -d 16384 -r 1 -o jsonl > /dev/null 2>&1 || exit 1
tail -5 gpurun_out/klog17_d16384.txt
for d in 16384 4096 0; do
  timeout -k 10 600 oracle/_ref/llama-bench -m $G8 -t 8 -ngl 99 -fa 1 -p 0 -n 128 -d $d -r 3 -o jsonl > gpurun_out/tg_d$d.log 2>&1 || exit 1
  echo "d=$d: $(grep -o '"samples_ts": \[[^]]*\]' gpurun_out/tg_d$d.log)"
done
timeout -k 10 600 oracle/_ref/llama-bench -m $G8 -t 8 -ngl 99 -fa 0 -p 0 -n 128 -d 16384 -r 3 -o jsonl > gpurun_out/tg_d16k_fa0.log 2>&1 || exit 1
echo "fa0 d=16384: $(grep -o '"samples_ts": \[[^]]*\]' gpurun_out/tg_d16k_fa0.log)"
timeout -k 10 900 python -u -m pytest tests/test_dropin_gpu.py -k "row_split" -x -q -s --timeout 800 --timeout-method thread > gpurun_out/r5_c17_rowsplit.log 2>&1
rc=$?; echo "rowsplit rc=$rc"; tail -3 gpurun_out/r5_c17_rowsplit.log; grep -E "^FAILED|Error|assert" gpurun_out/r5_c17_rowsplit.log | head -10
[ $rc -ne 0 ] && exit $rc
for arm in "none 1" "row 1,1" "row 1,1,1,1"; do
  set -- $arm
  n=$(echo $2 | tr ',' '\n' | wc -l)
  GGML_MI355X_VIRTUAL_DEVICES=$n GGML_MI355X_FORCE_PEER=1 timeout -k 10 600 oracle/_ref/llama-bench -m $G8 -t 8 -ngl 99 -fa 1 -p 0 -n 128 -sm $1 -ts $2 -r 3 -o jsonl > gpurun_out/rs_$n.log 2>&1 || exit 1
  echo "sm=$1 ts=$2: $(grep -o '"samples_ts": \[[^]]*\]' gpurun_out/rs_$n.log)"
done
