#!/bin/bash
# row split at HEAD: -sm row tg128 under FORCE_PEER (ts 1/1, 1/1/1/1) against the unsplit run, three passes
# suite), then -sm row tg128 under FORCE_PEER (ts 1/1, 1/1/1/1) against the unsplit run
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
G=$(python -c "import bench; print(bench.bench_gguf('llama3_8b', 'q4_k_m'))") || exit 1
export GGML_BACKEND_PATH=$PWD/llama-mi50.cpp_amd/lib/libggml-mi355x.so
O=gpurun_out/r5_c52_rowsplit.txt; : > $O
for pass in 1 2 3; do
  for arm in "4 1/1/1/1" "2 1/1" "1 -"; do
    set -- $arm
    if [ "$2" = "-" ]; then extra=""; else extra="-sm row -ts $2"; fi
    GGML_MI355X_VIRTUAL_DEVICES=$1 GGML_MI355X_FORCE_PEER=1 timeout -k 10 300 oracle/_ref/llama-bench -m $G -t 8 -ngl 99 -fa 1 -p 0 -n 128 -r 3 $extra -o jsonl > gpurun_out/r5_c52.jsonl 2> gpurun_out/r5_c52.err
    rc=$?; [ $rc -ne 0 ] && { echo "rc=$rc arm=$arm"; tail -5 gpurun_out/r5_c52.err; exit $rc; }
    echo "pass=$pass devices=$1 ts=$2 $(grep -o '"samples_ts": \[[^]]*\]' gpurun_out/r5_c52.jsonl)" >> $O
  done
done
cat $O
