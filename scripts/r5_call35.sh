#!/bin/bash
# Mixtral pp512: k_mmq4 token tile 128 (default) vs 64 (g_tune[17] = 2), two interleaved passes
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
GM=$(python -c "import bench; print(bench.bench_gguf('mixtral_8x7b', 'q5_k_m'))") || exit 1
export GGML_BACKEND_PATH=$PWD/llama-mi50.cpp_amd/lib/libggml-mi355x.so
O=gpurun_out/r5_moe_tt_ab.txt; : > $O
for pass in 1 2; do
  for arm in "" "17=2"; do
    GGML_MI355X_TUNE="$arm" timeout -k 10 300 oracle/_ref/llama-bench -m $GM -t 8 -ngl 99 -fa 1 -p 512 -n 0 -r 5 -o jsonl > gpurun_out/r5_moe_tt.jsonl 2> gpurun_out/r5_moe_tt.err
    rc=$?; [ $rc -ne 0 ] && { echo "rc=$rc"; tail -5 gpurun_out/r5_moe_tt.err; exit $rc; }
    python - "$pass" "$arm" >> $O <<'PY'
import json, sys
for l in open('gpurun_out/r5_moe_tt.jsonl'):
    d = json.loads(l)
    print('pass', sys.argv[1], 'arm', repr(sys.argv[2]), 'pp512 avg_ts %.1f' % d['avg_ts'], 'samples', [round(x) for x in d['samples_ts']])
PY
  done
done
cat $O
