#!/bin/bash
# capture at the first sighting (A/B vs the round-4 second-sighting capture): drop-in pp512 and tg128
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
G=$(python -c "import bench; print(bench.bench_gguf())") || exit 1
export GGML_BACKEND_PATH=$PWD/llama-mi50.cpp_amd/lib/libggml-mi355x.so
for pass in 1 2; do
  for arm in "GGML_MI355X_CAPTURE_SECOND=1" "X=0"; do
    r=$(env $arm timeout -k 10 300 oracle/_ref/llama-bench -m $G -t 8 -ngl 99 -fa 1 -p 512,2048 -n 128 -r 5 -o jsonl 2>/dev/null | grep -o '"n_prompt": [0-9]*, "n_gen": [0-9]*\|"samples_ts": \[[^]]*\]' | tr '\n' ' ')
    echo "pass=$pass arm=$arm $r"
  done
done
timeout -k 10 600 python -u -m pytest tests/test_dropin_gpu.py tests/test_llama_gpu.py -q -x --timeout 300 --timeout-method thread > gpurun_out/r5_c7_tests.log 2>&1
echo "tests rc=$?"; tail -3 gpurun_out/r5_c7_tests.log
