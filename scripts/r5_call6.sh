#!/bin/bash
# kernel traces of the drop-in pp512 (-r 3) and tg128 (-r 2) through the real llama-bench:
# GPU idle gaps per repetition (tools/trace_gaps.py)
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
G=$(python -c "import bench; print(bench.bench_gguf())") || exit 1
ROOTDIR=$PWD
cd /tmp && export TMPDIR=/tmp && cd "$ROOTDIR"
export GGML_BACKEND_PATH=$PWD/llama-mi50.cpp_amd/lib/libggml-mi355x.so DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
for t in "pp -p 512 -n 0 -r 3" "tg -p 0 -n 128 -r 2"; do
  set -- $t; name=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/trace_$name -o run --output-format csv -- \
    oracle/_ref/llama-bench -m $G -t 8 -ngl 99 -fa 1 "$@" -o jsonl > gpurun_out/trace_$name.log 2>&1
  echo "$name rc=$?"; grep '^{' gpurun_out/trace_$name.log | grep -o '"samples_ts": \[[^]]*\]'
  python tools/trace_gaps.py gpurun_out/trace_$name/run_kernel_trace.csv --gap-us 30 --segment-us 1500 | head -30
done
