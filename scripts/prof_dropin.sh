#!/bin/bash
# rocprofv3 kernel stats of the drop-in decode: the reference's libllama (ref-llama-bench)
# on libggml-mi355x.so, tg128 (RUN="-p 512 -n 0 -c 512" for pp512), -fa ${FA:-1}.
# GRAPHS=0 disables HIP-graph replay; with graphs on, DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 keeps
# rocprofv3 from faulting in hipGraphLaunch (a rocprofiler-sdk read past the end
# of the CLR's captured-packet buffer).
cd "$(dirname "$0")/.."
OUT=${OUT:-gpurun_out/prof_dropin}
mkdir -p $OUT
G=$(python -c "import bench; print(bench.bench_gguf())") || exit 1
ROOTDIR=$PWD
cd /tmp && export TMPDIR=/tmp && cd "$ROOTDIR"
export GGML_BACKEND_PATH=$PWD/llama-mi50.cpp_amd/lib/libggml-mi355x.so
[ "${GRAPHS:-1}" = 0 ] && export GGML_MI355X_DISABLE_GRAPHS=1
export DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
timeout -k 10 ${TMO:-300} rocprofv3 --kernel-trace --stats -d $OUT -o run --output-format csv -- \
  oracle/_ref/ref-llama-bench -m $G -t 8 -ngl 99 -fa ${FA:-1} ${RUN:--p 0 -n 128 -c 256} -r 1 ${CTK:+-ctk $CTK} > $OUT.log 2>&1
rc=$?
echo "prof_dropin rc=$rc"; head -30 $OUT/run_kernel_stats.csv
exit $rc
