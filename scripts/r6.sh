#!/bin/bash
# One GPU session as a list of steps (round 6; replaces the one-shot r4/r5 call wrappers).
#   bash scripts/r6.sh "<step>" "<step>" ...
# steps:
#   tests <pytest args...>        python -m pytest -m gpu (unbuffered, per-test timeout)
#   lb <name> <llama-bench flags> the reference llama-bench (oracle/_ref) on the 8B Q4_K_M GGUF,
#                                 -ngl 99 on this backend; jsonl -> $OUT/<name>.jsonl
#   prof <name> <ref flags>       rocprofv3 --kernel-trace --stats of ref-llama-bench (graphs on,
#                                 DEBUG_CLR_GRAPH_PACKET_CAPTURE=0) -> $OUT/<name>/
#   pmc <name> <counters> -- <ref flags>   one rocprofv3 --pmc pass of ref-llama-bench
#   bench <bench.py args>         bench.py
#   py <script args>              any python step
# Stops at the first crash / time limit / abort (rc >= 124, 134, 139): nothing further runs
# on the GPU in that call. Plain failures (rc 1) do not stop the later steps.
cd "$(dirname "$0")/.."
OUT=${OUT:-gpurun_out/r6}
mkdir -p $OUT
export TMPDIR=/tmp
LB=oracle/_ref/llama-bench
REFB=oracle/_ref/ref-llama-bench
LIB=${MXLIB:-$PWD/llama-mi50.cpp_amd/lib/libggml-mi355x.so}
G=""
gguf() { [ -n "$G" ] || G=$(python -c "import bench; print(bench.bench_gguf('${MODEL:-llama3_8b}', '${RECIPE:-q4_k_m}'))") || exit 1; }
fin() {  # name rc
  echo "$1 rc=$2"
  if [ $2 -ge 124 ] || [ $2 -eq 134 ] || [ $2 -eq 139 ]; then echo "stopping: $1 rc=$2"; exit $2; fi
}
n=0
for st in "$@"; do
  n=$((n + 1))
  set -- $st
  kind=$1; shift
  case $kind in
    tests)   # ('+' in an argument stands for a space: -k "a+or+b")
      set -- "${@//+/ }"
      [ $# -eq 0 ] && set -- tests
      timeout -k 10 ${TTMO:-1500} python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread "$@" > $OUT/tests_$n.log 2>&1
      rc=$?; tail -n 25 $OUT/tests_$n.log; fin tests_$n $rc ;;
    lb)
      gguf; name=$1; shift
      GGML_BACKEND_PATH=$LIB timeout -k 10 ${LTMO:-600} $LB -m $G -t 8 -ngl 99 -o jsonl -v "$@" > $OUT/$name.jsonl 2> $OUT/$name.err
      rc=$?
      echo "$name: $(grep -o '"n_prompt": [0-9]*, "n_gen": [0-9]*' $OUT/$name.jsonl | tr '\n' ' ') $(grep -o '"avg_ts": [0-9.]*' $OUT/$name.jsonl | tr '\n' ' ') splits: $(grep -o 'graph splits = .*' $OUT/$name.err | sort -u | tr '\n' ' ')"
      fin $name $rc ;;
    prof)
      gguf; name=$1; shift
      GGML_BACKEND_PATH=$LIB DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -k 10 ${PTMO:-600} rocprofv3 --kernel-trace --stats -d $OUT/$name -o run \
        --output-format csv -- $REFB -m $G -t 8 -ngl 99 "$@" > $OUT/$name.log 2>&1
      rc=$?
      f=$(find $OUT/$name -name '*kernel_stats.csv' | head -1); [ -n "$f" ] && cp "$f" $OUT/${name}_kernel_stats.csv && head -25 "$f"
      fin $name $rc ;;
    pmc)
      gguf; name=$1; ctr=$2; shift 3
      GGML_BACKEND_PATH=$LIB DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -s KILL 120 rocprofv3 --pmc $ctr -d $OUT/$name -o run \
        --output-format csv -- $REFB -m $G -t 8 -ngl 99 "$@" > $OUT/$name.log 2>&1
      rc=$?; fin $name $rc ;;
    tbo)     # the reference's test-backend-ops against MI355X0 (perf / test mode)
      name=$1; shift
      set -- "${@//+/ }"
      GGML_BACKEND_PATH=$LIB timeout -k 10 ${OTMO:-600} oracle/_ref/test-backend-ops "$@" > $OUT/$name.log 2>&1
      rc=$?; grep -E "us/run|tests passed|FAIL" $OUT/$name.log | tail -n 60; fin $name $rc ;;
    envlb)   # lb with env assignments first: envlb <name> VAR=val,VAR2=val -- flags
      name=$1; ev=$2; shift 3; gguf
      env ${ev//,/ } GGML_BACKEND_PATH=$LIB timeout -k 10 ${LTMO:-600} $LB -m $G -t 8 -ngl 99 -o jsonl -v "$@" > $OUT/$name.jsonl 2> $OUT/$name.err
      rc=$?
      echo "$name: $(grep -o '"avg_ts": [0-9.]*' $OUT/$name.jsonl | tr '\n' ' ') splits: $(grep -o 'graph splits = .*' $OUT/$name.err | sort -u | tr '\n' ' ')"
      fin $name $rc ;;
    bench)
      timeout -k 10 ${BTMO:-1200} python -u bench.py "$@" > $OUT/bench_$n.json 2> $OUT/bench_$n.err
      rc=$?; tail -c 3000 $OUT/bench_$n.json; fin bench_$n $rc ;;
    py)
      timeout -k 10 ${YTMO:-600} python -u "$@" > $OUT/py_$n.log 2>&1
      rc=$?; tail -n 30 $OUT/py_$n.log; fin py_$n $rc ;;
    *) echo "unknown step $kind"; exit 2 ;;
  esac
done
