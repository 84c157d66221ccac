#!/bin/bash
# Same-box bisect of the decode SwiGLU launch time (bench.py --roofline-only: the isolated
# k_gemv2 SwiGLU cycled over 32 layers' weights) across builds of earlier commits
# (ab_<commit>/, `git archive <commit>` built in place) and HEAD, interleaved twice.
cd "$(dirname "$0")/.."
O=$PWD/gpurun_out/bisect
mkdir -p $O
TREES=${TREES:-"ab_r1 ab_ed4257b ab_7a7ae32 ab_cc4907a ab_f67a99c ab_0d87f1f ."}
for i in 1 2; do
  for t in $TREES; do
    n=$(basename $(cd $t && pwd)); [ "$t" = "." ] && n=head
    (cd $t && timeout -k 10 240 python3 bench.py --roofline-only > $O/${n}_$i.log 2>&1) || { echo "$t failed"; exit 1; }
    echo "$i $n $(grep -o '"avg_launch_us": [0-9.]*' $O/${n}_$i.log)"
  done
done
