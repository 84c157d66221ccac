#!/bin/bash
# v4 (k_mmq4) for the q/k/v group and the K = 4096 projections (default) against round 2's
# choice (g_tune[17] = 5: k_mmq3m / k_mmq3 there): opbench GEMM cases after a warm-up arm,
# then the runner's pp512 / pp2048 interleaved, then the prefill GPU tests
cd "$(dirname "$0")/.."
CASES="pp_qkv pp_qkv_v6 pp_q_q4k pp_k_q4k" AB="17=5 0=0 17=5 0=0" bash scripts/ab_mmq4_x.sh > /dev/null 2>&1 || exit 1
grep -E '==|k_mmq|reduce' gpurun_out/mmx/report.txt
B="--steps 1 --warmup 1 --no-cpu-baseline --no-dropin --skip-roofline --tg 8"
for i in 1 2; do
  for arm in 17=5 0=0; do
    timeout -k 10 300 python3 bench.py $B --tune $arm > gpurun_out/pp_$arm.log 2>&1 || exit 2
    echo "$i arm=$arm $(grep -o '"pp512_tok_s": [0-9.]*\|"pp2048_tok_s": [0-9.]*' gpurun_out/pp_$arm.log | tr '\n' ' ')"
  done
done
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 -k "pp512 or pp2048 or mul_mat or qkv or prefill or mmq" > gpurun_out/t_pp.log 2>&1; rc=$?
tail -3 gpurun_out/t_pp.log; exit $rc
