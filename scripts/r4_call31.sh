#!/bin/bash
# -fa 0 decode attention in one memory round trip (k_attn_nofa_dec 1024-thread): parity + drop-in A/B (g_tune[2]=9: two-pass form)
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_ops_gpu.py -k "nofa or attn" tests/test_dropin_gpu.py > gpurun_out/r4_nofa_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r4_nofa_tests.log
[ $rc -eq 0 ] || exit 1
FA=0 AB="0=0 2=10 2=9" PASSES=2 R=5 timeout -k 10 600 bash scripts/ab_dropin.sh > gpurun_out/r4_nofa_ab.txt 2>&1; echo "ab rc=$?"; cat gpurun_out/r4_nofa_ab.txt
OUT=gpurun_out/prof_tg_fa0b FA=0 TMO=300 bash scripts/prof_dropin.sh > gpurun_out/r4_prof_tg_fa0b.txt 2>&1; echo "prof rc=$?"; grep -i "nofa" gpurun_out/prof_tg_fa0b/run_kernel_stats.csv | cut -c1-160
