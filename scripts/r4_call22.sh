#!/bin/bash
# k_mmq4 geometry sweep for the K=4096 projections and the down projection: tokens per tile
# (18=2: 64) and split-K shares (20=n)
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
OUT=gpurun_out/sw22 timeout -k 10 600 bash scripts/opbench.sh --only pp_q_q4k pp_qkv pp_down_q6k pp_down_q4k --ab 0=0 0=0 18=2 20=1 20=2 20=4 20=8 18=2,20=1 18=2,20=2 > gpurun_out/r4_sw22.txt 2>&1; echo "rc=$?"; grep -E "==|k_mmq" gpurun_out/sw22/report.txt
