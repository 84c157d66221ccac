#!/bin/bash
# L2 channel hot-spot hypothesis: f16 activation row stride 8 KB (K = 4096) vs padded by 64 / 128 halfs
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for pad in 0 64 0 128; do
GGML_MI355X_KP_PAD=$pad OUT=gpurun_out/kp$pad timeout -k 10 300 bash scripts/opbench.sh --only pp_glu_q4k pp_down_q4k pp_qkv --ab 0=0 0=0 3=8 > gpurun_out/r4_kp$pad.txt 2>&1; echo "pad $pad rc=$?"; grep -E "==|k_mmq" gpurun_out/kp$pad/report.txt
done
