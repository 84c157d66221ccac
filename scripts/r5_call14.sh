#!/bin/bash
# k_fattn_dec3 vs LONG at 16k keys in isolation: timing, wave-0 phases, per-workgroup spread
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python tools/opbench.py --only fa_4096 fa_16384 fa_32768 --ab 34=0 34=1 > gpurun_out/r5_c14_ab.log 2>&1 || { tail -20 gpurun_out/r5_c14_ab.log; exit 1; }
cat gpurun_out/r5_c14_ab.log | tail -12
timeout -k 10 300 python tools/opbench.py --only fa_16384 --trace --trace-blocks > gpurun_out/r5_c14_trace.log 2>&1 || { tail -20 gpurun_out/r5_c14_trace.log; exit 1; }
grep -E "trace|blocks" gpurun_out/r5_c14_trace.log | head -30
