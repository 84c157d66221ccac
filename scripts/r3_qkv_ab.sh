#!/bin/bash
# Balanced QKV layout (g_tune[30]) A/B: op tests, opbench attn_in, tg128 interleaved; then the
# SQ / FETCH counter passes of the prefill GEMMs and the decode kernels (scripts/pmc_sq.sh).
cd "$(dirname "$0")/.."
O=gpurun_out/qkvab
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_dropin_shapes_gpu.py tests/test_dropin_gpu.py tests/test_llama_gpu.py \
  -k "8b_width_decode or incremental or fusions_fire or unfused or q8_0_kv" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
OUT=$O/ob bash scripts/opbench.sh --only attn_in --ab 30=0 30=1 > $O/ob.txt 2>&1 || exit 2
grep -A3 "== " $O/ob/report.txt | grep -v copyBuffer
STEPS_N=3 AB="30=0 30=1 30=0 30=1" bash scripts/ab_bench.sh || exit 3
B="python3 bench.py --steps 1 --warmup 0 --tg 16 --pp 512 --no-cpu-baseline --no-dropin --skip-roofline --no-pp2048"
OUT=$O/pmc_pp KFILTER="k_mmq4|k_mmq3|k_fa_mma2" bash scripts/pmc_sq.sh $B || exit 4
OUT=$O/pmc_dec KFILTER="k_qkv|k_gemv2|k_fattn_dec2" COUNTERS="FETCH_SIZE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM GRBM_GUI_ACTIVE" \
  bash scripts/pmc_sq.sh $B || exit 5
