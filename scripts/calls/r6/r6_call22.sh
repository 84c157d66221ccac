#!/bin/bash
# q8_0 caches: LONG geometry at 16 key rows per lane (a real NI-16 instantiation this time)
cd "$(dirname "$0")/../../.."
mkdir -p gpurun_out/r6
bash scripts/r6.sh "tests tests/test_ops_gpu.py -k flash_attn_long_quantised+or+flash_attn_kv_types+or+mixed_kv" && \
bash scripts/r6.sh "lb t_q8kv_d16k_def -fa 1 -p 0 -n 64 -d 16384 -r 2 -ctk q8_0 -ctv q8_0" \
  "envlb t_q8kv_d16k_ni16 GGML_MI355X_TUNE=28=16 -- -fa 1 -p 0 -n 64 -d 16384 -r 2 -ctk q8_0 -ctv q8_0" \
  "lb t_q8kv_d8k_def -fa 1 -p 0 -n 64 -d 8192 -r 2 -ctk q8_0 -ctv q8_0" \
  "envlb t_q8kv_d8k_ni16 GGML_MI355X_TUNE=28=16 -- -fa 1 -p 0 -n 64 -d 8192 -r 2 -ctk q8_0 -ctv q8_0" \
  "lb t_q8kf16v_d16k_def -fa 1 -p 0 -n 64 -d 16384 -r 2 -ctk q8_0 -ctv f16" \
  "envlb t_q8kf16v_d16k_ni16 GGML_MI355X_TUNE=28=16 -- -fa 1 -p 0 -n 64 -d 16384 -r 2 -ctk q8_0 -ctv f16"
