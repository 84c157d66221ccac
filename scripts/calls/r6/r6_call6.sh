#!/bin/bash
cd "$(dirname "$0")/../../.."
bash scripts/r6.sh "tests tests/test_ops_gpu.py tests/test_dropin_gpu.py tests/test_dropin_shapes_gpu.py -k set_rows+or+flash_attn+or+dropin+or+pp512+or+pp2048+or+width_decode" "lb pp_f16 -fa 1 -p 512,2048 -n 0 -r 3" "lb pp_fa0 -fa 0 -p 512,2048 -n 0 -r 3" "lb pp_q8kv -fa 1 -p 512 -n 0 -r 3 -ctk q8_0 -ctv q8_0" "lb pp_q8k_f16v -fa 1 -p 512 -n 0 -r 3 -ctk q8_0 -ctv f16"
