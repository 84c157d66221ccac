#!/bin/bash
cd "$(dirname "$0")/../../.."
TTMO=1500 bash scripts/r6.sh "tests tests" ; \
bash scripts/r6.sh "lb pp_f16 -fa 1 -p 512,2048 -n 0 -r 3" "lb pp_fa0 -fa 0 -p 512,2048 -n 0 -r 3" "lb pp_q8kv -fa 1 -p 512 -n 0 -r 3 -ctk q8_0 -ctv q8_0" "lb pp_q8k_f16v -fa 1 -p 512 -n 0 -r 3 -ctk q8_0 -ctv f16" "lb tg_f16 -fa 1 -p 0 -n 128 -r 3" "lb tg_fa0 -fa 0 -p 0 -n 128 -r 3"
