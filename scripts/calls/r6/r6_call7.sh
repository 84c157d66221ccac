#!/bin/bash
cd "$(dirname "$0")/../../.."
TTMO=1500 bash scripts/r6.sh "tests tests" ; \
bash scripts/r6.sh "lb pp_f16 -fa 1 -p 512,2048 -n 0 -r 3" "lb pp_fa0 -fa 0 -p 512,2048 -n 0 -r 3" "lb pp_q8kv -fa 1 -p 512 -n 0 -r 3 -ctk q8_0 -ctv q8_0" "lb pp_q8k_f16v -fa 1 -p 512 -n 0 -r 3 -ctk q8_0 -ctv f16" "prof prof_pp512_fa0_v2 -fa 0 -p 512 -n 0 -c 512 -r 2" "prof prof_pp512_q8kv -fa 1 -p 512 -n 0 -c 512 -r 2 -ctk 8"
