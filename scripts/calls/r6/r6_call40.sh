#!/bin/bash
# shipped multi-column default: op tests + the reference harness's MUL_MAT chunk
cd "$(dirname "$0")/../../.."
mkdir -p gpurun_out/r6
bash scripts/r6.sh "tests tests/test_ops_gpu.py -k mul_mat" "tests tests/test_refops_gpu.py -k MUL_MAT" "tbo mm_test3 test -b MI355X0 -o MUL_MAT"
