#!/bin/bash
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
T="python -u -m pytest -v --timeout 600 --timeout-method thread -m gpu"
timeout -k 10 900 $T tests/test_dropin_gpu.py::test_dropin_row_split tests/test_dropin_gpu.py::test_dropin_layer_split tests/test_dropin_shapes_gpu.py::test_llama3_70b_width_layer_split_8 tests/test_dropin_shapes_gpu.py::test_llama3_8b_width_pp512 tests/test_dropin_shapes_gpu.py::test_llama3_70b_width_pp512 > gpurun_out/r4_c3_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "PASSED|FAILED|^E " gpurun_out/r4_c3_tests.log | head -30
[ $rc -ge 124 ] && exit $rc
timeout -k 10 600 bash scripts/r4_rowsplit.sh > gpurun_out/r4_rowsplit2.txt 2>&1; echo "rowsplit rc=$?"; cat gpurun_out/r4_rowsplit2.txt
OUT=gpurun_out/prof_pp512b RUN="-p 512 -n 0 -c 512" timeout -k 10 300 bash scripts/prof_dropin.sh > /dev/null 2>&1; echo "prof pp rc=$?"
python3 tools/trace_gaps.py gpurun_out/prof_pp512b/run_kernel_trace.csv --gap-us 100 > gpurun_out/prof_pp512b_gaps.txt; grep -E "k_add_rms|k_mmq4_reduce|k_rms_norm_v4" gpurun_out/prof_pp512b/run_kernel_stats.csv | cut -c1-120
G=${TMPDIR:-/tmp}/mx_bench_llama3_8b_q4_k_m.gguf
for i in 1 2; do GGML_BACKEND_PATH=$PWD/llama-mi50.cpp_amd/lib/libggml-mi355x.so timeout -k 10 300 oracle/_ref/ref-llama-bench -m $G -t 8 -ngl 99 -fa 1 -p 512 -n 0 -r 5 2>/dev/null | grep '^{'; done
AB="0=0" PASSES=1 EXTRA="" bash scripts/ab_dropin.sh
for pass in 1 2; do for arm in "" "GGML_MI355X_STAGE_IMMEDIATE=1"; do
  r=$(env $arm GGML_BACKEND_PATH=$PWD/llama-mi50.cpp_amd/lib/libggml-mi355x.so timeout -k 10 300 oracle/_ref/ref-llama-bench -m $G -t 8 -ngl 99 -fa 1 -p 512 -n 128 -r 5 2>/dev/null | grep '^{')
  echo "pass=$pass arm=[$arm] $(echo $r | grep -o '"pp_tok_s": [0-9.]*') $(echo $r | grep -o '"tg_tok_s": [0-9.]*')"
done; done
