#!/bin/bash
# round 4 call: new drop-in tests (KV state, 8-device layer split), the attribution with FA,
# then the default bench
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
T="python -u -m pytest -v --timeout 600 --timeout-method thread -m gpu"
timeout -k 10 600 $T tests/test_dropin_gpu.py -k "kv_state" tests/test_dropin_shapes_gpu.py::test_llama3_70b_width_layer_split_8 > gpurun_out/r4_new_dropin.log 2>&1
rc=$?; echo "new dropin tests rc=$rc"; grep -E "PASSED|FAILED|^E " gpurun_out/r4_new_dropin.log | head -20
[ $rc -ge 124 ] && exit $rc
timeout -k 10 600 bash scripts/r4_attrib.sh > /dev/null 2>&1; echo "attrib rc=$?"; tail -4 gpurun_out/attrib/llama3_70b_2l_fa1.txt
timeout -k 10 600 python bench.py > gpurun_out/r4_bench1.json 2> gpurun_out/r4_bench1.err; echo "bench rc=$?"; tail -c 1500 gpurun_out/r4_bench1.json
OUT=gpurun_out/fa256 timeout -k 10 300 bash scripts/opbench.sh --only fa_256 --ab 0=0 1=4 1=2 1=4,29=2 1=2,29=2 0=0 > gpurun_out/r4_fa256_ab.txt 2>&1; echo "fa ab rc=$?"; grep -E "==|fattn" gpurun_out/fa256/report.txt | head -40
AB="0=0 1=4 1=2 1=4,29=2" PASSES=2 timeout -k 10 400 bash scripts/ab_dropin.sh > gpurun_out/r4_ab_dropin_fa.txt 2>&1; echo "dropin ab rc=$?"; cat gpurun_out/r4_ab_dropin_fa.txt
OUT=gpurun_out/falong timeout -k 10 300 bash scripts/opbench.sh --only fa_4096 fa_16384 fa_32768 --ab 2=1 0=0 2=2 2=4 2=8 2=1 > gpurun_out/r4_falong_ab.txt 2>&1; echo "fa long ab rc=$?"; grep -E "==|fattn" gpurun_out/falong/report.txt | head -60
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_ops_gpu.py -k "flash_attn" > gpurun_out/r4_fa_tests.log 2>&1; echo "fa tests rc=$?"; tail -3 gpurun_out/r4_fa_tests.log
OUT=gpurun_out/prof_pp512 RUN="-p 512 -n 0 -c 512" timeout -k 10 300 bash scripts/prof_dropin.sh > /dev/null 2>&1; echo "prof pp rc=$?"; python tools/trace_gaps.py gpurun_out/prof_pp512/run_kernel_trace.csv --gap-us 100 | head -30
OUT=gpurun_out/prof_tg128 timeout -k 10 300 bash scripts/prof_dropin.sh > /dev/null 2>&1; echo "prof tg rc=$?"; python tools/trace_gaps.py gpurun_out/prof_tg128/run_kernel_trace.csv --gap-us 30 | head -30
timeout -k 10 600 bash scripts/r4_rowsplit.sh > gpurun_out/r4_rowsplit.txt 2>&1; echo "rowsplit rc=$?"; cat gpurun_out/r4_rowsplit.txt
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_dropin_gpu.py -k "split" > gpurun_out/r4_split_tests.log 2>&1; echo "split tests rc=$?"; grep -E "PASSED|FAILED|^E " gpurun_out/r4_split_tests.log | head
