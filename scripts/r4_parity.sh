#!/bin/bash
# round 4: k_mmq4 op tests (+ the same outlier cases against lib_old, the build before the
# range guard: expected to fail with non-finite rows), the split-K fusion test
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
T="python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu"
timeout -k 10 600 $T -x tests/test_mmq4_gpu.py "tests/test_llama_gpu.py::test_prefill_qkv_epilogue_fusion" > gpurun_out/r4_mmq4_tests.log 2>&1
rc=$?; echo "mmq4 tests rc=$rc"; tail -5 gpurun_out/r4_mmq4_tests.log
[ $rc -ge 124 ] && exit $rc
# GGML_MI355X_LIB=$PWD/llama-mi50.cpp_amd/lib_old/libggml-mi355x.so timeout -k 10 600 $T tests/test_mmq4_gpu.py -k "True or glu or group or moe or residual" > gpurun_out/r4_mmq4_tests_oldlib.log 2>&1
# echo "old lib rc=$?"; grep -E "passed|failed" gpurun_out/r4_mmq4_tests_oldlib.log | tail -3
# timeout -k 10 900 $T -x tests/test_dropin_gpu.py tests/test_dropin_shapes_gpu.py > gpurun_out/r4_dropin_tests.log 2>&1
# echo "dropin tests rc=$?"; tail -3 gpurun_out/r4_dropin_tests.log
MX_TEST_NO_KLOG=1 GGML_MI355X_LIB=$PWD/llama-mi50.cpp_amd/lib_old/libggml-mi355x.so timeout -k 10 600 $T tests/test_mmq4_gpu.py -k "True or glu or group or moe or residual" > gpurun_out/r4_mmq4_tests_oldlib_noklog.log 2>&1
echo "old lib numeric rc=$?"; grep -E "passed|failed" gpurun_out/r4_mmq4_tests_oldlib_noklog.log | tail -3
timeout -k 10 950 bash scripts/r4_attrib.sh; echo "attrib rc=$?"
