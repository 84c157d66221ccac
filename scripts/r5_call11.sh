#!/bin/bash
# MoE prefill gate/up/SwiGLU fused (k_mmq4 EPI 3): op tests, Mixtral per-position test, MoE bench leg, pp512 profile
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_mmq4_gpu.py -k "moe" -x -q -s --timeout 300 --timeout-method thread > gpurun_out/r5_c11_ops.log 2>&1
rc=$?; echo "ops rc=$rc"; tail -3 gpurun_out/r5_c11_ops.log; grep -E "^FAILED|Error|assert" gpurun_out/r5_c11_ops.log | head -10
[ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u -m pytest tests/test_dropin_shapes_gpu.py -k mixtral -x -q -s --timeout 800 --timeout-method thread \
   > gpurun_out/r5_c11_moe_test.log 2>&1
rc=$?; echo "moe test rc=$rc"; grep -E "prefill:|decode:|passed|failed|Error|assert" gpurun_out/r5_c11_moe_test.log | head -20
[ $rc -ne 0 ] && exit $rc
timeout -k 10 1200 python bench.py --moe-only --dropin-reps 3 > gpurun_out/r5_moe_leg4.json 2> gpurun_out/r5_moe_leg4.err
echo "moe leg rc=$?"; cut -c1-1500 gpurun_out/r5_moe_leg4.json
G=$(python -c "import bench; print(bench.bench_gguf('mixtral_8x7b', 'q5_k_m'))") || exit 1
export GGML_BACKEND_PATH=$PWD/llama-mi50.cpp_amd/lib/libggml-mi355x.so DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_moe4_pp -o run --output-format csv -- \
    oracle/_ref/llama-bench -m $G -t 8 -ngl 99 -fa 1 -p 512 -n 0 -r 2 -o jsonl > gpurun_out/prof_moe4_pp.log 2>&1
echo "pp rc=$?"; head -14 gpurun_out/prof_moe4_pp/run_kernel_stats.csv | cut -c1-150
