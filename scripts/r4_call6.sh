#!/bin/bash
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
T="python -u -m pytest -q --timeout 600 --timeout-method thread -m gpu"
timeout -k 10 600 $T tests/test_mmq4_gpu.py tests/test_ops_gpu.py tests/test_shapes_gpu.py tests/test_llama_gpu.py > gpurun_out/r4_c6_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r4_c6_tests.log; grep -E "^FAILED" gpurun_out/r4_c6_tests.log | head
[ $rc -ge 124 ] && exit $rc
timeout -k 10 600 $T tests/test_dropin_shapes_gpu.py -k "pp512 or pp2048 or mixtral" > gpurun_out/r4_c6_dropin.log 2>&1; echo "dropin rc=$?"; tail -2 gpurun_out/r4_c6_dropin.log; grep -E "^FAILED" gpurun_out/r4_c6_dropin.log | head
timeout -k 10 600 python bench.py --steps 5 --warmup 1 --depths "" > gpurun_out/r4_bench2.json 2> gpurun_out/r4_bench2.err; echo "bench rc=$?"
python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/r4_bench2.json') if l.startswith('{')][-1])
print('value', d['value'], 'pp512', d['pp512_tok_s'], 'runner', d['runner']['tg128_tok_s'], d['runner']['pp512_tok_s'], d['runner']['pp2048_tok_s'])
print({k: v for k, v in d['dropin'].items() if k.endswith('tok_s')})"
