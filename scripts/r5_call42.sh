#!/bin/bash
# PMC passes for the -fa 1 tg decode kernels at the round-5 end state (QKV, attention split
# partials, the O projection merging them, SwiGLU, down): SQ set + FETCH_SIZE
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
G8=$(python -c "import bench; print(bench.bench_gguf('llama3_8b', 'q4_k_m'))") || exit 1
export GGML_BACKEND_PATH=$PWD/llama-mi50.cpp_amd/lib/libggml-mi355x.so
OUT=gpurun_out/pmc_tg_fa1_sq KFILTER="k_qkv|k_fattn_dec2|k_gemv2" TMO=240 bash scripts/pmc_sq.sh oracle/_ref/llama-bench -m $G8 -t 8 -ngl 99 -fa 1 -p 0 -n 16 -r 1 -o jsonl && \
OUT=gpurun_out/pmc_tg_fa1_fetch KFILTER="k_qkv|k_fattn_dec2|k_gemv2" TMO=240 COUNTERS="FETCH_SIZE GRBM_GUI_ACTIVE" bash scripts/pmc_sq.sh oracle/_ref/llama-bench -m $G8 -t 8 -ngl 99 -fa 1 -p 0 -n 16 -r 1 -o jsonl
rc=$?; echo "rc=$rc"; python3 - <<'PY'
import json
for f in ("gpurun_out/pmc_tg_fa1_sq/summary.json", "gpurun_out/pmc_tg_fa1_fetch/summary.json"):
    try: d = json.load(open(f))
    except Exception as e: print(f, e); continue
    for k, v in d.items():
        print(f.split('/')[1], k[:60], {a: (round(b, 3) if isinstance(b, float) else b) for a, b in v.items() if a != 'per_dispatch'})
PY
exit $rc
