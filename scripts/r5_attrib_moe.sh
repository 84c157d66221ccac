#!/bin/bash
# Per-node attribution of the Mixtral-width (mixtral_2l Q5_K_M) prompt error: the reference
# libllama on mixtral_2l, 128 prompt tokens, node dumps from the reference CPU backend
# and from this backend, then tools/mm_attrib.py (every MUL_MAT against float64 W.x).
cd "$(dirname "$0")/.."
SHAPE=${SHAPE:-mixtral_2l}; N=${N:-128}; FA=${FA:-1}; RECIPE=${RECIPE:-q5_k_m}
OUT=${OUT:-gpurun_out/attrib}; W=${TMPDIR:-/tmp}/attrib_$SHAPE
mkdir -p $OUT $W/cpu $W/gpu
[ -f $W/m.gguf ] || timeout -k 10 600 python tools/gguf_synth.py --shape $SHAPE --recipe $RECIPE --out $W/m.gguf > /dev/null || exit 1
python -c "import numpy as np; np.random.default_rng(32).integers(0, 32000, $N).astype(np.int32).tofile('$W/t.i32')"
timeout -k 10 600 oracle/_ref/ref-llama-bench -m $W/m.gguf -t 16 -ngl 0 -fa $FA --logits $W/t.i32 $W/o_cpu.f32 \
  --last 16 --dump $W/cpu.txt --dump-dir $W/cpu > $OUT/cpu_run.txt 2>&1 || { tail $OUT/cpu_run.txt; exit 1; }
GGML_BACKEND_PATH=$PWD/llama-mi50.cpp_amd/lib/libggml-mi355x.so timeout -k 10 600 oracle/_ref/ref-llama-bench -m $W/m.gguf \
  -t 16 -ngl 99 -fa $FA --logits $W/t.i32 $W/o_gpu.f32 --last 16 --dump $W/gpu.txt --dump-dir $W/gpu > $OUT/gpu_run.txt 2>&1 || { tail $OUT/gpu_run.txt; exit 2; }
MOE_ROWS=${MOE_ROWS:-256} timeout -k 10 900 python tools/mm_attrib.py $W/m.gguf $W/cpu.txt $W/cpu $W/gpu.txt $W/gpu > $OUT/${SHAPE}_fa${FA}.txt 2>&1
rc=$?; cat $OUT/${SHAPE}_fa${FA}.txt; rm -rf $W/cpu $W/gpu; exit $rc
