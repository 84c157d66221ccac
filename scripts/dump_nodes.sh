#!/bin/bash
# Per-node parity of the reference libllama on the MI355X backend vs its CPU backend:
# SHAPE/RECIPE GGUF from tools/gguf_synth.py, N prompt tokens, both runs dumped with
# ref-llama-bench --dump/--dump-dir, compared by tools/dump_compare.py.
cd "$(dirname "$0")/.."
SHAPE=${SHAPE:-mixtral_2l}; RECIPE=${RECIPE:-q5_k_m}; N=${N:-64}; FA=${FA:-1}; LAST=${LAST:-8}
OUT=${OUT:-gpurun_out/dump}; W=/tmp/dumpw
mkdir -p $OUT $W/cpu $W/gpu
python tools/gguf_synth.py --shape $SHAPE --recipe $RECIPE --out $W/m.gguf > /dev/null || exit 1
python -c "import numpy as np; np.random.default_rng(25).integers(0, 32000, $N).astype(np.int32).tofile('$W/t.i32')"
timeout -k 10 300 oracle/_ref/ref-llama-bench -m $W/m.gguf -t 16 -ngl 0 -fa $FA --logits $W/t.i32 $W/o_cpu.f32 \
  --last $LAST --dump $W/cpu.txt --dump-dir $W/cpu ${EXTRA:-} > /dev/null || exit 1
GGML_BACKEND_PATH=$PWD/llama-mi50.cpp_amd/lib/libggml-mi355x.so timeout -k 10 300 oracle/_ref/ref-llama-bench -m $W/m.gguf \
  -t 16 -ngl 99 -fa $FA --logits $W/t.i32 $W/o_gpu.f32 --last $LAST --dump $W/gpu.txt --dump-dir $W/gpu ${EXTRA:-} > /dev/null || exit 1
python tools/dump_compare.py $W/cpu.txt $W/cpu $W/gpu.txt $W/gpu "${DETAIL:-}" > $OUT/${SHAPE}_fa${FA}.txt
cat $OUT/${SHAPE}_fa${FA}.txt
