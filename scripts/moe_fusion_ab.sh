#!/bin/bash
# A/B of the MoE fusions on a tiny synthetic MoE GGUF: reference libllama on this backend
# (-ngl 99) vs the reference CPU backend, prefill of 40 tokens and incremental decode.
cd "$(dirname "$0")/.."
python tools/gguf_synth.py --shape tiny_moe --recipe q4_k_m --out /tmp/tm.gguf > /dev/null
python -c "import numpy as np; np.random.default_rng(7).integers(0, 1000, 40).astype(np.int32).tofile('/tmp/t40.i32')"
for inc in "" --incremental; do
  oracle/_ref/ref-llama-bench -m /tmp/tm.gguf -t 8 -ngl 0 -fa 1 --logits /tmp/t40.i32 /tmp/cpu.f32 $inc > /dev/null 2>&1
  for v in NONE GGML_MI355X_NO_TOPK_FUSION GGML_MI355X_NO_COMBINE_FUSION; do
    rm -f /tmp/kl.txt
    env $v=1 GGML_MI355X_KLOG=/tmp/kl.txt GGML_BACKEND_PATH=$PWD/llama-mi50.cpp_amd/lib/libggml-mi355x.so timeout -k 5 60 \
      oracle/_ref/ref-llama-bench -m /tmp/tm.gguf -t 8 -ngl 99 -fa 1 --logits /tmp/t40.i32 /tmp/gpu.f32 $inc > /dev/null 2>&1
    python -c "
import numpy as np; a=np.fromfile('/tmp/cpu.f32',np.float32).reshape(40,-1); b=np.fromfile('/tmp/gpu.f32',np.float32).reshape(40,-1)
print('${inc:-prefill}', '$v', float(((a-b)**2).sum()/(a**2).sum()))"
    if [ "$v" = NONE ]; then grep -E "topk|combine" /tmp/kl.txt | sort | uniq -c; fi
  done
done
true
