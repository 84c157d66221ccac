#!/usr/bin/env python3
"""How fast is a plain f16 GEMM (torch -> hipBLASLt) at the prefill shapes? (MEASUREMENT
PROBE for the dequantised-weight-cache design question; not part of the product.)
y[N, M] = x[N, K] @ W[M, K]^T with f16 inputs, f32 accumulate, f16 or f32 out."""
import torch

def bench(fn, iters=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1000 / iters

dev = "cuda"
for N, K, M, name in [(512, 4096, 28672, "glu gate+up"), (512, 14336, 4096, "down"), (512, 4096, 6144, "qkv"),
                      (512, 4096, 4096, "o"), (2048, 4096, 28672, "glu pp2048"), (512, 8192, 57344, "70b glu")]:
    x = torch.randn(N, K, device=dev, dtype=torch.float16)
    ws = [torch.randn(M, K, device=dev, dtype=torch.float16) * 0.02 for _ in range(max(1, min(8, (320 << 20) // (M * K * 2) + 1)))]
    i = [0]
    def f():
        i[0] = (i[0] + 1) % len(ws)
        return x @ ws[i[0]].t()
    t = bench(f)
    print(f"{name:12s} N={N} K={K} M={M}: {t:8.1f} us  {2 * N * K * M / t / 1e6:7.1f} TFLOP/s  (weights rotated x{len(ws)})", flush=True)
