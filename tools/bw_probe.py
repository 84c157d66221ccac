"""HBM read-bandwidth calibration (torch reductions / copies over n MB): what a plain
streaming kernel reaches at the sizes the decode kernels move per launch"""
import sys, torch
dev = torch.device("cuda:0")
for mb in [16, 64, 256, 1024]:
    n = mb * 1024 * 1024 // 2
    x = torch.randn(n, device=dev, dtype=torch.float32).to(torch.float16)
    y = torch.empty_like(x)
    for name, fn, bytes_ in [("sum", lambda: x.sum(dtype=torch.float32), n * 2), ("copy", lambda: y.copy_(x), n * 4)]:
        for _ in range(5): fn()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        its = 50
        s.record()
        for _ in range(its): fn()
        e.record(); torch.cuda.synchronize()
        t = s.elapsed_time(e) / its * 1e-3
        print(f"{name} {mb} MB: {t*1e6:.1f} us  {bytes_/t/1e12:.2f} TB/s", flush=True)
