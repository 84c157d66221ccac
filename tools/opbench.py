#!/usr/bin/env python3
"""Per-op micro-benchmark of the decode hot path (Llama-3-8B shapes) on one MI355X.

Run under rocprofv3 (kernel trace) with HIP graphs off; each case is bracketed by a
separator launch (an ARGSORT graph) so tools/opbench_report.py can attribute kernel
durations to cases:

  GGML_MI355X_DISABLE_GRAPHS=1 rocprofv3 --kernel-trace -d gpurun_out/ob -o ob \
      --output-format csv -- python3 tools/opbench.py [--only NAME ...]

Inputs are random bytes/values of the real shapes (weights read once per launch from
HBM: every case rotates over enough weight copies to defeat the 256 MiB MALL).
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from mi355x_pkg import load_package  # noqa: E402
from qgen import NAMES, rand_quant  # noqa: E402

ITERS = 40
MALL_BYTES = 320 << 20


def separator(pkg, be):
    ctx = pkg.Context()
    a = ctx.new_tensor("f32", 16, 1)
    g = ctx.build(ctx.argsort(a))
    ctx.alloc(be)
    a.set(np.arange(16, dtype=np.float32))
    ctx.compute(be, g)
    ctx.free()


def copies_for(nbytes):
    return int(max(1, min(16, -(-MALL_BYTES // max(nbytes, 1)))))


def case_gemv(pkg, be, rng, tname, K, M, glu=False, add=False):
    tid = NAMES[tname]
    w, rb = rand_quant(tid, M, K, rng)
    n = copies_for(len(w) * (2 if glu else 1))
    ctx = pkg.Context()
    x = ctx.new_tensor("f32", K, 1)
    outs, ws = [], []
    for _ in range(n):
        tw = ctx.new_tensor(tid, K, M)
        ws.append(tw)
        y = ctx.mul_mat(tw, x)
        if glu:
            tu = ctx.new_tensor(tid, K, M)
            ws.append(tu)
            y = ctx.swiglu_split(y, ctx.mul_mat(tu, x))
        if add:
            r = ctx.new_tensor("f32", M, 1)
            y = ctx.add(y, r)
        outs.append(y)
    graphs = [ctx.build(o) for o in outs]
    ctx.alloc(be)
    for tw in ws:
        tw.set(w)
    x.set(rng.standard_normal(K).astype(np.float32))
    return ctx, graphs


def case_fa(pkg, be, rng, n_kv, H=32, Hkv=8, D=128):
    ctx = pkg.Context()
    q = ctx.new_tensor("f32", D, 1, H)
    k = ctx.new_tensor("f16", D, n_kv, Hkv)
    v = ctx.new_tensor("f16", D, n_kv, Hkv)
    m = ctx.new_tensor("f16", n_kv, 1)
    o = ctx.flash_attn_ext(q, k, v, m, 1.0 / np.sqrt(D))
    g = ctx.build(o)
    ctx.alloc(be)
    q.set(rng.standard_normal((H, D)).astype(np.float32))
    k.set(rng.standard_normal((Hkv, n_kv, D)).astype(np.float16).view(np.uint16))
    v.set(rng.standard_normal((Hkv, n_kv, D)).astype(np.float16).view(np.uint16))
    m.set(np.zeros(n_kv, np.float16).view(np.uint16))
    return ctx, [g]


def case_rms(pkg, be, rng, K=4096):
    ctx = pkg.Context()
    x = ctx.new_tensor("f32", K, 1)
    w = ctx.new_tensor("f32", K)
    y = ctx.mul(ctx.rms_norm(x, 1e-5), w)
    g = ctx.build(y)
    ctx.alloc(be)
    x.set(rng.standard_normal(K).astype(np.float32))
    w.set(np.ones(K, np.float32))
    return ctx, [g]


CASES = {
    "q_q4k": lambda p, b, r: case_gemv(p, b, r, "q4_K", 4096, 4096),
    "k_q4k": lambda p, b, r: case_gemv(p, b, r, "q4_K", 4096, 1024),
    "v_q6k": lambda p, b, r: case_gemv(p, b, r, "q6_K", 4096, 1024),
    "o_q4k_add": lambda p, b, r: case_gemv(p, b, r, "q4_K", 4096, 4096, add=True),
    "glu_q4k": lambda p, b, r: case_gemv(p, b, r, "q4_K", 4096, 14336, glu=True),
    "down_q4k_add": lambda p, b, r: case_gemv(p, b, r, "q4_K", 14336, 4096, add=True),
    "down_q6k_add": lambda p, b, r: case_gemv(p, b, r, "q6_K", 14336, 4096, add=True),
    "lm_head_q6k": lambda p, b, r: case_gemv(p, b, r, "q6_K", 4096, 128256),
    "fa_256": lambda p, b, r: case_fa(p, b, r, 256),
    "fa_1024": lambda p, b, r: case_fa(p, b, r, 1024),
    "fa_4096": lambda p, b, r: case_fa(p, b, r, 4096),
    "rms_mul": lambda p, b, r: case_rms(p, b, r),
}


SWEEP = [(16, 2), (16, 4), (16, 8), (32, 2), (32, 4), (32, 8), (64, 2), (64, 4), (64, 8)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", nargs="*")
    ap.add_argument("--iters", type=int, default=ITERS)
    ap.add_argument("--sweep", action="store_true", help="GEMV cases under every (lanes/row, units/lane) geometry")
    args = ap.parse_args()
    pkg = load_package()
    lib = pkg._lib.load()
    be = pkg.Backend(0)
    rng = np.random.default_rng(0)
    names = []
    for name in args.only or list(CASES):
        cfgs = [None]
        if args.sweep and not name.startswith(("fa_", "rms")):
            cfgs = [c for c in SWEEP if not (name.startswith("glu") and c[1] == 8)]
        ctx, graphs = CASES[name](pkg, be, rng)
        for cfg in cfgs:
            base = 2 if name.startswith("glu") else 0
            lib.ggml_backend_mi355x_set_tune(base, cfg[0] if cfg else 0)
            lib.ggml_backend_mi355x_set_tune(base + 1, cfg[1] if cfg else 0)
            label = name + (f"@{cfg[0]}x{cfg[1]}" if cfg else "")
            separator(pkg, be)
            for it in range(args.iters):
                ctx.compute(be, graphs[it % len(graphs)])
            be.synchronize()
            names.append(label)
            print(f"case {label}: {len(graphs)} weight copies x {args.iters} iters", flush=True)
        lib.ggml_backend_mi355x_set_tune(0, 0); lib.ggml_backend_mi355x_set_tune(1, 0)
        lib.ggml_backend_mi355x_set_tune(2, 0); lib.ggml_backend_mi355x_set_tune(3, 0)
        ctx.free()
    separator(pkg, be)
    with open(os.environ.get("OPBENCH_CASES", "gpurun_out/opbench_cases.txt"), "w") as f:
        f.write("\n".join(names) + "\n")


if __name__ == "__main__":
    main()
