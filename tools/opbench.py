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


def case_gemm(pkg, be, rng, tname, K, M, N=512):
    """prefill GEMM: M weight rows x N tokens over K."""
    tid = NAMES[tname]
    w, _ = rand_quant(tid, M, K, rng)
    n = copies_for(len(w))
    ctx = pkg.Context()
    x = ctx.new_tensor("f32", K, N)
    tws = [ctx.new_tensor(tid, K, M) for _ in range(n)]
    gs = [ctx.build(ctx.mul_mat(tw, x)) for tw in tws]
    ctx.alloc(be)
    for tw in tws:
        tw.set(w)
    x.set(rng.standard_normal((N, K)).astype(np.float32))
    return ctx, gs


def case_gemm_qkv(pkg, be, rng, K=4096, Mq=4096, Mkv=1024, tv="q4_K", N=512):
    """prefill q/k/v projections sharing x (one graph: the executor's grouped GEMM)"""
    tq = NAMES["q4_K"]
    wq, _ = rand_quant(tq, Mq, K, rng)
    wk, _ = rand_quant(tq, Mkv, K, rng)
    wv, _ = rand_quant(NAMES[tv], Mkv, K, rng)
    n = copies_for(len(wq) + len(wk) + len(wv))
    ctx = pkg.Context()
    x = ctx.new_tensor("f32", K, N)
    sets = [(ctx.new_tensor(tq, K, Mq), ctx.new_tensor(tq, K, Mkv), ctx.new_tensor(NAMES[tv], K, Mkv)) for _ in range(n)]
    gs = [ctx.build(ctx.mul_mat(a, x), ctx.mul_mat(b, x), ctx.mul_mat(c, x)) for a, b, c in sets]
    ctx.alloc(be)
    for a, b, c in sets:
        a.set(wq); b.set(wk); c.set(wv)
    x.set(rng.standard_normal((N, K)).astype(np.float32))
    return ctx, gs


def case_gemm_glu(pkg, be, rng, tname, K, M, N=512):
    """prefill gate/up/SwiGLU GEMM pair (fused): 2 x M weight rows x N tokens over K."""
    tid = NAMES[tname]
    wg, _ = rand_quant(tid, M, K, rng)
    n = copies_for(2 * len(wg))
    ctx = pkg.Context()
    x = ctx.new_tensor("f32", K, N)
    pairs = [(ctx.new_tensor(tid, K, M), ctx.new_tensor(tid, K, M)) for _ in range(n)]
    gs = [ctx.build(ctx.swiglu_split(ctx.mul_mat(tg, x), ctx.mul_mat(tu, x))) for tg, tu in pairs]
    ctx.alloc(be)
    for tg, tu in pairs:
        tg.set(wg)
        tu.set(wg)
    x.set(rng.standard_normal((N, K)).astype(np.float32))
    return ctx, gs


def case_moe(pkg, be, rng, tname="q5_K", K=4096, M=14336, n_exp=8, used=2, T=512, skew=0.0):
    """MUL_MAT_ID at Mixtral shapes: T tokens x top-`used` of `n_exp` experts (uniform random
    routing; skew > 0 sends that fraction of the tokens to experts 0 and 1)"""
    tid = NAMES[tname]
    w1, _ = rand_quant(tid, M, K, rng)
    ctx = pkg.Context()
    tw = ctx.new_tensor(tid, K, M, n_exp)
    tx = ctx.new_tensor("f32", K, 1, T)
    ti = ctx.new_tensor("i32", used, T)
    g = ctx.build(ctx.mul_mat_id(tw, tx, ti))
    ctx.alloc(be)
    tw.set(np.tile(w1, n_exp))
    tx.set(rng.standard_normal((T, 1, K)).astype(np.float32))
    ids = np.stack([rng.permutation(n_exp)[:used] for _ in range(T)]).astype(np.int32)
    ns = int(skew * T)
    ids[:ns] = np.array([0, 1][:used], np.int32)
    ti.set(ids)
    return ctx, [g]


def case_ffn(pkg, be, rng, tname="q4_K", tdown="q4_K", K=4096, F=14336):
    """ffn_norm-less FFN block: gate/up SwiGLU GEMV (+q8 of its output) -> down + residual."""
    tid, tdn = NAMES[tname], NAMES[tdown]
    wg, _ = rand_quant(tid, F, K, rng)
    wd, _ = rand_quant(tdn, K, F, rng)
    n = copies_for(2 * len(wg) + len(wd))
    ctx = pkg.Context()
    x = ctx.new_tensor("f32", K, 1)
    graphs, ws = [], []
    for _ in range(n):
        tg, tu, td = ctx.new_tensor(tid, K, F), ctx.new_tensor(tid, K, F), ctx.new_tensor(tdn, F, K)
        ws += [(tg, wg), (tu, wg), (td, wd)]
        h = ctx.swiglu_split(ctx.mul_mat(tg, x), ctx.mul_mat(tu, x))
        graphs.append(ctx.add(ctx.mul_mat(td, h), x))
    graphs = [ctx.build(o) for o in graphs]
    ctx.alloc(be)
    for t, w in ws:
        t.set(w)
    x.set(rng.standard_normal(K).astype(np.float32))
    return ctx, graphs


def case_attn_in(pkg, be, rng, K=4096, H=32, Hkv=8, hd=128, n_ctx=512, tv="q6_K"):
    """attn_norm -> Q/K/V GEMVs -> RoPE(q, k) -> KV-cache stores: the fused QKV kernel."""
    tq = NAMES["q4_K"]
    wq, _ = rand_quant(tq, H * hd, K, rng)
    wk, _ = rand_quant(tq, Hkv * hd, K, rng)
    wv, _ = rand_quant(NAMES[tv], Hkv * hd, K, rng)
    n = copies_for(len(wq) + len(wk) + len(wv))
    ctx = pkg.Context()
    x = ctx.new_tensor("f32", K, 1)
    nw = ctx.new_tensor("f32", K)
    pos = ctx.new_tensor("i32", 1)
    kidx = ctx.new_tensor("i64", 1)
    graphs, ws = [], []
    for _ in range(n):
        a, b, c = ctx.new_tensor(tq, K, H * hd), ctx.new_tensor(tq, K, Hkv * hd), ctx.new_tensor(NAMES[tv], K, Hkv * hd)
        ws += [(a, wq), (b, wk), (c, wv)]
        kc = ctx.new_tensor("f16", Hkv * hd, n_ctx)
        vc = ctx.new_tensor("f16", Hkv * hd, n_ctx)
        cur = ctx.mul(ctx.rms_norm(x, 1e-5), nw)
        q = ctx.rope_ext(ctx.reshape(ctx.mul_mat(a, cur), hd, H, 1), pos, None, hd, 0, 8192, 500000.0)
        v = ctx.mul_mat(c, cur)
        k = ctx.rope_ext(ctx.reshape(ctx.mul_mat(b, cur), hd, Hkv, 1), pos, None, hd, 0, 8192, 500000.0)
        sk = ctx.set_rows(kc, ctx.reshape(k, Hkv * hd, 1), kidx)
        sv = ctx.set_rows(vc, v, kidx)
        graphs.append((q, sk, sv))
    graphs = [ctx.build(*o) for o in graphs]
    ctx.alloc(be)
    for t, w in ws:
        t.set(w)
    x.set(rng.standard_normal(K).astype(np.float32))
    nw.set(np.ones(K, np.float32))
    pos.set(np.array([17], np.int32))
    kidx.set(np.array([17], np.int64))
    return ctx, graphs


def case_ffn_block(pkg, be, rng, tname="q4_K", tdown="q4_K", K=4096, F=14336):
    """ffn_norm -> gate/up SwiGLU (norm absorbed, q8 out) -> down + residual: the decode FFN."""
    tid, tdn = NAMES[tname], NAMES[tdown]
    wg, _ = rand_quant(tid, F, K, rng)
    wd, _ = rand_quant(tdn, K, F, rng)
    n = copies_for(2 * len(wg) + len(wd))
    ctx = pkg.Context()
    x = ctx.new_tensor("f32", K, 1)
    nw = ctx.new_tensor("f32", K)
    graphs, ws = [], []
    for _ in range(n):
        tg, tu, td = ctx.new_tensor(tid, K, F), ctx.new_tensor(tid, K, F), ctx.new_tensor(tdn, F, K)
        ws += [(tg, wg), (tu, wg), (td, wd)]
        cur = ctx.mul(ctx.rms_norm(x, 1e-5), nw)
        h = ctx.swiglu_split(ctx.mul_mat(tg, cur), ctx.mul_mat(tu, cur))
        graphs.append(ctx.add(ctx.mul_mat(td, h), x))
    graphs = [ctx.build(o) for o in graphs]
    ctx.alloc(be)
    for t, w in ws:
        t.set(w)
    x.set(rng.standard_normal(K).astype(np.float32))
    nw.set(np.ones(K, np.float32))
    return ctx, graphs


def case_fa(pkg, be, rng, n_kv, H=32, Hkv=8, D=128, n_q=1):
    ctx = pkg.Context()
    q = ctx.new_tensor("f32", D, n_q, H)
    k = ctx.new_tensor("f16", D, n_kv, Hkv)
    v = ctx.new_tensor("f16", D, n_kv, Hkv)
    m = ctx.new_tensor("f16", n_kv, n_q)
    o = ctx.flash_attn_ext(q, k, v, m, 1.0 / np.sqrt(D))
    g = ctx.build(o)
    ctx.alloc(be)
    q.set(rng.standard_normal((H, n_q, D)).astype(np.float32))
    k.set(rng.standard_normal((Hkv, n_kv, D)).astype(np.float16).view(np.uint16))
    v.set(rng.standard_normal((Hkv, n_kv, D)).astype(np.float16).view(np.uint16))
    mask = np.zeros((n_q, n_kv), np.float32)
    for i in range(n_q):                      # causal, the prompt at the end of the cache
        mask[i, n_kv - n_q + i + 1:] = -np.inf
    m.set(mask.astype(np.float16).view(np.uint16))
    return ctx, [g]


def case_attn_o(pkg, be, rng, n_kv=256, H=32, Hkv=8, D=128, M=4096):
    """decode attention -> output projection (Q4_K) -> + residual: one k_attn_o launch
    (ops_attn_o.hip, opt-in): --ab 27=64 (v2), 27=96 (v2, one key split), 27=16 (v1); the
    default runs it unfused (k_fattn_dec2 + the GEMV)"""
    from qgen import NAMES
    K = D * H
    w, _ = rand_quant(NAMES["q4_K"], M, K, rng)
    n = copies_for(len(w))
    ctx = pkg.Context()
    q = ctx.new_tensor("f32", D, 1, H)
    k = ctx.new_tensor("f16", D, n_kv, Hkv)
    v = ctx.new_tensor("f16", D, n_kv, Hkv)
    m = ctx.new_tensor("f16", n_kv, 1)
    r = ctx.new_tensor("f32", M, 1)
    fa = ctx.flash_attn_ext(q, k, v, m, 1.0 / np.sqrt(D))
    ws, graphs = [], []
    for _ in range(n):
        tw = ctx.new_tensor(NAMES["q4_K"], K, M)
        ws.append(tw)
        graphs.append(None)
    outs = [ctx.add(ctx.mul_mat(tw, ctx.reshape(fa, K, 1)), r) for tw in ws]
    graphs = [ctx.build(o) for o in outs]
    ctx.alloc(be)
    for tw in ws:
        tw.set(w)
    q.set(rng.standard_normal((H, 1, D)).astype(np.float32))
    k.set(rng.standard_normal((Hkv, n_kv, D)).astype(np.float16).view(np.uint16))
    v.set(rng.standard_normal((Hkv, n_kv, D)).astype(np.float16).view(np.uint16))
    m.set(np.zeros((1, n_kv), np.float16).view(np.uint16))
    r.set(rng.standard_normal(M).astype(np.float32))
    return ctx, graphs


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
    "attn_in": lambda p, b, r: case_attn_in(p, b, r),
    "pp_q_q4k": lambda p, b, r: case_gemm(p, b, r, "q4_K", 4096, 4096),
    "pp_gate_q4k": lambda p, b, r: case_gemm(p, b, r, "q4_K", 4096, 14336),
    "pp_down_q6k": lambda p, b, r: case_gemm(p, b, r, "q6_K", 14336, 4096),
    "pp_k_q4k": lambda p, b, r: case_gemm(p, b, r, "q4_K", 4096, 1024),
    "pp_glu_q4k": lambda p, b, r: case_gemm_glu(p, b, r, "q4_K", 4096, 14336),
    "pp_qkv": lambda p, b, r: case_gemm_qkv(p, b, r),
    "pp_qkv_v6": lambda p, b, r: case_gemm_qkv(p, b, r, tv="q6_K"),
    "pp_glu_q4k_2048": lambda p, b, r: case_gemm_glu(p, b, r, "q4_K", 4096, 14336, N=2048),
    "pp_q_q4k_2048": lambda p, b, r: case_gemm(p, b, r, "q4_K", 4096, 4096, N=2048),
    "pp_glu_q5k": lambda p, b, r: case_gemm_glu(p, b, r, "q5_K", 4096, 14336),
    "pp_moe_q5k": lambda p, b, r: case_moe(p, b, r),
    "pp_moe_q5k_skew": lambda p, b, r: case_moe(p, b, r, skew=0.9),
    "tg_moe_q5k": lambda p, b, r: case_moe(p, b, r, T=1),
    "pp_down_q4k": lambda p, b, r: case_gemm(p, b, r, "q4_K", 14336, 4096),
    "ffn_q4k": lambda p, b, r: case_ffn(p, b, r),
    "ffn_block": lambda p, b, r: case_ffn_block(p, b, r),
    # workgroup-balance probes: 448 SwiGLU workgroups (F 14336) are 1.75 per CU; F 16384 /
    # 8192 / 12288 give exactly 2 / 1 / 1.5 per CU
    "ffn_block_16384": lambda p, b, r: case_ffn_block(p, b, r, F=16384),
    "ffn_block_12288": lambda p, b, r: case_ffn_block(p, b, r, F=12288),
    "ffn_block_8192": lambda p, b, r: case_ffn_block(p, b, r, F=8192),
    "ffn_q4k_q6k": lambda p, b, r: case_ffn(p, b, r, tdown="q6_K"),
    "fa_256": lambda p, b, r: case_fa(p, b, r, 256),
    "fa_1024": lambda p, b, r: case_fa(p, b, r, 1024),
    "fa_4096": lambda p, b, r: case_fa(p, b, r, 4096),
    "fa_16384": lambda p, b, r: case_fa(p, b, r, 16384),
    "fa_32768": lambda p, b, r: case_fa(p, b, r, 32768),
    "fa_pp512": lambda p, b, r: case_fa(p, b, r, 512, n_q=512),
    "fa_pp2048": lambda p, b, r: case_fa(p, b, r, 2048, n_q=512),
    "rms_mul": lambda p, b, r: case_rms(p, b, r),
    "attn_o": lambda p, b, r: case_attn_o(p, b, r),
}


SWEEP = [(16, 2), (16, 4), (16, 8), (32, 2), (32, 4), (32, 8), (64, 2), (64, 4), (64, 8)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", nargs="*")
    ap.add_argument("--iters", type=int, default=ITERS)
    ap.add_argument("--sweep", action="store_true", help="GEMV cases under every (lanes/row, units/lane) geometry")
    ap.add_argument("--trace", action="store_true", help="print phase timestamps of workgroup 0")
    ap.add_argument("--trace-blocks", action="store_true", help="GEMV cases: per-workgroup start/end spread")
    ap.add_argument("--sweep-mm", action="store_true", help="pp_* cases under both GEMM row tiles (64, 128)")
    ap.add_argument("--sweep-glu8", action="store_true", help="ffn cases under every q8-emitting SwiGLU geometry")
    ap.add_argument("--sweep3", action="store_true", help="GEMV v3 cases under every geometry id x workgroups per CU")
    ap.add_argument("--bpc", nargs="*", type=int, default=[1, 2, 4], help="--sweep3 workgroups per CU")
    ap.add_argument("--ab", nargs="*", default=None, help="repeat each case under these tune settings, e.g. 14=0 14=1,11=2")
    ap.add_argument("--dbg", nargs="*", type=int, default=None,
                    help="timing experiments: repeat each case under these GEMV dbg masks (1 no prologue, 2 no dots, 4 no epilogue math)")
    args = ap.parse_args()
    pkg = load_package()
    lib = pkg._lib.load()
    be = pkg.Backend(0)
    rng = np.random.default_rng(0)
    names = []
    for name in args.only or list(CASES):
        cfgs = [None]
        if args.sweep_mm and name.startswith("pp_"):
            ctx, graphs = CASES[name](pkg, be, rng)
            for bm in (64, 128):
                lib.ggml_backend_mi355x_set_tune(8, bm)
                separator(pkg, be)
                for it in range(args.iters):
                    ctx.compute(be, graphs[it % len(graphs)])
                be.synchronize()
                names.append(f"{name}@bm{bm}")
            lib.ggml_backend_mi355x_set_tune(8, 0)
            ctx.free()
            continue
        if args.sweep and not name.startswith(("fa_", "rms", "ffn")):
            cfgs = [c for c in SWEEP if not (name.startswith("glu") and c[1] == 8)]
        ctx, graphs = CASES[name](pkg, be, rng)
        if args.sweep_glu8 and name.startswith("ffn"):
            for v in range(4):
                for mode in range(3):
                    lib.ggml_backend_mi355x_set_tune(4, v)
                    lib.ggml_backend_mi355x_set_tune(9, mode)
                    separator(pkg, be)
                    for it in range(args.iters):
                        ctx.compute(be, graphs[it % len(graphs)])
                    be.synchronize()
                    names.append(f"{name}@glu8v{v}m{mode}")
            lib.ggml_backend_mi355x_set_tune(4, 0)
            lib.ggml_backend_mi355x_set_tune(9, 0)
            ctx.free()
            continue
        if args.trace:
            import ctypes
            lib.ggml_backend_mi355x_set_tune(6, 1)
            buf = (ctypes.c_ulonglong * 2048)()
            lib.ggml_backend_mi355x_trace_read(buf, 2048)        # clear
            for it in range(3):
                ctx.compute(be, graphs[it % len(graphs)])
            be.synchronize()
            lib.ggml_backend_mi355x_trace_read(buf, 2048)
            lib.ggml_backend_mi355x_set_tune(6, 0)
            for slot, sname in enumerate(["fa_dec", "gemv", "qkv", "mmq4"]):
                for w in range(16):
                    t = [buf[slot * 128 + w * 8 + k] for k in range(8)]
                    if t[0] == 0:
                        continue
                    print(f"trace {name} {sname} wave{w}: " + " ".join(str(x - t[0]) if x else "-" for x in t[1:]), flush=True)
        if args.trace_blocks:
            import ctypes
            lib.ggml_backend_mi355x_set_tune(6, 2)
            for it in range(3):
                ctx.compute(be, graphs[it % len(graphs)])
            be.synchronize()
            n = 2 * 65536
            buf = (ctypes.c_ulonglong * n)()
            lib.ggml_backend_mi355x_trace_blocks_read(buf, n)
            lib.ggml_backend_mi355x_set_tune(6, 0)
            a = np.frombuffer(buf, dtype=np.uint64).reshape(-1, 2).astype(np.int64)
            a = a[(a[:, 0] > 0) & (a[:, 1] > 0)]
            if len(a):
                t0 = a[:, 0].min()
                st, en = (a[:, 0] - t0) * 10, (a[:, 1] - t0) * 10   # ns
                dur = en - st
                print(f"blocks {name}: n={len(a)} start[p50,p90,max]={np.percentile(st,50):.0f},{np.percentile(st,90):.0f},{st.max():.0f}ns "
                      f"end[min,p50,max]={en.min():.0f},{np.percentile(en,50):.0f},{en.max():.0f}ns dur[p10,p50,p90]={np.percentile(dur,10):.0f},"
                      f"{np.percentile(dur,50):.0f},{np.percentile(dur,90):.0f}ns", flush=True)
                q = [0, 10, 25, 50, 75, 90, 100]
                print(f"blocks {name}: dur pct {q} = {[int(np.percentile(dur, x)) for x in q]} ns; "
                      f"end pct = {[int(np.percentile(en, x)) for x in q]} ns", flush=True)
        if args.sweep3 and not name.startswith(("fa_", "rms", "pp_")):
            for cfg in range(6):
                for bpc in args.bpc:
                    lib.ggml_backend_mi355x_set_tune(12, cfg + 1)
                    lib.ggml_backend_mi355x_set_tune(13, bpc)
                    separator(pkg, be)
                    for it in range(args.iters):
                        ctx.compute(be, graphs[it % len(graphs)])
                    be.synchronize()
                    names.append(f"{name}@c{cfg}b{bpc}")
            lib.ggml_backend_mi355x_set_tune(12, 0)
            lib.ggml_backend_mi355x_set_tune(13, 0)
            ctx.free()
            continue
        if args.ab:
            for spec in args.ab:
                kv = [tuple(int(x) for x in t.split("=")) for t in spec.split(",") if t]
                for k, v in kv:
                    lib.ggml_backend_mi355x_set_tune(k, v)
                separator(pkg, be)
                for it in range(args.iters):
                    ctx.compute(be, graphs[it % len(graphs)])
                be.synchronize()
                names.append(f"{name}@{spec}")
                for k, _ in kv:
                    lib.ggml_backend_mi355x_set_tune(k, 0)
            ctx.free()
            continue
        if args.dbg:
            for d in args.dbg:
                lib.ggml_backend_mi355x_set_tune(11, d)
                separator(pkg, be)
                for it in range(args.iters):
                    ctx.compute(be, graphs[it % len(graphs)])
                be.synchronize()
                names.append(f"{name}@dbg{d}")
            lib.ggml_backend_mi355x_set_tune(11, 0)
            ctx.free()
            continue
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
