"""Op-level parity of the default prefill GEMM, k_mmq4 (ops_mmq4.hip), against the CPU
oracle — every epilogue the executor launches it with, each asserted from the
kernel-choice log:

* EPI 0 plain and + residual (MUL_MAT, MUL_MAT -> ADD; reference mul_mat_q,
  ggml-cuda/mmq.cuh:3364-3700), split-K off and forced on (g_tune[20]: the partial
  planes and k_mmq4_reduce, the reference's stream-k fixup role, mmq.cuh:3701);
* EPI 0 grouped (q/k/v: 2-3 weights sharing src1, mixed K-quant types in one launch);
* EPI 1 gate/up SwiGLU (ggml-cuda.cu:2145-2181 semantics);
* EPI 2 MoE expert tiles (MUL_MAT_ID, device-side expert sort; ggml-cuda/mmid.cu:28-160).

Ragged shapes throughout (M not a multiple of the 256-row tile, N not a multiple of the
128-token tile). Tolerance: NMSE 5e-4 against the float64 product of the dequantised
weights and the f32 input (tests/test-backend-ops.cpp:3718).

Outlier rows: k_mmq4 dequantises weights into f16 MFMA operands scaled by 2^10; a block
whose scaled values would pass the f16 range (|w| > 32 at 2^10) lowers its row's scale
(m4_range). The outlier cases put |w| up to ~200 in whole rows, in the LAST super-block of
a row (the rescale happens after accumulation started) and in the first one."""
import os

import numpy as np
import pytest

from qgen import NAMES, nmse, rand_quant

pytestmark = pytest.mark.gpu

BLOCK = {12: 144, 13: 176, 14: 210, 8: 34}
QK = {12: 256, 13: 256, 14: 256, 8: 32}                # weights per block
BIG_D = {12: (0, 0.2), 13: (0, 0.1), 14: (208, 0.05), 8: (0, 1.6)}   # (f16 d offset, d): |w| up to ~190-205


def with_outliers(raw, tid, M, K, rng):
    """rows 5 (last super-block), 77 (first super-block) and M-3 (every block) get d so
    large that the dequantised weights reach |w| ~ 200; returns (raw, outlier row list)"""
    raw = raw.copy()
    bs, nb = BLOCK[tid], K // QK[tid]
    off, d = BIG_D[tid]
    blocks = raw.reshape(M, nb, bs)
    sel = [(5, [nb - 1]), (77 % M, [0]), (M - 3, list(range(nb)))]
    for r, bl in sel:
        for b in bl:
            v = np.float16(d * rng.uniform(0.8, 1.0))
            blocks[r, b, off:off + 2] = np.frombuffer(v.tobytes(), np.uint8)
    return blocks.reshape(-1), sorted({r for r, _ in sel})


def check(y, ref, rows_out=()):
    assert np.all(np.isfinite(y)), "non-finite output (f16 operand overflow?)"
    normal = np.setdiff1d(np.arange(ref.shape[1]), rows_out)
    assert nmse(y[:, normal], ref[:, normal]) < 5e-4
    if len(rows_out):
        assert nmse(y[:, rows_out], ref[:, rows_out]) < 5e-4


def run(pkg, be, build, tune=()):
    lib = pkg._lib.load()
    for k, v in tune:
        lib.ggml_backend_mi355x_set_tune(k, v)
    try:
        ctx = pkg.Context()
        outs, feed = build(ctx)
        g = ctx.build(*outs)
        ctx.alloc(be)
        for t, arr in feed:
            t.set(arr)
        be.klog(True)
        ctx.compute(be, g)
        res = [o.numpy() for o in outs]
        log = be.klog_read()
        be.klog(False)
        ctx.free()
    finally:
        for k, _ in tune:
            lib.ggml_backend_mi355x_set_tune(k, 0)
    return res, log


# MX_TEST_NO_KLOG=1: numeric checks only (running these cases against an older build whose
# kernel-choice log lacks the launch lines, profiles/r04/mmq4_outlier_old_vs_new.txt)
NO_KLOG = os.environ.get("MX_TEST_NO_KLOG") == "1"


def launch_lines(log):
    return [l for l in log if l.startswith("mmq4 launch ")]


def klog_has(log, pred):
    return NO_KLOG or any(pred(l) for l in log)


@pytest.mark.parametrize("tname", ["q4_K", "q5_K", "q6_K", "q8_0"])
@pytest.mark.parametrize("ks", [1, 2, 4])
@pytest.mark.parametrize("outlier", [False, True])
def test_mmq4_plain(pkg, backend, orc, tname, ks, outlier):
    tid = NAMES[tname]
    rng = np.random.default_rng(1000 * tid + 10 * ks + outlier)
    K, M, N = 2048, 300, 150
    w, rb = rand_quant(tid, M, K, rng)
    rows_out = []
    if outlier:
        w, rows_out = with_outliers(w, tid, M, K, rng)
    x = rng.standard_normal((N, K)).astype(np.float32)

    def build(ctx):
        tw = ctx.new_tensor(tid, K, M)
        tx = ctx.new_tensor("f32", K, N)
        return [ctx.mul_mat(tw, tx)], [(tw, w), (tx, x)]

    (y,), log = run(pkg, backend, build, [(20, ks)])
    assert klog_has(log, lambda l: l.startswith(f"mmq4 qt={tid} ")), log
    assert NO_KLOG or (launch_lines(log) and all(f"epi=0 ks={ks} " in l for l in launch_lines(log))), log
    check(y.reshape(N, M), orc.mul_mat(tid, w, rb, x, exact=True), rows_out)


@pytest.mark.parametrize("tname", ["q4_K", "q6_K"])
@pytest.mark.parametrize("ks", [1, 2])
def test_mmq4_residual(pkg, backend, orc, tname, ks):
    """MUL_MAT -> ADD: the residual added in the k_mmq4 epilogue (ks 1) or in k_mmq4_reduce"""
    tid = NAMES[tname]
    rng = np.random.default_rng(77 + ks + tid)
    K, M, N = 2048, 300, 150
    w, rb = rand_quant(tid, M, K, rng)
    w, rows_out = with_outliers(w, tid, M, K, rng)
    x = rng.standard_normal((N, K)).astype(np.float32)
    r = rng.standard_normal((N, M)).astype(np.float32)

    def build(ctx):
        tw = ctx.new_tensor(tid, K, M)
        tx = ctx.new_tensor("f32", K, N)
        tr = ctx.new_tensor("f32", M, N)
        return [ctx.add(ctx.mul_mat(tw, tx), tr)], [(tw, w), (tx, x), (tr, r)]

    (y,), log = run(pkg, backend, build, [(20, ks)])
    assert klog_has(log, lambda l: l.startswith(f"mmq4 qt={tid} ") and "res=1" in l), log
    assert klog_has(launch_lines(log), lambda l: f"epi=0 ks={ks} " in l), log
    check(y.reshape(N, M), orc.mul_mat(tid, w, rb, x, exact=True) + r, rows_out)


@pytest.mark.parametrize("types", [("q4_K", "q4_K", "q6_K"), ("q6_K", "q4_K"), ("q5_K", "q5_K", "q6_K"),
                                   ("q5_K", "q5_K", "q5_K"), ("q5_K", "q8_0", "q8_0"), ("q4_K", "q8_0", "q8_0"),
                                   ("q8_0", "q8_0", "q8_0")])
@pytest.mark.parametrize("ks", [1, 2])
def test_mmq4_group(pkg, backend, orc, types, ks):
    """2-3 GEMMs sharing src1 in ONE k_mmq4 launch (segments, two weight types at most);
    the last segment carries outlier rows"""
    rng = np.random.default_rng(41 + ks + len(types))
    K, N = 2048, 150
    Ms = [300, 128, 200][:len(types)]
    ws, outs_rows = [], []
    for i, (t, M) in enumerate(zip(types, Ms)):
        w, rb = rand_quant(NAMES[t], M, K, rng)
        ro = []
        if i == len(types) - 1:
            w, ro = with_outliers(w, NAMES[t], M, K, rng)
        ws.append((w, rb))
        outs_rows.append(ro)
    x = rng.standard_normal((N, K)).astype(np.float32)

    def build(ctx):
        tx = ctx.new_tensor("f32", K, N)
        tws = [ctx.new_tensor(NAMES[t], K, M) for t, M in zip(types, Ms)]
        outs = [ctx.mul_mat(tw, tx) for tw in tws]
        return outs, [(tx, x)] + [(tw, w) for tw, (w, _) in zip(tws, ws)]

    ys, log = run(pkg, backend, build, [(20, ks)])
    assert klog_has(log, lambda l: l.startswith(f"mmq4 group n={len(types)} ")), log
    assert klog_has(launch_lines(log), lambda l: f"epi=0 ks={ks} " in l), log
    for y, t, M, (w, rb), ro in zip(ys, types, Ms, ws, outs_rows):
        check(y.reshape(N, M), orc.mul_mat(NAMES[t], w, rb, x, exact=True), ro)


@pytest.mark.parametrize("tname", ["q4_K", "q5_K", "q6_K", "q8_0"])
@pytest.mark.parametrize("N", [150, 40])
def test_mmq4_glu(pkg, backend, orc, tname, N):
    """gate/up/SwiGLU in one k_mmq4 launch (EPI 1): gate and up waves keep separate weight
    scales (outliers in up only)"""
    tid = NAMES[tname]
    rng = np.random.default_rng(21 + tid + N)
    K, M = 2048, 300
    wg, rb = rand_quant(tid, M, K, rng)
    wu, _ = rand_quant(tid, M, K, rng)
    wu, rows_out = with_outliers(wu, tid, M, K, rng)
    x = rng.standard_normal((N, K)).astype(np.float32)

    def build(ctx):
        tg = ctx.new_tensor(tid, K, M)
        tu = ctx.new_tensor(tid, K, M)
        tx = ctx.new_tensor("f32", K, N)
        up = ctx.mul_mat(tu, tx)
        gate = ctx.mul_mat(tg, tx)
        return [ctx.swiglu_split(gate, up)], [(tg, wg), (tu, wu), (tx, x)]

    (y,), log = run(pkg, backend, build)
    assert klog_has(log, lambda l: l.startswith(f"mmq4 glu qt={tid} ")), log
    assert klog_has(launch_lines(log), lambda l: "epi=1 " in l), log
    g = orc.mul_mat(tid, wg, rb, x, exact=True)
    u = orc.mul_mat(tid, wu, rb, x, exact=True)
    check(y.reshape(N, M), orc.swiglu(g, u), rows_out)


@pytest.mark.parametrize("M,N", [(300, 300), (1024, 512), (2048, 700)])
@pytest.mark.parametrize("outlier", [False, True])
def test_mmq5_glu(pkg, backend, orc, M, N, outlier):
    """gate/up/SwiGLU from 256 tokens on: k_mmq5 (256-token tiles, one wave per SIMD, the
    row pair's weight scale fixed up front from a scan of its super-block headers); M = 300
    ragged rows (linear tile order), 1024 / 2048 (row tiles a multiple of 8: the XCD-aware
    order), N ragged"""
    tid = NAMES["q4_K"]
    rng = np.random.default_rng(3 * M + N + outlier)
    K = 2048
    wg, rb = rand_quant(tid, M, K, rng)
    wu, _ = rand_quant(tid, M, K, rng)
    rows_out = []
    if outlier:
        wg, rows_out = with_outliers(wg, tid, M, K, rng)
        wu, _ = with_outliers(wu, tid, M, K, rng)
    x = rng.standard_normal((N, K)).astype(np.float32)

    def build(ctx):
        tg = ctx.new_tensor(tid, K, M)
        tu = ctx.new_tensor(tid, K, M)
        tx = ctx.new_tensor("f32", K, N)
        return [ctx.swiglu_split(ctx.mul_mat(tg, tx), ctx.mul_mat(tu, tx))], [(tg, wg), (tu, wu), (tx, x)]

    (y,), log = run(pkg, backend, build)
    assert klog_has(launch_lines(log), lambda l: "epi=1 " in l and "wide=1" in l), log
    g = orc.mul_mat(tid, wg, rb, x, exact=True)
    u = orc.mul_mat(tid, wu, rb, x, exact=True)
    check(y.reshape(N, M), orc.swiglu(g, u), rows_out)


@pytest.mark.parametrize("tname", ["q4_K", "q5_K", "q6_K", "q8_0"])
@pytest.mark.parametrize("T", [70, 300])
def test_mmq4_moe(pkg, backend, orc, tname, T):
    """MUL_MAT_ID prefill: items sorted by expert on the device, expert-grouped k_mmq4 tiles
    (EPI 2, activation rows gathered, outputs scattered); a skewed routing (expert 3 unused,
    expert 1 takes most items) and outliers in expert 2. T 300: full 128-token tiles plus
    partial last tiles in both the 128- and the 64-token launch (round 6)"""
    tid = NAMES[tname]
    rng = np.random.default_rng(5 + tid + T)
    K, M, E, used = 2048, 200, 4, 2
    parts = [rand_quant(tid, M, K, rng) for _ in range(E)]
    rb = parts[0][1]
    w2, rows_out = with_outliers(parts[2][0], tid, M, K, rng)
    parts[2] = (w2, rb)
    w = np.concatenate([p for p, _ in parts])
    x = rng.standard_normal((T, 1, K)).astype(np.float32)
    ids = np.stack([np.where(rng.random(T) < 0.8, 1, 0), np.where(rng.random(T) < 0.3, 2, 0)], 1).astype(np.int32)
    ids[:, 1] = np.where(ids[:, 1] == ids[:, 0], 2, ids[:, 1])

    def build(ctx):
        tw = ctx.new_tensor(tid, K, M, E)
        tx = ctx.new_tensor("f32", K, 1, T)
        ti = ctx.new_tensor("i32", used, T)
        return [ctx.mul_mat_id(tw, tx, ti)], [(tw, w), (tx, x), (ti, ids)]

    (y,), log = run(pkg, backend, build)
    assert klog_has(log, lambda l: l.startswith(f"mmq4 moe qt={tid} ")), log
    assert klog_has(launch_lines(log), lambda l: "epi=2 " in l), log
    y = y.reshape(T, used, M)
    for e in range(E):
        sel = np.argwhere(ids == e)
        if not len(sel):
            continue
        ref = orc.mul_mat(tid, parts[e][0], rb, x[sel[:, 0], 0], exact=True)
        check(y[sel[:, 0], sel[:, 1]], ref, rows_out if e == 2 else ())


@pytest.mark.parametrize("tname", ["q4_K", "q5_K", "q6_K", "q8_0"])
@pytest.mark.parametrize("T", [70, 300])
def test_mmq4_moe_glu(pkg, backend, orc, tname, T):
    """MoE prefill gate/up/SwiGLU (llama build_moe_ffn) in ONE k_mmq4 launch (EPI 3): the
    expert-grouped tiles with gate waves and up waves over the same gathered activations,
    silu(g) * u scattered to the GLU output and its f16 copy claimed for the down
    projection's expert GEMM (checked through the down product too); skewed routing,
    outliers in one expert's up rows"""
    tid = NAMES[tname]
    rng = np.random.default_rng(77 + tid + T)
    K, M, Md, E, used = 2048, 512, 200, 4, 2
    wg = [rand_quant(tid, M, K, rng) for _ in range(E)]
    wu = [rand_quant(tid, M, K, rng) for _ in range(E)]
    rb = wg[0][1]
    w2, rows_out = with_outliers(wu[2][0], tid, M, K, rng)
    wu[2] = (w2, rb)
    wd = [rand_quant(tid, Md, M, rng) for _ in range(E)]
    rbd = wd[0][1]
    x = rng.standard_normal((T, 1, K)).astype(np.float32)
    ids = np.stack([np.where(rng.random(T) < 0.8, 1, 0), np.where(rng.random(T) < 0.3, 2, 0)], 1).astype(np.int32)
    ids[:, 1] = np.where(ids[:, 1] == ids[:, 0], 2, ids[:, 1])

    def build(ctx):
        tg = ctx.new_tensor(tid, K, M, E)
        tu = ctx.new_tensor(tid, K, M, E)
        td = ctx.new_tensor(tid, M, Md, E)
        tx = ctx.new_tensor("f32", K, 1, T)
        ti = ctx.new_tensor("i32", used, T)
        up = ctx.mul_mat_id(tu, tx, ti)
        gate = ctx.mul_mat_id(tg, tx, ti)
        glu = ctx.swiglu_split(gate, up)
        down = ctx.mul_mat_id(td, glu, ti)
        return [glu, down], [(tg, np.concatenate([w for w, _ in wg])), (tu, np.concatenate([w for w, _ in wu])),
                             (td, np.concatenate([w for w, _ in wd])), (tx, x), (ti, ids)]

    (y, yd), log = run(pkg, backend, build)
    assert klog_has(log, lambda l: l.startswith(f"mmq4 moe_glu qt={tid} ") and l.endswith(" h=1")), log
    assert klog_has(launch_lines(log), lambda l: "epi=3 " in l), log
    y = y.reshape(T, used, M)
    yd = yd.reshape(T, used, Md)
    for e in range(E):
        sel = np.argwhere(ids == e)
        if not len(sel):
            continue
        xe = x[sel[:, 0], 0]
        g = orc.mul_mat(tid, wg[e][0], rb, xe, exact=True)
        u = orc.mul_mat(tid, wu[e][0], rb, xe, exact=True)
        ye = y[sel[:, 0], sel[:, 1]]
        check(ye, orc.swiglu(g, u), rows_out if e == 2 else ())
        check(yd[sel[:, 0], sel[:, 1]], orc.mul_mat(tid, wd[e][0], rbd, ye, exact=True), ())
