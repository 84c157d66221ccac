"""Parity at the shapes the Llama-3-8B / Mixtral benches time (BASELINE configs 2, 3, 5).

Every decode GEMV instantiation that `profiles/r01/decode_v6_kernel_stats.csv` lists runs
here at its bench shape, against the CPU oracle (oracle/oracle.c, `exact` = f32
activations, the reference CPU backend's arithmetic up to its q8_K activation rounding),
and each test asserts through the kernel-choice log (ggml_backend_mi355x_klog) that the
instantiation it meant to pin is the one that ran:

  SwiGLU 4096 -> 14336 (gate+up Q4_K, deferred ffn_norm, LDS-DMA staged x, q8 emission)
      k_gemv2<12,16,2,1,8,XS_NORM_LDS>
  down 14336 -> 4096 + residual, Q4_K and Q6_K (q8 input from the SwiGLU)
      k_gemv2<12,32,4,2,4,XS_Q8>, k_gemv2<14,32,2,2,4,XS_Q8>
  O projection 4096 -> 4096 + residual (f32 input)       k_gemv2<12,16,4,2,4,XS_F32>
  lm_head 4096 -> 128256 Q6_K after the output_norm+q8 launch  k_gemv2<14,16,4,0,4,XS_Q8>
  Mixtral MUL_MAT_ID 4096 -> 14336 Q5_K, 8 experts, top-2, T in {1, 64}

Tolerance: NMSE 5e-4 (tests/test-backend-ops.cpp:3718, MUL_MAT / MUL_MAT_ID).
"""
import re

import numpy as np
import pytest

from qgen import NAMES, nmse, rand_quant

pytestmark = pytest.mark.gpu

XS_F32, XS_NORM, XS_Q8, XS_F32_LDS, XS_NORM_LDS = 0, 1, 2, 3, 4
E, FF, VOCAB = 4096, 14336, 128256
TOL = 5e-4


def run(pkg, be, build):
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
    return res, log


def gemv_lines(log):
    out = []
    for ln in log:
        if ln.startswith("gemv2 "):
            out.append({k: int(v) for k, v in re.findall(r"(\w+)=(-?\d+)", ln)})
    return out


def find(lines, **kw):
    hits = [d for d in lines if all(d.get(k) == v for k, v in kw.items())]
    assert hits, f"no gemv2 launch with {kw}; launched: {lines}"
    return hits[0]


@pytest.mark.parametrize("down_t", ["q4_K", "q6_K"])
def test_ffn_block_llama3_8b(pkg, backend, orc, down_t):
    """ffn_norm -> gate/up -> SwiGLU -> down + residual, one token, Llama-3-8B widths"""
    rng = np.random.default_rng(101)
    q4k, dt = NAMES["q4_K"], NAMES[down_t]
    wg, rb = rand_quant(q4k, FF, E, rng)
    wu, _ = rand_quant(q4k, FF, E, rng)
    wd, rbd = rand_quant(dt, E, FF, rng)
    x = rng.standard_normal((1, E)).astype(np.float32)
    nw = rng.uniform(0.5, 1.5, E).astype(np.float32)
    before = backend.stats()["nodes_fused"]

    def build(ctx):
        tx = ctx.new_tensor("f32", E, 1)
        tn = ctx.new_tensor("f32", E)
        tg = ctx.new_tensor(q4k, E, FF)
        tu = ctx.new_tensor(q4k, E, FF)
        td = ctx.new_tensor(dt, FF, E)
        cur = ctx.mul(ctx.rms_norm(tx, 1e-5), tn)
        h = ctx.swiglu_split(ctx.mul_mat(tg, cur), ctx.mul_mat(tu, cur))
        y = ctx.add(ctx.mul_mat(td, h), tx)
        return [y], [(tx, x), (tn, nw), (tg, wg), (tu, wu), (td, wd)]

    (y,), log = run(pkg, backend, build)
    xn = orc.rms_norm(x, 1e-5) * nw
    h = orc.swiglu(orc.mul_mat(q4k, wg, rb, xn, exact=True), orc.mul_mat(q4k, wu, rb, xn, exact=True))
    ref = orc.mul_mat(dt, wd, rbd, h, exact=True) + x
    err = nmse(y.reshape(1, E), ref)
    assert err < TOL, err
    lines = gemv_lines(log)
    find(lines, qt=q4k, lpr=16, upl=2, epi=1, w=8, mode=XS_NORM_LDS, K=E, M=FF, q8o=1)
    find(lines, qt=dt, lpr=32, upl=4 if down_t == "q4_K" else 2, epi=2, w=4, mode=XS_Q8, K=FF, M=E)
    assert len(lines) == 2, lines
    assert backend.stats()["nodes_fused"] >= before + 5, "norm deferral / GLU / residual fusion did not fire"


def test_attn_output_llama3_8b(pkg, backend, orc):
    """O projection + residual (f32 input: the attention output), Q4_K 4096 -> 4096"""
    rng = np.random.default_rng(102)
    q4k = NAMES["q4_K"]
    w, rb = rand_quant(q4k, E, E, rng)
    x = rng.standard_normal((1, E)).astype(np.float32)
    r = rng.standard_normal((1, E)).astype(np.float32)

    def build(ctx):
        tw = ctx.new_tensor(q4k, E, E)
        tx = ctx.new_tensor("f32", E, 1)
        tr = ctx.new_tensor("f32", E, 1)
        return [ctx.add(ctx.mul_mat(tw, tx), tr)], [(tw, w), (tx, x), (tr, r)]

    (y,), log = run(pkg, backend, build)
    ref = orc.mul_mat(q4k, w, rb, x, exact=True) + r
    assert nmse(y.reshape(1, E), ref) < TOL
    find(gemv_lines(log), qt=q4k, lpr=16, upl=4, epi=2, w=4, mode=XS_F32, K=E, M=E)


def test_lm_head_llama3_8b(pkg, backend, orc):
    """output_norm -> lm_head Q6_K 4096 -> 128256 (the largest decode GEMV, 431 MB); the norm
    is not deferred into the 8016 workgroups (exec.cpp try_defer_norm): it runs once and
    emits q8, which the GEMV stages"""
    rng = np.random.default_rng(103)
    q6k = NAMES["q6_K"]
    w, rb = rand_quant(q6k, VOCAB, E, rng)
    x = rng.standard_normal((1, E)).astype(np.float32)
    nw = rng.uniform(0.5, 1.5, E).astype(np.float32)

    def build(ctx):
        tx = ctx.new_tensor("f32", E, 1)
        tn = ctx.new_tensor("f32", E)
        tw = ctx.new_tensor(q6k, E, VOCAB)
        return [ctx.mul_mat(tw, ctx.mul(ctx.rms_norm(tx, 1e-5), tn))], [(tx, x), (tn, nw), (tw, w)]

    (y,), log = run(pkg, backend, build)
    ref = orc.mul_mat(q6k, w, rb, orc.rms_norm(x, 1e-5) * nw, exact=True)
    assert nmse(y.reshape(1, VOCAB), ref) < TOL
    find(gemv_lines(log), qt=q6k, lpr=16, upl=4, epi=0, w=4, mode=XS_Q8, K=E, M=VOCAB)


@pytest.mark.parametrize("T", [1, 64])
def test_mul_mat_id_mixtral(pkg, backend, orc, T):
    """Mixtral-8x7B ffn_gate_exps: Q5_K [4096 -> 14336] x 8 experts, top-2 routing"""
    rng = np.random.default_rng(104 + T)
    q5k = NAMES["q5_K"]
    n_exp, used = 8, 2
    ws = [rand_quant(q5k, FF, E, rng) for _ in range(n_exp)]
    rb = ws[0][1]
    w = np.concatenate([a for a, _ in ws])
    x = rng.standard_normal((T, 1, E)).astype(np.float32)
    ids = np.stack([rng.permutation(n_exp)[:used] for _ in range(T)]).astype(np.int32)

    def build(ctx):
        tw = ctx.new_tensor(q5k, E, FF, n_exp)
        tx = ctx.new_tensor("f32", E, 1, T)
        ti = ctx.new_tensor("i32", used, T)
        return [ctx.mul_mat_id(tw, tx, ti)], [(tw, w), (tx, x), (ti, ids)]

    (y,), log = run(pkg, backend, build)
    y = y.reshape(T, used, FF)
    for e in range(n_exp):
        sel = np.argwhere(ids == e)
        if len(sel) == 0:
            continue
        ref = orc.mul_mat(q5k, ws[e][0], rb, x[sel[:, 0], 0], exact=True)
        got = y[sel[:, 0], sel[:, 1]]
        assert nmse(got, ref) < TOL, (e, nmse(got, ref))
    assert any(ln.startswith(("moe_", "mmid", "mmq4 moe", "gemv2 moe")) for ln in log), log
    if T >= 32:
        assert any(ln.startswith("mmq4 moe") for ln in log), log   # the expert-grouped GEMM
