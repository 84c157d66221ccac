"""Per-op parity of libggml-mi355x.so against the CPU oracle (oracle/oracle.c), driven
through the backend C-ABI (graph_compute) with seeded inputs.

Tolerances are the reference parity harness's (tests/test-backend-ops.cpp): NMSE
5e-4 for MUL_MAT/MUL_MAT_ID/FLASH_ATTN_EXT (:3718, :3854, :6082), 1e-7 for
RMS_NORM/ROPE (:1124), 1e-6 SOFT_MAX (:4427); SET_ROWS (f16 KV store) and GET_ROWS
(dequantisation) must be bit-exact.
"""
import numpy as np
import pytest

from qgen import NAMES, nmse, rand_quant

pytestmark = pytest.mark.gpu

F16 = 1


def run(pkg, be, build):
    ctx = pkg.Context()
    outs, feed = build(ctx)
    g = ctx.build(*outs)
    ctx.alloc(be)
    for t, arr in feed:
        t.set(arr)
    ctx.compute(be, g)
    res = [o.numpy() for o in outs]
    ctx.free()
    return res


@pytest.mark.parametrize("tname", ["q4_K", "q6_K", "q5_K", "q4_0", "q8_0", "q4_1", "q5_0"])
@pytest.mark.parametrize("N", [1, 2, 3, 8, 17, 130])
def test_mul_mat_quant(pkg, backend, orc, tname, N):
    tid = NAMES[tname]
    rng = np.random.default_rng(hash((tname, N)) % 2**32)
    K, M = (512, 200) if N > 8 else (1024, 333)
    w, rb = rand_quant(tid, M, K, rng)
    x = rng.standard_normal((N, K)).astype(np.float32)

    def build(ctx):
        tw = ctx.new_tensor(tid, K, M)
        tx = ctx.new_tensor("f32", K, N)
        return [ctx.mul_mat(tw, tx)], [(tw, w), (tx, x)]

    y = run(pkg, backend, build)[0].reshape(N, M)
    ref_cpu = orc.mul_mat(tid, w, rb, x)          # CPU backend semantics (q8 activations)
    ref_exact = orc.mul_mat(tid, w, rb, x, exact=True)
    assert np.all(np.isfinite(y))
    assert nmse(y, ref_cpu) < 5e-4
    assert nmse(y, ref_exact) < 5e-4


@pytest.mark.parametrize("tname", ["q4_K", "q6_K", "q5_K", "q4_0", "q8_0"])
@pytest.mark.parametrize("N,K", [(2, 1024), (4, 1024), (5, 1024), (7, 2048), (8, 14336), (3, 14336)])
def test_mul_mat_multicolumn(pkg, backend, orc, tname, N, K):
    """2..8 activation columns on the LDS-staged multi-column GEMV (ops_gemv_nc.hip): every
    column count class (5 and 7 run with a padding column), K 14336 = the down projection's
    width with the 143 KB LDS image of 8 columns, a ragged last row tile (M % 16 != 0)"""
    tid = NAMES[tname]
    rng = np.random.default_rng(hash((tname, N, K, 5)) % 2**32)
    M = 333 if K <= 2048 else 1000
    w, rb = rand_quant(tid, M, K, rng)
    x = rng.standard_normal((N, K)).astype(np.float32)

    def build(ctx):
        tw = ctx.new_tensor(tid, K, M)
        tx = ctx.new_tensor("f32", K, N)
        return [ctx.mul_mat(tw, tx)], [(tw, w), (tx, x)]

    backend.klog(True)
    try:
        y = run(pkg, backend, build)[0].reshape(N, M)
        log = backend.klog_read()
    finally:
        backend.klog(False)
    nc = N if N <= 4 else (6 if N <= 6 else 8)
    assert any(ln.startswith(f"gemv_nc qt={tid} nc={nc} ncols={N} K={K} M={M} ") for ln in log), log
    assert np.all(np.isfinite(y))
    assert nmse(y, orc.mul_mat(tid, w, rb, x)) < 5e-4


@pytest.mark.parametrize("tname", ["q4_K", "q6_K", "q5_K"])
@pytest.mark.parametrize("kernel", [1, 2])
def test_mul_mat_quant_prefill_kernels(pkg, backend, orc, tname, kernel):
    """both K-quant prefill GEMMs (ops_mm.hip): 8-wave k_mmq3 (g_tune[5] = 1) and 4-wave
    k_mmq2 (g_tune[5] = 2), ragged token and row tiles, K over 8 steps"""
    lib = pkg._lib.load()
    lib.ggml_backend_mi355x_set_tune(5, kernel)
    try:
        tid = NAMES[tname]
        rng = np.random.default_rng(7 + kernel)
        K, M, N = 1024, 200, 150
        w, rb = rand_quant(tid, M, K, rng)
        x = rng.standard_normal((N, K)).astype(np.float32)

        def build(ctx):
            tw = ctx.new_tensor(tid, K, M)
            tx = ctx.new_tensor("f32", K, N)
            return [ctx.mul_mat(tw, tx)], [(tw, w), (tx, x)]

        y = run(pkg, backend, build)[0].reshape(N, M)
        assert np.all(np.isfinite(y))
        assert nmse(y, orc.mul_mat(tid, w, rb, x, exact=True)) < 5e-4
    finally:
        lib.ggml_backend_mi355x_set_tune(5, 0)


@pytest.mark.parametrize("tname", ["q4_K", "q6_K", "q5_K", "q4_0", "q8_0", "q4_1", "q5_0", "q5_1"])
def test_get_rows_dequant_bit_exact(pkg, backend, orc, tname):
    tid = NAMES[tname]
    rng = np.random.default_rng(3)
    K, M = 512, 40
    w, rb = rand_quant(tid, M, K, rng)
    idx = np.array([5, 0, 39, 5, 17], np.int32)

    def build(ctx):
        tw = ctx.new_tensor(tid, K, M)
        ti = ctx.new_tensor("i32", len(idx))
        return [ctx.get_rows(tw, ti)], [(tw, w), (ti, idx)]

    y = run(pkg, backend, build)[0].reshape(len(idx), K)
    for j, r in enumerate(idx):
        ref = orc.dequantize(tid, w[r * rb:(r + 1) * rb], K)
        assert np.array_equal(y[j].view(np.uint32), ref.view(np.uint32)), f"row {r}"


@pytest.mark.parametrize("idx_type", ["i64", "i32"])
def test_set_rows_f16_bit_exact(pkg, backend, orc, idx_type):
    rng = np.random.default_rng(5)
    D, cells, n = 1024, 64, 7
    src = (rng.standard_normal((n, D)) * 3).astype(np.float32)
    src[0, :4] = [65504.0, 1e-8, -0.0, 70000.0]   # max f16, subnormal, signed zero, overflow
    idx = rng.permutation(cells)[:n].astype(np.int64 if idx_type == "i64" else np.int32)

    def build(ctx):
        cache = ctx.new_tensor("f16", D, cells)
        ts = ctx.new_tensor("f32", D, n)
        ti = ctx.new_tensor(idx_type, n)
        return [ctx.set_rows(cache, ts, ti), cache], [(cache, np.zeros((cells, D), np.uint16)), (ts, src), (ti, idx)]

    out = run(pkg, backend, build)[1].reshape(cells, D).view(np.uint16)
    ref = orc.f32_to_f16(src)
    for j, c in enumerate(idx):
        assert np.array_equal(out[c], ref[j])
    untouched = np.setdiff1d(np.arange(cells), idx)
    assert not out[untouched].any()


@pytest.mark.parametrize("kind,idx_type", [("q8_0", "i64"), ("q4_0", "i64"), ("q4_0", "i32")])
def test_set_rows_quantised_bit_exact(pkg, backend, orc, kind, idx_type):
    """SET_ROWS into a q8_0 / q4_0 KV cache (-ctk / -ctv q8_0 / q4_0): every stored row equals
    the oracle's quantize_row_<type>_ref bytes (tests/test_oracle.py pins those to the
    reference's C quantiser); cells not indexed stay untouched"""
    rng = np.random.default_rng(6)
    D, cells, n = 1024, 48, 5
    src = (rng.standard_normal((n, D)) * np.array([1e-3, 1, 5, 200, 1])[:, None]).astype(np.float32)
    src[1, :32] = 0.0                               # an all-zero block: d = 0
    idx = rng.permutation(cells)[:n].astype(np.int64 if idx_type == "i64" else np.int32)
    bs = 34 if kind == "q8_0" else 18
    row = D // 32 * bs

    ctx = pkg.Context()
    cache = ctx.new_tensor(kind, D, cells)
    ts = ctx.new_tensor("f32", D, n)
    ti = ctx.new_tensor(idx_type, n)
    g = ctx.build(ctx.set_rows(cache, ts, ti))
    ctx.alloc(backend)
    cache.set(np.zeros(cells * row, np.uint8)); ts.set(src); ti.set(idx)
    ctx.compute(backend, g)
    out = cache.get_bytes().reshape(cells, row)
    ctx.free()
    quant = orc.quantize_q8_0 if kind == "q8_0" else orc.quantize_q4_0
    for j, cidx in enumerate(idx):
        assert np.array_equal(out[cidx], quant(src[j])), j
    untouched = np.setdiff1d(np.arange(cells), idx)
    assert not out[untouched].any()


@pytest.mark.parametrize("idx_type,n_tok,dtype", [("i64", 512, "f16"), ("i64", 7, "f16"), ("i32", 100, "f32")])
def test_set_rows_transposed_v(pkg, backend, orc, idx_type, n_tok, dtype):
    """the non-flash-attention V store (llama_kv_cache::cpy_v, v_trans): v_cur [D, n_tok]
    reshaped to [1, D * n_tok], one index per element, element (d, t) -> cache element
    d * kv + cell(t); set_elems transposes through LDS (klog) and must be bit-exact"""
    rng = np.random.default_rng(n_tok)
    D, kv = 1024, 768
    v = (rng.standard_normal((n_tok, D)) * 3).astype(np.float32)
    cells = np.sort(rng.permutation(kv)[:n_tok]) if n_tok < 16 else np.arange(100, 100 + n_tok)
    idx = (np.arange(D)[None, :] * kv + cells[:, None]).astype(np.int64 if idx_type == "i64" else np.int32)  # [n_tok, D]

    def build(ctx):
        cache = ctx.new_tensor(dtype, D * kv)
        tv = ctx.new_tensor("f32", D, n_tok)
        ti = ctx.new_tensor(idx_type, D * n_tok)
        dst = ctx.set_rows(ctx.reshape(cache, 1, D * kv), ctx.reshape(tv, 1, D * n_tok), ti)
        zero = np.zeros(D * kv, np.uint16 if dtype == "f16" else np.float32)
        return [dst, cache], [(cache, zero), (tv, v), (ti, idx.reshape(-1))]

    backend.klog(True)
    out = run(pkg, backend, build)[1].reshape(D, kv)
    log = backend.klog_read()
    backend.klog(False)
    assert any(ln.startswith("set_elems") and "R=1024" in ln for ln in log), log
    ref = orc.f32_to_f16(v).view(np.uint16) if dtype == "f16" else v
    out = out.view(np.uint16) if dtype == "f16" else out
    assert np.array_equal(out[:, cells], ref.T.reshape(D, n_tok))
    mask = np.ones(kv, bool); mask[cells] = False
    assert not out[:, mask].any()


@pytest.mark.parametrize("ne0,nrows", [(4096, 3), (64, 5), (1025, 4), (8192, 1)])
def test_rms_norm_fused_mul(pkg, backend, orc, ne0, nrows):
    rng = np.random.default_rng(ne0)
    x = rng.standard_normal((nrows, ne0)).astype(np.float32)
    w = rng.standard_normal(ne0).astype(np.float32)

    def build(ctx):
        tx = ctx.new_tensor("f32", ne0, nrows)
        tw = ctx.new_tensor("f32", ne0)
        n = ctx.rms_norm(tx, 1e-5)
        return [ctx.mul(n, tw), ], [(tx, x), (tw, w)]

    y = run(pkg, backend, build)[0].reshape(nrows, ne0)
    ref = orc.rms_norm(x, 1e-5) * w
    assert nmse(y, ref) < 1e-7


@pytest.mark.parametrize("mode", [0, 2])
@pytest.mark.parametrize("ndims,heads", [(128, 8), (64, 8), (128, 1)])
def test_rope(pkg, backend, orc, mode, ndims, heads):
    """heads > 1: per-token table kernel (k_rope2), partial rotation with ndims < head dim;
    heads = 1: per-row kernel"""
    rng = np.random.default_rng(11)
    hd, ntok = 128, 5
    x = rng.standard_normal((ntok, heads, hd)).astype(np.float32)
    pos = np.array([0, 1, 7, 300, 4095], np.int32)

    def build(ctx):
        tx = ctx.new_tensor("f32", hd, heads, ntok)
        tp = ctx.new_tensor("i32", ntok)
        return [ctx.rope_ext(tx, tp, None, ndims, mode, 8192, 500000.0)], [(tx, x), (tp, pos)]

    y = run(pkg, backend, build)[0].reshape(ntok, heads, hd)
    ref = orc.rope(x, pos, ndims, mode, 8192, 500000.0)
    assert nmse(y, ref) < 1e-7


@pytest.mark.parametrize("ne00,ne01,heads", [(256, 1, 32), (1000, 7, 4), (4096, 3, 2)])
def test_soft_max_masked(pkg, backend, orc, ne00, ne01, heads):
    rng = np.random.default_rng(ne00)
    x = rng.standard_normal((heads, ne01, ne00)).astype(np.float32)
    mask = np.zeros((ne01, ne00), np.float32)
    mask[:, ne00 // 2:] = -np.inf
    m16 = mask.astype(np.float16).view(np.uint16)

    def build(ctx):
        tx = ctx.new_tensor("f32", ne00, ne01, heads)
        tm = ctx.new_tensor("f16", ne00, ne01)
        return [ctx.soft_max_ext(tx, tm, 0.125)], [(tx, x), (tm, m16)]

    y = run(pkg, backend, build)[0].reshape(heads, ne01, ne00)
    ref = orc.soft_max(x, m16, 0.125)
    assert nmse(y, ref) < 1e-6


@pytest.mark.parametrize("types", [("q4_K", "q4_K", "q6_K"), ("q6_K", "q4_K"), ("q5_K", "q5_K", "q5_K")])
def test_grouped_prefill_mul_mats(pkg, backend, orc, types):
    """prefill GEMMs sharing src1 (q/k/v) in one k_mmq3m launch, mixed weight types"""
    rng = np.random.default_rng(41)
    K, N = 1024, 150
    Ms = [256, 128, 200][:len(types)]
    ws = [rand_quant(NAMES[t], M, K, rng) for t, M in zip(types, Ms)]
    x = rng.standard_normal((N, K)).astype(np.float32)
    before = backend.stats()["nodes_fused"]

    def build(ctx):
        tx = ctx.new_tensor("f32", K, N)
        tws = [ctx.new_tensor(NAMES[t], K, M) for t, M in zip(types, Ms)]
        outs = [ctx.mul_mat(tw, tx) for tw in tws]
        return outs, [(tx, x)] + [(tw, w) for tw, (w, _) in zip(tws, ws)]

    ys = run(pkg, backend, build)
    for y, t, M, (w, rb) in zip(ys, types, Ms, ws):
        ref = orc.mul_mat(NAMES[t], w, rb, x, exact=True)
        assert nmse(y.reshape(N, M), ref) < 5e-4
    assert backend.stats()["nodes_fused"] >= before + len(types) - 1, "grouped GEMM did not fire"


@pytest.mark.parametrize("tname", ["q4_K", "q6_K"])
@pytest.mark.parametrize("N", [1, 150])
def test_fused_mul_mat_add(pkg, backend, orc, tname, N):
    """MUL_MAT -> ADD(residual): decode GEMV epilogue (N = 1), prefill GEMM epilogue (N = 150)"""
    tid = NAMES[tname]
    rng = np.random.default_rng(31)
    K, M = 1024, 200
    w, rb = rand_quant(tid, M, K, rng)
    x = rng.standard_normal((N, K)).astype(np.float32)
    r = rng.standard_normal((N, M)).astype(np.float32)
    before = backend.stats()["nodes_fused"]

    def build(ctx):
        tw = ctx.new_tensor(tid, K, M)
        tx = ctx.new_tensor("f32", K, N)
        tr = ctx.new_tensor("f32", M, N)
        return [ctx.add(ctx.mul_mat(tw, tx), tr)], [(tw, w), (tx, x), (tr, r)]

    y = run(pkg, backend, build)[0].reshape(N, M)
    ref = orc.mul_mat(tid, w, rb, x, exact=True) + r
    assert nmse(y, ref) < 5e-4
    assert backend.stats()["nodes_fused"] >= before + 1, "MUL_MAT -> ADD fusion did not fire"


@pytest.mark.parametrize("tname", ["q4_K", "q6_K", "q5_K"])
@pytest.mark.parametrize("N", [1, 150])
def test_fused_gate_up_swiglu(pkg, backend, orc, tname, N):
    """N = 1: decode GEMV (gemv2 EPI 1); N = 150: prefill k_mmq3g (ragged token and row tiles)"""
    tid = NAMES[tname]
    rng = np.random.default_rng(21)
    K, M = 1024, (512 if N == 1 else 200)
    wg, rb = rand_quant(tid, M, K, rng)
    wu, _ = rand_quant(tid, M, K, rng)
    x = rng.standard_normal((N, K)).astype(np.float32)
    before = backend.stats()["nodes_fused"]

    def build(ctx):
        tg = ctx.new_tensor(tid, K, M)
        tu = ctx.new_tensor(tid, K, M)
        tx = ctx.new_tensor("f32", K, N)
        up = ctx.mul_mat(tu, tx)
        gate = ctx.mul_mat(tg, tx)
        return [ctx.swiglu_split(gate, up)], [(tg, wg), (tu, wu), (tx, x)]

    y = run(pkg, backend, build)[0].reshape(N, M)
    g = orc.mul_mat(tid, wg, rb, x, exact=True)
    u = orc.mul_mat(tid, wu, rb, x, exact=True)
    ref = orc.swiglu(g, u)
    assert nmse(y, ref) < 5e-4
    assert backend.stats()["nodes_fused"] >= before + 2, "gate/up/GLU fusion did not fire"


@pytest.mark.parametrize("n_q,n_kv,H,Hkv,D", [(1, 256, 32, 8, 128), (1, 700, 8, 8, 128), (5, 512, 8, 2, 128),
                                               (64, 300, 4, 4, 128), (100, 333, 8, 2, 128), (130, 130, 4, 1, 64),
                                               (1, 4096, 8, 2, 128), (3, 1000, 4, 2, 64),
                                               # decode kernel v2 (ops_fattn_dec.hip): one split (direct
                                               # store), ragged last split, GQA 8, D 64 with 2 query rows
                                               (1, 64, 8, 8, 128), (1, 100, 32, 4, 128), (2, 65, 16, 2, 64),
                                               (4, 1500, 32, 8, 128),
                                               # prefill kernel v2 (k_fa_mma2, D 128): 4 / 2 / 1 heads
                                               # per workgroup, GQA 8 (two head groups), ragged tiles
                                               (512, 512, 32, 8, 128), (200, 450, 6, 3, 128), (77, 77, 16, 2, 128),
                                               (33, 1000, 4, 4, 128),
                                               # decode LONG geometry (one 128-key chunk per workgroup,
                                               # parallel combine): llama-bench -d 16384, GQA 8 (70B:
                                               # two head groups), a ragged 33000-key cache
                                               (1, 16384, 32, 8, 128), (1, 8000, 64, 8, 128), (1, 33000, 8, 8, 128)])
def test_flash_attn(pkg, backend, orc, n_q, n_kv, H, Hkv, D):
    rng = np.random.default_rng(n_q * 1000 + n_kv)
    q = rng.standard_normal((H, n_q, D)).astype(np.float32)
    k = rng.standard_normal((Hkv, n_kv, D)).astype(np.float16).view(np.uint16)
    v = rng.standard_normal((Hkv, n_kv, D)).astype(np.float16).view(np.uint16)
    mask = np.zeros((n_q, n_kv), np.float32)
    for i in range(n_q):
        mask[i, n_kv - n_q + i + 1:] = -np.inf   # causal tail
    m16 = mask.astype(np.float16).view(np.uint16)
    scale = 1.0 / np.sqrt(D)

    def build(ctx):
        tq = ctx.new_tensor("f32", D, n_q, H)
        tk = ctx.new_tensor("f16", D, n_kv, Hkv)
        tv = ctx.new_tensor("f16", D, n_kv, Hkv)
        tm = ctx.new_tensor("f16", n_kv, n_q)
        return [ctx.flash_attn_ext(tq, tk, tv, tm, scale)], [(tq, q), (tk, k), (tv, v), (tm, m16)]

    y = run(pkg, backend, build)[0].reshape(n_q, H, D)
    ref = orc.flash_attn(q, k, v, m16, scale)
    assert nmse(y, ref) < 5e-4
    if n_q <= 4:
        # the split merge's arrival counters must be back at zero for the next launch
        y2 = run(pkg, backend, build)[0].reshape(n_q, H, D)
        assert np.array_equal(y, y2)


@pytest.mark.parametrize("n_q,n_kv,H,Hkv,D", [(1, 1500, 32, 8, 128), (2, 700, 8, 2, 64), (1, 300, 8, 8, 128)])
def test_flash_attn_split_merge(pkg, backend, orc, n_q, n_kv, H, Hkv, D):
    """decode FA v2's in-launch split merge (ops_fattn_dec.hip), forced with g_tune[10] = 3"""
    lib = pkg._lib.load()
    lib.ggml_backend_mi355x_set_tune(10, 3)
    try:
        test_flash_attn(pkg, backend, orc, n_q, n_kv, H, Hkv, D)
    finally:
        lib.ggml_backend_mi355x_set_tune(10, 0)


def test_flash_attn_stream_merge_visibility(pkg, backend, orc):
    """k_fattn_dec3's split merge counts arrivals with a RELAXED agent-scope add —
    it relies on the partials being agent-scope atomic (write-through) stores completed by
    s_waitcnt before the count, and on agent-scope loads in the merging workgroup. Pinned
    here at scale: 64K keys (the most splits per KV head, 8 XCDs), one graph run 24 times —
    every output bit-identical to the first and to the oracle's bound"""
    lib = pkg._lib.load()
    D, H, Hkv, n_kv = 128, 32, 8, 65536
    rng = np.random.default_rng(77)
    q = rng.standard_normal((H, 1, D)).astype(np.float32)
    k = rng.standard_normal((Hkv, n_kv, D)).astype(np.float16).view(np.uint16)
    v = rng.standard_normal((Hkv, n_kv, D)).astype(np.float16).view(np.uint16)
    m16 = np.zeros((1, n_kv), np.float16).view(np.uint16)
    scale = 1.0 / np.sqrt(D)
    ctx = pkg.Context()
    tq = ctx.new_tensor("f32", D, 1, H)
    tk = ctx.new_tensor("f16", D, n_kv, Hkv)
    tv = ctx.new_tensor("f16", D, n_kv, Hkv)
    tm = ctx.new_tensor("f16", n_kv, 1)
    y = ctx.flash_attn_ext(tq, tk, tv, tm, scale)
    g = ctx.build(y)
    ctx.alloc(backend)
    for t, a in ((tq, q), (tk, k), (tv, v), (tm, m16)):
        t.set(a)
    backend.klog(True)
    outs = []
    for _ in range(24):
        ctx.compute(backend, g)
        outs.append(y.numpy().copy())
    log = backend.klog_read()
    backend.klog(False)
    ctx.free()
    assert any(ln.startswith("fattn_dec3 ") for ln in log), log[:10]
    ref = orc.flash_attn(q, k, v, m16, scale)
    assert nmse(outs[0].reshape(1, H, D), ref) < 5e-4
    for o in outs[1:]:
        assert np.array_equal(o, outs[0])


@pytest.mark.parametrize("n_kv,H,Hkv,masked", [(16384, 32, 8, True), (2048, 8, 8, True), (5000, 16, 2, True),
                                                (33000, 8, 8, True), (8000, 64, 8, True), (4096, 4, 4, False),
                                                (30000, 32, 4, True)])
@pytest.mark.parametrize("stream", [True, False])
def test_flash_attn_stream(pkg, backend, orc, n_kv, H, Hkv, masked, stream):
    """long-cache decode attention: k_fattn_dec3 (one workgroup per CU streaming a key range
    of one KV head through its LDS-DMA ring, all Gt query heads, splits merged in-launch by
    the last arrival) — GQA 1 / 2 / 4 / 8, ragged last split, no mask; stream=False keeps
    the round-3 LONG geometry + combine (g_tune[39] = 1) for comparison. Run twice: the
    arrival counters must be back at zero for the next launch / replay"""
    lib = pkg._lib.load()
    lib.ggml_backend_mi355x_set_tune(39, 0 if stream else 1)
    lib.ggml_backend_mi355x_set_tune(35, 8)          # from 2048 keys (the default starts at 16384)
    D = 128
    rng = np.random.default_rng(n_kv + H)
    q = rng.standard_normal((H, 1, D)).astype(np.float32)
    k = rng.standard_normal((Hkv, n_kv, D)).astype(np.float16).view(np.uint16)
    v = rng.standard_normal((Hkv, n_kv, D)).astype(np.float16).view(np.uint16)
    mask = np.zeros((1, n_kv), np.float32)
    if masked:
        mask[0, n_kv - 37:] = -np.inf            # the padded tail of a KV cache view
        mask[0, 100:300] = -np.inf               # a masked run inside one split
    m16 = mask.astype(np.float16).view(np.uint16)
    scale = 1.0 / np.sqrt(D)

    def build(ctx):
        tq = ctx.new_tensor("f32", D, 1, H)
        tk = ctx.new_tensor("f16", D, n_kv, Hkv)
        tv = ctx.new_tensor("f16", D, n_kv, Hkv)
        if not masked:
            return [ctx.flash_attn_ext(tq, tk, tv, None, scale)], [(tq, q), (tk, k), (tv, v)]
        tm = ctx.new_tensor("f16", n_kv, 1)
        return [ctx.flash_attn_ext(tq, tk, tv, tm, scale)], [(tq, q), (tk, k), (tv, v), (tm, m16)]

    try:
        backend.klog(True)
        y = run(pkg, backend, build)[0].reshape(1, H, D)
        log = backend.klog_read()
        backend.klog(False)
        y2 = run(pkg, backend, build)[0].reshape(1, H, D)
    finally:
        lib.ggml_backend_mi355x_set_tune(39, 0)
        lib.ggml_backend_mi355x_set_tune(35, 0)
    assert any(ln.startswith("fattn_dec3 ") for ln in log) == stream, log
    ref = orc.flash_attn(q, k, v, m16, scale)
    assert nmse(y, ref) < 5e-4
    assert np.array_equal(y, y2)


@pytest.mark.parametrize("kind", ["q8_0", "q4_0", "bf16", "f32"])
@pytest.mark.parametrize("n_q,n_kv,H,Hkv,D,softcap", [
    (1, 256, 32, 8, 128, 0.0),      # tg128 decode step: k_fattn_dec2 (q8_0 native), tile kernel otherwise
    (1, 1500, 32, 8, 128, 0.0),     # long cache: dec2 split merge (q8_0)
    (2, 130, 8, 2, 64, 0.0),        # two query rows, D 64
    (512, 512, 32, 8, 128, 0.0),    # pp512 prefill: f16 copies + k_fa_mma2
    (40, 320, 8, 2, 64, 0.0),       # prefill D 64: f16 copies + k_fa_mma
    (5, 200, 4, 2, 128, 10.0),      # softcap: tile kernel
])
def test_flash_attn_kv_types(pkg, backend, orc, kind, n_q, n_kv, H, Hkv, D, softcap):
    """quantised / bf16 / f32 KV caches (llama-bench -ctk/-ctv, tests/test-backend-ops.cpp:8232)
    against orc_flash_attn_t, which is pinned to the reference CPU backend (test_oracle.py)"""
    from qgen import KV_TYPES, kv_rows
    if kind == "f32" and (n_q >= 512 or n_kv > 1000):
        pytest.skip("f32 caches: the tile kernel only; large shapes add nothing")
    rng = np.random.default_rng(n_q * 1000 + n_kv + D)
    q = rng.standard_normal((H, n_q, D)).astype(np.float32)
    k = kv_rows(kind, Hkv, n_kv, D, rng, orc)
    v = kv_rows(kind, Hkv, n_kv, D, rng, orc)
    mask = np.zeros((n_q, n_kv), np.float32)
    for i in range(n_q):
        mask[i, n_kv - n_q + i + 1:] = -np.inf
    m16 = mask.astype(np.float16).view(np.uint16)
    scale = 1.0 / np.sqrt(D)
    tid = KV_TYPES[kind]

    def build(ctx):
        tq = ctx.new_tensor("f32", D, n_q, H)
        tk = ctx.new_tensor(tid, D, n_kv, Hkv)
        tv = ctx.new_tensor(tid, D, n_kv, Hkv)
        tm = ctx.new_tensor("f16", n_kv, n_q)
        return [ctx.flash_attn_ext(tq, tk, tv, tm, scale, 0.0, softcap)], [(tq, q), (tk, k), (tv, v), (tm, m16)]

    backend.klog(True)
    y = run(pkg, backend, build)[0].reshape(n_q, H, D)
    log = backend.klog_read()
    backend.klog(False)
    ref = orc.flash_attn_t(q, k, v, m16, scale, tid, 0.0, softcap)
    assert nmse(y, ref) < 5e-4, nmse(y, ref)
    if kind == "q8_0" and n_q <= 4 and softcap == 0.0:
        assert any(ln.startswith("fattn_dec2") and "kq8=1" in ln for ln in log), log
    if n_q >= 16 and softcap == 0.0 and kind != "f32":
        assert any(ln.startswith("fa_kv_to_f16") for ln in log) and any(ln.startswith("fa_mma") for ln in log), log


@pytest.mark.parametrize("kt,vt", [("q8_0", "f16"), ("f16", "q8_0"), ("q4_0", "f16"), ("q8_0", "q4_0")])
@pytest.mark.parametrize("n_q,n_kv,H,Hkv,D", [
    (1, 256, 32, 8, 128),      # tg128 decode step (f16 / q8_0 pairs: k_fattn_dec2, KV 2 / 3)
    (1, 1500, 32, 8, 128),     # long cache: the LONG geometry + combine
    (512, 512, 32, 8, 128),    # pp512 prefill: the quantised side copied to f16, k_fa_mma2
    (3, 130, 8, 2, 64),        # a few query rows, D 64
])
def test_flash_attn_mixed_kv_types(pkg, backend, orc, kt, vt, n_q, n_kv, H, Hkv, D):
    """Round 6: K and V caches of different types (-ctk q8_0 -ctv f16, the fork's own line,
    AGENTS.md:166-176; the reference's FA_ALL_QUANTS pairs, fattn.cu:220-260) against the
    oracle with K's and V's own dequantisation (orc_flash_attn_kv)"""
    from qgen import KV_TYPES, kv_rows
    rng = np.random.default_rng(n_q * 1000 + n_kv + D + 7)
    q = rng.standard_normal((H, n_q, D)).astype(np.float32)
    k = kv_rows(kt, Hkv, n_kv, D, rng, orc)
    v = kv_rows(vt, Hkv, n_kv, D, rng, orc)
    mask = np.zeros((n_q, n_kv), np.float32)
    for i in range(n_q):
        mask[i, n_kv - n_q + i + 1:] = -np.inf
    m16 = mask.astype(np.float16).view(np.uint16)
    scale = 1.0 / np.sqrt(D)

    def build(ctx):
        tq = ctx.new_tensor("f32", D, n_q, H)
        tk = ctx.new_tensor(KV_TYPES[kt], D, n_kv, Hkv)
        tv = ctx.new_tensor(KV_TYPES[vt], D, n_kv, Hkv)
        tm = ctx.new_tensor("f16", n_kv, n_q)
        return [ctx.flash_attn_ext(tq, tk, tv, tm, scale, 0.0, 0.0)], [(tq, q), (tk, k), (tv, v), (tm, m16)]

    backend.klog(True)
    y = run(pkg, backend, build)[0].reshape(n_q, H, D)
    log = backend.klog_read()
    backend.klog(False)
    ref = orc.flash_attn_t(q, k, v, m16, scale, KV_TYPES[kt], v_type=KV_TYPES[vt])
    assert nmse(y, ref) < 5e-4, nmse(y, ref)
    if n_q <= 4 and {kt, vt} <= {"f16", "q8_0"}:
        assert any(ln.startswith("fattn_dec2") and f"kq8={int(kt == 'q8_0')} vq8={int(vt == 'q8_0')}" in ln for ln in log), log
    if n_q >= 16:
        assert any(ln.startswith("fa_mma") for ln in log), log


@pytest.mark.parametrize("ni", [0, 16])
@pytest.mark.parametrize("kt,vt", [("q8_0", "q8_0"), ("q8_0", "f16")])
def test_flash_attn_long_quantised_geometry(pkg, backend, orc, kt, vt, ni):
    """Decode attention over a long quantised cache (the LONG split geometry + combine) at the
    default keys rows per lane and at 16 (g_tune[28], the geometry swept for q8_0 caches in
    round 6): the splits must cover every key whichever NI the launch uses"""
    from qgen import KV_TYPES, kv_rows
    n_q, n_kv, H, Hkv, D = 1, 6000, 32, 8, 128
    rng = np.random.default_rng(n_kv + 31 * ni + len(vt))
    q = rng.standard_normal((H, n_q, D)).astype(np.float32)
    k = kv_rows(kt, Hkv, n_kv, D, rng, orc)
    v = kv_rows(vt, Hkv, n_kv, D, rng, orc)
    mask = np.zeros((n_q, n_kv), np.float32)
    mask[:, -17:] = -np.inf                       # the tail past the "current" token masked
    m16 = mask.astype(np.float16).view(np.uint16)
    scale = 1.0 / np.sqrt(D)

    def build(ctx):
        tq = ctx.new_tensor("f32", D, n_q, H)
        tk = ctx.new_tensor(KV_TYPES[kt], D, n_kv, Hkv)
        tv = ctx.new_tensor(KV_TYPES[vt], D, n_kv, Hkv)
        tm = ctx.new_tensor("f16", n_kv, n_q)
        return [ctx.flash_attn_ext(tq, tk, tv, tm, scale, 0.0, 0.0)], [(tq, q), (tk, k), (tv, v), (tm, m16)]

    lib = pkg._lib.load()
    lib.ggml_backend_mi355x_set_tune(28, ni)
    try:
        backend.klog(True)
        y = run(pkg, backend, build)[0].reshape(n_q, H, D)
        log = backend.klog_read()
        backend.klog(False)
    finally:
        lib.ggml_backend_mi355x_set_tune(28, 0)
    ref = orc.flash_attn_t(q, k, v, m16, scale, KV_TYPES[kt], v_type=KV_TYPES[vt])
    assert nmse(y, ref) < 5e-4, nmse(y, ref)
    assert any(ln.startswith("fattn_dec2") and "long=1" in ln for ln in log), log


def test_staged_write_dropped_when_buffer_freed(pkg, backend):
    """a small write is only queued (staged into the pinned ring, copied by the next
    flush). If its buffer is freed before that flush, the queued copy must be dropped — else
    it lands in freed memory or in the next allocation at that address. Write, free, reallocate
    the same size many times (hipMalloc hands the address back), write the new owner through a
    path that bypasses the queue (larger than a staged write), and read it back."""
    import ctypes
    lib = pkg._lib.load()
    st = (ctypes.c_uint64 * 3)()
    lib.ggml_backend_mi355x_stage_stats(0, st)
    dropped0 = st[2]
    n = (5 << 20) // 4                                  # 5 MB: above the 4 MB staging limit
    big = np.arange(n, dtype=np.float32)
    for trial in range(6):
        c1 = pkg.Context()
        a = c1.new_tensor("f32", n)
        c1.alloc(backend)
        # a staged write into a's buffer: the first 64 KB
        lib.mxg_tensor_set(a.ptr, np.full(16384, -1.0, np.float32).ctypes.data, 0, 65536)
        c1.free()                                       # freed with that write still queued
        c2 = pkg.Context()
        b = c2.new_tensor("f32", n)
        c2.alloc(backend)
        b.set(big)                                      # direct copy (not staged)
        got = b.numpy().reshape(-1)
        c2.free()
        assert np.array_equal(got, big), (trial, got[:4])
    lib.ggml_backend_mi355x_stage_stats(0, st)
    assert st[2] >= dropped0 + 6, (dropped0, list(st))


def test_mul_mat_id(pkg, backend, orc):
    tid = NAMES["q4_K"]
    rng = np.random.default_rng(8)
    K, M, E, used, T = 512, 96, 4, 2, 3
    ws = [rand_quant(tid, M, K, rng) for _ in range(E)]
    rb = ws[0][1]
    w = np.concatenate([a for a, _ in ws])
    x = rng.standard_normal((T, 1, K)).astype(np.float32)
    ids = np.array([[1, 3], [0, 1], [2, 2]], np.int32)

    def build(ctx):
        tw = ctx.new_tensor(tid, K, M, E)
        tx = ctx.new_tensor("f32", K, 1, T)
        ti = ctx.new_tensor("i32", used, T)
        return [ctx.mul_mat_id(tw, tx, ti)], [(tw, w), (tx, x), (ti, ids)]

    y = run(pkg, backend, build)[0].reshape(T, used, M)
    for t in range(T):
        for e in range(used):
            ex = ids[t, e]
            ref = orc.mul_mat(tid, w[ex * M * rb:(ex + 1) * M * rb], rb, x[t])[0]
            assert nmse(y[t, e], ref) < 5e-4


@pytest.mark.parametrize("extra_use", [False, True])
def test_norm_absorbed_by_gemv(pkg, backend, orc, extra_use):
    """RMS_NORM -> MUL(w) consumed only by single-token GEMVs is folded into the GEMV
    prologues (deferred norm); with an extra non-GEMV consumer it is materialised."""
    tid = NAMES["q4_K"]
    rng = np.random.default_rng(31)
    K, M1, M2 = 2048, 384, 128
    w1, rb = rand_quant(tid, M1, K, rng)
    w2, _ = rand_quant(tid, M2, K, rng)
    x = rng.standard_normal((1, K)).astype(np.float32)
    nw = rng.uniform(0.5, 1.5, K).astype(np.float32)
    before = backend.stats()["nodes_fused"]

    def build(ctx):
        tx = ctx.new_tensor("f32", K, 1)
        tn = ctx.new_tensor("f32", K)
        t1 = ctx.new_tensor(tid, K, M1)
        t2 = ctx.new_tensor(tid, K, M2)
        cur = ctx.mul(ctx.rms_norm(tx, 1e-5), tn)
        outs = [ctx.mul_mat(t1, cur), ctx.mul_mat(t2, cur)]
        if extra_use:
            outs.append(ctx.scale(cur, 2.0))
        return outs, [(tx, x), (tn, nw), (t1, w1), (t2, w2)]

    res = run(pkg, backend, build)
    xn = orc.rms_norm(x, 1e-5) * nw
    for y, w, M in ((res[0], w1, M1), (res[1], w2, M2)):
        ref = orc.mul_mat(tid, w, rb, xn, exact=True)
        assert nmse(y.reshape(1, M), ref) < 5e-4
    if extra_use:
        assert nmse(res[2].reshape(1, K), 2.0 * xn) < 1e-10
    else:
        assert backend.stats()["nodes_fused"] >= before + 2, "norm was not deferred"


@pytest.mark.parametrize("tname", ["q4_K", "q6_K", "q5_K", "q4_0", "q8_0"])
@pytest.mark.parametrize("norm", [False, True])
def test_gemv_lds_dma_staging_forced(pkg, backend, orc, tname, norm):
    """the LDS-DMA activation prologue (XS_F32_LDS / XS_NORM_LDS: counted vmcnt wait + raw
    s_barrier, gemv.cuh stage_finish) normally runs only on grids of >= 2048 waves;
    g_tune[9] = 1 forces it at a small shape, K over several weight batches"""
    lib = pkg._lib.load()
    tid = NAMES[tname]
    rng = np.random.default_rng(61)
    K, M = 2048, 320
    w, rb = rand_quant(tid, M, K, rng)
    x = rng.standard_normal((1, K)).astype(np.float32)
    nw = rng.uniform(0.5, 1.5, K).astype(np.float32)

    def build(ctx):
        tw = ctx.new_tensor(tid, K, M)
        tx = ctx.new_tensor("f32", K, 1)
        tn = ctx.new_tensor("f32", K)
        src = ctx.mul(ctx.rms_norm(tx, 1e-5), tn) if norm else tx
        return [ctx.mul_mat(tw, src)], [(tw, w), (tx, x), (tn, nw)]

    lib.ggml_backend_mi355x_set_tune(9, 1)
    backend.klog(True)
    try:
        y = run(pkg, backend, build)[0].reshape(1, M)
        log = backend.klog_read()
    finally:
        backend.klog(False)
        lib.ggml_backend_mi355x_set_tune(9, 0)
    xin = orc.rms_norm(x, 1e-5) * nw if norm else x
    assert nmse(y, orc.mul_mat(tid, w, rb, xin, exact=True)) < 5e-4
    mode = 4 if norm else 3
    assert any(ln.startswith("gemv2 ") and f" mode={mode} " in ln for ln in log), log


@pytest.mark.parametrize("n_tok,n_exp,producer", [(1, 8, False), (40, 8, False), (40, 4, True), (1, 4, True), (64, 8, True)])
def test_moe_router_fusion(pkg, backend, n_tok, n_exp, producer):
    """llama build_moe_ffn's router chain (SOFT_MAX -> ARGSORT -> top-k GET_ROWS -> SUM_ROWS
    -> CLAMP -> DIV) runs as one k_topk_moe launch; every node's output is checked against
    numpy (softmax 1e-6 like test-backend-ops, selection exact)"""
    rng = np.random.default_rng(91 + n_tok)
    k, E = 2, 256
    wr = (rng.standard_normal((n_exp, E)) * 0.1).astype(np.float32)
    xr = rng.standard_normal((n_tok, E)).astype(np.float32)
    logits = rng.standard_normal((n_tok, n_exp)).astype(np.float32) * 2
    if producer:   # the logits come from the router MUL_MAT in the same graph (f32 weights)
        logits = (xr.astype(np.float64) @ wr.T.astype(np.float64)).astype(np.float32)

    def build(ctx):
        if producer:
            tw = ctx.new_tensor("f32", E, n_exp)
            tx = ctx.new_tensor("f32", E, n_tok)
            tl = ctx.mul_mat(tw, tx)
            feed = [(tw, wr), (tx, xr)]
        else:
            tl = ctx.new_tensor("f32", n_exp, n_tok)
            feed = [(tl, logits)]
        probs = ctx.soft_max_ext(tl, None, 1.0)
        order = ctx.argsort(probs, desc=True)
        nb1 = order.nb[1]
        topk = ctx.view_4d(order, k, n_tok, 1, 1, nb1, nb1 * n_tok, nb1 * n_tok, 0)
        w = ctx.get_rows(ctx.reshape(probs, 1, n_exp, n_tok), topk)
        w2 = ctx.reshape(w, k, n_tok)
        cl = ctx.clamp(ctx.sum_rows(w2), 6.103515625e-5, float("inf"))
        wn = ctx.div(w2, cl)
        return [probs, order, w, wn], feed

    backend.klog(True)
    probs, order, w, wn = run(pkg, backend, build)
    log = backend.klog_read()
    backend.klog(False)
    e = np.exp(logits - logits.max(1, keepdims=True))
    ref_p = e / e.sum(1, keepdims=True)
    assert nmse(probs.reshape(n_tok, n_exp), ref_p) < (1e-5 if producer else 1e-6)
    ref_o = np.argsort(-ref_p, axis=1, kind="stable")
    assert np.array_equal(order.reshape(n_tok, n_exp)[:, :k], ref_o[:, :k])
    ref_w = np.take_along_axis(ref_p, ref_o[:, :k], 1)
    assert nmse(w.reshape(n_tok, k), ref_w) < 1e-6
    assert nmse(wn.reshape(n_tok, k), ref_w / ref_w.sum(1, keepdims=True)) < 1e-6
    assert any(ln.startswith("topk_moe") for ln in log), log


@pytest.mark.parametrize("n_kv,H,Hkv,D,mask_t", [(256, 32, 8, 128, "f32"), (512, 8, 8, 128, "f16"), (96, 4, 2, 64, "f32"),
                                                 (256, 32, 8, 128, None), (48, 4, 2, 64, "f32"), (16384, 8, 8, 128, "f16"),
                                                 (16640, 32, 8, 128, "f16"), (17000, 16, 2, 128, "f32"), (8192, 64, 8, 128, "f16"),
                                                 (20008, 4, 4, 128, None), (4096, 32, 8, 128, "f16"), (2056, 8, 2, 128, "f32")])
def test_attn_nofa_decode_chain(pkg, backend, n_kv, H, Hkv, D, mask_t):
    """-fa 0 decode attention (llama-bench's default): MUL_MAT(k, q) -> SOFT_MAX(mask, scale)
    -> MUL_MAT(v^T, kq) -> PERMUTE -> CONT (src/llama-graph.cpp:1740-1796) as one launch
    (k_attn_nofa_dec), against the node-by-node semantics in float64: q and p rounded to
    f16 as the two mul_mats' vec_dot_type conversions do. n_kv = 48 at D 64 does not split
    into the kernel's 4 parts of 8-key steps: the chain must run unfused (and stay right);
    n_kv = 16384 needs 64 KB of scores in LDS (max dynamic LDS raised past the default).
    Round 5: caches from 512 keys (and all beyond the one-workgroup kernel's 16384) take
    the three-launch long form (klog attn_nofa_long: chunked scores + (max, sum) partials,
    block P·V partials, their ordered sum) — llama-bench -d 16384 pads n_kv to 16640; GQA 8,
    4, 2 and 1; a ragged last chunk and block (17000, 20008)."""
    rng = np.random.default_rng(n_kv + H + D)
    q = rng.standard_normal((H, 1, D)).astype(np.float32)
    k = rng.standard_normal((Hkv, n_kv, D)).astype(np.float16)
    vt = rng.standard_normal((Hkv, D, n_kv)).astype(np.float16)     # transposed V cache view
    mask = np.zeros((1, n_kv), np.float32)
    mask[0, n_kv - 5:] = -np.inf
    scale = 1.0 / np.sqrt(D)

    def build(ctx):
        tq = ctx.new_tensor("f32", D, 1, H)
        tk = ctx.new_tensor("f16", D, n_kv, Hkv)
        tv = ctx.new_tensor("f16", n_kv, D, Hkv)
        tm = ctx.new_tensor(mask_t, n_kv, 1) if mask_t else None
        kq = ctx.mul_mat(tk, tq)
        sm = ctx.soft_max_ext(kq, tm, scale)
        kqv = ctx.mul_mat(tv, sm)
        out = ctx.cont(ctx.permute(kqv, 0, 2, 1, 3))
        feed = [(tq, q), (tk, k.view(np.uint16)), (tv, vt.view(np.uint16))]
        if mask_t:
            feed.append((tm, mask if mask_t == "f32" else mask.astype(np.float16).view(np.uint16)))
        return [out], feed

    backend.klog(True)
    y = run(pkg, backend, build)[0].reshape(H, D)
    log = backend.klog_read()
    backend.klog(False)
    lng = D == 128 and n_kv % 8 == 0 and n_kv >= 512
    fused = lng or (n_kv % (8 * (256 // D)) == 0 and n_kv <= 16384)
    assert any(ln.startswith("attn_nofa") for ln in log) == fused, log
    assert any(ln.startswith("attn_nofa_long ") for ln in log) == lng, log
    G = H // Hkv
    ref = np.empty((H, D))
    for h in range(H):
        s = (q[h, 0].astype(np.float16).astype(np.float64) @ k[h // G].astype(np.float64).T) * scale
        if mask_t:
            s = s + mask[0]
        e = np.exp(s - s.max())
        pr = (e / e.sum()).astype(np.float16).astype(np.float64)
        ref[h] = vt[h // G].astype(np.float64) @ pr
    assert nmse(y, ref) < 1e-6, nmse(y, ref)


@pytest.mark.parametrize("n_q,n_kv,H,Hkv,mask_t", [(512, 512, 32, 8, "f32"), (64, 256, 8, 8, "f16"), (100, 192, 16, 4, "f32"),
                                                   (512, 2048, 32, 8, "f32")])
def test_attn_nofa_prefill_chain(pkg, backend, n_q, n_kv, H, Hkv, mask_t):
    """-fa 0 prefill attention (llama-bench's default): the same node chain as the decode
    case with n_q query rows, run as one transposed-V MFMA flash kernel (k_fa_mma2<HG, VT>,
    klog attn_nofa_mma) against the node-by-node semantics in float64 (q and p rounded to
    f16 as the mul_mats convert them). Causal mask with the queries at the end of the cache
    (the prefill of a later ubatch), f32 as libllama's non-FA graph builds it or f16."""
    D = 128
    rng = np.random.default_rng(n_q + n_kv + H)
    q = rng.standard_normal((H, n_q, D)).astype(np.float32)
    k = rng.standard_normal((Hkv, n_kv, D)).astype(np.float16)
    vt = rng.standard_normal((Hkv, D, n_kv)).astype(np.float16)
    mask = np.zeros((n_q, n_kv), np.float32)
    for i in range(n_q):
        mask[i, n_kv - n_q + i + 1:] = -np.inf
    scale = 1.0 / np.sqrt(D)

    def build(ctx):
        tq = ctx.new_tensor("f32", D, n_q, H)
        tk = ctx.new_tensor("f16", D, n_kv, Hkv)
        tv = ctx.new_tensor("f16", n_kv, D, Hkv)
        tm = ctx.new_tensor(mask_t, n_kv, n_q)
        kq = ctx.mul_mat(tk, tq)
        sm = ctx.soft_max_ext(kq, tm, scale)
        kqv = ctx.mul_mat(tv, sm)
        out = ctx.cont(ctx.permute(kqv, 0, 2, 1, 3))
        feed = [(tq, q), (tk, k.view(np.uint16)), (tv, vt.view(np.uint16)),
                (tm, mask if mask_t == "f32" else mask.astype(np.float16).view(np.uint16))]
        return [out], feed

    backend.klog(True)
    y = run(pkg, backend, build)[0].reshape(n_q, H, D)
    log = backend.klog_read()
    backend.klog(False)
    assert any(ln.startswith("attn_nofa_mma") for ln in log), log
    G = H // Hkv
    ref = np.empty((n_q, H, D))
    for h in range(H):
        s = (q[h].astype(np.float16).astype(np.float64) @ k[h // G].astype(np.float64).T) * scale + mask
        e = np.exp(s - s.max(1, keepdims=True))
        pr = (e / e.sum(1, keepdims=True)).astype(np.float16).astype(np.float64)
        ref[:, h] = pr @ vt[h // G].astype(np.float64).T
    assert nmse(y, ref) < 1e-5, nmse(y, ref)


@pytest.mark.parametrize("kind", ["f16", "q8_0"])
@pytest.mark.parametrize("n_kv,H,Hkv,M,wt,mask_tail,ni", [
    (256, 32, 8, 4096, "q4_K", 0, 4),      # llama-bench tg128: 4 splits of 64 keys
    (256, 32, 8, 4096, "q4_K", 200, 4),    # mostly masked: splits 1-3 fully masked (max -inf)
    (256, 32, 8, 4096, "q4_K", 0, 2),      # 8 splits of 32 keys (XS_FAP8)
    (37, 32, 8, 4096, "q5_K", 5, 4),       # one ragged split
    (130, 32, 4, 1000, "q6_K", 0, 4),      # 3 splits, ragged rows (M % 16 != 0), GQA 8
    (1, 8, 2, 512, "q4_0", 0, 4),          # one key, small model (lpr 64 geometry)
    (200, 16, 16, 2048, "q8_0", 17, 2),    # no GQA, 7 splits
])
def test_attn_split_oproj_decode(pkg, backend, orc, kind, n_kv, H, Hkv, M, wt, mask_tail, ni):
    """Round 5: FLASH_ATTN_EXT -> RESHAPE -> MUL_MAT(wo) -> ADD(residual) of one decode token
    as the attention's split partials (fa_dec2_partials, 64- or 32-key chunks) merged in the
    residual GEMV's prologue (XStage::fap, modes 8 / 9) — the default decode path (exec.cpp
    fuse_attn_split_o) — against the node-by-node oracle, and against the round-4 path
    (g_tune[32] = 1: one-split attention, O projection from x)"""
    from qgen import KV_TYPES, kv_rows
    D = 128
    rng = np.random.default_rng(n_kv * 7 + H + M)
    q = rng.standard_normal((H, 1, D)).astype(np.float32)
    k = kv_rows(kind, Hkv, n_kv, D, rng, orc)
    v = kv_rows(kind, Hkv, n_kv, D, rng, orc)
    mask = np.zeros((1, n_kv), np.float32)
    if mask_tail:
        mask[0, n_kv - mask_tail:] = -np.inf
    m16 = mask.astype(np.float16).view(np.uint16)
    scale = 1.0 / np.sqrt(D)
    K = D * H
    tw_t = NAMES[wt]
    w, rb = rand_quant(tw_t, M, K, rng)
    r = rng.standard_normal((1, M)).astype(np.float32)
    tid = KV_TYPES[kind]

    def build(ctx):
        tq = ctx.new_tensor("f32", D, 1, H)
        tk = ctx.new_tensor(tid, D, n_kv, Hkv)
        tv = ctx.new_tensor(tid, D, n_kv, Hkv)
        tm = ctx.new_tensor("f16", n_kv, 1)
        tw = ctx.new_tensor(tw_t, K, M)
        tr = ctx.new_tensor("f32", M, 1)
        fa = ctx.flash_attn_ext(tq, tk, tv, tm, scale)
        y = ctx.add(ctx.mul_mat(tw, ctx.reshape(fa, K, 1)), tr)
        return [y], [(tq, q), (tk, k), (tv, v), (tm, m16), (tw, w), (tr, r)]

    lib = pkg._lib.load()
    lib.ggml_backend_mi355x_set_tune(33, ni)
    try:
        backend.klog(True)
        y = run(pkg, backend, build)[0].reshape(M)
        log = backend.klog_read()
        backend.klog(False)
        ns = -(-n_kv // (16 * ni))
        assert any(l.startswith("fattn_dec2_part ") and f"NI={ni} nsplit={ns} " in l for l in log), log
        mode = 8 if ns <= 4 else 9
        assert any(l.startswith("gemv2 ") and "epi=2" in l and f"mode={mode} " in l for l in log), log
        y2 = run(pkg, backend, build)[0].reshape(M)
        lib.ggml_backend_mi355x_set_tune(32, 1)
        backend.klog(True)
        y3 = run(pkg, backend, build)[0].reshape(M)
        log3 = backend.klog_read()
        backend.klog(False)
        assert not any(l.startswith("fattn_dec2_part ") for l in log3), log3
    finally:
        lib.ggml_backend_mi355x_set_tune(32, 0)
        lib.ggml_backend_mi355x_set_tune(33, 0)
    att = orc.flash_attn_t(q, k, v, m16, scale, tid, 0.0, 0.0).reshape(1, K)
    ref = orc.mul_mat(tw_t, w, rb, att)[0] + r[0]
    ref_exact = orc.mul_mat(tw_t, w, rb, att, exact=True)[0] + r[0]
    assert np.all(np.isfinite(y))
    assert nmse(y, ref) < 5e-4, nmse(y, ref)
    assert nmse(y, ref_exact) < 5e-4, nmse(y, ref_exact)
    assert np.array_equal(y, y2)                  # deterministic (no atomics in either launch)
    assert nmse(y, y3) < 1e-5, nmse(y, y3)


@pytest.mark.parametrize("per_expert", [False, True])
@pytest.mark.parametrize("n_exp,E,wtype,knorm", [(8, 4096, "f32", True), (8, 4096, "f16", True), (4, 256, "f32", False),
                                                 (16, 1024, "f32", True), (8, 6144, "f32", True), (8, 6144, "f16", False)])
def test_moe_router_head_fusion(pkg, backend, orc, n_exp, E, wtype, knorm, per_expert):
    """Round 5: the MoE block's head of one decoded token — RMS_NORM -> MUL(ffn_norm) ->
    MUL_MAT(router) -> SOFT_MAX -> ARGSORT -> top-k GET_ROWS [-> SUM_ROWS -> CLAMP -> DIV] —
    as ONE launch (ops_moe.hip fuse_moe_router), every node's output checked against numpy,
    and against the node-by-node launches (g_tune[34] = 1). Round 6: <= 8 experts run the
    single 1024-thread workgroup k_moe_router1; per_expert (g_tune[46] = 1) the round-5 one
    workgroup per expert with the last-arriver top-k"""
    rng = np.random.default_rng(7 + n_exp + E)
    k = 2
    x = rng.standard_normal((1, E)).astype(np.float32)
    nw = (1 + 0.1 * rng.standard_normal(E)).astype(np.float32)
    wr = (rng.standard_normal((n_exp, E)) * 0.05).astype(np.float32)
    wr_feed = wr.astype(np.float16).view(np.uint16) if wtype == "f16" else wr
    wr_ref = wr.astype(np.float16).astype(np.float32) if wtype == "f16" else wr

    def build(ctx):
        tx = ctx.new_tensor("f32", E, 1)
        tn = ctx.new_tensor("f32", E)
        tw = ctx.new_tensor(wtype, E, n_exp)
        cur = ctx.mul(ctx.rms_norm(tx, 1e-5), tn)
        tl = ctx.mul_mat(tw, cur)
        probs = ctx.soft_max_ext(tl, None, 1.0)
        order = ctx.argsort(probs, desc=True)
        nb1 = order.nb[1]
        topk = ctx.view_4d(order, k, 1, 1, 1, nb1, nb1, nb1, 0)
        w = ctx.get_rows(ctx.reshape(probs, 1, n_exp, 1), topk)
        outs = [cur, tl, probs, order, w]
        if knorm:
            w2 = ctx.reshape(w, k, 1)
            cl = ctx.clamp(ctx.sum_rows(w2), 6.103515625e-5, float("inf"))
            outs.append(ctx.div(w2, cl))
        return outs, [(tx, x), (tn, nw), (tw, wr_feed)]

    lib = pkg._lib.load()
    lib.ggml_backend_mi355x_set_tune(46, int(per_expert))
    try:
        backend.klog(True)
        res = run(pkg, backend, build)
        log = backend.klog_read()
        backend.klog(False)
    finally:
        lib.ggml_backend_mi355x_set_tune(46, 0)
    lib.ggml_backend_mi355x_set_tune(34, 1)
    try:
        res_u = run(pkg, backend, build)
    finally:
        lib.ggml_backend_mi355x_set_tune(34, 0)
    one = not per_expert and n_exp <= 8 and E % 128 == 0 and E <= 8192
    assert any(ln.startswith("moe_router1 " if one else "moe_router ") for ln in log), log
    cur_ref = orc.rms_norm(x, 1e-5) * nw
    assert nmse(res[0].reshape(1, E), cur_ref) < 1e-7
    lg_ref = (cur_ref.astype(np.float64) @ wr_ref.T.astype(np.float64))[0]
    assert nmse(res[1].reshape(n_exp), lg_ref) < 1e-6
    e = np.exp(lg_ref - lg_ref.max())
    p_ref = e / e.sum()
    assert nmse(res[2].reshape(n_exp), p_ref) < 1e-5
    o_ref = np.argsort(-p_ref, kind="stable")
    assert np.array_equal(res[3].reshape(n_exp)[:k], o_ref[:k])
    w_ref = p_ref[o_ref[:k]]
    assert nmse(res[4].reshape(k), w_ref) < 1e-6
    if knorm:
        assert nmse(res[5].reshape(k), w_ref / w_ref.sum()) < 1e-6
    for a, b in zip(res, res_u):   # fused == node by node (ordering / selection identical)
        if a.dtype == np.int32:
            assert np.array_equal(a.reshape(-1)[:k], b.reshape(-1)[:k])
        else:
            assert nmse(a.reshape(-1), b.reshape(-1)) < 1e-9


@pytest.mark.parametrize("n_kv,H,Hkv,M,wt,mask_t", [(256, 32, 8, 4096, "q4_K", "f16"), (512, 8, 8, 1024, "q6_K", "f32"),
                                                  (64, 16, 4, 2048, "q5_K", None), (448, 8, 2, 1024, "q4_K", "f16")])
def test_attn_nofa_split_oproj_decode(pkg, backend, orc, n_kv, H, Hkv, M, wt, mask_t):
    """Round 5: the -fa 0 decode chain MUL_MAT(k, q) -> SOFT_MAX -> MUL_MAT(v^T, p) ->
    PERMUTE -> CONT -> RESHAPE -> MUL_MAT(wo) -> ADD(residual) of one token as split partials
    of 64 keys (k_nofa_part) merged in the output projection's prologue (XStage::fap) —
    the default for caches of <= 512 keys (ops_fattn_dec.hip nofa_split_o) — against the
    node-by-node semantics in float64 (q rounded to f16, p normalised then rounded to f16 as
    the node chain does; the partial form keeps p in f32) and against the chain kernel path
    (g_tune[38] = 1)"""
    D = 128
    rng = np.random.default_rng(n_kv * 3 + H + M)
    q = rng.standard_normal((H, 1, D)).astype(np.float32)
    k = rng.standard_normal((Hkv, n_kv, D)).astype(np.float16)
    vt = rng.standard_normal((Hkv, D, n_kv)).astype(np.float16)
    mask = np.zeros((1, n_kv), np.float32)
    mask[0, n_kv - 7:] = -np.inf
    scale = 1.0 / np.sqrt(D)
    K = D * H
    tw_t = NAMES[wt]
    w, rb = rand_quant(tw_t, M, K, rng)
    r = rng.standard_normal((1, M)).astype(np.float32)

    def build(ctx):
        tq = ctx.new_tensor("f32", D, 1, H)
        tk = ctx.new_tensor("f16", D, n_kv, Hkv)
        tv = ctx.new_tensor("f16", n_kv, D, Hkv)
        tm = ctx.new_tensor(mask_t, n_kv, 1) if mask_t else None
        tw = ctx.new_tensor(tw_t, K, M)
        tr = ctx.new_tensor("f32", M, 1)
        kq = ctx.mul_mat(tk, tq)
        sm = ctx.soft_max_ext(kq, tm, scale)
        kqv = ctx.mul_mat(tv, sm)
        out = ctx.cont(ctx.permute(kqv, 0, 2, 1, 3))
        y = ctx.add(ctx.mul_mat(tw, ctx.reshape(out, K, 1)), tr)
        feed = [(tq, q), (tk, k.view(np.uint16)), (tv, vt.view(np.uint16)), (tw, w), (tr, r)]
        if mask_t:
            feed.append((tm, mask if mask_t == "f32" else mask.astype(np.float16).view(np.uint16)))
        return [y], feed

    lib = pkg._lib.load()
    try:
        backend.klog(True)
        y = run(pkg, backend, build)[0].reshape(M)
        log = backend.klog_read()
        backend.klog(False)
        assert any(l.startswith("attn_nofa_part ") and f"nsplit={n_kv // 64}" in l for l in log), log
        assert any(l.startswith("gemv2 ") and "epi=2" in l and (" mode=8 " in l or " mode=9 " in l) for l in log), log
        lib.ggml_backend_mi355x_set_tune(38, 1)
        backend.klog(True)
        y2 = run(pkg, backend, build)[0].reshape(M)
        log2 = backend.klog_read()
        backend.klog(False)
        assert not any(l.startswith("attn_nofa_part ") for l in log2), log2
    finally:
        lib.ggml_backend_mi355x_set_tune(38, 0)
    G = H // Hkv
    att = np.empty((H, D))
    for h in range(H):
        s_ = (q[h, 0].astype(np.float16).astype(np.float64) @ k[h // G].astype(np.float64).T) * scale
        if mask_t:
            s_ = s_ + mask[0]
        e = np.exp(s_ - s_.max())
        pr = (e / e.sum()).astype(np.float16).astype(np.float64)
        att[h] = vt[h // G].astype(np.float64) @ pr
    ref = orc.mul_mat(tw_t, w, rb, att.reshape(1, K).astype(np.float32), exact=True)[0] + r[0]
    assert np.all(np.isfinite(y))
    assert nmse(y, ref) < 5e-4, nmse(y, ref)
    assert nmse(y2, ref) < 5e-4, nmse(y2, ref)
    assert nmse(y, y2) < 1e-4, nmse(y, y2)
