"""The oracle pinned to the reference's own outputs (CPU only).

Golden vectors: tests/golden/quant_*.npz, produced by tests/golden/make_golden.py from
the reference's gguf-py (de)quantisers and, for the K-quants gguf-py cannot quantise,
the reference C quantiser (ggml_quantize_chunk) built in oracle/_ref, on the data of the
reference KAT tests/test-quantize-fns.cpp:31-35.
"""
import glob
import os

import numpy as np
import pytest

from qgen import NAMES, nmse, rand_quant

GOLD = os.path.join(os.path.dirname(__file__), "golden")
FIXTURES = sorted(glob.glob(os.path.join(GOLD, "quant_*.npz")))


def test_fixtures_present():
    names = {os.path.basename(f)[6:-4] for f in FIXTURES}
    assert {"q4_0", "q8_0", "q4_K", "q5_K", "q6_K"} <= names


@pytest.mark.parametrize("path", FIXTURES, ids=lambda p: os.path.basename(p))
def test_dequant_bit_exact_vs_gguf_py(orc, path):
    name = os.path.basename(path)[6:-4]
    tid = NAMES[name]
    z = np.load(path, allow_pickle=False)
    q, deq = z["q"], z["deq"]
    rows, n = deq.shape
    q = q.reshape(rows, -1)
    for r in range(rows):
        y = orc.dequantize(tid, q[r], n)
        assert np.array_equal(y.view(np.uint32), deq[r].view(np.uint32)), f"{name} row {r}"


@pytest.mark.parametrize("path", FIXTURES, ids=lambda p: os.path.basename(p))
def test_quantisation_error_within_kat_bound(orc, path):
    # test-quantize-fns.cpp:18 MAX_QUANTIZATION_TOTAL_ERROR = 0.002 with the KAT's own
    # error measure array_rmse = sqrt(Σ diff²) / n (test-quantize-fns.cpp:38-45)
    z = np.load(path, allow_pickle=False)
    x, deq = z["x"], z["deq"]
    # the KAT quantises test_size = 4096 values (test-quantize-fns.cpp:103): all 4 rows together
    err = float(np.sqrt(np.sum((x.astype(np.float64) - deq) ** 2)) / x.size)
    assert x.size == 4096 and err < 0.002


def test_q8_0_quantiser_matches_golden(orc):
    z = np.load(os.path.join(GOLD, "quant_q8_0.npz"), allow_pickle=False)
    x, q = z["x"], z["q"].reshape(z["x"].shape[0], -1)
    for r in range(x.shape[0]):
        mine = orc.quantize_q8_0(x[r])
        # d fields must match exactly; quants may differ only on exact .5 ties (roundf vs np.round)
        a = mine.reshape(-1, 34)
        b = q[r].reshape(-1, 34)
        assert np.array_equal(a[:, :2], b[:, :2])
        diff = np.abs(a[:, 2:].view(np.int8).astype(int) - b[:, 2:].view(np.int8).astype(int))
        assert diff.max() <= 1 and (diff > 0).mean() < 0.01


def test_q4_0_quantiser_matches_golden(orc):
    """orc_quantize_row_q4_0 (SET_ROWS into a q4_0 KV cache) against gguf-py's Q4_0
    quantiser (tests/golden/quant_q4_0.npz): scales exact, nibbles equal but for rounding
    ties of the +8.5 truncation"""
    z = np.load(os.path.join(GOLD, "quant_q4_0.npz"), allow_pickle=False)
    x, q = z["x"], z["q"].reshape(z["x"].shape[0], -1)
    for r in range(x.shape[0]):
        a = orc.quantize_q4_0(x[r]).reshape(-1, 18)
        b = q[r].reshape(-1, 18)
        assert np.array_equal(a[:, :2], b[:, :2])
        na = np.concatenate([a[:, 2:] & 15, a[:, 2:] >> 4], 1).astype(int)
        nb = np.concatenate([b[:, 2:] & 15, b[:, 2:] >> 4], 1).astype(int)
        d = np.abs(na - nb)
        assert d.max() <= 1 and (d > 0).mean() < 0.01, (d.max(), (d > 0).mean())
    # and bit-exact against the reference's own C quantiser (ggml_quantize_chunk -> quantize_row_q4_0_ref,
    # oracle/_ref/libggml-ref.so built from /root/reference), where that build is present
    ref = os.path.join(os.path.dirname(GOLD), "..", "oracle", "_ref", "libggml-ref.so")
    if os.path.exists(ref):
        import ctypes
        L = ctypes.CDLL(ref)
        L.ggml_quantize_chunk.restype = ctypes.c_size_t
        L.ggml_quantize_chunk.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64,
                                          ctypes.c_int64, ctypes.c_void_p]
        rng = np.random.default_rng(3)
        xr = (rng.standard_normal((8, 1024)) * np.array([1e-3, 1, 7, 300, 1, 1, 1, 1])[:, None]).astype(np.float32)
        xr[4, :32] = 0.0
        xr[5, :64:2] = -xr[5, 1:64:2]                     # equal-magnitude pairs: the first one wins
        out = np.zeros((8, 1024 // 32 * 18), np.uint8)
        L.ggml_quantize_chunk(2, xr.ctypes.data, out.ctypes.data, 0, 8, 1024, None)   # GGML_TYPE_Q4_0 = 2
        for r in range(8):
            assert np.array_equal(orc.quantize_q4_0(xr[r]), out[r]), r


def test_fp16_conversion_matches_numpy(orc):
    rng = np.random.default_rng(0)
    vals = np.concatenate([rng.standard_normal(20000) * s for s in (1e-7, 1e-5, 1e-3, 1, 100, 1e4)]).astype(np.float32)
    vals = np.concatenate([vals, np.array([0.0, -0.0, 65504, 65519.99, 65520, 1e9, -1e9, 6e-8, 2.98e-8, np.inf, -np.inf], np.float32)])
    ours = orc.f32_to_f16(vals)
    ref = vals.astype(np.float16).view(np.uint16)
    assert np.array_equal(ours, ref)
    back = np.array([orc.lib.orc_fp16_to_fp32(int(h)) for h in ref[:5000]], np.float32)
    assert np.array_equal(back, ref[:5000].view(np.float16).astype(np.float32))


@pytest.mark.parametrize("tname", ["q4_K", "q5_K", "q6_K", "q4_0", "q8_0"])
def test_mul_mat_cpu_semantics_close_to_exact(orc, tname):
    tid = NAMES[tname]
    rng = np.random.default_rng(1)
    K, M, N = 1024, 64, 3
    w, rb = rand_quant(tid, M, K, rng)
    x = rng.standard_normal((N, K)).astype(np.float32)
    a = orc.mul_mat(tid, w, rb, x)
    b = orc.mul_mat(tid, w, rb, x, exact=True)
    assert nmse(a, b) < 5e-4


def test_rms_norm_rope_softmax_swiglu_numpy(orc):
    rng = np.random.default_rng(2)
    x = rng.standard_normal((3, 4096)).astype(np.float32)
    ref = x / np.sqrt(np.mean(x.astype(np.float64) ** 2, axis=1, keepdims=True) + 1e-5)
    assert nmse(orc.rms_norm(x, 1e-5), ref) < 1e-12
    # rope: rotation preserves the norm of each rotated pair, position 0 is identity
    q = rng.standard_normal((2, 4, 128)).astype(np.float32)
    y = orc.rope(q, np.array([0, 9], np.int32), 128, 0, 8192, 500000.0)
    assert np.allclose(y[0], q[0])
    assert np.allclose(np.linalg.norm(y[1], axis=-1), np.linalg.norm(q[1], axis=-1), rtol=1e-5)
    s = rng.standard_normal((2, 3, 50)).astype(np.float32)
    sm = orc.soft_max(s, None, 0.5)
    e = np.exp(0.5 * s - (0.5 * s).max(-1, keepdims=True))
    assert np.allclose(sm, e / e.sum(-1, keepdims=True), rtol=1e-5, atol=1e-7)
    a, b = rng.standard_normal(100).astype(np.float32), rng.standard_normal(100).astype(np.float32)
    assert np.allclose(orc.swiglu(a, b), a / (1 + np.exp(-a)) * b, rtol=1e-6)


def test_flash_attn_oracle_vs_dense_softmax(orc):
    rng = np.random.default_rng(3)
    H, Hkv, n_q, n_kv, D = 4, 2, 3, 40, 64
    q = rng.standard_normal((H, n_q, D)).astype(np.float32)
    k = rng.standard_normal((Hkv, n_kv, D)).astype(np.float16)
    v = rng.standard_normal((Hkv, n_kv, D)).astype(np.float16)
    out = orc.flash_attn(q, k.view(np.uint16), v.view(np.uint16), None, 0.125)
    qh = q.astype(np.float16).astype(np.float64)
    for h in range(H):
        kv = h // (H // Hkv)
        s = 0.125 * qh[h] @ k[kv].astype(np.float64).T
        p = np.exp(s - s.max(-1, keepdims=True))
        p /= p.sum(-1, keepdims=True)
        ref = p @ v[kv].astype(np.float64)
        assert np.allclose(out[:, h], ref, rtol=1e-4, atol=1e-5)


# ---------------------------------------------------------------------------
# the oracle op by op against the reference's own CPU ggml (oracle/ref_ops.cpp over
# oracle/_ref/libggml-ref.so, compiled from /root/reference by oracle/Makefile)
# ---------------------------------------------------------------------------
@pytest.fixture(scope="module")
def refops():
    import oracle_lib
    r = oracle_lib.load_ref_ops()
    if r is None:
        pytest.skip("oracle/_ref/libref-ops.so not built (make -C oracle ref)")
    return r


def _mask(n_q, n_kv):
    m = np.zeros((n_q, n_kv), np.float32)
    for i in range(n_q):
        m[i, n_kv - n_q + i + 1:] = -np.inf
    return m.astype(np.float16).view(np.uint16)


@pytest.mark.parametrize("kind", ["f16", "f32", "bf16", "q8_0", "q4_0"])
@pytest.mark.parametrize("n_q,n_kv,H,Hkv,D,max_bias,softcap", [(1, 113, 8, 2, 64, 0.0, 0.0), (7, 96, 4, 4, 128, 0.0, 0.0),
                                                               (3, 64, 4, 1, 64, 8.0, 0.0), (2, 70, 4, 2, 128, 0.0, 10.0)])
def test_flash_attn_oracle_vs_reference(orc, refops, kind, n_q, n_kv, H, Hkv, D, max_bias, softcap):
    """orc_flash_attn_t against ggml_flash_attn_ext on the reference CPU backend, every
    cache type of the harness grid (tests/test-backend-ops.cpp:8232), mask, ALiBi, softcap"""
    from qgen import KV_TYPES, kv_rows
    rng = np.random.default_rng(n_kv * 7 + D)
    q = rng.standard_normal((H, n_q, D)).astype(np.float32)
    k = kv_rows(kind, Hkv, n_kv, D, rng, orc)
    v = kv_rows(kind, Hkv, n_kv, D, rng, orc)
    m = _mask(n_q, n_kv)
    scale = 1.0 / np.sqrt(D)
    mine = orc.flash_attn_t(q, k, v, m, scale, KV_TYPES[kind], max_bias, softcap)
    ref = refops.flash_attn(q, k, v, m, scale, KV_TYPES[kind], max_bias, softcap)
    # the reference accumulates f16 V rows in f16 (VKQ16, ops.cpp one_chunk); the oracle in double
    assert nmse(mine, ref) < (2e-5 if kind == "f16" else 1e-9), nmse(mine, ref)


@pytest.mark.parametrize("mode,n_dims,ext", [(0, 128, 0.0), (2, 128, 0.0), (0, 64, 0.0), (2, 128, 1.0)])
def test_rope_oracle_vs_reference(orc, refops, mode, n_dims, ext):
    rng = np.random.default_rng(11 + mode + n_dims)
    x = rng.standard_normal((5, 4, 128)).astype(np.float32)
    pos = np.array([0, 1, 17, 300, 4095], np.int32)
    args = (pos, n_dims, mode, 8192, 500000.0, 0.5 if ext else 1.0, ext, 1.0, 32.0, 1.0)
    mine = orc.rope(x, *args)
    ref = refops.rope(x, *args)
    assert nmse(mine, ref) < 1e-12, nmse(mine, ref)


@pytest.mark.parametrize("masked,max_bias", [(False, 0.0), (True, 0.0), (True, 8.0)])
def test_soft_max_oracle_vs_reference(orc, refops, masked, max_bias):
    rng = np.random.default_rng(21)
    x = rng.standard_normal((4, 6, 77)).astype(np.float32) * 3
    m = None
    if masked:
        mm = np.where(rng.random((6, 77)) < 0.3, -np.inf, rng.standard_normal((6, 77))).astype(np.float16)
        m = mm.view(np.uint16)
    mine = orc.soft_max(x, m, 0.7, max_bias)
    ref = refops.soft_max(x, m, 0.7, max_bias)
    assert nmse(mine, ref) < 1e-12, nmse(mine, ref)


def test_rms_norm_oracle_vs_reference(orc, refops):
    rng = np.random.default_rng(31)
    x = rng.standard_normal((5, 4096)).astype(np.float32) * 2
    assert nmse(orc.rms_norm(x, 1e-5), refops.rms_norm(x, 1e-5)) < 1e-12
