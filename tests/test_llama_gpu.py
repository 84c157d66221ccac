"""End-to-end decode through the backend: the Llama graph of src/models/llama.cpp built
by the runner, executed by libggml-mi355x.so. Size-independent properties:
prefill logits == incremental-decode logits, flash-attn graph == KQ/softmax graph,
fused == unfused executor, HIP-graph replay == eager, determinism."""
import os

import numpy as np
import pytest

from qgen import nmse

pytestmark = pytest.mark.gpu

TINY = dict(n_vocab=1000, n_embd=256, n_layer=3, n_head=8, n_head_kv=2, n_ff=512, n_ctx_train=2048,
            rope_freq_base=10000.0, norm_eps=1e-5)


@pytest.fixture(scope="module")
def tiny(pkg, backend):
    m = pkg.Model.random(backend, TINY, "q4_k_m", seed=3)
    yield m
    m.free()


def test_prefill_matches_incremental_decode(pkg, tiny):
    rng = np.random.default_rng(0)
    toks = rng.integers(0, TINY["n_vocab"], 40).astype(np.int32)
    s1 = pkg.Session(tiny, n_ctx=256, flash_attn=True)
    all_logits = s1.decode_all(toks)          # one 40-token ubatch (MFMA GEMM path)
    s2 = pkg.Session(tiny, n_ctx=256, flash_attn=True)
    inc = np.stack([s2.decode(toks[i:i + 1]) for i in range(len(toks))])  # 40 single-token steps (GEMV path)
    assert np.all(np.isfinite(all_logits))
    assert nmse(inc, all_logits) < 5e-4
    s1.free(); s2.free()


def test_flash_attn_graph_matches_softmax_graph(pkg, tiny):
    rng = np.random.default_rng(1)
    toks = rng.integers(0, TINY["n_vocab"], 12).astype(np.int32)
    a = pkg.Session(tiny, n_ctx=256, flash_attn=True)
    b = pkg.Session(tiny, n_ctx=256, flash_attn=False)
    la = np.stack([a.decode(toks[i:i + 1]) for i in range(len(toks))])
    lb = np.stack([b.decode(toks[i:i + 1]) for i in range(len(toks))])
    assert nmse(la, lb) < 5e-4
    a.free(); b.free()


def test_graph_replay_deterministic(pkg, backend, tiny):
    rng = np.random.default_rng(2)
    toks = rng.integers(0, TINY["n_vocab"], 20).astype(np.int32)
    s = pkg.Session(tiny, n_ctx=256)
    before = backend.stats()["graph_replay"]
    r1 = np.stack([s.decode(toks[i:i + 1]) for i in range(len(toks))])
    s.reset()
    r2 = np.stack([s.decode(toks[i:i + 1]) for i in range(len(toks))])
    assert backend.stats()["graph_replay"] > before, "decode graphs were not replayed"
    assert np.array_equal(r1, r2)
    s.free()


def test_unfused_executor_matches(pkg, tiny):
    rng = np.random.default_rng(4)
    toks = rng.integers(0, TINY["n_vocab"], 6).astype(np.int32)
    s = pkg.Session(tiny, n_ctx=256)
    fused = np.stack([s.decode(toks[i:i + 1]) for i in range(len(toks))])
    s.free()
    os.environ["GGML_MI355X_DISABLE_FUSION"] = "1"
    os.environ["GGML_MI355X_DISABLE_GRAPHS"] = "1"
    try:
        be2 = pkg.Backend(0)
        m2 = pkg.Model.random(be2, TINY, "q4_k_m", seed=3)
        s2 = pkg.Session(m2, n_ctx=256)
        plain = np.stack([s2.decode(toks[i:i + 1]) for i in range(len(toks))])
        s2.free(); m2.free(); be2.free()
    finally:
        del os.environ["GGML_MI355X_DISABLE_FUSION"]
        del os.environ["GGML_MI355X_DISABLE_GRAPHS"]
    assert nmse(fused, plain) < 1e-6


@pytest.mark.parametrize("recipe", ["q4_0", "q8_0", "q5_k_m"])
def test_other_recipes_finite(pkg, backend, recipe):
    m = pkg.Model.random(backend, TINY, recipe, seed=5)
    s = pkg.Session(m, n_ctx=256)
    toks = np.arange(1, 30, dtype=np.int32)
    pre = s.decode(toks)
    assert np.all(np.isfinite(pre))
    s.free(); m.free()


def test_moe_decode_matches_prefill(pkg, backend):
    shape = dict(TINY, n_expert=4, n_expert_used=2)
    m = pkg.Model.random(backend, shape, "q4_k_m", seed=9)
    rng = np.random.default_rng(6)
    toks = rng.integers(0, TINY["n_vocab"], 10).astype(np.int32)
    a = pkg.Session(m, n_ctx=256)
    full = a.decode_all(toks)
    b = pkg.Session(m, n_ctx=256)
    inc = np.stack([b.decode(toks[i:i + 1]) for i in range(len(toks))])
    assert np.all(np.isfinite(full))
    assert nmse(inc, full) < 5e-4
    a.free(); b.free(); m.free()


@pytest.mark.parametrize("fa", [True, False])
def test_decode_fusions_fire(pkg, backend, tiny, fa):
    """Every decode layer runs the fused chains: rms_norm·w (1), Q/K/V+RoPE+KV-store (6),
    wo+residual (1), rms_norm·w (1), gate/up/GLU (2), down+residual (1)."""
    s = pkg.Session(tiny, n_ctx=256, flash_attn=fa)
    before = backend.stats()["nodes_fused"]
    s.decode(np.array([5], dtype=np.int32))
    fused = backend.stats()["nodes_fused"] - before
    s.free()
    assert fused >= 12 * TINY["n_layer"], f"only {fused} nodes fused"
