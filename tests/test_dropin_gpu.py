"""Drop-in parity: the reference's own libllama (oracle/_ref, built from /root/reference
sources) runs a GGUF unmodified with libggml-mi355x.so loaded through
GGML_BACKEND_PATH and all layers offloaded (-ngl 99); its logits must match the same
libllama on the reference CPU backend (-ngl 0). Also: this package's own runner on the
same GGUF against the reference CPU logits.

Tolerance: NMSE 2e-3 on whole-model logits (the reference's test-backend-ops bound for
full graphs); prefill (one ubatch, MFMA GEMM path) and incremental decode
(one token per llama_decode: GEMV / decode-FA / fused QKV path) are both checked.
Synthetic GGUFs come from tools/gguf_synth.py (random weights, seeded)."""
import json
import os
import re
import subprocess
import sys

import numpy as np
import pytest

from dropin_util import assert_unsplit, graph_splits
from qgen import nmse

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = os.path.join(ROOT, "oracle", "_ref", "ref-llama-bench")
LIB = os.path.join(ROOT, "llama-mi50.cpp_amd", "lib", "libggml-mi355x.so")
TOL = 2e-3


def _need_ref():
    if not os.path.exists(REF):
        pytest.skip("oracle/_ref/ref-llama-bench not built")


@pytest.fixture(scope="module")
def ggufs(tmp_path_factory):
    d = tmp_path_factory.mktemp("gguf")
    out = {}
    for shape, recipe in [("tiny", "q4_k_m"), ("small", "q4_k_m"), ("small", "q4_0"), ("small", "q8_0"), ("tiny_moe", "q4_k_m")]:
        path = str(d / f"{shape}_{recipe}.gguf")
        subprocess.run([sys.executable, os.path.join(ROOT, "tools", "gguf_synth.py"), "--shape", shape,
                        "--recipe", recipe, "--out", path], check=True, timeout=300)
        out[(shape, recipe)] = path
    return out


def run_ref(tmp_path, gguf, toks, ngl, fa, incremental=False, ctk=None, klog=None, extra=(), env_extra=None, ctv=None,
            splits="auto"):
    """splits: the graph-split count libllama must report on the MI355X run ("auto": 2 —
    CPU input embedding + MI355X — unless a multi-device split mode is requested; None:
    not checked)"""
    tf = tmp_path / "toks.i32"
    of = tmp_path / f"logits_{ngl}_{fa}_{int(incremental)}.f32"
    np.asarray(toks, np.int32).tofile(tf)
    env = dict(os.environ)
    if ngl > 0:
        env["GGML_BACKEND_PATH"] = LIB
        if klog:
            env["GGML_MI355X_KLOG"] = str(klog)
    cmd = [REF, "-m", gguf, "-t", "8", "-ngl", str(ngl), "-fa", str(fa), "--logits", str(tf), str(of)]
    if incremental:
        cmd.append("--incremental")
    if ctk is not None:
        cmd += ["-ctk", str(ctk)]        # K and V cache type (ggml type id)
    if ctv is not None:
        cmd += ["-ctv", str(ctv)]        # V cache type alone
    cmd += list(extra)
    if env_extra and ngl > 0:
        env.update(env_extra)
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    if splits == "auto":
        splits = 2 if "-sm" not in extra else None
    if ngl > 0 and splits is not None:
        assert_unsplit(r.stderr, splits)
    n_vocab = int(r.stdout.strip().splitlines()[-1].split('"n_vocab": ')[1].split(",")[0].rstrip("}"))
    return np.fromfile(of, np.float32).reshape(len(toks), n_vocab), r.stderr


CASES = [("tiny", "q4_k_m"), ("small", "q4_k_m"), ("small", "q4_0"), ("small", "q8_0"), ("tiny_moe", "q4_k_m")]


@pytest.mark.parametrize("shape,recipe", CASES)
@pytest.mark.parametrize("fa", [1, 0])
def test_dropin_prefill(ggufs, tmp_path, shape, recipe, fa):
    _need_ref()
    toks = np.random.default_rng(7).integers(0, 1000, 40)
    cpu, _ = run_ref(tmp_path, ggufs[(shape, recipe)], toks, 0, fa)
    gpu, log = run_ref(tmp_path, ggufs[(shape, recipe)], toks, 99, fa)
    assert "MI355X" in log, "the MI355X backend was not loaded:\n" + log[-1000:]
    assert np.all(np.isfinite(gpu))
    assert nmse(gpu, cpu) < TOL


@pytest.mark.parametrize("shape,recipe", [("tiny", "q4_k_m"), ("small", "q4_k_m"), ("small", "q4_0")])
@pytest.mark.parametrize("fa", [1, 0])
def test_dropin_incremental_decode(ggufs, tmp_path, shape, recipe, fa):
    _need_ref()
    toks = np.random.default_rng(8).integers(0, 1000, 24)
    cpu, _ = run_ref(tmp_path, ggufs[(shape, recipe)], toks, 0, fa, incremental=True)
    gpu, log = run_ref(tmp_path, ggufs[(shape, recipe)], toks, 99, fa, incremental=True)
    assert "MI355X" in log
    assert nmse(gpu, cpu) < TOL


@pytest.mark.parametrize("incremental", [False, True])
def test_dropin_q8_0_kv_cache(ggufs, tmp_path, incremental):
    """-ctk q8_0 -ctv q8_0 (the fork's preferred setting): SET_ROWS into q8_0 caches and
    FLASH_ATTN_EXT on them, against the reference CPU backend with the same caches; the
    decode steps must take the fused QKV (q8_0 rows) and the q8_0 decode attention kernel"""
    _need_ref()
    toks = np.random.default_rng(9).integers(0, 1000, 24 if incremental else 40)
    g = ggufs[("small", "q4_k_m")]
    klog = tmp_path / "klog.txt"
    cpu, _ = run_ref(tmp_path, g, toks, 0, 1, incremental=incremental, ctk=8)
    gpu, log = run_ref(tmp_path, g, toks, 99, 1, incremental=incremental, ctk=8, klog=klog)
    assert "MI355X" in log
    assert nmse(gpu, cpu) < TOL, nmse(gpu, cpu)
    if not incremental:   # (round 6) prefill: q/k/v + RoPE fused, the q8_0 rows by their SET_ROWS nodes
        kl = klog.read_text().splitlines()
        assert any(ln.startswith("qkv_pp ") and "k_mode=1 v_mode=1" in ln for ln in kl), kl[-40:]
    if incremental:
        kl = klog.read_text()
        assert "kq8=1" in kl and any(ln.startswith("qkv ") and "kq8=1" in ln for ln in kl.splitlines()), kl[-2000:]
        assert any(ln.startswith("fattn_dec2") and "kq8=1" in ln for ln in kl.splitlines()), kl[-2000:]
        # round 6: the token's q8_0 rows are quantised and stored by the attention launch
        # (KvNewRow), not by a k_kv_store_q8 launch of their own
        assert all("newrow=1" in ln for ln in kl.splitlines() if ln.startswith("fattn_dec2")), kl[-2000:]
        assert not any(ln.startswith("kv_store_q8") for ln in kl.splitlines()), kl[-2000:]


@pytest.mark.parametrize("ctk,ctv", [(8, 1), (1, 8), (8, 2), (2, 1)])
@pytest.mark.parametrize("incremental", [False, True])
def test_dropin_mixed_kv_cache(ggufs, tmp_path, incremental, ctk, ctv):
    """Round 6: K and V caches of different types. -ctk q8_0 -ctv f16 is the fork's own
    llama-bench line (AGENTS.md:166-176; the reference enables the K-q8_0 / V-f16 kernels
    with GGML_CUDA_FA_ALL_QUANTS, fattn.cu:220-226) — SET_ROWS into each cache in its own
    type, FLASH_ATTN_EXT over the pair, against the reference CPU backend with the same
    caches. The graph must stay in two splits (no CPU fallback of the attention), decode
    must take the fused QKV (q8_0 rows for the q8_0 side only) and, for f16 / q8_0 pairs,
    the split-partials decode attention; q4_0 pairs run the tile kernel."""
    _need_ref()
    toks = np.random.default_rng(9).integers(0, 1000, 24 if incremental else 40)
    g = ggufs[("small", "q4_k_m")]
    klog = tmp_path / "klog.txt"
    cpu, _ = run_ref(tmp_path, g, toks, 0, 1, incremental=incremental, ctk=ctk, ctv=ctv)
    gpu, log = run_ref(tmp_path, g, toks, 99, 1, incremental=incremental, ctk=ctk, ctv=ctv, klog=klog)
    assert "MI355X" in log
    # a q4_0 K cache: 16 levels per block, so a last-bit difference in a K value computed by
    # the two backends (the projections' own rounding) moves a quantised K element by a whole
    # step d = amax/8 (q8_0: amax/127) — the stored keys themselves differ, before any
    # attention arithmetic (SET_ROWS q4_0 is bit-exact on equal input, test_ops_gpu.py)
    tol = 5e-3 if ctk == 2 else TOL
    assert nmse(gpu, cpu) < tol, nmse(gpu, cpu)
    kl = klog.read_text().splitlines()
    if incremental and {ctk, ctv} <= {1, 8}:
        kq, vq = int(ctk == 8), int(ctv == 8)
        assert any(ln.startswith("qkv ") and f"kq8={kq} vq8={vq}" in ln for ln in kl), kl[-40:]
        assert any(ln.startswith("fattn_dec2") and f"kq8={kq} vq8={vq} " in ln and "newrow=1" in ln for ln in kl), kl[-40:]
        assert not any(ln.startswith("kv_store_q8") for ln in kl), kl[-40:]
    elif incremental:
        assert any(ln.startswith("fattn_tile") and f"type={ctk} vtype={ctv}" in ln for ln in kl), kl[-40:]
    else:
        assert any(ln.startswith("fa_mma") for ln in kl), kl[-40:]


@pytest.mark.parametrize("incremental", [False, True])
def test_dropin_nofa_q8_0_k_cache(ggufs, tmp_path, incremental):
    """-fa 0 -ctk q8_0 (V stays f16: libllama refuses a quantised V cache without flash
    attention): the KQ MUL_MAT reads the q8_0 K cache view, V is stored transposed in f16"""
    _need_ref()
    toks = np.random.default_rng(19).integers(0, 1000, 24 if incremental else 40)
    g = ggufs[("small", "q4_k_m")]
    cpu, _ = run_ref(tmp_path, g, toks, 0, 0, incremental=incremental, ctk=8, ctv=1)
    gpu, log = run_ref(tmp_path, g, toks, 99, 0, incremental=incremental, ctk=8, ctv=1)
    assert "MI355X" in log
    assert nmse(gpu, cpu) < TOL, nmse(gpu, cpu)


def test_dropin_split_count_catches_cpu_fallback(ggufs, tmp_path):
    """The split assertion itself: with FLASH_ATTN_EXT refused by supports_op
    (GGML_MI355X_REFUSE_OP, a test knob) libllama schedules every layer's attention on the
    CPU backend — logits still match, and only the split count shows it"""
    _need_ref()
    toks = np.random.default_rng(9).integers(0, 1000, 24)
    g = ggufs[("small", "q4_k_m")]
    env = {"GGML_MI355X_REFUSE_OP": "FLASH_ATTN_EXT"}
    cpu, _ = run_ref(tmp_path, g, toks, 0, 1)
    with pytest.raises(AssertionError, match="graph splits"):
        run_ref(tmp_path, g, toks, 99, 1, env_extra=env)
    gpu, log = run_ref(tmp_path, g, toks, 99, 1, env_extra=env, splits=None)
    assert nmse(gpu, cpu) < TOL
    assert graph_splits(log) and min(graph_splits(log)) > 2, graph_splits(log)


@pytest.mark.parametrize("shape,recipe", [("small", "q4_k_m"), ("tiny_moe", "q4_k_m")])
def test_runner_matches_reference_cpu(pkg, backend, ggufs, tmp_path, shape, recipe):
    """This package's Llama runner (graph builder + executor) on the same GGUF."""
    _need_ref()
    toks = np.random.default_rng(9).integers(0, 1000, 24).astype(np.int32)
    cpu, _ = run_ref(tmp_path, ggufs[(shape, recipe)], toks, 0, 1)
    m = pkg.Model.load_gguf(backend, ggufs[(shape, recipe)])
    s = pkg.Session(m, n_ctx=256, flash_attn=True)
    pre = s.decode_all(toks)
    s.reset()
    inc = np.stack([s.decode(toks[i:i + 1]) for i in range(len(toks))])
    s.free(); m.free()
    assert nmse(pre, cpu) < TOL
    assert nmse(inc, cpu) < TOL


def test_layer_split_handoff_cpy_tensor_async(tmp_path):
    """The layer-split hand-off as libllama's scheduler performs it, through the reference's
    own ggml-backend (oracle/cpy_async_probe.cpp over libggml-ref.so): two MI355X backends,
    ggml_backend_tensor_copy_async into the second one's buffer, then a graph on it that
    reads the copy without a host synchronisation (be_cpy_async's event orders them)."""
    probe = os.path.join(ROOT, "oracle", "_ref", "cpy-async-probe")
    if not os.path.exists(probe):
        pytest.skip("oracle/_ref/cpy-async-probe not built")
    r = subprocess.run([probe, LIB], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr[-2000:]
    assert '"mismatches": 0' in r.stdout and "MI355X" in r.stdout, r.stdout


@pytest.mark.parametrize("incremental,no_peer,force_peer,ts", [(False, False, True, "1,1"), (True, False, True, "1,1"),
                                                             (True, True, True, "1,1"), (False, False, False, "1,1"),
                                                             (True, False, False, "1,1"), (True, False, True, "1,1,1,1"),
                                                             (False, False, True, "1,1,1,1"), (True, False, False, "1,1,1,1"),
                                                             (True, False, True, "3,1")])
def test_dropin_row_split(ggufs, tmp_path, incremental, no_peer, force_peer, ts):
    """llama -sm row -ts 1,1 / 1,1,1,1 / 3,1: libllama puts every matrix in the backend's
    split buffer type (proc ggml_backend_split_buffer_type), rows divided over the devices —
    here logical devices of the one MI355X (GGML_MI355X_VIRTUAL_DEVICES) — and every
    MUL_MAT runs its slices on each and gathers them (split.cpp). Logits against the
    reference CPU backend. Decode's gate/up/SwiGLU and MUL_MAT -> ADD run as per-slice fused
    GEMVs (klog glu_split / mm_split_add): on the main stream when the slices are this GPU's,
    and (round 5) forked onto each other slice device's own stream under
    GGML_MI355X_FORCE_PEER — the branch separate GPUs with peer access take (remote =
    slices - 1: the main device's slice stays on the main stream). Without peer access
    (GGML_MI355X_NO_PEER) they fall back to the staged per-matrix path."""
    _need_ref()
    n_dev = len(ts.split(","))
    toks = np.random.default_rng(10).integers(0, 1000, 24 if incremental else 40)
    g = ggufs[("small", "q4_k_m")]
    klog = tmp_path / "klog.txt"
    cpu, _ = run_ref(tmp_path, g, toks, 0, 1, incremental=incremental)
    env = {"GGML_MI355X_VIRTUAL_DEVICES": str(n_dev)}
    if force_peer:
        env["GGML_MI355X_FORCE_PEER"] = "1"
    if no_peer:
        env["GGML_MI355X_NO_PEER"] = "1"
    gpu, log = run_ref(tmp_path, g, toks, 99, 1, incremental=incremental, klog=klog, extra=["-sm", "row", "-ts", ts],
                       env_extra=env)
    assert "MI355X" in log
    assert nmse(gpu, cpu) < TOL, nmse(gpu, cpu)
    kl = klog.read_text()
    assert "mm_split" in kl and f"devices={n_dev}" in kl, kl[-2000:]
    fused = [ln for ln in kl.splitlines() if ln.startswith(("glu_split ", "mm_split_add "))]
    if force_peer:
        # GGML_MI355X_FORCE_PEER: the cross-device broadcast / gather branches of split.cpp ran
        # (no_peer: the slices come back by one contiguous peer copy and a 2D copy on main)
        assert all("peer=1" in ln and f"direct={int(not no_peer)}" in ln for ln in kl.splitlines() if ln.startswith("mm_split ")), kl[-2000:]
        if no_peer:
            assert not fused, kl[-2000:]
        elif incremental:
            assert any(ln.startswith("glu_split ") for ln in fused) and any(ln.startswith("mm_split_add ") for ln in fused), kl[-2000:]
            sr = [re.search(r"slices=(\d+) remote=(\d+)", ln).groups() for ln in fused]
            # every slice but the main device's own runs on its device's stream
            assert all(int(b) == int(a) - 1 for a, b in sr) and any(int(a) == n_dev for a, _ in sr), fused[:4]
    elif incremental:
        # one-token steps: the per-slice fused SwiGLU and residual GEMVs on this stream
        assert any(ln.startswith("glu_split ") for ln in fused) and any(ln.startswith("mm_split_add ") for ln in fused), kl[-2000:]
        assert all("remote=0" in ln for ln in fused), fused[:4]


@pytest.mark.parametrize("ts", ["1,1", "1,1,1,1"])
@pytest.mark.parametrize("incremental", [False, True])
def test_dropin_layer_split(ggufs, tmp_path, ts, incremental):
    """llama -sm layer -ts 1,1 / 1,1,1,1 (llama-bench's default split mode) over 2 or 4
    logical devices of the one MI355X (GGML_MI355X_VIRTUAL_DEVICES): libllama gives each
    device a contiguous layer range (src/llama-model.cpp:2599-2609) and, with every layer
    offloaded, turns on pipeline parallelism (src/llama-context.cpp:307-334: the
    scheduler's n_copies = 4 input copies ordered by this backend's events,
    ggml/src/ggml-backend.cpp:1445-1629). Each boundary activation crosses through
    be_cpy_async, forced onto its peer-copy branch (GGML_MI355X_FORCE_PEER=1) so the code a
    real multi-GPU run takes executes here. Logits against the reference CPU backend,
    prefill (one ubatch) and incremental decode."""
    _need_ref()
    n_dev = len(ts.split(","))
    toks = np.random.default_rng(14).integers(0, 1000, 24 if incremental else 40)
    g = ggufs[("small", "q4_k_m")]          # 4 layers: one per device at -ts 1,1,1,1
    klog = tmp_path / "klog.txt"
    cpu, _ = run_ref(tmp_path, g, toks, 0, 1, incremental=incremental)
    gpu, log = run_ref(tmp_path, g, toks, 99, 1, incremental=incremental, klog=klog, extra=["-sm", "layer", "-ts", ts],
                       env_extra={"GGML_MI355X_VIRTUAL_DEVICES": str(n_dev), "GGML_MI355X_FORCE_PEER": "1"})
    assert "MI355X" in log
    assert nmse(gpu, cpu) < TOL, nmse(gpu, cpu)
    cp = [ln for ln in klog.read_text().splitlines() if ln.startswith("cpy_async")]
    assert cp and all("peer=1" in ln for ln in cp), cp[:8]
    for i in range(n_dev - 1):     # every layer boundary handed its activation over
        assert any(f"MI355X{i} -> MI355X{i + 1} " in ln for ln in cp), (i, cp[:8])


@pytest.fixture(scope="module")
def tinyllama(tmp_path_factory):
    path = str(tmp_path_factory.mktemp("gguf_tl") / "tinyllama_q4_0.gguf")
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "gguf_synth.py"), "--shape", "tinyllama",
                    "--recipe", "q4_0", "--out", path], check=True, timeout=600)
    return path


def test_tinyllama_q4_0_dropin(tinyllama, tmp_path):
    """BASELINE configs[0]: the TinyLlama-1.1B shape (2048 / 22 layers / 32 heads / 4 KV /
    5632 / 32000) in Q4_0, the reference's CPU-runnable plumbing config (llama-bench pp64 /
    tg32). The same libllama on the reference CPU backend (-ngl 0) and on this backend
    (-ngl 99): logits of a 64-token prefill and of 32 incremental decode steps within the
    whole-graph bound, then both run llama-bench's pp64 / tg32 loop."""
    _need_ref()
    toks = np.random.default_rng(15).integers(0, 32000, 64)
    cpu, _ = run_ref(tmp_path, tinyllama, toks, 0, 1)
    gpu, log = run_ref(tmp_path, tinyllama, toks, 99, 1)
    assert "MI355X" in log
    assert nmse(gpu, cpu) < TOL, nmse(gpu, cpu)
    cpu_i, _ = run_ref(tmp_path, tinyllama, toks[:32], 0, 1, incremental=True)
    gpu_i, _ = run_ref(tmp_path, tinyllama, toks[:32], 99, 1, incremental=True)
    assert nmse(gpu_i, cpu_i) < TOL, nmse(gpu_i, cpu_i)
    res = {}
    for ngl in (0, 99):
        env = dict(os.environ, GGML_BACKEND_PATH=LIB) if ngl else dict(os.environ)
        r = subprocess.run([REF, "-m", tinyllama, "-t", str(min(16, os.cpu_count() or 8)), "-ngl", str(ngl), "-p", "64",
                            "-n", "32", "-r", "2"], capture_output=True, text=True, timeout=600, env=env)
        assert r.returncode == 0, r.stderr[-2000:]
        res[ngl] = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
        assert res[ngl]["pp_tok_s"] > 0 and res[ngl]["tg_tok_s"] > 0, res[ngl]
    print(f"tinyllama q4_0 pp64/tg32: cpu {res[0]['pp_tok_s']:.0f}/{res[0]['tg_tok_s']:.1f}  "
          f"mi355x {res[99]['pp_tok_s']:.0f}/{res[99]['tg_tok_s']:.1f} tok/s")


def test_dropin_async_upload_no_mmap(ggufs, tmp_path):
    """llama -mmp 0: the model loader uploads the weights through this backend's pinned
    host buffers, set_tensor_async and events (src/llama-model-loader.cpp:999-1180, the
    path taken when the device reports async + host_buffer + events) instead of mmap +
    set_tensor. The weights must land identically: logits bit-equal to the mmap load, and
    the upload backend's counters show the file's bytes went through set_tensor_async."""
    _need_ref()
    toks = np.random.default_rng(13).integers(0, 1000, 24)
    g = ggufs[("small", "q4_k_m")]
    a, _ = run_ref(tmp_path, g, toks, 99, 1)
    b, err = run_ref(tmp_path, g, toks, 99, 1, extra=["-mmp", "0"], env_extra={"GGML_MI355X_STATS": "1"})
    assert np.array_equal(a, b)
    st = [json.loads(ln.split("stats ", 1)[1]) for ln in err.splitlines() if "[mi355x] stats" in ln]
    assert st and max(x["bytes_set"] for x in st) > 0.5 * os.path.getsize(g), st


def _kld_stats(p_logits, q_logits):
    """llama-perplexity --kl-divergence's per-token statistics (tools/perplexity/perplexity.cpp:
    KL(P_ref || Q) of the softmaxed logits, top-1 agreement), in float64"""
    def logsm(x):
        x = x.astype(np.float64)
        x = x - x.max(-1, keepdims=True)
        return x - np.log(np.exp(x).sum(-1, keepdims=True))
    lp, lq = logsm(p_logits), logsm(q_logits)
    kld = (np.exp(lp) * (lp - lq)).sum(-1)
    same_top = float(np.mean(np.argmax(lp, -1) == np.argmax(lq, -1)))
    return kld, same_top


@pytest.mark.parametrize("shape,recipe,ctk,ctv", [("small", "q4_k_m", None, None), ("small", "q8_0", None, None),
                                                   ("small", "q4_k_m", 8, None), ("small", "q4_k_m", 8, 1)])
def test_dropin_kl_divergence(ggufs, tmp_path, shape, recipe, ctk, ctv):
    """End-to-end parity the way the fork checks a backend: KL divergence of the token
    distributions (the reference CPU backend's as P) over a 64-token prompt, prefill and
    incremental decode, and top-1 agreement. Bounds: mean KLD 5e-4, max 5e-3 (measured
    0.6-1.6e-4 mean, <= 6e-4 max), top-1 >= 90 % — the synthetic models' random weights give
    near-flat distributions whose top token flips under 1e-4 KLD (measured 94-98 %)."""
    _need_ref()
    toks = np.random.default_rng(11).integers(0, 1000, 64)
    g = ggufs[(shape, recipe)]
    for inc in (False, True):
        cpu, _ = run_ref(tmp_path, g, toks, 0, 1, incremental=inc, ctk=ctk, ctv=ctv)
        gpu, _ = run_ref(tmp_path, g, toks, 99, 1, incremental=inc, ctk=ctk, ctv=ctv)
        kld, top = _kld_stats(cpu, gpu)
        print(f"kld {shape} {recipe} ctk={ctk} ctv={ctv} inc={inc}: mean {kld.mean():.3e} p99 {np.percentile(kld, 99):.3e} "
              f"max {kld.max():.3e} top1 {top:.3f}")
        assert kld.mean() < 5e-4 and kld.max() < 5e-3 and top >= 0.90, (kld.mean(), kld.max(), top)


def parse_seq_state(blob):
    """a llama_state_seq_get_data blob (src/llama-kv-cache.cpp:1648-1867): returns the
    bit-exact part (stream / cell counts, every cell's position and sequence ids, the
    per-layer type / row-size headers) and the K / V payloads (one uint8 array per layer
    and kind)"""
    o = 0

    def take(n):
        nonlocal o
        b = blob[o:o + n]
        o += n
        return b

    u32 = lambda: int(np.frombuffer(take(4), np.uint32)[0])   # noqa: E731
    exact, payload = [], []
    n_stream = u32()
    exact.append(("n_stream", n_stream))
    for _ in range(n_stream):
        cells = u32()
        exact.append(("cells", cells))
        if cells == 0:
            continue
        for _ in range(cells):
            pos = int(np.frombuffer(take(4), np.int32)[0])
            ns = u32()
            exact.append(("cell", pos, tuple(np.frombuffer(take(4 * ns), np.int32).tolist())))
        v_trans, n_layer = u32(), u32()
        exact.append(("v_trans", v_trans, "n_layer", n_layer))
        for _ in range(n_layer):
            kt = int(np.frombuffer(take(4), np.int32)[0])
            row = int(np.frombuffer(take(8), np.uint64)[0])
            exact.append(("k", kt, row))
            payload.append((kt, take(cells * row)))
        for _ in range(n_layer):
            vt = int(np.frombuffer(take(4), np.int32)[0])
            if not v_trans:
                row = int(np.frombuffer(take(8), np.uint64)[0])
                exact.append(("v", vt, row))
                payload.append((vt, take(cells * row)))
            else:
                el, nv = u32(), u32()
                exact.append(("vt", vt, el, nv))
                payload.append((vt, take(cells * el * nv)))
    assert o == len(blob), (o, len(blob))
    return exact, payload


@pytest.mark.parametrize("fa,ctk,ctv", [(1, None, None), (0, None, None), (1, 8, None), (1, 8, 1), (0, 8, 1)])
def test_dropin_kv_state(ggufs, tmp_path, fa, ctk, ctv):
    """KV state save / restore through this backend (SURVEY §5 checkpoint/resume):
    llama_state_seq_get_data / set_data and llama_state_save_file / load_file
    (src/llama-context.cpp:3416-3431) read and write the raw KV rows through get_tensor /
    set_tensor. oracle/state_probe.cpp (built against the reference libllama) prefills a
    prompt on a GPU context, saves, and continues; then restores into fresh GPU contexts,
    a CPU context, and the CPU's own state into a GPU context. Bit-exact: the GPU state
    read back after a restore, the continued logits after either restore (seq blob and
    state file), and the cell occupancy (positions, sequence ids, row headers) against the
    reference CPU backend's state; the K/V rows themselves (computed by two backends) and
    the cross-backend continuations within the whole-graph bound. fa 0 stores V
    transposed; ctk 8 is the q8_0 cache; ctk 8 ctv 1 (round 6) K q8_0 with V f16."""
    probe = os.path.join(ROOT, "oracle", "_ref", "state-probe")
    if not os.path.exists(probe):
        pytest.skip("oracle/_ref/state-probe not built")
    rng = np.random.default_rng(40 + fa)
    rng.integers(0, 1000, 37).astype(np.int32).tofile(tmp_path / "p.i32")
    rng.integers(0, 1000, 6).astype(np.int32).tofile(tmp_path / "g.i32")
    cmd = [probe, "-m", ggufs[("small", "q4_k_m")], "-fa", str(fa), "--prompt", str(tmp_path / "p.i32"),
           "--gen", str(tmp_path / "g.i32"), "--out", str(tmp_path)] + (["-ctk", str(ctk)] if ctk else []) + \
          (["-ctv", str(ctv)] if ctv else [])
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=dict(os.environ, GGML_BACKEND_PATH=LIB))
    assert r.returncode == 0, r.stderr[-2000:]
    info = json.loads(r.stdout.strip().splitlines()[-1])
    n = info["blob_bytes"]
    assert n > 0 and info["set_b"] == n and info["set_d"] == n and info["set_e"] == n, info
    assert info["saved"] == 1 and info["loaded"] == 1 and info["file_tokens"] == 37, info
    blob = {k: np.fromfile(tmp_path / f"blob_{k}.bin", np.uint8) for k in "abc"}
    lg = {k: np.fromfile(tmp_path / f"logits_{k}.f32", np.float32).reshape(6, -1) for k in "abcdef"}
    # GPU -> GPU: the state survives set_tensor / get_tensor bit for bit, and so does the
    # continuation (seq blob and whole-context state file)
    assert np.array_equal(blob["b"], blob["a"])
    assert np.array_equal(lg["b"].view(np.uint32), lg["a"].view(np.uint32))
    assert np.array_equal(lg["f"].view(np.uint32), lg["a"].view(np.uint32))
    # KV indexing bit-exact against the reference CPU backend's own state
    ea, pa = parse_seq_state(blob["a"])
    ec, pc = parse_seq_state(blob["c"])
    assert ea == ec
    assert sum(1 for e in ea if e[0] == "cell") == 37
    for (ta, xa), (tc, xc) in zip(pa, pc):
        if ta == 1:     # f16 rows: values within the whole-graph bound
            assert nmse(xa.view(np.float16).astype(np.float64), xc.view(np.float16).astype(np.float64)) < TOL
        elif ta == 8:   # q8_0 rows: dequantise (f16 scale + 32 int8)
            def deq(x):
                b = x.reshape(-1, 34)
                return (b[:, :2].copy().view(np.float16).astype(np.float64) * b[:, 2:].view(np.int8).astype(np.float64))
            assert nmse(deq(xa), deq(xc)) < TOL
    # across backends: the GPU state continued on the CPU, the CPU state on the GPU
    assert nmse(lg["a"], lg["c"]) < TOL
    assert nmse(lg["d"], lg["a"]) < TOL
    assert nmse(lg["e"], lg["c"]) < TOL
