"""Drop-in parity at the bench widths: the reference's own libllama (oracle/_ref) runs
two-layer GGUFs with the full Llama-3-8B / Mixtral-8x7B widths (tools/gguf_synth.py
shapes `llama3_8b_2l`, `mixtral_2l`) on libggml-mi355x.so (-ngl 99) and on the reference
CPU backend (-ngl 0); logits must agree within NMSE 2e-3 (SURVEY §8c whole-graph bound).

Covered configs (BASELINE.json):
  * Llama-3-8B Q4_K_M tg (config 2): incremental decode, fa 1 and fa 0 — every decode
    kernel at its bench shape (fused QKV+RoPE+KV store, decode FA, SwiGLU GEMV with the
    LDS-DMA norm prologue, down Q4_K (layer 0) and Q6_K (layer 1), lm_head 128256);
  * Llama-3-8B pp512 (one ubatch) and pp2048 (-b 2048 -ub 512: four ubatches, the KV
    cache growing to 2048 cells; config 3) — the MFMA GEMMs and prefill attention;
  * Mixtral-8x7B Q5_K_M (config 5): MUL_MAT_ID prefill and decode with FA, the fused QKV
    on its (q Q5_K, k Q8_0, v Q8_0) recipe;
  * Llama-3-70B Q4_K_M widths (config 4, `llama3_70b_2l`: 8192 / 64 heads / 8 KV / 28672,
    attn_v Q5_K by the 70B rule on layer 0, Q6_K on layer 1): decode at fa 1 / fa 0 and
    pp512, asserting the K = 8192 / 28672 instantiations.
Besides logits, the kernel-choice log (GGML_MI355X_KLOG) shows which kernels libllama's
graph reached, and the executor's per-token launch mix under libllama must equal the
package runner's on the same GGUF (the fusions fire on the reference's node order).
"""
import collections
import os
import re
import subprocess
import sys

import numpy as np
import pytest

from dropin_util import assert_unsplit
from qgen import nmse

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = os.path.join(ROOT, "oracle", "_ref", "ref-llama-bench")
LIB = os.path.join(ROOT, "llama-mi50.cpp_amd", "lib", "libggml-mi355x.so")
TOL = 2e-3
MOE_TOL = 5e-3   # routing flips at router near-ties (test_mixtral_width_moe)


@pytest.fixture(scope="module")
def gguf_dir(tmp_path_factory):
    if not os.path.exists(REF):
        pytest.skip("oracle/_ref/ref-llama-bench not built")
    return tmp_path_factory.mktemp("gguf_shapes")


def make_gguf(d, shape, recipe):
    path = str(d / f"{shape}_{recipe}.gguf")
    if not os.path.exists(path):
        subprocess.run([sys.executable, os.path.join(ROOT, "tools", "gguf_synth.py"), "--shape", shape,
                        "--recipe", recipe, "--out", path], check=True, timeout=600)
    return path


@pytest.fixture(scope="module")
def l8b(gguf_dir):
    return make_gguf(gguf_dir, "llama3_8b_2l", "q4_k_m")


@pytest.fixture(scope="module")
def l70b(gguf_dir):
    return make_gguf(gguf_dir, "llama3_70b_2l", "q4_k_m")


@pytest.fixture(scope="module")
def l70b8(gguf_dir):
    return make_gguf(gguf_dir, "llama3_70b_8l", "q4_k_m")


@pytest.fixture(scope="module")
def mixtral(gguf_dir):
    return make_gguf(gguf_dir, "mixtral_2l", "q5_k_m")


def run_ref(tmp_path, gguf, toks, ngl, fa, incremental=False, last=0, extra=(), env_extra=None, tag="", splits="auto"):
    """splits: libllama's graph-split count the MI355X run must report (tests/dropin_util.py;
    "auto" = 2 unless a multi-device split mode is requested, None = unchecked)"""
    tf = tmp_path / f"toks{tag}.i32"
    of = tmp_path / f"logits_{ngl}_{fa}_{int(incremental)}{tag}.f32"
    kl = tmp_path / f"klog_{ngl}_{fa}_{int(incremental)}{tag}.txt"
    np.asarray(toks, np.int32).tofile(tf)
    env = dict(os.environ)
    if ngl > 0:
        env["GGML_BACKEND_PATH"] = LIB
        env["GGML_MI355X_KLOG"] = str(kl)
        env["GGML_MI355X_STATS"] = "1"
    env.update(env_extra or {})
    cmd = [REF, "-m", gguf, "-t", str(min(16, os.cpu_count() or 8)), "-ngl", str(ngl), "-fa", str(fa),
           "--logits", str(tf), str(of)] + list(extra)
    if incremental:
        cmd.append("--incremental")
    if last:
        cmd += ["--last", str(last)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=900, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    if splits == "auto":
        splits = 2 if "-sm" not in extra else None
    if ngl > 0 and splits is not None:
        assert_unsplit(r.stderr, splits)
    n_vocab = int(re.search(r'"n_vocab": (\d+)', r.stdout).group(1))
    logits = np.fromfile(of, np.float32).reshape(-1, n_vocab)
    klog = open(kl).read().splitlines() if kl.exists() else []
    return logits, r.stderr, klog


def kinds(klog):
    """launch counts keyed by kernel name (+ the GEMV's epilogue/mode and row count)"""
    c = collections.Counter()
    for ln in klog:
        f = dict(re.findall(r"(\w+)=(-?\d+)", ln))
        name = ln.split()[0]
        if name == "mmq4" and ln.split()[1] in ("glu", "group"):
            name = "mmq4 " + ln.split()[1]
        if name == "gemv2":
            name = f"gemv2 epi={f['epi']} mode={f['mode']} M={f['M']} q8o={f['q8o']}"
        c[name] += 1
    return c


def stats_of(stderr):
    m = re.findall(r"\[mi355x\] stats (\{.*\})", stderr)
    import json
    return [json.loads(s) for s in m]


@pytest.mark.parametrize("fa", [1, 0])
def test_llama3_8b_width_decode(l8b, tmp_path, fa):
    toks = np.random.default_rng(21).integers(0, 128000, 12)
    cpu, _, _ = run_ref(tmp_path, l8b, toks, 0, fa, incremental=True)
    gpu, log, klog = run_ref(tmp_path, l8b, toks, 99, fa, incremental=True,
                             env_extra={"GGML_MI355X_DISABLE_GRAPHS": "1"})
    assert "MI355X" in log, log[-2000:]
    assert np.all(np.isfinite(gpu))
    err = nmse(gpu, cpu)
    assert err < TOL, err
    k = kinds(klog)
    n, L = len(toks), 2
    # per token and layer: fused QKV+RoPE+KV store, SwiGLU (deferred norm, LDS-DMA staged,
    # q8 emission), down + residual from the q8 input, O projection + residual
    assert k["qkv"] == n * L, k
    assert k["gemv2 epi=1 mode=4 M=14336 q8o=1"] == n * L, k
    # lm_head: libllama marks result_norm an output, so the norm is not deferred; its
    # fused RMS_NORM+MUL kernel emits the q8 copy the lm_head GEMV stages
    assert k["gemv2 epi=0 mode=2 M=128256 q8o=0"] == n, k
    # O projection: + residual in the epilogue in every layer — in the last one across
    # libllama's one-row inp_out_ids GET_ROWS pair (exec.cpp try_fuse_mm_rows_add), whose
    # ADD the allocator puts over the dead attention output: that GEMV streams from a q8
    # copy of x (mode 2, like the down projections), the others read x itself (mode 0)
    assert k["gemv2 epi=0 mode=0 M=4096 q8o=0"] == 0, k
    if fa:
        # round 5 (exec.cpp fuse_attn_split_o): the attention writes split partials and the
        # O projection merges them in its prologue (mode 8 = XS_FAP4) in every layer, the
        # last one's GET_ROWS chain included; the down projections stream the q8 copy (mode 2)
        assert k["fattn_dec2_part"] == n * L, k
        assert k["gemv2 epi=2 mode=8 M=4096 q8o=0"] == n * L, k
        assert k["gemv2 epi=2 mode=2 M=4096 q8o=0"] == n * L, k
        assert k["gemv2 epi=2 mode=0 M=4096 q8o=0"] == 0, k
    else:
        # round 5: -fa 0 likewise — the chain writes split partials (attn_nofa_part) and the O
        # projection merges them (mode 8) in every layer; the down projections stream q8
        assert k["attn_nofa_part"] == n * L, k
        assert k["gemv2 epi=2 mode=8 M=4096 q8o=0"] == n * L, k
        assert k["gemv2 epi=2 mode=2 M=4096 q8o=0"] == n * L, k
    assert k["mmvq1"] == 0, k                                  # no first-generation fallback GEMV


def test_llama3_8b_width_decode_at_depth(l8b, tmp_path):
    """decode against a 4096-position cache (llama-bench -d's regime): a long-cache decode
    attention in every layer, and the decode fusions intact at depth — the
    SwiGLU absorbs the deferred ffn norm even where libllama's allocator puts the GLU output
    over the (never materialised) normed x (round 4 materialised the norm there and fell
    back to the first-generation GEMV: 30 us per layer at -d 16384)"""
    depth, n = 4096, 6
    toks = np.random.default_rng(24).integers(0, 128000, depth + n)
    extra = ("--prefix", str(depth))
    cpu, _, _ = run_ref(tmp_path, l8b, toks, 0, 1, incremental=True, extra=extra)
    gpu, log, klog = run_ref(tmp_path, l8b, toks, 99, 1, incremental=True, extra=extra,
                             env_extra={"GGML_MI355X_DISABLE_GRAPHS": "1"})
    assert cpu.shape[0] == n and gpu.shape[0] == n
    assert np.all(np.isfinite(gpu))
    err = nmse(gpu, cpu)
    assert err < TOL, err
    k = kinds(klog)
    L = 2
    assert k["fattn_dec3"] + k["fattn_dec2"] == n * L, k     # (the long-cache forms)
    # (+1: the prefix batch's last layer runs its one output row — llama's inp_out_ids)
    assert k["gemv2 epi=1 mode=4 M=14336 q8o=1"] == n * L + 1, k
    assert k["mmvq1"] == 0, k


@pytest.mark.parametrize("fa", [1, 0])
@pytest.mark.parametrize("ts", ["1,1", "1,1,1,1"])
def test_llama3_8b_width_row_split_decode(l8b, tmp_path, ts, fa):
    """-sm row at the 8B widths over 2 / 4 logical devices under GGML_MI355X_FORCE_PEER (the
    branch separate GPUs with peer access take): q/k/v + RoPE + K/V stores run as ONE fused
    launch per slice (round 5, ops_qkv.hip: slices split at head boundaries), the other
    slices on their devices' own streams; -fa 0 stores V transposed (per-element cache
    indices); each remote slice's activation staged on its device once per op (round 6).
    Logits against the reference CPU backend; graph capture on (the production path on one
    GPU)."""
    n_dev = len(ts.split(","))
    toks = np.random.default_rng(25).integers(0, 128000, 10)
    cpu, _, _ = run_ref(tmp_path, l8b, toks, 0, fa, incremental=True)
    env = {"GGML_MI355X_VIRTUAL_DEVICES": str(n_dev), "GGML_MI355X_FORCE_PEER": "1"}
    gpu, log, klog = run_ref(tmp_path, l8b, toks, 99, fa, incremental=True, extra=("-sm", "row", "-ts", ts),
                             env_extra=env, tag=f"rs{n_dev}")
    assert "MI355X" in log, log[-2000:]
    assert np.all(np.isfinite(gpu))
    err = nmse(gpu, cpu)
    assert err < TOL, err
    qs = [ln for ln in klog if ln.startswith("qkv_split ")]
    # one fused launch set per decoded token and layer (the capture repeats the eager pass's
    # choices without logging them: at least one token's worth)
    assert len(qs) >= 2, klog[-40:]
    sr = [tuple(map(int, re.search(r"slices=(\d+) remote=(\d+)", ln).groups())) for ln in qs]
    assert all(a == n_dev and b == n_dev - 1 for a, b in sr), sr[:4]
    assert not any(ln.startswith("qkv ") for ln in klog), klog[-40:]
    # round 6: every slice on another device gets its activation copied there ONCE per op
    # (split.cpp split_local_xs: x or its q8 image, and the norm weight the first time) instead
    # of each workgroup reading it over the link; the attention is merged on the main device
    # (16 KB per slice device instead of 66 KB of split partials), so the O projection runs as
    # the residual GEMV per slice
    st = [ln for ln in klog if ln.startswith("split_stage ")]
    assert st and not any("src=fap" in ln for ln in st), klog[-40:]
    moved = [int(re.search(r"bytes=(\d+)", ln).group(1)) for ln in st]
    assert max(moved) <= 2 * 4 * 4096 + 2 * 14336, moved[:12]    # (x + the norm weight once; the down q8 image)
    assert not any(ln.startswith("fap_split ") for ln in klog), klog[-40:]
    adds = [ln for ln in klog if ln.startswith("mm_split_add ")]
    assert adds and all(f"slices={n_dev} remote={n_dev - 1}" in ln for ln in adds), klog[-40:]


def test_llama3_8b_width_decode_graph_replay(l8b, tmp_path):
    """the production path: decode captured into a hipGraph and replayed per token"""
    toks = np.random.default_rng(22).integers(0, 128000, 10)
    cpu, _, _ = run_ref(tmp_path, l8b, toks, 0, 1, incremental=True)
    gpu, log, _ = run_ref(tmp_path, l8b, toks, 99, 1, incremental=True, tag="g")
    assert nmse(gpu, cpu) < TOL
    st = stats_of(log)
    assert st and st[0]["graph_replay"] >= len(toks) - 3, st


@pytest.mark.parametrize("fa", [1, 0])
def test_llama3_8b_width_pp512(l8b, tmp_path, fa):
    toks = np.random.default_rng(23).integers(0, 128000, 512)
    cpu, _, _ = run_ref(tmp_path, l8b, toks, 0, fa, last=16)
    gpu, _, klog = run_ref(tmp_path, l8b, toks, 99, fa, last=16)
    err = nmse(gpu, cpu)
    assert err < TOL, err
    k = kinds(klog)
    assert k["mmq3g"] + k["mmq4 glu"] == 2, k     # fused gate/up/SwiGLU per layer
    assert k["mmq3m"] + k["mmq4 group"] == 2, k   # q/k/v in one launch per layer
    # GEMM -> ADD -> RMS_NORM -> MUL as the GEMM + one k_add_rms_norm pass under libllama's
    # allocator (the norm reuses the dead GEMM input's memory): layer 0's two sites (the last
    # layer's attention output meets libllama's inp_out_ids GET_ROWS first)
    assert k["add_rms_norm"] >= 2, k
    # q/k/v GEMM + both ROPEs + the K/V stores fused (ops_qkv.hip qkv_prefill); -fa 0's
    # transposed V (round 6): the epilogue fills the V projection, its SET_ROWS node stores it
    qp = [ln for ln in klog if ln.startswith("qkv_pp ")]
    assert len(qp) == 2 and all(f"v_mode={0 if fa else 2}" in ln for ln in qp), qp
    if fa:
        assert k["fa_mma2"] == 2, k
    else:   # the KQ -> softmax -> KQV chain as one transposed-V flash launch per layer
        assert k["attn_nofa_mma"] == 2, k


def gemv_fields(klog):
    return [dict(re.findall(r"(\w+)=(-?\d+)", ln)) for ln in klog if ln.startswith("gemv2 qt")]


@pytest.mark.parametrize("fa", [1, 0])
def test_llama3_70b_width_decode(l70b, tmp_path, fa):
    """Llama-3-70B Q4_K_M widths, incremental decode through libllama. Every launch of the
    70B decode at its shape: the fused QKV with (Q4_K, Q4_K, Q5_K) on layer 0 (the 70B
    attn_v rule, src/llama-quant.cpp:305-310) and (Q4_K, Q4_K, Q6_K) on layer 1 at K = 8192,
    the SwiGLU GEMV over 2 x 28672 rows (K = 8192: the LDS-DMA norm prologue would need
    75,840 B, so x and the norm weight are staged in registers, one 16-value half per thread
    of the 512-thread workgroup: XS_NORM = 1), the down projection at
    K = 28672 from the SwiGLU's q8 copy (Q4_K layer 0, Q6_K layer 1), the 128256-row lm_head."""
    toks = np.random.default_rng(31).integers(0, 128000, 8)
    cpu, _, _ = run_ref(tmp_path, l70b, toks, 0, fa, incremental=True)
    gpu, log, klog = run_ref(tmp_path, l70b, toks, 99, fa, incremental=True,
                             env_extra={"GGML_MI355X_DISABLE_GRAPHS": "1"})
    assert "MI355X" in log, log[-2000:]
    assert np.all(np.isfinite(gpu))
    err = nmse(gpu, cpu)
    assert err < TOL, err
    n, L = len(toks), 2
    qkv = [ln for ln in klog if ln.startswith("qkv ")]
    assert len(qkv) == n * L and all("K=8192" in ln for ln in qkv), qkv[:4]
    assert sum("qta=12 qtk=12 qtv=13" in ln for ln in qkv) == n, qkv[:4]
    assert sum("qta=12 qtk=12 qtv=14" in ln for ln in qkv) == n, qkv[:4]
    g = gemv_fields(klog)
    glu = [f for f in g if f["epi"] == "1" and f["M"] == "28672"]
    assert len(glu) == n * L and all(f["K"] == "8192" and f["q8o"] == "1" and f["mode"] == "1" for f in glu), glu[:2]
    down = [f for f in g if f["K"] == "28672" and f["M"] == "8192"]
    assert len(down) == n * L and sorted({f["qt"] for f in down}) == ["12", "14"] and all(f["mode"] == "2" for f in down), down[:2]
    lm = [f for f in g if f["M"] == "128256"]
    assert len(lm) == n and all(f["K"] == "8192" and f["qt"] == "14" for f in lm), lm[:2]
    k = kinds(klog)
    assert k["mmvq1"] == 0, k
    if fa:
        assert k["fattn_dec2"] + k["fattn_dec"] == n * L, k
    else:
        assert k["attn_nofa"] == n * L, k


TOL_70B_PP = 5e-3   # see test_llama3_70b_width_pp512


@pytest.mark.parametrize("fa", [1, 0])
def test_llama3_70b_width_pp512(l70b, tmp_path, fa):
    """70B widths, one 512-token ubatch: the MFMA GEMMs at K = 8192 / 28672, M = 28672.
    Bound 5e-3 instead of 2e-3: against the reference CPU backend the logits differ by NMSE
    2.4e-3 at these widths (8.6e-4 at the 8B widths), while this backend's own paths agree
    with each other to 7e-5 (k_mmq4 vs k_mmq3 GEMMs) and 1.5e-7 (fused vs unfused executor)
    — profiles/r03/diag_70b_width_pp512_nmse.txt: the spread is the CPU's q8_K activation
    rounding (one scale per 256 values) accumulated over K = 8192 / 28672, which the f16
    MFMA operands here do not share. The decode path (q8 activations per 32 values, closer
    to the CPU's) holds the 2e-3 bound at the same widths."""
    toks = np.random.default_rng(32).integers(0, 128000, 512)
    cpu, _, _ = run_ref(tmp_path, l70b, toks, 0, fa, last=16)
    gpu, _, klog = run_ref(tmp_path, l70b, toks, 99, fa, last=16)
    err = nmse(gpu, cpu)
    assert err < TOL_70B_PP, err
    k = kinds(klog)
    assert k["mmq3g"] + k["mmq4 glu"] == 2, k
    assert any(ln.startswith("mmq4 glu") and "M=28672" in ln and "K=8192" in ln for ln in klog), k
    assert k["fa_mma2" if fa else "attn_nofa_mma"] == 2, k


@pytest.mark.parametrize("incremental", [False, True])
def test_llama3_70b_width_layer_split_8(l70b8, tmp_path, incremental):
    """BASELINE configs[3] in miniature: an eight-layer GGUF at the Llama-3-70B widths,
    libllama -sm layer -ts 1,1,1,1,1,1,1,1 over eight logical devices of the one MI355X
    (GGML_MI355X_VIRTUAL_DEVICES=8): one layer per device (src/llama-model.cpp:2599-2609),
    pipeline parallelism on, every one of the seven boundary activations handed over by
    be_cpy_async on its peer-copy branch (GGML_MI355X_FORCE_PEER=1, the branch eight real
    GPUs take). Logits against the same backend on one device (incremental decode and a
    40-token prefill)."""
    toks = np.random.default_rng(35).integers(0, 128000, 6 if incremental else 40)
    one, _, _ = run_ref(tmp_path, l70b8, toks, 99, 1, incremental=incremental, tag="one")
    gpu, log, klog = run_ref(tmp_path, l70b8, toks, 99, 1, incremental=incremental,
                             extra=["-sm", "layer", "-ts", ",".join(["1"] * 8)],
                             env_extra={"GGML_MI355X_VIRTUAL_DEVICES": "8", "GGML_MI355X_FORCE_PEER": "1"})
    assert "MI355X7" in log, log[-2000:]
    assert np.all(np.isfinite(gpu))
    # the split must not change the arithmetic: against the same backend on one device (the
    # per-layer kernels are the same; the boundaries only copy). The one-device path itself
    # is pinned to the reference CPU backend at these widths by the two-layer tests; over
    # eight random-weight layers the two backends' small per-node differences (the CPU's
    # q8_K activation rounding, profiles/r04/attrib_llama3_70b_2l_fa1.txt) grow by the
    # attention's amplification to NMSE ~1e-2, so the CPU is not the bound here.
    err = nmse(gpu, one)
    assert err < 1e-6, err
    cp = [ln for ln in klog if ln.startswith("cpy_async")]
    assert cp and all("peer=1" in ln for ln in cp), cp[:8]
    for i in range(7):
        assert any(f"MI355X{i} -> MI355X{i + 1} " in ln for ln in cp), (i, cp[:10])


def test_llama3_8b_width_pp2048(l8b, tmp_path):
    """pp2048 as llama-bench runs it: -b 2048 -ub 512, four ubatches, causal attention over
    a KV cache growing to 2048 cells (512 queries x up to 2048 keys in the last one)"""
    toks = np.random.default_rng(24).integers(0, 128000, 2048)
    ex = ["-b", "2048", "-ub", "512", "-c", "2304"]
    cpu, _, _ = run_ref(tmp_path, l8b, toks, 0, 1, last=8, extra=ex)
    gpu, _, klog = run_ref(tmp_path, l8b, toks, 99, 1, last=8, extra=ex)
    err = nmse(gpu, cpu)
    assert err < TOL, err
    k = kinds(klog)
    # ubatches without outputs (the first three: --last 8) skip the last layer's FFN
    # (inp_out_ids selects no rows); the 8 output rows of the last take the GEMV path
    assert k["fa_mma2"] == 4 * 2 and k["mmq3g"] + k["mmq4 glu"] == 4 + 0, k
    assert any("n_kv=2048" in ln or "n_kv=2304" in ln for ln in klog if ln.startswith("fa_mma2")), \
        [ln for ln in klog if ln.startswith("fa_mma2")]


def dump_run(tmp_path, gguf, toks, ngl, tag, incremental=False, last=8, with_logits=False):
    d = tmp_path / f"dump_{ngl}{tag}"
    d.mkdir()
    logits, _, _ = run_ref(tmp_path, gguf, toks, ngl, 1, incremental=incremental, last=last,
                           extra=["--dump", str(d / "nodes.txt"), "--dump-dir", str(d)], tag=f"d{ngl}{tag}")
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import dump_compare
    nodes = [(n, op, ne, np.fromfile(d / f"{i:03d}.f32", np.float32))
             for i, (n, op, ne) in enumerate(dump_compare.names(str(d / "nodes.txt")))]
    return (nodes, logits) if with_logits else nodes


def moe_flip_tokens(cpu, gpu, n_used=2):
    """{layer: tokens} whose MUL_MAT_ID rows ran a different expert on the two backends
    (row NMSE >= 0.5: an unrelated expert's output). Rows between 1e-2 and 0.5 are a bug, not
    a flip — except for tokens an earlier layer's flip already reached (at and after its
    first flipped token: their inputs differ). A decode dump holds one token per node."""
    rows = {}
    for (n, op, ne, a), (n2, _, _, b) in zip(cpu, gpu):
        assert n == n2
        if op != "MUL_MAT_ID":
            continue
        try:
            layer = int(n.rsplit("-", 1)[1])
        except (IndexError, ValueError):
            continue
        A = a.astype(np.float64).reshape(-1, ne[0]); B = b.astype(np.float64).reshape(-1, ne[0])
        rows.setdefault(layer, []).append((n, np.sum((A - B) ** 2, 1) / np.maximum(np.sum(A ** 2, 1), 1e-30)))
    flips, t0 = {}, 10 ** 9
    for layer in sorted(rows):
        for n, r in rows[layer]:
            tok = np.arange(len(r)) // n_used
            live = tok < t0
            assert not ((r > 1e-2) & (r < 0.5) & live).any(), (n, t0, np.sort(r[live])[-10:])
            flips.setdefault(layer, set()).update(int(t) for t in tok[(r >= 0.5) & live])
        t0 = min(flips.get(layer, set()) | {t0})
    return flips


def per_position_moe(cpu_logits, gpu_logits, flips, positions):
    """Round 5: every logits position that no routing flip can reach must be
    within MOE_TOL — a layer-0 flip at token t reaches every position >= t (layer 1's causal
    attention reads token t), a layer-1 flip only its own position. Returns (clean, reached)
    NMSE lists."""
    t0 = min(flips.get(0, set()) | {10 ** 9})
    clean, reached = [], []
    for i, p in enumerate(positions):
        e = nmse(gpu_logits[i], cpu_logits[i])
        (reached if p >= t0 or p in flips.get(1, set()) else clean).append(e)
    assert clean, (flips, positions)
    assert max(clean) < MOE_TOL, (clean, flips)
    # (reached positions carry another expert's output somewhere upstream — a flip in the
    # last layer changes its own position's logits wholesale: reported, not bounded)
    return clean, reached


def check_moe_layer0(cpu, gpu):
    """per (token, slot) row of every layer-0 MUL_MAT_ID node: either the same expert ran
    (NMSE < 1e-2: q8_1 vs the CPU's q8_K activation rounding over inputs that already carry
    the upstream noise — the dense 8B graph's ffn_out shows the same 1e-3) or routing
    flipped at a near-tie of the router probabilities (NMSE ~ 2: an unrelated expert's
    output); nothing in between, and flips must be rare"""
    flips = rows = 0
    for (n, op, ne, a), (n2, _, _, b) in zip(cpu, gpu):
        assert n == n2
        if op != "MUL_MAT_ID" or not n.endswith("-0"):
            continue
        A = a.astype(np.float64).reshape(-1, ne[0]); B = b.astype(np.float64).reshape(-1, ne[0])
        r = np.sum((A - B) ** 2, 1) / np.maximum(np.sum(A ** 2, 1), 1e-30)
        bad = (r > 1e-2) & (r < 0.5)
        assert not bad.any(), (n, np.sort(r)[-10:])
        flips += int(np.sum(r >= 0.5)); rows += len(r)
    assert rows > 0
    assert flips <= 0.1 * rows, (flips, rows)
    return flips, rows


def test_mixtral_width_moe(mixtral, tmp_path):
    """Mixtral-8x7B widths (8 experts top-2, Q5_K experts, Q8_0 attn_k/v) with FA, prefill of
    64 tokens (grouped MUL_MAT_ID) and incremental decode. Router logits carry the activation
    quantisation noise of the q8/f16 GEMMs (NMSE ~1e-4 against the CPU's q8_K arithmetic),
    so top-2 selection flips wherever two experts' probabilities nearly tie; those tokens
    then legitimately run different experts, and a flipped token in layer 0 perturbs every
    later token through layer 1's attention. Checked: expert rows match per (token, slot) in
    every layer unless a flip happened, layer-0 flips are rare (~5 % of rows measured), and
    (round 5) EVERY logits position no flip can reach is within MOE_TOL — prefill (all 64
    positions) and incremental decode (12 steps)."""
    toks = np.random.default_rng(25).integers(0, 32000, 64)
    n = len(toks)
    dc, lc = dump_run(tmp_path, mixtral, toks, 0, "p", last=n, with_logits=True)
    dg, lg = dump_run(tmp_path, mixtral, toks, 99, "p", last=n, with_logits=True)
    f, r = check_moe_layer0(dc, dg)
    print(f"prefill: {f} of {r} layer-0 expert rows flipped")
    flips = moe_flip_tokens(dc, dg)
    clean, reached = per_position_moe(lc, lg, flips, list(range(n)))
    print(f"prefill: {len(clean)} positions no flip reaches (max NMSE {max(clean):.2e}), {len(reached)} reached "
          f"(max {max(reached or [0]):.2e}); flips {flips}")
    # the ordinary (fused, non-callback) run: the kernels the dumps' node-by-node run cannot fuse
    cpu, _, _ = run_ref(tmp_path, mixtral, toks, 0, 1, last=8)
    gpu, log, klog = run_ref(tmp_path, mixtral, toks, 99, 1, last=8)
    assert np.all(np.isfinite(gpu))
    #  the fused run's own logits: its kernels (grouped Q8_0 q/k/v, EPI 3 expert
    # GEMM, skinny router) are not the dump run's node-by-node ones, so its flips may differ;
    # per position within MOE_TOL at the median (flipped positions are the outliers)
    per = [nmse(gpu[i], cpu[i]) for i in range(len(gpu))]
    assert np.median(per) < MOE_TOL, per
    assert any(ln.startswith(("moe_", "mmid", "mmq4 moe", "gemv2 moe")) for ln in klog), klog[:40]
    # round 5: the 8-expert recipe's Q8_0 k / v run grouped with q in k_mmq4 (Q8_0 B operand),
    # the router's few f32 rows in k_mm_skinny (both were the generic k_mmq: 32 % + 9 % of
    # the Mixtral pp512 GPU time, profiles/r05/)
    assert any(ln.startswith("mmq4 group n=3 qta=13 qtb=8 ") for ln in klog), [l for l in klog if "mmq" in l][:10]
    assert any(ln.startswith("mm_skinny ") for ln in klog), klog[:40]
    assert not any(ln.startswith("mmq1 ") for ln in klog), [l for l in klog if l.startswith("mmq1 ")][:5]
    t2 = toks[:12]
    dci, lci = dump_run(tmp_path, mixtral, t2, 0, "i", True, last=len(t2), with_logits=True)
    dgi, lgi = dump_run(tmp_path, mixtral, t2, 99, "i", True, last=len(t2), with_logits=True)
    assert len(lci) == len(t2) and len(dci) % len(t2) == 0 and len(dci) == len(dgi), (len(lci), len(dci), len(dgi))
    f, r = check_moe_layer0(dci, dgi)
    print(f"decode: {f} of {r} layer-0 expert rows flipped")
    # incremental: one dump per decoded token, in order — node k of token t is dump entry t * per + k
    per = len(dci) // len(t2)
    fl = {}
    for t in range(len(t2)):
        ft = moe_flip_tokens(dci[t * per:(t + 1) * per], dgi[t * per:(t + 1) * per])
        for layer, s_ in ft.items():
            if s_:
                fl.setdefault(layer, set()).add(t)
    clean, reached = per_position_moe(lci, lgi, fl, list(range(len(t2))))
    print(f"decode: {len(clean)} clean positions (max NMSE {max(clean):.2e}), {len(reached)} reached; flips {fl}")
    cpu_i, _, _ = run_ref(tmp_path, mixtral, t2, 0, 1, incremental=True, tag="i")
    gpu_i, _, klog_i = run_ref(tmp_path, mixtral, t2, 99, 1, incremental=True, tag="i",
                               env_extra={"GGML_MI355X_DISABLE_GRAPHS": "1"})
    assert np.all(np.isfinite(gpu_i))
    per_i = [nmse(gpu_i[i], cpu_i[i]) for i in range(len(t2))]
    assert np.median(per_i) < MOE_TOL, per_i
    # graphs on (the production decode): the router's last-arriver counter is reset inside
    # the launch, so every replay must route as the eager run does — logits equal to the
    # eager (graphs-off) run's (a stale counter would pick other experts: NMSE ~1), and
    # replays actually happened
    gpu_g, log_g, _ = run_ref(tmp_path, mixtral, t2, 99, 1, incremental=True, tag="ig")
    st = stats_of(log_g)
    assert st and max(x["graph_replay"] for x in st) >= len(t2) - 3, st
    dg = [nmse(gpu_g[i], gpu_i[i]) for i in range(len(t2))]
    assert max(dg) < 1e-6, dg
    qkv = [ln for ln in klog_i if ln.startswith("qkv ")]
    assert len(qkv) == 2 * len(t2) and all("qta=13 qtk=8 qtv=8" in ln for ln in qkv), (qkv[:4], klog_i[:20])
    # round 5: norm + router + top-k of every decoded token's MoE block in one launch
    # (round 6: Mixtral's 8 experts take the one-workgroup form, k_moe_router1)
    assert sum(ln.startswith("moe_router1 ") for ln in klog_i) == 2 * len(t2), [l for l in klog_i if "moe" in l][:8]
    # round 6: the down projection's MUL_MAT_ID + the expert combine (+ residual) in one launch
    # per layer; its per-row dots run the unfused GEMV's lane order, so the logits equal the
    # two-launch form's (GGML_MI355X_NO_MOE_DOWN_COMBINE=1)
    assert sum(ln.startswith("moe_down_comb ") and "res=1" in ln for ln in klog_i) == 2 * len(t2), \
        [l for l in klog_i if "moe" in l][:8]
    assert not any(ln.startswith("moe_combine ") for ln in klog_i), [l for l in klog_i if "moe" in l][:8]
    gpu_u, _, klog_u = run_ref(tmp_path, mixtral, t2, 99, 1, incremental=True, tag="iu",
                               env_extra={"GGML_MI355X_DISABLE_GRAPHS": "1", "GGML_MI355X_NO_MOE_DOWN_COMBINE": "1"})
    assert sum(ln.startswith("moe_combine ") for ln in klog_u) == 2 * len(t2), [l for l in klog_u if "moe" in l][:8]
    du = [nmse(gpu_u[i], gpu_i[i]) for i in range(len(t2))]
    assert max(du) < 1e-9, du


def test_runner_launch_mix_equals_dropin(pkg, backend, l8b, tmp_path):
    """the package's runner and the reference's libllama, same GGUF, one decoded token
    each (eager): the same kernels launch the same number of times"""
    toks = np.random.default_rng(26).integers(0, 128000, 3).astype(np.int32)
    _, _, klog = run_ref(tmp_path, l8b, toks, 99, 1, incremental=True,
                         env_extra={"GGML_MI355X_DISABLE_GRAPHS": "1"}, tag="mix")
    m = pkg.Model.load_gguf(backend, l8b)
    s = pkg.Session(m, n_ctx=256, flash_attn=True)
    runner = []
    for i in range(len(toks)):
        backend.klog(True)
        s.decode(toks[i:i + 1])
        backend.synchronize()
        if i == 0:      # first sighting of the decode graph runs eagerly (no capture)
            runner = backend.klog_read()
        backend.klog(False)
    s.free(); m.free()
    ours = kinds(runner)
    theirs = kinds(klog)
    per_tok = collections.Counter({kk: v // len(toks) for kk, v in theirs.items()})
    hot = [kk for kk in set(ours) | set(per_tok) if kk.startswith(("gemv2", "qkv", "fattn"))]
    assert hot, ours
    # libllama's graph has the inp_out_ids GET_ROWS pair after the last layer's attention;
    # for one token exec.cpp folds MUL_MAT -> GET_ROWS x2 -> ADD into the residual GEMV
    # (round 4), so the hot launches are the same kernels, the same number of times. The
    # lm_head reads the RMS_NORM+MUL+q8 launch's q8 copy in both (exec.cpp never defers a
    # norm into a 128256-row grid)
    ours_adj = collections.Counter(ours)
    moved = per_tok["gemv2 epi=2 mode=2 M=4096 q8o=0"] - ours["gemv2 epi=2 mode=2 M=4096 q8o=0"]
    assert moved in (0, 1), (per_tok, ours)   # the last layer's O projection from the q8 copy
    ours_adj["gemv2 epi=2 mode=0 M=4096 q8o=0"] -= moved
    ours_adj["gemv2 epi=2 mode=2 M=4096 q8o=0"] += moved
    for kk in hot:
        assert per_tok[kk] == ours_adj[kk], (kk, per_tok, ours)
