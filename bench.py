#!/usr/bin/env python3
"""bench.py — llama-bench tg128 (+ pp512) tokens/s for Llama-3-8B Q4_K_M on MI355X.

Workload (BASELINE.json configs[1]): Llama-3-8B shapes (n_embd 4096, 32 layers, 32/8
heads, n_ff 14336, vocab 128256) with Q4_K_M weights (Q4_K + Q6_K attn_v/ffn_down on
the 16 use_more_bits layers + Q6_K output), synthetic random weights (no checkpoints
offline).

Headline (`value`, round 4; round 5: measured by the reference's own llama-bench, built
unmodified from tools/llama-bench/llama-bench.cpp + common/ into oracle/_ref/llama-bench) —
the drop-in path the north star names: the reference's libllama loading
libggml-mi355x.so through GGML_BACKEND_PATH, -ngl 99,
-fa 1, on a synthetic GGUF of that shape (tools/gguf_synth.py). A *step* is one tg128
repetition (llama-bench -r K after its own untimed warmup run: W - 1 further untimed
repetitions run first); value = K * 128 tokens / the sum of the K repetitions' times as
llama-bench measures them (llama_decode + synchronize per token). This package's own
runner (the same backend driven by mx_llama, device-side random weights) is reported
beside it under `runner` (tg128, pp512, pp2048), as are the drop-in's -fa 0 / q8_0-KV /
pp2048 / depth legs.

Multi-GPU (torchrun, one process per GPU): libllama's own layer split, as llama-bench
-sm layer -ts 1,..,1 measures it — rank 0 drives GPUs 0..N-1 through this backend
(contiguous layer ranges, boundary activations by cpy_tensor_async peer copies over xGMI,
pipeline parallelism on: src/llama-context.cpp:307-334); the other ranks only wait in a
gloo barrier (no RCCL kernel resident on their GPUs during the measurement). ONE sequence
passes all N devices in turn, so the total work is fixed ("strong") and the curve is
expected flat to declining. --mode pipeline runs this package's own RCCL
send/recv pipeline instead (reported as before), --mode replicas a whole model per GPU.
--model picks the BASELINE.json config (llama3_8b, llama3_70b, mixtral_8x7b, tinyllama)
for the runner modes.
"""
import argparse
import ctypes
import json
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "llama-bench tg128 + pp512 tok/s, Llama-3-8B Q4_K_M, 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s peak
MFMA_F16_PEAK_TFS = 2500.0  # MI355X_MICROARCH.md: dense f16/bf16 MFMA (no sparsity)
# prefill matmul FLOPs per token (2 x weight-matrix parameters of all layers; the causal
# attention adds ~1 % at pp512 and is left out): Llama-3-8B 2 * 218,103,808 * 32
PP_FLOPS_PER_TOKEN = {"llama3_8b": 2 * 218103808 * 32}


def dist_setup(n_gpus, backend=None):
    """backend: None = nccl (RCCL) when a GPU is visible, else gloo; "gloo" for the drop-in
    layer-split headline (only rank 0's child process touches the GPUs)"""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as tdist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        backend = os.environ.get("MX_DIST_BACKEND") or backend or ("nccl" if torch.cuda.device_count() > 0 else "gloo")
        if backend == "nccl":
            torch.cuda.set_device(local)
        tdist.init_process_group(backend=backend)
        dist = tdist
    return world, rank, local, dist


def barrier(dist, local):
    if dist is None:
        return
    import torch
    if dist.get_backend() == "nccl":
        torch.cuda.synchronize(local)
    dist.barrier()


def max_over_ranks(dist, v):
    if dist is None:
        return v
    import torch
    dev = "cuda" if dist.get_backend() == "nccl" else "cpu"
    t = torch.tensor([v], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(dist, v):
    if dist is None:
        return v
    import torch
    dev = "cuda" if dist.get_backend() == "nccl" else "cpu"
    t = torch.tensor([v], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())


def tg_step(sess, rng, n_vocab, n_gen):
    sess.reset()
    toks = rng.integers(0, n_vocab, size=n_gen, dtype=np.int32)
    for t in toks:
        sess.decode(np.array([t], dtype=np.int32), want_logits=True)


def roofline_glu(pkg, be, model, iters=256):
    """Dominant decode kernel: the fused gate/up SwiGLU GEMV (2.1 GB of the 4.6 GB read
    per token), launched exactly as in decode (ffn_norm absorbed in the prologue, q8 of
    the output emitted for the down projection). Timed with HIP events on the backend's
    stream over back-to-back launches that cycle through all 32 layers' real
    ffn_gate/ffn_up weights (4.2 GB, so every launch streams from HBM, not the 256 MiB
    MALL). Algorithmic bytes per launch = both Q4_K weight matrices + the f32 activation
    and norm weight read + the f32 and q8 outputs written."""
    lib = pkg._lib.load()
    l0, l1 = model.stage
    n_layer = l1 - l0
    P = ctypes.c_void_p
    wg = (P * n_layer)(*[model.layer_tensor(i, "ffn_gate") for i in range(l0, l1)])
    wu = (P * n_layer)(*[model.layer_tensor(i, "ffn_up") for i in range(l0, l1)])
    t0 = pkg.Tensor(None, wg[0])
    K, M = t0.ne[0], t0.ne[1]
    ctx = pkg.Context()
    x = ctx.new_tensor("f32", K, 1)
    out = ctx.new_tensor("f32", M, 1)
    ctx.alloc(be)
    x.set(np.random.default_rng(7).standard_normal(K).astype(np.float32))
    us = lib.ggml_backend_mi355x_time_mmvq(be.ptr, wg, wu, n_layer, x.ptr, out.ptr, iters)
    bytes_per_launch = 2 * t0.nbytes() + 2 * K * 4 + M * 4 + M + (M // 32) * 8
    ctx.free()
    achieved = bytes_per_launch / (us * 1e-6) / 1e9
    traffic, traffic_src = None, None
    # scripts/pmc_roofline.sh (separate FETCH_SIZE / WRITE_SIZE passes of --roofline-only):
    # the newest round's counter file for this exact launch
    for rnd in ("r06", "r05", "r04", "r03", "r02", "r01"):
        pmc = os.path.join(ROOT, "profiles", rnd, "pmc_glu.json")
        if not os.path.exists(pmc):
            continue
        try:
            rec = json.load(open(pmc))
            if rec.get("bytes_per_launch") == int(bytes_per_launch):
                traffic, traffic_src = rec["hbm_bytes_per_launch"], os.path.relpath(pmc, ROOT)
                break
        except Exception:  # noqa: BLE001
            pass
    return {"bound": "hbm", "kernel": f"k_gemv2 SwiGLU (ffn gate+up, {K}->{M} x2, cycled over {n_layer} layers)",
            "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic, "traffic_source": traffic_src,
            "bytes_per_launch": int(bytes_per_launch), "avg_launch_us": round(us, 2)}


REF_BENCH = os.path.join(ROOT, "oracle", "_ref", "ref-llama-bench")
LIB = os.path.join(ROOT, "llama-mi50.cpp_amd", "lib", "libggml-mi355x.so")


def bench_gguf(model="llama3_8b", recipe="q4_k_m"):
    """the synthetic GGUF of the bench shape (tools/gguf_synth.py), written once per box"""
    gguf = os.path.join(os.environ.get("TMPDIR", "/tmp"), f"mx_bench_{model}_{recipe}.gguf")
    if not os.path.exists(gguf):
        subprocess.run([sys.executable, os.path.join(ROOT, "tools", "gguf_synth.py"), "--shape", model,
                        "--recipe", recipe, "--out", gguf + ".part"], check=True, timeout=900,
                       stdout=subprocess.DEVNULL)
        os.replace(gguf + ".part", gguf)
    return gguf


def host_threads():
    """CPU threads this process may use: the affinity mask, capped by the cgroup CPU quota
    (a GPU box shows the whole machine's CPUs but grants a share of them)"""
    n = len(os.sched_getaffinity(0))
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            n = min(n, max(1, int(int(q) / int(per))))
    except (OSError, ValueError):
        pass
    return int(os.environ.get("MX_CPU_THREADS", n))


def cpu_model():
    """lscpu's model name (record the host CPU beside the baseline)"""
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def cpu_baseline(args):
    """Reference CPU backend (oracle/_ref, built from /root/reference sources) on the same
    GGUF, bounded sample, every CPU thread this process is granted (-t nproc).
    Returns None when the reference build is absent."""
    if not (os.path.exists(REF_BENCH) or os.path.exists(LLAMA_BENCH)) or args.no_cpu_baseline:
        return None
    threads = host_threads()
    try:
        gguf = bench_gguf()
        res, err = ref_bench(gguf, dict(os.environ), ["-t", threads, "-ngl", 0, "-fa", 1, "-p", args.cpu_pp,
                                                      "-n", args.cpu_tg, "-r", args.cpu_reps])
        if isinstance(res, str):
            raise RuntimeError(res)
        return {"value": res["tg_tok_s"], "unit": "tok/s", "cores": threads, "kind": "reference", "tool": bench_tool(),
                "pp_tok_s": res.get("pp_tok_s"), "tg_samples": res.get("tg_samples"), "pp_samples": res.get("pp_samples"),
                "cpu_model": cpu_model(), "host_cpus": os.cpu_count(),
                "sample": f"reference CPU backend (libllama+ggml-cpu from /root/reference), same GGUF, the bench's own "
                          f"llama-bench flags at -ngl 0 -fa 1: tg{args.cpu_tg} and pp{args.cpu_pp}, one warmup then "
                          f"{args.cpu_reps} repetitions each "
                          f"(llama-bench's loop), {threads} threads (the cgroup CPU quota of os.cpu_count() = "
                          f"{os.cpu_count()})"}
    except Exception as e:  # noqa: BLE001 — the GPU number stays valid without the baseline
        return {"value": None, "unit": "tok/s", "cores": threads, "kind": "reference", "sample": f"failed: {e}"}


# Round 5: the reference's own llama-bench, unmodified (oracle/Makefile builds
# tools/llama-bench/llama-bench.cpp with the common/ sources it links from /root/reference);
# ref-llama-bench (the round-4 restatement of its loop) stays as the fallback when absent.
LLAMA_BENCH = os.path.join(ROOT, "oracle", "_ref", "llama-bench")


def bench_tool():
    return "llama-bench" if os.path.exists(LLAMA_BENCH) else "ref-llama-bench"


def ref_bench(gguf, env, flags, timeout=900):
    """one llama-bench run -> {tg_tok_s, tg_samples, pp_tok_s, pp_samples} (or an error
    string). With the real tool: `-o jsonl`, one line per test; its own defaults for
    everything not passed (-b 2048 -ub 512, its warmup run); -c is the restatement's flag
    only (llama-bench sizes the context from -p + -n + -d itself)."""
    flags = [str(f) for f in flags]
    if bench_tool() == "llama-bench":
        fl = []
        i = 0
        tname = {"8": "q8_0", "2": "q4_0", "1": "f16", "30": "bf16"}
        has_ctv = "-ctv" in flags
        while i < len(flags):
            if flags[i] == "-c":
                i += 2
                continue
            if flags[i] in ("-ctk", "-ctv"):   # the restatement takes ggml_type ids (-ctk: K and V), llama-bench names
                name = tname.get(flags[i + 1], flags[i + 1])
                fl += [flags[i], name] + (["-ctv", name] if flags[i] == "-ctk" and not has_ctv else [])
                i += 2
                continue
            fl.append(flags[i])
            i += 1
        # -v: llama-bench keeps libllama's log (only that: llama-bench.cpp:2067), whose
        # "graph splits = N" per context shows any node that fell back to the CPU backend
        r = subprocess.run([LLAMA_BENCH, "-m", gguf, "-o", "jsonl", "-v"] + fl, capture_output=True, text=True,
                           timeout=timeout, env=env)
        lines = [json.loads(ln) for ln in r.stdout.splitlines() if ln.startswith("{")]
        if r.returncode != 0 or not lines:
            return f"failed rc={r.returncode}: {r.stderr[-300:]}", r.stderr
        res = {"tool": "llama-bench", "pp_tok_s": 0.0, "tg_tok_s": 0.0, "pp_samples": [], "tg_samples": [],
               "graph_splits": graph_splits(r.stderr)}
        for t in lines:
            kind = "tg" if t["n_gen"] > 0 and t["n_prompt"] == 0 else "pp"
            res[f"{kind}_tok_s"] = t["avg_ts"]
            res[f"{kind}_samples"] = t["samples_ts"]
            res[f"{kind}_test"] = {k: t[k] for k in ("n_prompt", "n_gen", "n_depth", "n_batch", "n_ubatch", "n_threads",
                                                     "flash_attn", "type_k", "type_v", "split_mode", "avg_ts", "stddev_ts")}
        return res, r.stderr
    r = subprocess.run([REF_BENCH, "-m", gguf] + flags, capture_output=True, text=True,
                       timeout=timeout, env=env)
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    if r.returncode != 0 or not line:
        return f"failed rc={r.returncode}: {r.stderr[-300:]}", r.stderr
    return dict(json.loads(line[-1]), graph_splits=graph_splits(r.stderr)), r.stderr


def graph_splits(stderr):
    """libllama's "graph splits = N" counts (src/llama-context.cpp:523-533), one per context
    reserve: 2 = CPU input embedding + MI355X, i.e. no node fell back to the CPU backend"""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import dropin_util
    return sorted(set(dropin_util.graph_splits(stderr)))


def tg_from_samples(samples, n_tok):
    """whole-job rate of llama-bench repetitions: K * n_tok tokens over the summed times
    (the samples are per-repetition tok/s), and the mean ms per repetition"""
    secs = [n_tok / x for x in samples]
    return len(samples) * n_tok / sum(secs), 1000.0 * sum(secs) / len(secs)


def dropin_tg(args, env, flags, key):
    """the timed drop-in tg: W - 1 untimed repetitions (llama-bench runs one warmup of its
    own), then exactly K = --steps timed ones; returns a result dict or an error string"""
    gguf = bench_gguf()
    base = ["-t", "8", "-ngl", "99", "-p", 0, "-n", args.tg]
    if args.warmup > 1:
        ref_bench(gguf, env, base + flags + ["-r", args.warmup - 1])
    t0 = time.perf_counter()
    res, err = ref_bench(gguf, env, base + flags + ["-r", args.steps])
    wall = time.perf_counter() - t0
    if isinstance(res, str):
        return res
    value, ms = tg_from_samples(res["tg_samples"], args.tg)
    st = [json.loads(x.split("stats ", 1)[1]) for x in err.splitlines() if "[mi355x] stats" in x]
    st.sort(key=lambda e: -e.get("graph_compute", 0))   # the decode context's backend (llama-bench frees several)
    return {"key": key, "tok_s": value, "ms_per_step": ms, "samples": res["tg_samples"], "avg_ts": res["tg_tok_s"],
            "tool": bench_tool(), "test": res.get("tg_test"), "wall_s_incl_load": round(wall, 2), "executor": st[0] if st else None,
            "graph_splits": res.get("graph_splits")}


def dropin_bench(args, skip=()):
    """The drop-in path as a user of the reference runs it: the reference's own libllama
    (oracle/_ref/ref-llama-bench, llama-bench's test_prompt / test_gen loop,
    tools/llama-bench/llama-bench.cpp:1962-2010, warmup + -r repetitions) loads
    libggml-mi355x.so through GGML_BACKEND_PATH with every layer offloaded (-ngl 99), on
    the same Llama-3-8B Q4_K_M GGUF. The extra legs beside the headline: tg128 at -fa 0
    and with a q8_0 KV cache (-ctk q8_0 -ctv q8_0: keys *_q8kv; -ctk q8_0 -ctv f16, the fork's
    line: *_q8k_f16v), pp512 at each, pp2048
    (-b 2048 -ub 512, BASELINE configs[2]), tg128 at depth (-d: llama-bench.cpp:2191-2226,
    the KV cache filled with D tokens first)."""
    if not (os.path.exists(REF_BENCH) or os.path.exists(LLAMA_BENCH)) or args.no_dropin:
        return None
    out = {"how": f"the reference's {bench_tool()} (oracle/_ref) + GGML_BACKEND_PATH=libggml-mi355x.so, -ngl 99, "
                  f"-r {args.dropin_reps}, llama-bench warmup"}
    try:
        gguf = bench_gguf()
        env = dict(os.environ, GGML_BACKEND_PATH=LIB, GGML_MI355X_STATS="1")
        base = ["-t", "8", "-ngl", "99", "-r", args.dropin_reps]
        runs = []
        # K / V cache types (ggml ids, 8 = q8_0, 1 = f16): f16, q8_0 / q8_0, and (round 6) the
        # fork's own line -ctk q8_0 -ctv f16 (AGENTS.md:166-176)
        for fa, ctk, ctv, tag in ((1, None, None, ""), (0, None, None, ""), (1, 8, 8, "_q8kv"), (1, 8, 1, "_q8k_f16v")):
            for test, pp, tg in (("tg128", 0, args.tg), ("pp512", args.pp, 0)):
                if (pp or tg) == 0:
                    continue
                key = f"{test}_fa{fa}{tag}"
                if key in skip:
                    continue
                runs.append((key, tg > 0, ["-fa", fa, "-p", pp, "-n", tg, "-c", max(256, pp + tg)] +
                             (["-ctk", ctk, "-ctv", ctv] if ctk else [])))
        if args.pp2048:
            for fa in (1, 0):
                runs.append((f"pp2048_fa{fa}", False, ["-fa", fa, "-p", 2048, "-n", 0, "-b", 2048, "-ub", 512, "-c", 2304]))
        for d in args.depths:
            runs.append((f"tg128_d{d}_fa1", True, ["-fa", 1, "-p", 0, "-n", args.tg, "-d", d, "-c", d + args.tg + 256]))
        for key, is_tg, flags in runs:
            res, err = ref_bench(gguf, env, base + flags)
            if isinstance(res, str):
                out[key] = res
                continue
            out[f"{key}_tok_s"] = res["tg_tok_s"] if is_tg else res["pp_tok_s"]
            out[f"{key}_samples"] = res["tg_samples"] if is_tg else res["pp_samples"]
            out[f"{key}_graph_splits"] = res.get("graph_splits")
    except Exception as e:  # noqa: BLE001
        out["error"] = str(e)
    return out


def dropin_layer_split(args, world, tg_leg=True):
    """N > 1: libllama's own layer split as llama-bench -sm layer measures it — ONE process
    (rank 0's child) drives the first N GPUs through this backend, contiguous layer ranges
    per device, boundary activations by cpy_tensor_async (hipMemcpyPeerAsync over xGMI),
    pipeline parallelism on (src/llama-context.cpp:307-334). The timed tg128 (-r K after
    W untimed repetitions) is the N > 1 headline; pp512 at -fa 1 beside it."""
    if not (os.path.exists(REF_BENCH) or os.path.exists(LLAMA_BENCH)) or args.no_dropin:
        return None
    vis = os.environ.get("HIP_VISIBLE_DEVICES")
    devs = vis.split(",")[:world] if vis else [str(i) for i in range(world)]
    env = dict(os.environ, GGML_BACKEND_PATH=LIB, HIP_VISIBLE_DEVICES=",".join(devs), GGML_MI355X_STATS="1")
    if os.environ.get("MX_BENCH_VIRTUAL") == "1":
        # rehearsal on a one-GPU box: N logical devices of GPU 0 (GGML_MI355X_VIRTUAL_DEVICES),
        # every layer boundary on the peer-copy branch — the control flow of the real N-GPU run
        devs = [devs[0]]
        env.update(HIP_VISIBLE_DEVICES=devs[0], GGML_MI355X_VIRTUAL_DEVICES=str(world), GGML_MI355X_FORCE_PEER="1")
    virtual = os.environ.get("MX_BENCH_VIRTUAL") == "1"
    ts = ",".join(["1"] * world)
    split = ["-fa", "1", "-sm", "layer", "-ts", ts]
    out = {"how": f"reference libllama -sm layer -ts {ts} over HIP devices {','.join(devs)}, -ngl 99, -fa 1",
           "devices": devs}
    if virtual:   # a rehearsal must not pass for a multi-GPU number
        out["virtual_devices"] = True
    try:
        if tg_leg:
            out["tg"] = dropin_tg(args, env, split + ["-c", 256], "tg128_split")
        gguf = bench_gguf()
        res, _ = ref_bench(gguf, env, ["-t", "8", "-ngl", "99", "-p", args.pp, "-n", 0, "-c", max(512, args.pp),
                                       "-r", args.dropin_reps] + split)
        if isinstance(res, str):
            out["pp512"] = res
        else:
            out["pp512_tok_s"], out["pp512_samples"] = res["pp_tok_s"], res["pp_samples"]
    except Exception as e:  # noqa: BLE001
        out["error"] = str(e)
    return out


def plan_decode_bytes(shape, recipe):
    """HBM bytes one decoded token streams for a synthetic GGUF (tools/gguf_synth.py's own
    tensor plan): every weight once, the experts' tensors (*_exps) by n_expert_used /
    n_expert, token_embd one row (a GET_ROWS)"""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import gguf_synth as gs
    s = gs.SHAPES[shape]
    used = s.get("n_expert_used", 1) / s.get("n_expert", 1) if s.get("n_expert") else 1.0
    tot = 0
    for name, tname, ne in gs.tensor_plan(s, recipe):
        b = gs.nbytes(tname, ne)
        if name.startswith("token_embd"):
            b = gs.nbytes(tname, [ne[0], 1])
        elif "_exps" in name:
            b = b * used
        tot += b
    return int(tot)


def moe_leg(args):
    """BASELINE configs[4]: Mixtral-8x7B Q5_K_M (MUL_MAT_ID, 8-expert recipe: k/v Q8_0) + flash
    attention, through the reference's llama-bench like the headline: tg128 and pp512 at -fa 1,
    with its own decode roofline (the experts streamed by 2 of 8)"""
    if not (os.path.exists(REF_BENCH) or os.path.exists(LLAMA_BENCH)):
        return None
    out = {"how": f"the reference's {bench_tool()} + GGML_BACKEND_PATH=libggml-mi355x.so, Mixtral-8x7B Q5_K_M synthetic GGUF, "
                  f"-ngl 99 -fa 1 -r {args.dropin_reps}"}
    try:
        gguf = bench_gguf("mixtral_8x7b", "q5_k_m")
        env = dict(os.environ, GGML_BACKEND_PATH=LIB, GGML_MI355X_STATS="1")
        res, _ = ref_bench(gguf, env, ["-t", "8", "-ngl", "99", "-fa", "1", "-p", args.pp, "-n", args.tg,
                                       "-r", args.dropin_reps], timeout=1500)
        if isinstance(res, str):
            out["error"] = res
            return out
        bpt = plan_decode_bytes("mixtral_8x7b", "q5_k_m")
        out.update({"tg128_tok_s": res["tg_tok_s"], "tg128_samples": res["tg_samples"], "pp512_tok_s": res["pp_tok_s"],
                    "pp512_samples": res["pp_samples"], "decode_bytes_per_token": bpt,
                    "decode_roofline": {"achieved_GBs": round(bpt * res["tg_tok_s"] / 1e9, 1), "peak_GBs": HBM_PEAK_GBS,
                                        "frac": round(bpt * res["tg_tok_s"] / 1e9 / HBM_PEAK_GBS, 4)}})
    except Exception as e:  # noqa: BLE001
        out["error"] = str(e)
    return out


MODELS = {  # BASELINE.json configs -> (shape name in the package, default recipe, label)
    "llama3_8b": ("LLAMA3_8B", "q4_k_m", "Llama-3-8B"),
    "llama3_70b": ("LLAMA3_70B", "q4_k_m", "Llama-3-70B"),
    "mixtral_8x7b": ("MIXTRAL_8X7B", "q5_k_m", "Mixtral-8x7B"),
    "tinyllama": ("TINYLLAMA_1B", "q4_0", "TinyLlama-1.1B"),
}


class PipelineStage:
    """One rank of the layer split: layers [l0, l1) of the model, the hidden
    state handed to the next rank by RCCL point-to-point send/recv over xGMI. S sequences
    are kept in flight so that every stage works on a different sequence at a time
    (llama-bench tg feeds random tokens, so no token travels backwards)."""

    def __init__(self, pkg, dist, rank, world, local, shape, recipe, fa, n_ctx, n_seq, seed=1234):
        import torch
        self.dist, self.rank, self.world = dist, rank, world
        L = shape["n_layer"]
        self.l0, self.l1 = rank * L // world, (rank + 1) * L // world
        self.be = pkg.Backend(local % max(pkg.device_count(), 1))
        self.model = pkg.Model.random_stage(self.be, shape, (self.l0, self.l1), recipe, seed=seed)
        self.sessions = [pkg.Session(self.model, n_ctx=n_ctx, n_ubatch=512, flash_attn=fa) for _ in range(n_seq)]
        self.n_embd = shape["n_embd"]
        self.torch = torch
        # MX_PIPE_HOST=1: hand-off through pinned host buffers (gloo; lets several ranks
        # share one GPU for testing). Default: device buffers, RCCL over xGMI.
        self.host = os.environ.get("MX_PIPE_HOST") == "1"
        self.dev = torch.device("cpu") if self.host else torch.device("cuda", local)
        mk = (lambda: torch.empty((512, self.n_embd), dtype=torch.float32).pin_memory()) if self.host else \
             (lambda: torch.empty((512, self.n_embd), dtype=torch.float32, device=self.dev))
        self.hin = mk()
        self.hout = [mk(), mk()]
        self.pending = [None, None]
        self.flip = 0

    @property
    def first(self):
        return self.rank == 0

    @property
    def last(self):
        return self.rank == self.world - 1

    def item(self, si, tokens):
        """Run one ubatch of sequence si through this stage (recv -> compute -> send)."""
        n = len(tokens)
        hin = 0
        if not self.first:
            self.dist.recv(self.hin[:n], src=self.rank - 1)
            if not self.host:
                self.torch.cuda.current_stream(self.dev).synchronize()
            hin = self.hin.data_ptr()
        s = self.sessions[si]
        if self.last:
            s.decode_stage(tokens=tokens if self.first else None, h_in=hin, n_tokens=n, want_logits=True)
            return
        b = self.flip
        self.flip ^= 1
        if self.pending[b] is not None:
            self.pending[b].wait()
        s.decode_stage(tokens=tokens if self.first else None, h_in=hin, n_tokens=n, h_out=self.hout[b].data_ptr())
        self.pending[b] = self.dist.isend(self.hout[b][:n], dst=self.rank + 1)

    def drain(self):
        for w in self.pending:
            if w is not None:
                w.wait()
        self.pending = [None, None]
        if not self.host:
            self.torch.cuda.synchronize(self.dev)

    def tg(self, rng, n_vocab, n_gen, n_active=None):
        """n_active sequences (default all) decode n_gen tokens each, interleaved so that
        with n_active == N every stage works on a different sequence at a time"""
        n_active = n_active or len(self.sessions)
        for s in self.sessions[:n_active]:
            s.reset()
        toks = rng.integers(0, n_vocab, size=(n_active, n_gen), dtype=np.int32)
        for k in range(n_gen):
            for si in range(n_active):
                self.item(si, toks[si, k:k + 1])
        self.drain()

    def pp(self, rng, n_vocab, n_tok):
        s = self.sessions[0]
        s.reset()
        toks = rng.integers(0, n_vocab, size=n_tok, dtype=np.int32)
        for i in range(0, n_tok, 512):
            self.item(0, toks[i:i + 512])
        self.drain()

    def free(self):
        for s in self.sessions:
            s.free()
        self.model.free()


def base_line(args, world, value, ms_per_step, scaling, workload, parallelism, recipe, label):
    return {
        "metric": METRIC,
        "value": round(value, 2) if value else value,
        "unit": "tok/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 3) if ms_per_step else ms_per_step,
        "higher_is_better": True,
        "scaling": scaling,
        "vs_baseline": None,
        "dtype": "quantised weights (%s), int8 x int8 dot (v_dot4) + f32 accumulate" % recipe,
        "data": "synthetic (random %s weights, random tokens)" % recipe,
        "config": {"workload": workload, "model_shape": args.model, "recipe": recipe, "tg": args.tg, "pp": args.pp,
                   "flash_attn": not args.no_fa, "parallelism": parallelism},
    }


def split_headline(args, world, rank, local, dist, run_split=None):
    """N > 1 drop-in headline (libllama -sm layer): rank 0 runs the child over GPUs
    0..N-1; every rank meets in gloo barriers around it (no collective kernel on any GPU).
    Returns the JSON line on rank 0, None elsewhere. run_split is injectable (CPU tests)."""
    run_split = run_split or dropin_layer_split
    barrier(dist, local)
    t0 = time.perf_counter()
    split = run_split(args, world) if rank == 0 else None
    barrier(dist, local)
    wall = max_over_ranks(dist, time.perf_counter() - t0)
    if rank != 0:
        return None
    tg = (split or {}).get("tg")
    ok = isinstance(tg, dict)
    line = base_line(args, world, tg["tok_s"] if ok else None, tg["ms_per_step"] if ok else None, "strong",
                     f"Llama-3-8B Q4_K_M tg{args.tg} decode: the reference's {bench_tool()} on the reference libllama, "
                     f"layer split over {world} GPUs", f"libllama -sm layer -ts {','.join(['1'] * world)} "
                     "(cpy_tensor_async peer hand-off over xGMI), one sequence", "q4_k_m", "Llama-3-8B")
    line["dropin_layer_split"] = split
    if os.environ.get("MX_BENCH_VIRTUAL") == "1":
        line["virtual_devices"] = True
        line["scaling_note"] = (f"rehearsal: {world} logical devices of ONE GPU (GGML_MI355X_VIRTUAL_DEVICES), "
                                "not a multi-GPU measurement; keep out of any scaling curve")
    line["wall_s_all_legs"] = round(wall, 2)
    line["roofline"] = None
    line["cpu_baseline"] = None
    return line


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--tg", type=int, default=128)
    ap.add_argument("--pp", type=int, default=512)
    ap.add_argument("--model", default="llama3_8b", choices=sorted(MODELS))
    ap.add_argument("--recipe", default=None)
    ap.add_argument("--mode", default="auto", choices=["auto", "dropin", "single", "pipeline", "replicas"],
                    help="auto = dropin (the reference libllama on this backend; N>1: its -sm layer split) when "
                         "oracle/_ref is built and --model llama3_8b, else the package runner (single / pipeline)")
    ap.add_argument("--seqs", type=int, default=0,
                    help="pipeline: sequences of the pipelined_tok_s extra (default = number of GPUs); the headline is 1")
    ap.add_argument("--no-fa", action="store_true", help="llama-bench -fa 0 graph (KQ mul_mat + softmax)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-dropin", action="store_true", help="skip the reference-libllama drop-in legs (runner headline)")
    ap.add_argument("--dropin-reps", type=int, default=5, help="llama-bench -r of the extra legs (SURVEY §8d: 5)")
    ap.add_argument("--depths", type=lambda v: [int(x) for x in v.split(",") if x], default=[4096, 16384],
                    help="drop-in tg128 at these KV depths (llama-bench -d), comma list, '' for none")
    ap.add_argument("--no-pp2048", dest="pp2048", action="store_false", help="skip the pp2048 legs (BASELINE configs[2])")
    ap.add_argument("--cpu-pp", type=int, default=512)
    ap.add_argument("--cpu-tg", type=int, default=128)
    ap.add_argument("--cpu-reps", type=int, default=2)
    ap.add_argument("--skip-roofline", action="store_true")
    ap.add_argument("--moe-leg", action="store_true", help="add the Mixtral-8x7B Q5_K_M drop-in leg (BASELINE configs[4]; "
                    "writes a 32 GB GGUF)")
    ap.add_argument("--moe-only", action="store_true", help="run only the Mixtral drop-in leg and print it")
    ap.add_argument("--roofline-only", action="store_true",
                    help="only the dominant-kernel timing (for scripts/pmc_roofline.sh's rocprofv3 --pmc passes)")
    ap.add_argument("--tune", nargs="*", default=[], help="backend tuning knobs IDX=VAL (A/B experiments)")
    args = ap.parse_args()
    if args.tune:
        from mi355x_pkg import load_package
        lib = load_package()._lib.load()
        for t in args.tune:
            k, v = (int(x) for x in t.split("="))
            lib.ggml_backend_mi355x_set_tune(k, v)
    if args.moe_only:
        print(json.dumps({"moe": moe_leg(args)}), flush=True)
        return
    if args.roofline_only:
        from mi355x_pkg import load_package
        pkg = load_package()
        be = pkg.Backend(0)
        model = pkg.Model.random(be, getattr(pkg, MODELS[args.model][0]), args.recipe or MODELS[args.model][1], seed=1234)
        print(json.dumps(roofline_glu(pkg, be, model)), flush=True)
        model.free()
        return

    world_env = int(os.environ.get("WORLD_SIZE", "1"))
    dropin_ok = (os.path.exists(REF_BENCH) or os.path.exists(LLAMA_BENCH)) and not args.no_dropin and args.model == "llama3_8b" and not args.no_fa
    mode = args.mode
    if mode == "auto":
        mode = "dropin" if dropin_ok else ("pipeline" if world_env > 1 else "single")
    if mode == "dropin" and world_env > 1:
        world, rank, local, dist = dist_setup(args.gpus, backend="gloo")
        line = split_headline(args, world, rank, local, dist)
        if line is not None:
            print(json.dumps(line), flush=True)
        dist.destroy_process_group()
        return
    world, rank, local, dist = dist_setup(args.gpus)
    runner_mode = "single" if mode == "dropin" else mode
    from mi355x_pkg import load_package
    pkg = load_package()
    shape_name, def_recipe, label = MODELS[args.model]
    shape = getattr(pkg, shape_name)
    recipe = args.recipe or def_recipe
    # llama-bench sizes the context per test: n_ctx = n_prompt + n_gen, padded to 256 cells
    # (src/llama-context.cpp) — tg128 runs in a 256-cell cache, pp512 in a 512-cell one
    pad256 = lambda n: max(256, (n + 255) // 256 * 256)   # noqa: E731
    n_ctx_tg, n_ctx_pp = pad256(args.tg), pad256(args.pp)
    n_ctx = max(n_ctx_tg, n_ctx_pp)
    rng = np.random.default_rng(42 + rank)
    n_vocab = shape["n_vocab"]

    if runner_mode == "pipeline":
        n_seq = args.seqs or world
        stage = PipelineStage(pkg, dist, rank, world, local, shape, recipe, not args.no_fa, n_ctx, n_seq)
        be, model = stage.be, stage.model
        run_tg = lambda: stage.tg(rng, n_vocab, args.tg, 1)   # noqa: E731 — llama-bench -sm layer: one sequence
        tokens_per_step = args.tg                             # whole job (all ranks together)
    else:
        be = pkg.Backend(local if world > 1 else 0)
        model = pkg.Model.random(be, shape, recipe, seed=1234 + rank)
        sess = pkg.Session(model, n_ctx=n_ctx_tg, n_ubatch=512, flash_attn=not args.no_fa)
        run_tg = lambda: tg_step(sess, rng, n_vocab, args.tg)   # noqa: E731
        tokens_per_step = args.tg                                # per rank; summed below

    for _ in range(args.warmup):
        run_tg()
    barrier(dist, local)
    be.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        run_tg()
    be.synchronize()
    barrier(dist, local)
    dt = max_over_ranks(dist, time.perf_counter() - t0)
    if runner_mode == "pipeline":
        tokens = args.steps * tokens_per_step
    else:
        tokens = sum_over_ranks(dist, args.steps * tokens_per_step)
    tg_value = tokens / dt

    pipelined = None
    if runner_mode == "pipeline" and n_seq > 1:   # extra: N sequences in flight, one per stage
        stage.tg(rng, n_vocab, args.tg)
        barrier(dist, local)
        t2 = time.perf_counter()
        stage.tg(rng, n_vocab, args.tg)
        barrier(dist, local)
        pipelined = {"tok_s": round(n_seq * args.tg / max_over_ranks(dist, time.perf_counter() - t2), 2),
                     "sequences": n_seq}

    # pp512 beside it (not the headline value)
    pp_tok_s = None
    if args.pp > 0:
        if runner_mode == "pipeline":
            stage.pp(rng, n_vocab, args.pp)   # warm
            barrier(dist, local)
            t1 = time.perf_counter()
            reps = 3
            for _ in range(reps):
                stage.pp(rng, n_vocab, args.pp)
            barrier(dist, local)
            pp_tok_s = reps * args.pp / max_over_ranks(dist, time.perf_counter() - t1)
        else:
            sess.free()
            sess = pkg.Session(model, n_ctx=n_ctx_pp, n_ubatch=512, flash_attn=not args.no_fa)
            toks = rng.integers(0, n_vocab, size=args.pp, dtype=np.int32)
            sess.reset(); sess.decode(toks)  # warm the prefill graph
            reps = 3
            be.synchronize()
            t1 = time.perf_counter()
            for _ in range(reps):
                sess.reset()
                sess.decode(toks)
            be.synchronize()
            pp_tok_s = reps * args.pp / (time.perf_counter() - t1)
    # pp2048 (BASELINE configs[2]): llama-bench -p 2048 -b 2048 -ub 512, four 512-token
    # ubatches into a cache growing to 2048 cells; single GPU only
    pp2048_tok_s = None
    if args.pp2048 and runner_mode != "pipeline" and args.pp > 0:
        sess.free()
        sess = pkg.Session(model, n_ctx=2304, n_ubatch=512, flash_attn=not args.no_fa)
        toks = rng.integers(0, n_vocab, size=2048, dtype=np.int32)
        sess.reset(); sess.decode(toks)
        be.synchronize()
        t1 = time.perf_counter()
        for _ in range(2):
            sess.reset()
            sess.decode(toks)
        be.synchronize()
        pp2048_tok_s = 2 * 2048 / (time.perf_counter() - t1)

    stats = be.stats()
    # weights one decoded token reads (all stages together)
    decode_bytes = int(sum_over_ranks(dist, model.decode_bytes())) if runner_mode == "pipeline" else model.decode_bytes()
    roof = None if (args.skip_roofline or shape.get("n_expert")) else roofline_glu(pkg, be, model)
    cpu = cpu_baseline(args) if (rank == 0 and world == 1 and args.model == "llama3_8b") else None
    head_dropin = None
    if mode == "dropin" and rank == 0:
        env = dict(os.environ, GGML_BACKEND_PATH=LIB, GGML_MI355X_STATS="1")
        head_dropin = dropin_tg(args, env, ["-fa", 1, "-c", 256], "tg128_fa1")
    dropin = dropin_bench(args, skip=("tg128_fa1",) if mode == "dropin" else ()) \
        if (rank == 0 and world == 1 and args.model == "llama3_8b") else None
    moe = moe_leg(args) if (rank == 0 and world == 1 and args.moe_leg) else None
    barrier(dist, local)

    if rank == 0:
        par = {"single": "single", "replicas": f"replicas x{world}",
               "pipeline": f"layer split x{world} (RCCL p2p hidden-state hand-off), one sequence (llama-bench -sm layer)"}[runner_mode]
        runner = {"how": "this package's runner (mx_llama: the same backend, device-side random weights) "
                         f"-> {par}, {args.warmup} warmup + {args.steps} timed tg steps",
                  "tg128_tok_s": round(tg_value, 2), "ms_per_step": round(1000.0 * dt / args.steps, 3),
                  "pp512_tok_s": round(pp_tok_s, 1) if pp_tok_s else None,
                  "pp2048_tok_s": round(pp2048_tok_s, 1) if pp2048_tok_s else None,
                  "executor": stats, "pipelined": pipelined}
        if isinstance(head_dropin, dict):
            out = base_line(args, world, head_dropin["tok_s"], head_dropin["ms_per_step"], "weak",
                            f"{label} {recipe.upper()} tg{args.tg} decode: the reference's {bench_tool()} (-o jsonl, its own "
                            "defaults otherwise) on the reference libllama (GGML_BACKEND_PATH=libggml-mi355x.so, -ngl 99, -fa 1)",
                            "single", recipe, label)
            out["headline"] = head_dropin
            hv = head_dropin["tok_s"]
        else:
            # runner headline (no reference build, another model, or the drop-in failed)
            out = base_line(args, world, tg_value, 1000.0 * dt / args.steps, "strong" if runner_mode == "pipeline" else "weak",
                            f"{label} {recipe.upper()} tg{args.tg} decode (llama-bench test_gen), package runner", par,
                            recipe, label)
            if head_dropin is not None:
                out["headline_dropin_error"] = head_dropin
            hv = tg_value
        if moe is not None:
            out["moe"] = moe
        pp_ref = (dropin or {}).get("pp512_fa1_tok_s") if isinstance(head_dropin, dict) else pp_tok_s
        out.update({
            "pp512_tok_s": round(pp_ref, 1) if pp_ref else None,
            "pp_roofline": ({"bound": "mfma", "achieved": round(pp_ref * PP_FLOPS_PER_TOKEN[args.model] / 1e12 / world, 1),
                             "peak": MFMA_F16_PEAK_TFS, "unit": "TFLOP/s",
                             "frac": round(pp_ref * PP_FLOPS_PER_TOKEN[args.model] / 1e12 / world / MFMA_F16_PEAK_TFS, 4),
                             "flops_per_token": PP_FLOPS_PER_TOKEN[args.model]}
                            if pp_ref and args.model in PP_FLOPS_PER_TOKEN else None),
            "decode_bytes_per_token": decode_bytes,
            "decode_roofline": {"achieved_GBs": round(decode_bytes * hv / world / 1e9, 1), "peak_GBs": HBM_PEAK_GBS,
                                "frac": round(decode_bytes * hv / world / 1e9 / HBM_PEAK_GBS, 4)},
            "roofline": roof,
            "cpu_baseline": cpu,
            "runner": runner,
            "dropin": dropin,
        })
        print(json.dumps(out), flush=True)
    if runner_mode == "pipeline":
        stage.free()
    else:
        sess.free()
        model.free()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
