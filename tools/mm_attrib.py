#!/usr/bin/env python3
"""Per-node error attribution of the prefill MUL_MATs (TEST/DEBUG INFRASTRUCTURE).

Two node dumps of the same prompt through the reference libllama (oracle/_ref/
ref-llama-bench --dump/--dump-dir, scripts/dump_nodes.sh): the reference CPU backend
(-ngl 0) and this backend (-ngl 99). The eval callback makes the scheduler compute the
graph node by node, so every MUL_MAT output in the GPU dump is one k_mmq4 launch on the
input the GPU dump also holds. For every MUL_MAT of the llama graph (src/models/llama.cpp:
Qcur/Kcur/Vcur <- attn_norm, attn_out <- kqv_out, ffn_gate/ffn_up <- ffn_norm, ffn_out <-
ffn_swiglu, result_output <- result_norm) and every FLASH_ATTN_EXT (roped Qcur/Kcur and
Vcur, causal, K/V rounded to f16 as the cache holds them) this prints, per backend B:

    own  = NMSE(out_B, W . x_B)   the error THIS node adds on B's own input, against the
                                  float64 product of the dequantised weight and the
                                  unquantised f32 input (the CPU rounds x to q8_K /
                                  q8_0 first: ggml-cpu vec_dot_type; the GPU to f16)
    in   = NMSE(x_gpu, x_cpu)     how far the two inputs already are apart
    out  = NMSE(out_gpu, out_cpu)

    python tools/mm_attrib.py model.gguf cpu.txt cpu_dir gpu.txt gpu_dir
"""
import os
import struct
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))

BLK = {0: (1, 4), 1: (1, 2), 2: (32, 18), 8: (32, 34), 12: (256, 144), 13: (256, 176), 14: (256, 210)}
INPUT = {"Qcur": "attn_norm", "Kcur": "attn_norm", "Vcur": "attn_norm", "attn_out": "kqv_out",
         "ffn_gate": "ffn_norm", "ffn_up": "ffn_norm", "ffn_out": "ffn_swiglu"}
WEIGHT = {"Qcur": "attn_q", "Kcur": "attn_k", "Vcur": "attn_v", "attn_out": "attn_output",
          "ffn_gate": "ffn_gate", "ffn_up": "ffn_up", "ffn_out": "ffn_down"}


def gguf_tensors(path):
    """name -> (type, [ne0, ne1, ...], absolute byte offset) of a GGUF v3 file
    (ggml/src/gguf.cpp layout)"""
    f = open(path, "rb")
    rd = lambda fmt: struct.unpack("<" + fmt, f.read(struct.calcsize("<" + fmt)))   # noqa: E731
    assert f.read(4) == b"GGUF"
    _, n_t, n_kv = rd("IQQ")
    sizes = {0: 1, 1: 1, 2: 2, 3: 2, 4: 4, 5: 4, 6: 4, 7: 1, 10: 8, 11: 8, 12: 8}
    align = 32

    def rstr():
        n, = rd("Q")
        return f.read(n).decode()

    def rval(t):
        if t == 8:
            return rstr()
        if t == 9:
            et, n = rd("IQ")
            return [rval(et) for _ in range(n)] if et in (8, 9) else f.read(sizes[et] * n)
        return f.read(sizes[t])

    for _ in range(n_kv):
        k = rstr()
        t, = rd("I")
        v = rval(t)
        if k == "general.alignment":
            align = struct.unpack("<I", v)[0]
    infos = {}
    for _ in range(n_t):
        name = rstr()
        nd, = rd("I")
        ne = list(rd("Q" * nd))
        typ, off = rd("IQ")
        infos[name] = (typ, ne, off)
    base = (f.tell() + align - 1) // align * align
    return {k: (t, ne, base + off) for k, (t, ne, off) in infos.items()}


def weight_f64(path, info, orc):
    typ, ne, off = info
    K, M = ne[0], ne[1]
    be, bb = BLK[typ]
    rb = K // be * bb
    raw = np.fromfile(path, np.uint8, count=rb * M, offset=off)
    if typ == 0:
        return raw.view(np.float32).reshape(M, K).astype(np.float64)
    if typ == 1:
        return raw.view(np.float16).reshape(M, K).astype(np.float64)
    return np.stack([orc.dequantize(typ, raw[r * rb:(r + 1) * rb], K) for r in range(M)]).astype(np.float64)


def nodes(path):
    out = []
    for ln in open(path):
        t = ln.split()
        for i in range(1, len(t)):
            try:
                ne = [int(x) for x in t[i + 1:i + 5]]
                out.append((" ".join(t[:i]), t[i], ne))
                break
            except (ValueError, IndexError):
                continue
    return out


def nmse(a, b):
    return float(np.sum((a - b) ** 2) / max(np.sum(b ** 2), 1e-300))


def main():
    import oracle_lib
    orc = oracle_lib.load()
    gguf, ct, cd, gt, gd = sys.argv[1:6]
    tens = gguf_tensors(gguf)
    nc, ng = nodes(ct), nodes(gt)
    assert [n[:2] for n in nc] == [n[:2] for n in ng], "the two dumps observed different node lists"
    load = lambda d, i, ne: np.fromfile(f"{d}/{i:03d}.f32", np.float32).astype(np.float64).reshape(ne[1], ne[0])  # noqa: E731
    last = {}
    print(f"{'node':16s} {'weight':22s} {'type':5s} {'rows':>6s} {'N':>4s}  {'own cpu':>9s} {'own gpu':>9s} "
          f"{'gpu/cpu':>8s}  {'in g-c':>9s} {'out g-c':>9s}")
    rows = []
    for i, (name, op, ne) in enumerate(nc):
        base, _, il = name.partition("-")
        last[name] = (i, ne)
        if op != "MUL_MAT":
            continue
        if name == "result_output":
            src, wname = "result_norm", "output.weight"
        elif base in INPUT and il.isdigit():
            src, wname = f"{INPUT[base]}-{il}", f"blk.{il}.{WEIGHT[base]}.weight"
        else:
            continue
        if src not in last or wname not in tens:
            continue
        j, nej = last[src]
        xc, xg = load(cd, j, nej), load(gd, j, nej)
        if xc.shape[0] != ne[1]:       # (the last layer's GET_ROWS of the output rows sits between)
            continue
        W = weight_f64(gguf, tens[wname], orc)
        yc, yg = load(cd, i, ne), load(gd, i, ne)
        ec, eg = nmse(yc, xc @ W.T), nmse(yg, xg @ W.T)
        typ = {0: "f32", 1: "f16", 2: "q4_0", 8: "q8_0", 12: "q4_K", 13: "q5_K", 14: "q6_K"}[tens[wname][0]]
        r = (name, wname, typ, ne[0], ne[1], ec, eg, eg / max(ec, 1e-300), nmse(xg, xc), nmse(yg, yc))
        rows.append(r)
        print(f"{r[0]:16s} {r[1]:22s} {r[2]:5s} {r[3]:6d} {r[4]:4d}  {r[5]:9.2e} {r[6]:9.2e} {r[7]:8.4f}  {r[8]:9.2e} {r[9]:9.2e}",
              flush=True)
    # MUL_MAT_ID (MoE experts, round 5): each (token, slot) item against float64 W_e . x of
    # that backend's own routing (ffn_moe_topk) and input; MOE_ROWS rows of every expert
    # used (the full 14336 x 4096 x 8 tensors do not fit a float64 dequantisation)
    moe_rows = int(os.environ.get("MOE_ROWS", "256"))
    # (the routing: the first n_used columns of ffn_moe_argsort; the down projection's input:
    # the layer's SWIGLU node, whatever its callback name)
    MOE = {"ffn_moe_up": ("ffn_norm", "ffn_up_exps"), "ffn_moe_gate": ("ffn_norm", "ffn_gate_exps"),
           "ffn_moe_down": ("@glu", "ffn_down_exps")}
    seen = {}
    for i, (name, op, ne) in enumerate(nc):
        base, _, il = name.partition("-")
        seen[name] = (i, ne)
        if op in ("SWIGLU", "GLU") and il.isdigit():
            seen[f"@glu-{il}"] = (i, ne)
        if op != "MUL_MAT_ID" or base not in MOE or not il.isdigit():
            continue
        src, wn = MOE[base]
        src, wname, tk = f"{src}-{il}", f"blk.{il}.{wn}.weight", f"ffn_moe_argsort-{il}"
        if src not in seen or tk not in seen or wname not in tens:
            continue
        typ, wne, off = tens[wname]
        K, M, E = wne[0], wne[1], wne[2]
        be, bb = BLK[typ]
        rb = K // be * bb
        rows_ = min(moe_rows, M)
        n_used, n_tok = ne[1], ne[2]
        (jx, nex), (jt, net) = seen[src], seen[tk]
        cache = {}

        def wexp(e):
            if e not in cache:
                raw = np.fromfile(gguf, np.uint8, count=rb * rows_, offset=off + e * rb * M)
                cache[e] = np.stack([orc.dequantize(typ, raw[r * rb:(r + 1) * rb], K) for r in range(rows_)]).astype(np.float64)
            return cache[e]

        errs, outs = [], []
        for d in (cd, gd):
            ids = np.fromfile(f"{d}/{jt:03d}.f32", np.float32).reshape(net[1], net[0]).astype(np.int64)[:, :n_used]
            x = np.fromfile(f"{d}/{jx:03d}.f32", np.float32).astype(np.float64)
            x = x.reshape(n_tok, -1, K)          # [n_tok, 1 or n_used, K]
            y = np.fromfile(f"{d}/{i:03d}.f32", np.float32).astype(np.float64).reshape(n_tok, n_used, M)[:, :, :rows_]
            ref = np.empty_like(y)
            for t in range(n_tok):
                for sl in range(n_used):
                    ref[t, sl] = wexp(int(ids[t, sl])) @ x[t, sl % x.shape[1]]
            errs.append(nmse(y, ref))
            outs.append((ids, y))
        same = outs[0][0] == outs[1][0]          # items both backends routed alike
        og = nmse(outs[1][1][same], outs[0][1][same]) if same.any() else float("nan")
        tname = {12: "q4_K", 13: "q5_K", 14: "q6_K", 8: "q8_0"}.get(typ, str(typ))
        r = (name, wname, tname, rows_, n_tok * n_used, errs[0], errs[1], errs[1] / max(errs[0], 1e-300), float("nan"), og)
        rows.append(r)
        print(f"{r[0]:16s} {r[1][-22:]:22s} {r[2]:5s} {r[3]:6d} {r[4]:4d}  {r[5]:9.2e} {r[6]:9.2e} {r[7]:8.4f}  {'':9s} {r[9]:9.2e}"
              f"  (items routed alike {int(same.sum())}/{same.size})", flush=True)
    # FLASH_ATTN_EXT: float64 causal attention of each backend's own roped q / k and v
    # (k, v rounded to f16 as the cache stores them: SET_ROWS is bit-exact on both)
    idx = {}
    for i, (name, op, ne) in enumerate(nc):
        idx[(name, op)] = (i, ne)
    for i, (name, op, ne) in enumerate(nc):
        if op != "FLASH_ATTN_EXT" or not name.startswith("__fattn__-"):
            continue
        il = name.split("-")[1]
        try:
            (iq, neq), (ik, nek), (iv, nev) = idx[(f"Qcur-{il}", "ROPE")], idx[(f"Kcur-{il}", "ROPE")], idx[(f"Vcur-{il}", "RESHAPE")]
        except KeyError:
            continue
        D, H, N = ne[0], ne[1], ne[2]
        Hkv = nek[1]
        errs, outs = [], []
        for d in (cd, gd):
            q = np.fromfile(f"{d}/{iq:03d}.f32", np.float32).astype(np.float64).reshape(N, H, D)
            k = np.fromfile(f"{d}/{ik:03d}.f32", np.float32).astype(np.float16).astype(np.float64).reshape(N, Hkv, D)
            v = np.fromfile(f"{d}/{iv:03d}.f32", np.float32).astype(np.float16).astype(np.float64).reshape(N, Hkv, D)
            o = np.fromfile(f"{d}/{i:03d}.f32", np.float32).astype(np.float64).reshape(N, H, D)
            ref = np.empty_like(o)
            causal = np.triu(np.full((N, N), -np.inf), 1)
            for h in range(H):
                kv = h // (H // Hkv)
                sc = q[:, h, :] @ k[:, kv, :].T / np.sqrt(D) + causal
                p_ = np.exp(sc - sc.max(1, keepdims=True))
                ref[:, h, :] = (p_ / p_.sum(1, keepdims=True)) @ v[:, kv, :]
            errs.append(nmse(o, ref))
            outs.append(o)
        r = (name, "(K/V f16 cache)", "fa", D * H, N, errs[0], errs[1], errs[1] / max(errs[0], 1e-300), float("nan"),
             nmse(outs[1], outs[0]))
        rows.append(r)
        print(f"{r[0]:16s} {r[1]:22s} {r[2]:5s} {r[3]:6d} {r[4]:4d}  {r[5]:9.2e} {r[6]:9.2e} {r[7]:8.4f}  {'':9s} {r[9]:9.2e}",
              flush=True)
    worst = max(r[7] for r in rows) if rows else float("nan")
    print(f"nodes {len(rows)}; max over nodes of own-error ratio gpu/cpu = {worst:.4f} "
          f"({'the GPU adds less error than the reference CPU at every node' if worst < 1 else 'NOT below the CPU at every node'})")


if __name__ == "__main__":
    main()
