#!/usr/bin/env python3
"""Write a synthetic Llama-architecture GGUF (v3) with random quantised weights.

The file layout follows the reference's GGUF container (ggml/src/gguf.cpp,
ggml/include/gguf.h); the quantisation recipe follows llama_model_quantize's Q4_K_M
rules (src/llama-quant.cpp:185-187, 302-303, 358-365). There are no real checkpoints
offline, so block bytes are random with the f16 scale fields set to give weights of
std ~0.02 (same generator family as the device-side synthetic weights).
The vocab is a synthetic SentencePiece list (<unk>, <s>, </s>, 256 byte tokens, then
"▁t<i>") that the reference's llama vocab loader accepts.

    python tools/gguf_synth.py --shape llama3_8b --recipe q4_k_m --out /tmp/l3.gguf
    python tools/gguf_synth.py --shape tiny --out /tmp/tiny.gguf
"""
import argparse
import struct

import numpy as np

SHAPES = {
    "llama3_8b": dict(n_vocab=128256, n_embd=4096, n_layer=32, n_head=32, n_head_kv=8, n_ff=14336,
                      n_ctx=8192, rope_base=500000.0),
    "tinyllama": dict(n_vocab=32000, n_embd=2048, n_layer=22, n_head=32, n_head_kv=4, n_ff=5632,
                      n_ctx=2048, rope_base=10000.0),
    "tiny": dict(n_vocab=1024, n_embd=256, n_layer=2, n_head=4, n_head_kv=2, n_ff=512, n_ctx=1024,
                 rope_base=10000.0),
    "small": dict(n_vocab=4096, n_embd=1024, n_layer=4, n_head=8, n_head_kv=2, n_ff=2816, n_ctx=2048,
                  rope_base=500000.0),
    # two-layer models at the full widths of the bench configs: every decode / prefill
    # kernel instantiation the Llama-3-8B / Mixtral benches time, in a GGUF the reference
    # CPU backend runs in seconds (Q4_K_M over 2 layers: layer 0 Q4_K, layer 1 Q6_K v/down)
    "llama3_8b_2l": dict(n_vocab=128256, n_embd=4096, n_layer=2, n_head=32, n_head_kv=8, n_ff=14336,
                         n_ctx=8192, rope_base=500000.0),
    "llama3_70b": dict(n_vocab=128256, n_embd=8192, n_layer=80, n_head=64, n_head_kv=8, n_ff=28672,
                       n_ctx=8192, rope_base=500000.0),
    # Llama-3-70B widths over two layers, with the 70B model's attn_v rule (LLM_TYPE_70B
    # is an 80-layer model, so the flag stands in for the layer count): layer 0 attn_v Q5_K,
    # layer 1 (use_more_bits) attn_v / ffn_down Q6_K
    "llama3_70b_2l": dict(n_vocab=128256, n_embd=8192, n_layer=2, n_head=64, n_head_kv=8, n_ff=28672,
                          n_ctx=8192, rope_base=500000.0, rule70b=True),
    # eight layers at 70B widths: one per device of an 8-way layer split (-sm layer -ts 1x8,
    # BASELINE configs[3]); use_more_bits layers 0, 3, 6, 7 carry the Q6_K attn_v / ffn_down
    "llama3_70b_8l": dict(n_vocab=128256, n_embd=8192, n_layer=8, n_head=64, n_head_kv=8, n_ff=28672,
                          n_ctx=8192, rope_base=500000.0, rule70b=True),
    "mixtral_8x7b": dict(n_vocab=32000, n_embd=4096, n_layer=32, n_head=32, n_head_kv=8, n_ff=14336,
                         n_ctx=32768, rope_base=1e6, n_expert=8, n_expert_used=2),
    "mixtral_2l": dict(n_vocab=32000, n_embd=4096, n_layer=2, n_head=32, n_head_kv=8, n_ff=14336,
                       n_ctx=32768, rope_base=1e6, n_expert=8, n_expert_used=2),
    "tiny_moe": dict(n_vocab=1024, n_embd=256, n_layer=2, n_head=4, n_head_kv=2, n_ff=512, n_ctx=1024,
                     rope_base=10000.0, n_expert=4, n_expert_used=2),
}
# ggml type id -> (block elements, block bytes)
TYPES = {"f32": (0, 1, 4), "f16": (1, 1, 2), "q4_0": (2, 32, 18), "q8_0": (8, 32, 34), "q4_K": (12, 256, 144),
         "q5_K": (13, 256, 176), "q6_K": (14, 256, 210)}
FILE_TYPE = {"q4_k_m": 15, "q5_k_m": 17, "q4_0": 2, "q8_0": 7, "f16": 1}
ALIGN = 32


def use_more_bits(i, n):
    return i < n // 8 or i >= 7 * n // 8 or (i - n // 8) % 3 == 2


def tensor_plan(s, recipe):
    L, E, F, V = s["n_layer"], s["n_embd"], s["n_ff"], s["n_vocab"]
    kv = E // s["n_head"] * s["n_head_kv"]
    n_exp = s.get("n_expert", 0)
    plan = []

    def main_t(i, kind):
        # 8-expert models: attn_k / attn_v Q8_0 (llama-quant.cpp:311-321); 70B: attn_v
        # Q4_K -> Q5_K (:305-310)
        if n_exp == 8 and kind in ("k", "v") and recipe in ("q4_k_m", "q5_k_m"):
            return "q8_0"
        if kind == "v" and recipe == "q4_k_m" and (s.get("rule70b") or (E == 8192 and L == 80)) and not use_more_bits(i, L):
            return "q5_K"
        if recipe == "q4_k_m":
            return "q6_K" if kind in ("v", "down") and use_more_bits(i, L) else "q4_K"
        if recipe == "q5_k_m":
            return "q6_K" if kind in ("v", "down") and use_more_bits(i, L) else "q5_K"
        return {"q4_0": "q4_0", "q8_0": "q8_0", "f16": "f16"}[recipe]

    emb_t = {"q4_k_m": "q4_K", "q5_k_m": "q5_K", "q4_0": "q4_0", "q8_0": "q8_0", "f16": "f16"}[recipe]
    out_t = {"q4_k_m": "q6_K", "q5_k_m": "q6_K", "q4_0": "q6_K", "q8_0": "q8_0", "f16": "f16"}[recipe]
    plan.append(("token_embd.weight", emb_t, [E, V]))
    for i in range(L):
        p = f"blk.{i}."
        plan.append((p + "attn_norm.weight", "f32", [E]))
        plan.append((p + "attn_q.weight", main_t(i, "q"), [E, E]))
        plan.append((p + "attn_k.weight", main_t(i, "k"), [E, kv]))
        plan.append((p + "attn_v.weight", main_t(i, "v"), [E, kv]))
        plan.append((p + "attn_output.weight", main_t(i, "o"), [E, E]))
        plan.append((p + "ffn_norm.weight", "f32", [E]))
        if n_exp:
            plan.append((p + "ffn_gate_inp.weight", "f32", [E, n_exp]))
            plan.append((p + "ffn_gate_exps.weight", main_t(i, "gate"), [E, F, n_exp]))
            plan.append((p + "ffn_up_exps.weight", main_t(i, "up"), [E, F, n_exp]))
            plan.append((p + "ffn_down_exps.weight", main_t(i, "down"), [F, E, n_exp]))
        else:
            plan.append((p + "ffn_gate.weight", main_t(i, "gate"), [E, F]))
            plan.append((p + "ffn_up.weight", main_t(i, "up"), [E, F]))
            plan.append((p + "ffn_down.weight", main_t(i, "down"), [F, E]))
    plan.append(("output_norm.weight", "f32", [E]))
    plan.append(("output.weight", out_t, [E, V]))
    return plan


def nbytes(tname, ne):
    _, blk, sz = TYPES[tname]
    n = int(np.prod(ne))
    return n // blk * sz


def fill(tname, name, n_elems, rng):
    """random bytes with sane scale fields (std ~0.02 after dequantisation)"""
    tid, blk, sz = TYPES[tname]
    if tname == "f32":
        if name.endswith("norm.weight"):
            return np.ones(n_elems, np.float32).tobytes()
        return (rng.standard_normal(n_elems, dtype=np.float32) * 0.02).tobytes()
    if tname == "f16":
        return (rng.standard_normal(n_elems, dtype=np.float32) * 0.02).astype(np.float16).tobytes()
    nb = n_elems // blk
    raw = rng.integers(0, 256, size=(nb, sz), dtype=np.uint8)
    u = rng.uniform(0.75, 1.25, size=nb).astype(np.float32)

    def put(off, vals):
        raw[:, off:off + 2] = vals.astype(np.float16).view(np.uint8).reshape(nb, 2)

    if tname == "q4_K":
        put(0, 9.3e-5 * u); put(2, 9.3e-5 * 7.5 * u)
    elif tname == "q5_K":
        put(0, 4.6e-5 * u); put(2, 4.6e-5 * 15.5 * u)
    elif tname == "q6_K":
        raw[:, 192:208] = ((raw[:, 192:208].astype(np.int16) & 0x1F) - 16).astype(np.int8).view(np.uint8)
        put(208, 1.2e-4 * u)
    elif tname == "q4_0":
        put(0, 4.3e-3 * u)
    elif tname == "q8_0":
        put(0, 2.7e-4 * u)
    return raw.tobytes()


class W:
    def __init__(self, f):
        self.f = f

    def u32(self, v): self.f.write(struct.pack("<I", v))
    def u64(self, v): self.f.write(struct.pack("<Q", v))
    def i32(self, v): self.f.write(struct.pack("<i", v))
    def f32(self, v): self.f.write(struct.pack("<f", v))

    def s(self, x):
        b = x.encode() if isinstance(x, str) else x
        self.u64(len(b))
        self.f.write(b)

    def kv(self, key, typ, val):
        self.s(key)
        self.u32(typ)
        if typ == 8:
            self.s(val)
        elif typ == 4:
            self.u32(val)
        elif typ == 6:
            self.f32(val)
        elif typ == 7:
            self.f.write(struct.pack("<B", 1 if val else 0))
        elif typ == 9:
            et, items = val
            self.u32(et)
            self.u64(len(items))
            if et == 8:
                for it in items:
                    self.s(it)
            elif et == 6:
                self.f.write(np.asarray(items, np.float32).tobytes())
            elif et == 5:
                self.f.write(np.asarray(items, np.int32).tobytes())


def write(path, shape, recipe, seed=1234):
    s = SHAPES[shape]
    rng = np.random.default_rng(seed)
    plan = tensor_plan(s, recipe)
    V = s["n_vocab"]
    toks = [b"<unk>", b"<s>", b"</s>"] + [("<0x%02X>" % i).encode() for i in range(256)]
    toks += [("▁t%d" % i).encode() for i in range(V - len(toks))]
    types = [2, 3, 3] + [6] * 256 + [1] * (V - 259)
    kvs = [
        ("general.architecture", 8, "llama"), ("general.name", 8, f"synthetic-{shape}"),
        ("general.file_type", 4, FILE_TYPE[recipe]),
        ("llama.block_count", 4, s["n_layer"]), ("llama.context_length", 4, s["n_ctx"]),
        ("llama.embedding_length", 4, s["n_embd"]), ("llama.feed_forward_length", 4, s["n_ff"]),
        ("llama.attention.head_count", 4, s["n_head"]), ("llama.attention.head_count_kv", 4, s["n_head_kv"]),
        ("llama.rope.freq_base", 6, s["rope_base"]), ("llama.attention.layer_norm_rms_epsilon", 6, 1e-5),
        ("llama.rope.dimension_count", 4, s["n_embd"] // s["n_head"]), ("llama.vocab_size", 4, V),
        ("tokenizer.ggml.model", 8, "llama"), ("tokenizer.ggml.pre", 8, "default"),
        ("tokenizer.ggml.tokens", 9, (8, toks)), ("tokenizer.ggml.scores", 9, (6, [-float(i) for i in range(V)])),
        ("tokenizer.ggml.token_type", 9, (5, types)),
        ("tokenizer.ggml.bos_token_id", 4, 1), ("tokenizer.ggml.eos_token_id", 4, 2),
        ("tokenizer.ggml.unknown_token_id", 4, 0), ("tokenizer.ggml.add_bos_token", 7, True),
    ]
    if s.get("n_expert"):
        kvs += [("llama.expert_count", 4, s["n_expert"]), ("llama.expert_used_count", 4, s["n_expert_used"])]
    with open(path, "wb") as f:
        w = W(f)
        f.write(b"GGUF")
        w.u32(3)
        w.u64(len(plan))
        w.u64(len(kvs))
        for k, t, v in kvs:
            w.kv(k, t, v)
        off = 0
        offsets = []
        for name, tname, ne in plan:
            w.s(name)
            w.u32(len(ne))
            for d in ne:
                w.u64(d)
            w.u32(TYPES[tname][0])
            w.u64(off)
            offsets.append(off)
            off += (nbytes(tname, ne) + ALIGN - 1) // ALIGN * ALIGN
        pad = (-f.tell()) % ALIGN
        f.write(b"\0" * pad)
        for (name, tname, ne), o in zip(plan, offsets):
            n = int(np.prod(ne))
            data = fill(tname, name, n, rng)
            f.write(data)
            f.write(b"\0" * ((-len(data)) % ALIGN))
    return path


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="tiny", choices=sorted(SHAPES))
    ap.add_argument("--recipe", default="q4_k_m", choices=sorted(FILE_TYPE))
    ap.add_argument("--seed", type=int, default=1234)
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    write(a.out, a.shape, a.recipe, a.seed)
    print(a.out)


if __name__ == "__main__":
    main()
