"""Seeded synthetic ggml super-blocks for tests (valid bytes of every field; scale
fields set so dequantised values are O(1e-2), like real checkpoints)."""
import numpy as np

# type id -> (block elements, block bytes, [(byte offset of an f16 scale field, magnitude)])
LAYOUT = {
    2: (32, 18, [(0, 4e-3)]),                 # q4_0
    3: (32, 20, [(0, 4e-3), (2, 1e-2)]),      # q4_1
    6: (32, 22, [(0, 2e-3)]),                 # q5_0
    7: (32, 24, [(0, 2e-3), (2, 1e-2)]),      # q5_1
    8: (32, 34, [(0, 3e-4)]),                 # q8_0
    12: (256, 144, [(0, 1e-4), (2, 7e-4)]),   # q4_K
    13: (256, 176, [(0, 5e-5), (2, 7e-4)]),   # q5_K
    14: (256, 210, [(208, 1.2e-4)]),          # q6_K
}
NAMES = {"q4_0": 2, "q4_1": 3, "q5_0": 6, "q5_1": 7, "q8_0": 8, "q4_K": 12, "q5_K": 13, "q6_K": 14}


def rand_quant(type_id, rows, k, rng):
    blk, sz, scales = LAYOUT[type_id]
    nb = rows * (k // blk)
    raw = rng.integers(0, 256, size=(nb, sz), dtype=np.uint8)
    for off, mag in scales:
        d = (mag * rng.uniform(0.5, 1.5, size=nb)).astype(np.float16)
        raw[:, off:off + 2] = d.view(np.uint8).reshape(nb, 2)
    return raw.reshape(-1), (k // blk) * sz


def nmse(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.sum((a - b) ** 2) / max(np.sum(b ** 2), 1e-30))


# KV-cache rows of every cache type FLASH_ATTN_EXT takes: name -> ggml type id
KV_TYPES = {"f32": 0, "f16": 1, "q4_0": 2, "q8_0": 8, "bf16": 30}


def kv_rows(kind, Hkv, n_kv, D, rng, orc):
    """[Hkv, n_kv, row bytes] uint8 K or V rows of cache type `kind` holding N(0, 1) data
    (q8_0 by the oracle's quantize_row_q8_0_ref; q4_0 as random nibbles with d ~ 0.25)"""
    x = rng.standard_normal((Hkv, n_kv, D)).astype(np.float32)
    if kind == "f32":
        return x.view(np.uint8).reshape(Hkv, n_kv, -1)
    if kind == "f16":
        return x.astype(np.float16).view(np.uint8).reshape(Hkv, n_kv, -1)
    if kind == "bf16":
        u = x.view(np.uint32)
        u = (u + 0x7FFF + ((u >> 16) & 1)) >> 16
        return u.astype(np.uint16).view(np.uint8).reshape(Hkv, n_kv, -1)
    if kind == "q8_0":
        rows = [orc.quantize_q8_0(r) for r in x.reshape(-1, D)]
        return np.stack(rows).reshape(Hkv, n_kv, -1)
    if kind == "q4_0":
        nb = Hkv * n_kv * D // 32
        raw = rng.integers(0, 256, size=(nb, 18), dtype=np.uint8)
        raw[:, 0:2] = (0.25 * rng.uniform(0.5, 1.5, size=nb)).astype(np.float16).view(np.uint8).reshape(nb, 2)
        return raw.reshape(Hkv, n_kv, -1)
    raise ValueError(kind)
