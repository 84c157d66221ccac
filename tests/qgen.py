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
