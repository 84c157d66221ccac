"""Generate the golden fixtures under tests/golden/ (run in the build container only).

Source of truth: the reference's own gguf-py quantiser (gguf-py/gguf/quants.py:220-575,
imported read-only from /root/reference) on the deterministic data of the reference's
quantisation KAT, tests/test-quantize-fns.cpp:31-35 (x[i] = 0.1 + 2*cos(i + offset)).

Output: quant_<type>.npz with
    x      float32 input (4 rows x 1024 values, offsets 0..3)
    q      uint8   quantised bytes as gguf-py writes them
    deq    float32 gguf-py dequantisation of q
Only data is committed; the reference source itself is never copied.
"""
import os
import sys

import numpy as np

REF = os.environ.get("REF", "/root/reference")
HERE = os.path.dirname(os.path.abspath(__file__))


def ref_quantize(x, qtype):
    import ctypes
    lib = ctypes.CDLL(os.path.join(HERE, "..", "..", "oracle", "_ref", "libggml-ref.so"))
    lib.ggml_row_size.restype = ctypes.c_size_t
    lib.ggml_row_size.argtypes = [ctypes.c_int, ctypes.c_int64]
    lib.ggml_quantize_chunk.restype = ctypes.c_size_t
    lib.ggml_quantize_chunk.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                                        ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p]
    rows, n = x.shape
    rs = lib.ggml_row_size(qtype, n)
    out = np.zeros((rows, rs), dtype=np.uint8)
    xc = np.ascontiguousarray(x, dtype=np.float32)
    lib.ggml_quantize_chunk(qtype, xc.ctypes.data, out.ctypes.data, 0, rows, n, None)
    return out


def main():
    sys.path.insert(0, os.path.join(REF, "gguf-py"))
    from gguf import quants, GGMLQuantizationType as T  # noqa: E402

    n = 1024
    rows = 4
    x = np.stack([0.1 + 2.0 * np.cos(np.arange(n, dtype=np.float64) + off) for off in range(rows)]).astype(np.float32)
    for name, qt in [("q4_0", T.Q4_0), ("q8_0", T.Q8_0), ("q4_1", T.Q4_1), ("q5_0", T.Q5_0), ("q5_1", T.Q5_1),
                     ("q4_K", T.Q4_K), ("q5_K", T.Q5_K), ("q6_K", T.Q6_K)]:
        try:
            q = quants.quantize(x, qt)
        except NotImplementedError:
            # gguf-py has no K-quant quantiser: use the reference C quantiser
            # (ggml_quantize_chunk, ggml.c:7537) from the oracle/_ref build
            q = ref_quantize(x, int(qt))
        deq = quants.dequantize(q, qt).astype(np.float32)
        np.savez_compressed(os.path.join(HERE, f"quant_{name}.npz"), x=x, q=np.ascontiguousarray(q).view(np.uint8), deq=deq)
        print(name, q.shape, deq.shape)


if __name__ == "__main__":
    main()
