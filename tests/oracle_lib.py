"""ctypes access to oracle/liboracle.so — the CPU restatement used as the checker
(TEST INFRASTRUCTURE; see oracle/oracle.h)."""
import ctypes
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "oracle", "liboracle.so")
P = ctypes.c_void_p


class Oracle:
    def __init__(self, lib):
        self.lib = lib
        L = lib
        L.orc_fp16_to_fp32.restype = ctypes.c_float; L.orc_fp16_to_fp32.argtypes = [ctypes.c_uint16]
        L.orc_fp32_to_fp16.restype = ctypes.c_uint16; L.orc_fp32_to_fp16.argtypes = [ctypes.c_float]
        L.orc_dequantize_row.restype = ctypes.c_int; L.orc_dequantize_row.argtypes = [ctypes.c_int, P, P, ctypes.c_int64]
        for n in ("orc_quantize_row_q8_0", "orc_quantize_row_q4_0", "orc_quantize_row_q8_1", "orc_quantize_row_q8_K"):
            getattr(L, n).restype = None; getattr(L, n).argtypes = [P, P, ctypes.c_int64]
        for n in ("orc_mul_mat", "orc_mul_mat_exact"):
            getattr(L, n).restype = ctypes.c_int
            getattr(L, n).argtypes = [ctypes.c_int, P, ctypes.c_size_t, P, P, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64]
        L.orc_rms_norm.argtypes = [P, P, ctypes.c_int64, ctypes.c_int64, ctypes.c_float]
        L.orc_rope.argtypes = [P, P, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, P, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                               ctypes.c_float, ctypes.c_float, ctypes.c_float, ctypes.c_float, ctypes.c_float, ctypes.c_float, P]
        L.orc_soft_max.argtypes = [P, P, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, P, ctypes.c_float, ctypes.c_float, P]
        L.orc_swiglu.argtypes = [P, P, P, ctypes.c_int64]
        L.orc_f32_to_f16.argtypes = [P, P, ctypes.c_int64]
        L.orc_flash_attn.argtypes = [P, P, P, P, P] + [ctypes.c_int64] * 5 + [ctypes.c_float] * 3
        L.orc_flash_attn_t.restype = ctypes.c_int
        L.orc_flash_attn_t.argtypes = [P, P, P, P, P] + [ctypes.c_int64] * 5 + [ctypes.c_float] * 3 + [ctypes.c_int]
        L.orc_flash_attn_kv.restype = ctypes.c_int
        L.orc_flash_attn_kv.argtypes = [P, P, P, P, P] + [ctypes.c_int64] * 5 + [ctypes.c_float] * 3 + [ctypes.c_int] * 2

    @staticmethod
    def _p(a):
        return None if a is None else a.ctypes.data

    def dequantize(self, type_id, q, k):
        y = np.empty(k, dtype=np.float32)
        q = np.ascontiguousarray(q)
        assert self.lib.orc_dequantize_row(type_id, q.ctypes.data, y.ctypes.data, k) == 0
        return y

    def quantize_q8_0(self, x):
        x = np.ascontiguousarray(x, np.float32)
        y = np.zeros(len(x) // 32 * 34, np.uint8)
        self.lib.orc_quantize_row_q8_0(x.ctypes.data, y.ctypes.data, len(x))
        return y

    def quantize_q4_0(self, x):
        x = np.ascontiguousarray(x, np.float32)
        y = np.zeros(len(x) // 32 * 18, np.uint8)
        self.lib.orc_quantize_row_q4_0(x.ctypes.data, y.ctypes.data, len(x))
        return y

    def mul_mat(self, type_id, w, row_bytes, x, exact=False):
        """w: bytes [M rows], x: [N, K] f32 -> y [N, M]"""
        x = np.ascontiguousarray(x, np.float32)
        N, K = x.shape
        M = len(w) // row_bytes
        y = np.empty((N, M), np.float32)
        fn = self.lib.orc_mul_mat_exact if exact else self.lib.orc_mul_mat
        assert fn(type_id, np.ascontiguousarray(w).ctypes.data, row_bytes, x.ctypes.data, y.ctypes.data, K, M, N) == 0
        return y

    def rms_norm(self, x, eps):
        x = np.ascontiguousarray(x, np.float32)
        y = np.empty_like(x)
        self.lib.orc_rms_norm(x.ctypes.data, y.ctypes.data, x.shape[-1], x.size // x.shape[-1], eps)
        return y

    def rope(self, x, pos, n_dims, mode, n_ctx_orig, base, freq_scale=1.0, ext=0.0, attn=1.0, bf=32.0, bs=1.0, ff=None):
        """x: [ne2 tokens, ne1 heads, ne0] contiguous"""
        x = np.ascontiguousarray(x, np.float32)
        y = np.empty_like(x)
        pos = np.ascontiguousarray(pos, np.int32)
        ne2, ne1, ne0 = x.shape
        self.lib.orc_rope(x.ctypes.data, y.ctypes.data, ne0, ne1, ne2, pos.ctypes.data, n_dims, mode, n_ctx_orig,
                          base, freq_scale, ext, attn, bf, bs, self._p(ff))
        return y

    def soft_max(self, x, mask_f16, scale, max_bias=0.0, sinks=None):
        """x: [ne02, ne01, ne00]; mask f16 (uint16) [ne01, ne00] or None"""
        x = np.ascontiguousarray(x, np.float32)
        y = np.empty_like(x)
        ne02, ne01, ne00 = x.shape
        self.lib.orc_soft_max(x.ctypes.data, y.ctypes.data, ne00, ne01, ne02, self._p(mask_f16), scale, max_bias, self._p(sinks))
        return y

    def swiglu(self, a, b):
        a = np.ascontiguousarray(a, np.float32); b = np.ascontiguousarray(b, np.float32)
        y = np.empty_like(a)
        self.lib.orc_swiglu(a.ctypes.data, b.ctypes.data, y.ctypes.data, a.size)
        return y

    def f32_to_f16(self, x):
        x = np.ascontiguousarray(x, np.float32)
        y = np.empty(x.shape, np.uint16)
        self.lib.orc_f32_to_f16(x.ctypes.data, y.ctypes.data, x.size)
        return y

    def flash_attn(self, q, k, v, mask, scale, max_bias=0.0, softcap=0.0):
        """q [H, n_q, D] f32; k, v [Hkv, n_kv, D] uint16(f16); mask [n_q, n_kv] uint16 or None -> out [n_q, H, D]"""
        H, n_q, D = q.shape
        Hkv, n_kv, _ = k.shape
        out = np.empty((n_q, H, D), np.float32)
        q = np.ascontiguousarray(q, np.float32); k = np.ascontiguousarray(k); v = np.ascontiguousarray(v)
        self.lib.orc_flash_attn(q.ctypes.data, k.ctypes.data, v.ctypes.data, self._p(mask), out.ctypes.data,
                                D, n_q, n_kv, H, Hkv, scale, max_bias, softcap)
        return out

    def flash_attn_t(self, q, k, v, mask, scale, kv_type, max_bias=0.0, softcap=0.0, v_type=None):
        """k, v: [Hkv, n_kv, row_bytes] uint8 rows of ggml type kv_type (f32 0, f16 1, q4_0 2, q8_0 8, bf16 30);
        v_type: V's own type when it differs from K's"""
        H, n_q, D = q.shape
        Hkv, n_kv = k.shape[:2]
        out = np.empty((n_q, H, D), np.float32)
        q = np.ascontiguousarray(q, np.float32); k = np.ascontiguousarray(k); v = np.ascontiguousarray(v)
        vt = kv_type if v_type is None else v_type
        assert self.lib.orc_flash_attn_kv(q.ctypes.data, k.ctypes.data, v.ctypes.data, self._p(mask), out.ctypes.data,
                                          D, n_q, n_kv, H, Hkv, scale, max_bias, softcap, kv_type, vt) == 0
        return out


REF_OPS = os.path.join(ROOT, "oracle", "_ref", "libref-ops.so")


class RefOps:
    """single ops on the reference's own CPU ggml (oracle/ref_ops.cpp over libggml-ref.so)"""

    def __init__(self, lib):
        self.lib = lib
        lib.refop_flash_attn.restype = ctypes.c_int
        lib.refop_flash_attn.argtypes = [P, P, P, P, P] + [ctypes.c_int64] * 5 + [ctypes.c_float] * 3 + [ctypes.c_int]
        lib.refop_rope.restype = ctypes.c_int
        lib.refop_rope.argtypes = [P, P, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, P, ctypes.c_int, ctypes.c_int,
                                   ctypes.c_int] + [ctypes.c_float] * 6 + [P]
        lib.refop_soft_max.restype = ctypes.c_int
        lib.refop_soft_max.argtypes = [P, P, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, P, ctypes.c_float, ctypes.c_float]
        lib.refop_rms_norm.restype = ctypes.c_int
        lib.refop_rms_norm.argtypes = [P, P, ctypes.c_int64, ctypes.c_int64, ctypes.c_float]

    def flash_attn(self, q, k, v, mask, scale, kv_type, max_bias=0.0, softcap=0.0):
        H, n_q, D = q.shape
        Hkv, n_kv = k.shape[:2]
        out = np.empty((n_q, H, D), np.float32)
        q = np.ascontiguousarray(q, np.float32); k = np.ascontiguousarray(k); v = np.ascontiguousarray(v)
        assert self.lib.refop_flash_attn(q.ctypes.data, k.ctypes.data, v.ctypes.data, Oracle._p(mask), out.ctypes.data,
                                         D, n_q, n_kv, H, Hkv, scale, max_bias, softcap, kv_type) == 0
        return out

    def rope(self, x, pos, n_dims, mode, n_ctx_orig, base, freq_scale=1.0, ext=0.0, attn=1.0, bf=32.0, bs=1.0, ff=None):
        x = np.ascontiguousarray(x, np.float32)
        y = np.empty_like(x)
        pos = np.ascontiguousarray(pos, np.int32)
        ne2, ne1, ne0 = x.shape
        assert self.lib.refop_rope(x.ctypes.data, y.ctypes.data, ne0, ne1, ne2, pos.ctypes.data, n_dims, mode, n_ctx_orig,
                                   base, freq_scale, ext, attn, bf, bs, Oracle._p(ff)) == 0
        return y

    def soft_max(self, x, mask_f16, scale, max_bias=0.0):
        x = np.ascontiguousarray(x, np.float32)
        y = np.empty_like(x)
        ne02, ne01, ne00 = x.shape
        assert self.lib.refop_soft_max(x.ctypes.data, y.ctypes.data, ne00, ne01, ne02, Oracle._p(mask_f16), scale, max_bias) == 0
        return y

    def rms_norm(self, x, eps):
        x = np.ascontiguousarray(x, np.float32)
        y = np.empty_like(x)
        assert self.lib.refop_rms_norm(x.ctypes.data, y.ctypes.data, x.shape[-1], x.size // x.shape[-1], eps) == 0
        return y


def load_ref_ops():
    """None when the reference build (oracle/_ref) is absent"""
    return RefOps(ctypes.CDLL(REF_OPS)) if os.path.exists(REF_OPS) else None


def load():
    if not os.path.exists(LIB):
        subprocess.run(["make", "-C", os.path.join(ROOT, "oracle"), "liboracle.so"], check=True,
                       stdout=subprocess.DEVNULL)
    return Oracle(ctypes.CDLL(LIB))
