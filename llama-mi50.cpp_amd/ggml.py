"""Python mirror of the reference's graph API for the MI355X backend.

Names and argument meaning follow ggml/include/ggml.h (ggml_mul_mat, ggml_rms_norm,
ggml_rope_ext, ggml_soft_max_ext, ggml_flash_attn_ext, ggml_get_rows, ggml_set_rows,
ggml_swiglu_split, ...); every call goes through libggml-mi355x.so (mx_graph.h), and
compute() hands the graph to backend_i.graph_compute — the same C-ABI entry the
reference scheduler uses (ggml/src/ggml-backend-impl.h:114).
"""
import ctypes

import numpy as np

from . import _lib
from ._lib import GGML_TYPE, BLOCK

NP_OF = {0: np.float32, 1: np.float16, 26: np.int32, 27: np.int64, 24: np.int8}


class Backend:
    """One HIP stream on one MI355X (ggml_backend_mi355x_init)."""

    def __init__(self, device=0):
        self.lib = _lib.load()
        n = self.lib.ggml_backend_mi355x_get_device_count()
        if n <= device:
            raise RuntimeError(f"MI355X device {device} not visible ({n} devices)")
        self.ptr = self.lib.ggml_backend_mi355x_init(device)
        if not self.ptr:
            raise RuntimeError("ggml_backend_mi355x_init failed")
        self.buft = self.lib.ggml_backend_mi355x_buffer_type(device)

    def stats(self):
        out = (ctypes.c_uint64 * 4)()
        self.lib.ggml_backend_mi355x_stats(self.ptr, out)
        return dict(graph_compute=out[0], graph_replay=out[1], nodes_run=out[2], nodes_fused=out[3])

    def synchronize(self):
        self.lib.mxg_synchronize(self.ptr)

    def klog(self, on=True):
        """start (clear) / stop the kernel-choice log (ggml_backend_mi355x_klog)"""
        self.lib.ggml_backend_mi355x_klog(1 if on else 0)

    def klog_read(self):
        """the kernel-choice lines recorded since klog(True)"""
        n = self.lib.ggml_backend_mi355x_klog_read(None, 0)
        buf = ctypes.create_string_buffer(n + 1)
        self.lib.ggml_backend_mi355x_klog_read(buf, n + 1)
        return buf.value.decode().splitlines()

    def free(self):
        if self.ptr:
            self.lib.mxg_backend_free(self.ptr)
            self.ptr = None


class Tensor:
    def __init__(self, ctx, ptr):
        self.ctx = ctx
        self.ptr = ptr

    @property
    def raw(self):
        return _lib.tensor(self.ptr)

    @property
    def ne(self):
        return tuple(self.raw.ne)

    @property
    def nb(self):
        return tuple(self.raw.nb)

    @property
    def type(self):
        return self.raw.type

    @property
    def op(self):
        return self.raw.op

    def op_params(self, n=16):
        return list(self.raw.op_params)[:n]

    def nbytes(self):
        return _lib.load().mxg_nbytes(self.ptr)

    def set(self, arr):
        a = np.ascontiguousarray(arr)
        if a.nbytes != self.nbytes():
            raise ValueError(f"set: {a.nbytes} bytes for a {self.nbytes()}-byte tensor")
        self.ctx.lib.mxg_tensor_set(self.ptr, a.ctypes.data, 0, a.nbytes)

    def get_bytes(self):
        out = np.empty(self.nbytes(), dtype=np.uint8)
        self.ctx.lib.mxg_tensor_get(self.ptr, out.ctypes.data, 0, out.nbytes)
        return out

    def numpy(self):
        """Contiguous tensors only: returns an array shaped [ne3, ne2, ne1, ne0]."""
        t = self.type
        dt = NP_OF[t]
        ne = self.ne
        return self.get_bytes().view(dt).reshape(ne[3], ne[2], ne[1], ne[0])


class Context:
    """A graph-building context (ggml_context analogue)."""

    def __init__(self):
        self.lib = _lib.load()
        self.ptr = self.lib.mxg_init()

    def free(self):
        if self.ptr:
            self.lib.mxg_free(self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass

    def _t(self, p):
        if not p:
            raise RuntimeError("graph construction failed")
        return Tensor(self, p)

    @staticmethod
    def _p(t):
        return t.ptr if t is not None else None

    def new_tensor(self, type_, *ne, name=None, input=False):
        ne = list(ne) + [1] * (4 - len(ne))
        ty = GGML_TYPE[type_] if isinstance(type_, str) else type_
        t = self._t(self.lib.mxg_new_tensor_4d(self.ptr, ty, *ne))
        if name:
            self.lib.mxg_set_name(t.ptr, name.encode())
        if input:
            self.lib.mxg_set_input(t.ptr)
        return t

    def reshape(self, a, *ne):
        ne = list(ne) + [1] * (4 - len(ne))
        return self._t(self.lib.mxg_reshape_4d(self.ptr, a.ptr, *ne))

    def view_4d(self, a, ne0, ne1, ne2, ne3, nb1, nb2, nb3, offset):
        return self._t(self.lib.mxg_view_4d(self.ptr, a.ptr, ne0, ne1, ne2, ne3, nb1, nb2, nb3, offset))

    def permute(self, a, *ax):
        return self._t(self.lib.mxg_permute(self.ptr, a.ptr, *ax))

    def transpose(self, a):
        return self._t(self.lib.mxg_transpose(self.ptr, a.ptr))

    def cont(self, a):
        return self._t(self.lib.mxg_cont(self.ptr, a.ptr))

    def cpy(self, a, b):
        return self._t(self.lib.mxg_cpy(self.ptr, a.ptr, b.ptr))

    def cast(self, a, type_):
        return self._t(self.lib.mxg_cast(self.ptr, a.ptr, GGML_TYPE[type_]))

    def get_rows(self, a, b):
        return self._t(self.lib.mxg_get_rows(self.ptr, a.ptr, b.ptr))

    def set_rows(self, a, b, c):
        return self._t(self.lib.mxg_set_rows(self.ptr, a.ptr, b.ptr, c.ptr))

    def mul_mat(self, a, b):
        return self._t(self.lib.mxg_mul_mat(self.ptr, a.ptr, b.ptr))

    def mul_mat_id(self, as_, b, ids):
        return self._t(self.lib.mxg_mul_mat_id(self.ptr, as_.ptr, b.ptr, ids.ptr))

    def add(self, a, b):
        return self._t(self.lib.mxg_binary(self.ptr, 2, a.ptr, b.ptr))

    def mul(self, a, b):
        return self._t(self.lib.mxg_binary(self.ptr, 7, a.ptr, b.ptr))

    def div(self, a, b):
        return self._t(self.lib.mxg_binary(self.ptr, 8, a.ptr, b.ptr))

    def clamp(self, a, lo, hi):
        return self._t(self.lib.mxg_clamp(self.ptr, a.ptr, lo, hi))

    def scale(self, a, s):
        return self._t(self.lib.mxg_scale(self.ptr, a.ptr, s))

    def unary(self, a, op):
        return self._t(self.lib.mxg_unary(self.ptr, a.ptr, op))

    def swiglu_split(self, a, b):
        return self._t(self.lib.mxg_glu_split(self.ptr, a.ptr, b.ptr, 2))

    def rms_norm(self, a, eps):
        return self._t(self.lib.mxg_rms_norm(self.ptr, a.ptr, eps))

    def rope_ext(self, a, pos, ff, n_dims, mode, n_ctx_orig, freq_base, freq_scale=1.0, ext_factor=0.0,
                 attn_factor=1.0, beta_fast=32.0, beta_slow=1.0):
        return self._t(self.lib.mxg_rope_ext(self.ptr, a.ptr, pos.ptr, self._p(ff), n_dims, mode, n_ctx_orig,
                                             freq_base, freq_scale, ext_factor, attn_factor, beta_fast, beta_slow))

    def soft_max_ext(self, a, mask, scale, max_bias=0.0):
        return self._t(self.lib.mxg_soft_max_ext(self.ptr, a.ptr, self._p(mask), scale, max_bias))

    def flash_attn_ext(self, q, k, v, mask, scale, max_bias=0.0, softcap=0.0):
        return self._t(self.lib.mxg_flash_attn_ext(self.ptr, q.ptr, k.ptr, v.ptr, self._p(mask), scale, max_bias, softcap))

    def argsort(self, a, desc=False):
        return self._t(self.lib.mxg_argsort(self.ptr, a.ptr, 1 if desc else 0))

    def sum_rows(self, a):
        return self._t(self.lib.mxg_sum_rows(self.ptr, a.ptr))

    def build(self, *outs):
        g = self.lib.mxg_build(self.ptr, outs[0].ptr)
        for o in outs[1:]:
            self.lib.mxg_expand(self.ptr, g, o.ptr)
        return g

    def alloc(self, backend):
        if self.lib.mxg_alloc(self.ptr, backend.buft) != 0:
            raise MemoryError("mxg_alloc failed")

    def compute(self, backend, graph):
        st = self.lib.mxg_compute(backend.ptr, graph)
        if st != 0:
            raise RuntimeError(f"graph_compute returned status {st}")


def row_bytes(type_id, ne0):
    blk, sz = BLOCK[type_id]
    return ne0 // blk * sz
