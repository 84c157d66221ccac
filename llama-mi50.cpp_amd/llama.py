"""Llama-family decode driver on the MI355X backend (include/mx_llama.h).

Counterpart of the reference's llama_decode path (src/llama-context.cpp:1469,
process_ubatch :1117) for the bench and end-to-end tests: the graph it hands to the
backend is node-for-node llm_build_llama (src/models/llama.cpp:4-165).
"""
import ctypes

import numpy as np

from . import _lib
from ._lib import MxrHparams

# Model shapes named in BASELINE.json configs
LLAMA3_8B = dict(n_vocab=128256, n_embd=4096, n_layer=32, n_head=32, n_head_kv=8, n_ff=14336,
                 n_ctx_train=8192, rope_freq_base=500000.0, norm_eps=1e-5)
LLAMA3_70B = dict(n_vocab=128256, n_embd=8192, n_layer=80, n_head=64, n_head_kv=8, n_ff=28672,
                  n_ctx_train=8192, rope_freq_base=500000.0, norm_eps=1e-5)
TINYLLAMA_1B = dict(n_vocab=32000, n_embd=2048, n_layer=22, n_head=32, n_head_kv=4, n_ff=5632,
                    n_ctx_train=2048, rope_freq_base=10000.0, norm_eps=1e-5)
MIXTRAL_8X7B = dict(n_vocab=32000, n_embd=4096, n_layer=32, n_head=32, n_head_kv=8, n_ff=14336,
                    n_ctx_train=32768, rope_freq_base=1e6, norm_eps=1e-5, n_expert=8, n_expert_used=2)


def hparams(**kw):
    h = MxrHparams()
    for k, v in kw.items():
        setattr(h, k, v)
    return h


class Model:
    def __init__(self, backend, ptr):
        self.backend = backend
        self.lib = _lib.load()
        self.ptr = ptr
        if not ptr:
            raise RuntimeError("model creation failed")
        self.hp = MxrHparams()
        self.lib.mxr_model_hparams(ptr, ctypes.byref(self.hp))

    @classmethod
    def random(cls, backend, shape, recipe="q4_k_m", seed=1234):
        lib = _lib.load()
        h = hparams(**shape)
        return cls(backend, lib.mxr_model_random(backend.ptr, ctypes.byref(h), recipe.encode(), seed))

    @classmethod
    def random_stage(cls, backend, shape, layers, recipe="q4_k_m", seed=1234):
        """Pipeline stage holding layers [layers[0], layers[1]) of Model.random's model."""
        lib = _lib.load()
        h = hparams(**shape)
        return cls(backend, lib.mxr_model_random_stage(backend.ptr, ctypes.byref(h), recipe.encode(), seed,
                                                       int(layers[0]), int(layers[1])))

    @property
    def stage(self):
        a, b = ctypes.c_int32(), ctypes.c_int32()
        self.lib.mxr_model_stage(self.ptr, ctypes.byref(a), ctypes.byref(b))
        return a.value, b.value

    @property
    def is_first_stage(self):
        return self.stage[0] == 0

    @property
    def is_last_stage(self):
        return self.stage[1] == self.hp.n_layer

    @classmethod
    def load_gguf(cls, backend, path):
        lib = _lib.load()
        return cls(backend, lib.mxr_model_load_gguf(backend.ptr, str(path).encode()))

    def layer_tensor(self, il, which):
        """Raw ggml_tensor* of layer il's weight by GGUF role (e.g. "ffn_gate")."""
        return self.lib.mxr_model_layer_tensor(self.ptr, il, which.encode())

    def decode_bytes(self):
        """Algorithmic weight bytes read per decoded token (all weights but token_embd)."""
        return int(self.lib.mxr_model_decode_bytes(self.ptr))

    def type_bytes(self):
        out = (ctypes.c_int64 * 40)()
        self.lib.mxr_model_type_bytes(self.ptr, out)
        return {i: out[i] for i in range(40) if out[i]}

    def free(self):
        if self.ptr:
            self.lib.mxr_model_free(self.ptr)
            self.ptr = None


class Session:
    def __init__(self, model, n_ctx=512, n_ubatch=512, flash_attn=True):
        self.model = model
        self.lib = model.lib
        self.ptr = self.lib.mxr_context_new(model.ptr, n_ctx, n_ubatch, 1 if flash_attn else 0)
        if not self.ptr:
            raise RuntimeError("context creation failed")
        self.n_vocab = model.hp.n_vocab
        self._logits = np.empty(self.n_vocab, dtype=np.float32)

    def reset(self):
        self.lib.mxr_context_reset(self.ptr)

    @property
    def pos(self):
        return self.lib.mxr_context_pos(self.ptr)

    def decode(self, tokens, want_logits=True):
        toks = np.ascontiguousarray(tokens, dtype=np.int32)
        lp = self._logits.ctypes.data_as(ctypes.POINTER(ctypes.c_float)) if want_logits else None
        r = self.lib.mxr_decode(self.ptr, toks.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), len(toks), lp)
        if r != 0:
            raise RuntimeError(f"mxr_decode failed ({r})")
        return self._logits.copy() if want_logits else None

    def decode_stage(self, tokens=None, h_in=0, n_tokens=None, h_out=0, want_logits=False):
        """One ubatch through a pipeline stage. tokens (first stage) or h_in (an address of
        f32 [n_tokens, n_embd], device or host) in; h_out (address) or the last token's
        logits out. Returns the logits (last stage, want_logits) or None."""
        tp = None
        if tokens is not None:
            toks = np.ascontiguousarray(tokens, dtype=np.int32)
            n_tokens = len(toks)
            tp = toks.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))
        lp = self._logits.ctypes.data_as(ctypes.POINTER(ctypes.c_float)) if want_logits else None
        r = self.lib.mxr_decode_stage(self.ptr, tp, ctypes.c_void_p(h_in or None), int(n_tokens),
                                      ctypes.c_void_p(h_out or None), lp)
        if r != 0:
            raise RuntimeError(f"mxr_decode_stage failed ({r})")
        return self._logits.copy() if want_logits else None

    def decode_all(self, tokens):
        toks = np.ascontiguousarray(tokens, dtype=np.int32)
        out = np.empty((len(toks), self.n_vocab), dtype=np.float32)
        r = self.lib.mxr_decode_all_logits(self.ptr, toks.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), len(toks),
                                           out.ctypes.data_as(ctypes.POINTER(ctypes.c_float)))
        if r != 0:
            raise RuntimeError(f"mxr_decode_all_logits failed ({r})")
        return out

    def free(self):
        if self.ptr:
            self.lib.mxr_context_free(self.ptr)
            self.ptr = None
