"""ctypes bindings of libggml-mi355x.so (include/ggml_mi355x.h, mx_graph.h, mx_llama.h).

The shared library is the product; this module only declares its C-ABI. It fails
loudly when the library has not been built — there is no CPU fallback.
"""
import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("GGML_MI355X_LIB") or os.path.join(HERE, "lib", "libggml-mi355x.so")   # override: A/B builds

# ggml_type ids (ggml.h:389-431)
GGML_TYPE = {"f32": 0, "f16": 1, "q4_0": 2, "q4_1": 3, "q5_0": 6, "q5_1": 7, "q8_0": 8, "q8_1": 9,
             "q2_K": 10, "q3_K": 11, "q4_K": 12, "q5_K": 13, "q6_K": 14, "q8_K": 15,
             "i8": 24, "i16": 25, "i32": 26, "i64": 27, "f64": 28, "bf16": 30}
# ggml_op ids used by the host API (ggml.h:469-576)
GGML_OP = {"ADD": 2, "SUB": 6, "MUL": 7, "DIV": 8}
BLOCK = {0: (1, 4), 1: (1, 2), 30: (1, 2), 26: (1, 4), 27: (1, 8), 24: (1, 1),
         2: (32, 18), 3: (32, 20), 6: (32, 22), 7: (32, 24), 8: (32, 34),
         12: (256, 144), 13: (256, 176), 14: (256, 210)}


class MxrHparams(ctypes.Structure):
    _fields_ = [("n_vocab", ctypes.c_int32), ("n_embd", ctypes.c_int32), ("n_layer", ctypes.c_int32),
                ("n_head", ctypes.c_int32), ("n_head_kv", ctypes.c_int32), ("n_ff", ctypes.c_int32),
                ("n_ctx_train", ctypes.c_int32), ("n_expert", ctypes.c_int32), ("n_expert_used", ctypes.c_int32),
                ("rope_freq_base", ctypes.c_float), ("norm_eps", ctypes.c_float)]


class GgmlTensor(ctypes.Structure):
    """Layout of struct ggml_tensor (ggml.h:655-687, 336 bytes)."""
    _fields_ = [("type", ctypes.c_int), ("buffer", ctypes.c_void_p),
                ("ne", ctypes.c_int64 * 4), ("nb", ctypes.c_size_t * 4), ("op", ctypes.c_int),
                ("op_params", ctypes.c_int32 * 16), ("flags", ctypes.c_int32),
                ("src", ctypes.c_void_p * 10), ("view_src", ctypes.c_void_p), ("view_offs", ctypes.c_size_t),
                ("data", ctypes.c_void_p), ("name", ctypes.c_char * 64), ("extra", ctypes.c_void_p),
                ("padding", ctypes.c_char * 8)]


assert ctypes.sizeof(GgmlTensor) == 336

_lib = None

P = ctypes.c_void_p
I64 = ctypes.c_int64
F = ctypes.c_float
I = ctypes.c_int


def _sig(lib, name, restype, *argtypes):
    fn = getattr(lib, name)
    fn.restype = restype
    fn.argtypes = list(argtypes)


def load():
    """Load the backend library (raises if it was not built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} missing: build it with `make -C llama-mi50.cpp_amd` "
                          "(or __graft_entry__.build()); there is no CPU fallback")
    lib = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
    _sig(lib, "ggml_backend_init", P)
    _sig(lib, "ggml_backend_score", I)
    _sig(lib, "ggml_backend_mi355x_reg", P)
    _sig(lib, "ggml_backend_mi355x_init", P, I)
    _sig(lib, "ggml_backend_mi355x_get_device_count", I)
    _sig(lib, "ggml_backend_is_mi355x", ctypes.c_bool, P)
    _sig(lib, "ggml_backend_mi355x_buffer_type", P, I)
    _sig(lib, "ggml_backend_mi355x_stats", None, P, ctypes.POINTER(ctypes.c_uint64))
    _sig(lib, "ggml_backend_mi355x_time_mmvq", ctypes.c_double, P, P, P, I, P, P, I)
    _sig(lib, "ggml_backend_mi355x_set_tune", None, I, I)
    _sig(lib, "ggml_backend_mi355x_trace_read", I, P, I)
    _sig(lib, "ggml_backend_mi355x_trace_blocks_read", I, P, I)
    _sig(lib, "ggml_backend_mi355x_klog", None, I)
    _sig(lib, "ggml_backend_mi355x_klog_read", ctypes.c_size_t, ctypes.c_char_p, ctypes.c_size_t)
    # graph builder
    _sig(lib, "mxg_init", P)
    _sig(lib, "mxg_free", None, P)
    _sig(lib, "mxg_new_tensor_4d", P, P, I, I64, I64, I64, I64)
    _sig(lib, "mxg_set_name", None, P, ctypes.c_char_p)
    _sig(lib, "mxg_set_input", None, P)
    _sig(lib, "mxg_set_output", None, P)
    _sig(lib, "mxg_reshape_4d", P, P, P, I64, I64, I64, I64)
    _sig(lib, "mxg_view_4d", P, P, P, I64, I64, I64, I64, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_size_t)
    _sig(lib, "mxg_permute", P, P, P, I, I, I, I)
    _sig(lib, "mxg_transpose", P, P, P)
    _sig(lib, "mxg_cont", P, P, P)
    _sig(lib, "mxg_cont_4d", P, P, P, I64, I64, I64, I64)
    _sig(lib, "mxg_cpy", P, P, P, P)
    _sig(lib, "mxg_cast", P, P, P, I)
    _sig(lib, "mxg_get_rows", P, P, P, P)
    _sig(lib, "mxg_set_rows", P, P, P, P, P)
    _sig(lib, "mxg_mul_mat", P, P, P, P)
    _sig(lib, "mxg_mul_mat_id", P, P, P, P, P)
    _sig(lib, "mxg_binary", P, P, I, P, P)
    _sig(lib, "mxg_scale", P, P, P, F)
    _sig(lib, "mxg_clamp", P, P, P, F, F)
    _sig(lib, "mxg_unary", P, P, P, I)
    _sig(lib, "mxg_glu_split", P, P, P, P, I)
    _sig(lib, "mxg_rms_norm", P, P, P, F)
    _sig(lib, "mxg_rope_ext", P, P, P, P, P, I, I, I, F, F, F, F, F, F)
    _sig(lib, "mxg_soft_max_ext", P, P, P, P, F, F)
    _sig(lib, "mxg_flash_attn_ext", P, P, P, P, P, P, F, F, F)
    _sig(lib, "mxg_argsort", P, P, P, I)
    _sig(lib, "mxg_sum_rows", P, P, P)
    _sig(lib, "mxg_build", P, P, P)
    _sig(lib, "mxg_expand", None, P, P, P)
    _sig(lib, "mxg_alloc", I, P, P)
    _sig(lib, "mxg_tensor_set", None, P, P, ctypes.c_size_t, ctypes.c_size_t)
    _sig(lib, "mxg_tensor_get", None, P, P, ctypes.c_size_t, ctypes.c_size_t)
    _sig(lib, "mxg_nbytes", ctypes.c_size_t, P)
    _sig(lib, "mxg_compute", I, P, P)
    _sig(lib, "mxg_synchronize", None, P)
    _sig(lib, "mxg_backend_free", None, P)
    # llama runner
    _sig(lib, "mxr_model_random", P, P, ctypes.POINTER(MxrHparams), ctypes.c_char_p, ctypes.c_uint64)
    _sig(lib, "mxr_model_random_stage", P, P, ctypes.POINTER(MxrHparams), ctypes.c_char_p, ctypes.c_uint64, I, I)
    _sig(lib, "mxr_model_stage", None, P, ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_int32))
    _sig(lib, "mxr_model_load_gguf", P, P, ctypes.c_char_p)
    _sig(lib, "mxr_model_free", None, P)
    _sig(lib, "mxr_model_hparams", None, P, ctypes.POINTER(MxrHparams))
    _sig(lib, "mxr_model_layer_tensor", P, P, I, ctypes.c_char_p)
    _sig(lib, "mxr_model_decode_bytes", I64, P)
    _sig(lib, "mxr_model_type_bytes", None, P, ctypes.POINTER(I64))
    _sig(lib, "mxr_context_new", P, P, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32)
    _sig(lib, "mxr_context_free", None, P)
    _sig(lib, "mxr_context_reset", None, P)
    _sig(lib, "mxr_context_pos", ctypes.c_int32, P)
    _sig(lib, "mxr_decode", ctypes.c_int32, P, ctypes.POINTER(ctypes.c_int32), ctypes.c_int32, ctypes.POINTER(ctypes.c_float))
    _sig(lib, "mxr_decode_all_logits", ctypes.c_int32, P, ctypes.POINTER(ctypes.c_int32), ctypes.c_int32, ctypes.POINTER(ctypes.c_float))
    _sig(lib, "mxr_decode_stage", ctypes.c_int32, P, ctypes.POINTER(ctypes.c_int32), P, ctypes.c_int32, P, ctypes.POINTER(ctypes.c_float))
    _lib = lib
    return lib


def tensor(ptr):
    """View a ggml_tensor* as its Python struct."""
    return GgmlTensor.from_address(ptr)
