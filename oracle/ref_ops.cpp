// oracle/ref_ops.cpp — TEST INFRASTRUCTURE ONLY (never linked into the product).
// Single ops run on the reference's own CPU ggml (libggml-ref.so, compiled from
// /root/reference by oracle/Makefile), so that tests/test_oracle.py can pin the C
// restatement in oracle.c op by op against the reference implementation itself:
// FLASH_ATTN_EXT (every cache type), ROPE, SOFT_MAX, RMS_NORM.
#include "ggml.h"
#include "ggml-cpu.h"

#include <cstdint>
#include <cstring>

namespace {

ggml_context * ctx_new(size_t bytes) {
    ggml_init_params ip = {bytes + (64u << 20), nullptr, false};
    return ggml_init(ip);
}

void compute(ggml_context * ctx, ggml_tensor * out) {
    ggml_cgraph * gf = ggml_new_graph(ctx);
    ggml_build_forward_expand(gf, out);
    ggml_graph_compute_with_ctx(ctx, gf, 4);
}

}  // namespace

extern "C" {

// q [H][n_q][D] f32, k/v [Hkv][n_kv] rows of kv_type, mask [n_q][n_kv] f16 (nullable)
// -> out [n_q][H][D] (ggml_flash_attn_ext's [D, H, n_q] result)
int refop_flash_attn(const float * q, const void * k, const void * v, const uint16_t * mask, float * out,
                     int64_t D, int64_t n_q, int64_t n_kv, int64_t H, int64_t Hkv, float scale, float max_bias,
                     float softcap, int kv_type) {
    const ggml_type t = (ggml_type) kv_type;
    const size_t kb = ggml_row_size(t, D) * n_kv * Hkv;
    ggml_context * ctx = ctx_new(2 * kb + (size_t) (D * n_q * H) * 8 + (size_t) (n_q * n_kv) * 2);
    if (!ctx) return -1;
    ggml_tensor * tq = ggml_new_tensor_3d(ctx, GGML_TYPE_F32, D, n_q, H);
    ggml_tensor * tk = ggml_new_tensor_3d(ctx, t, D, n_kv, Hkv);
    ggml_tensor * tv = ggml_new_tensor_3d(ctx, t, D, n_kv, Hkv);
    memcpy(tq->data, q, ggml_nbytes(tq));
    memcpy(tk->data, k, kb);
    memcpy(tv->data, v, kb);
    ggml_tensor * tm = nullptr;
    if (mask) {
        tm = ggml_new_tensor_2d(ctx, GGML_TYPE_F16, n_kv, n_q);
        memcpy(tm->data, mask, ggml_nbytes(tm));
    }
    ggml_tensor * o = ggml_flash_attn_ext(ctx, tq, tk, tv, tm, scale, max_bias, softcap);
    ggml_flash_attn_ext_set_prec(o, GGML_PREC_F32);
    compute(ctx, o);
    memcpy(out, o->data, ggml_nbytes(o));
    ggml_free(ctx);
    return 0;
}

// x [ne2 tokens][ne1 heads][ne0] f32, pos[ne2] -> y (same layout)
int refop_rope(const float * x, float * y, int64_t ne0, int64_t ne1, int64_t ne2, const int32_t * pos, int n_dims,
               int mode, int n_ctx_orig, float freq_base, float freq_scale, float ext_factor, float attn_factor,
               float beta_fast, float beta_slow, const float * freq_factors) {
    ggml_context * ctx = ctx_new((size_t) ne0 * ne1 * ne2 * 8 + 4 * ne2 + 4 * ne0);
    if (!ctx) return -1;
    ggml_tensor * tx = ggml_new_tensor_3d(ctx, GGML_TYPE_F32, ne0, ne1, ne2);
    ggml_tensor * tp = ggml_new_tensor_1d(ctx, GGML_TYPE_I32, ne2);
    memcpy(tx->data, x, ggml_nbytes(tx));
    memcpy(tp->data, pos, ggml_nbytes(tp));
    ggml_tensor * tf = nullptr;
    if (freq_factors) {
        tf = ggml_new_tensor_1d(ctx, GGML_TYPE_F32, n_dims / 2);
        memcpy(tf->data, freq_factors, ggml_nbytes(tf));
    }
    ggml_tensor * o = ggml_rope_ext(ctx, tx, tp, tf, n_dims, mode, n_ctx_orig, freq_base, freq_scale, ext_factor,
                                    attn_factor, beta_fast, beta_slow);
    compute(ctx, o);
    memcpy(y, o->data, ggml_nbytes(o));
    ggml_free(ctx);
    return 0;
}

// x [ne02][ne01][ne00] f32, mask [ne01][ne00] f16 (nullable, broadcast over ne02)
int refop_soft_max(const float * x, float * y, int64_t ne00, int64_t ne01, int64_t ne02, const uint16_t * mask,
                   float scale, float max_bias) {
    ggml_context * ctx = ctx_new((size_t) ne00 * ne01 * ne02 * 8 + (size_t) ne00 * ne01 * 2);
    if (!ctx) return -1;
    ggml_tensor * tx = ggml_new_tensor_3d(ctx, GGML_TYPE_F32, ne00, ne01, ne02);
    memcpy(tx->data, x, ggml_nbytes(tx));
    ggml_tensor * tm = nullptr;
    if (mask) {
        tm = ggml_new_tensor_2d(ctx, GGML_TYPE_F16, ne00, ne01);
        memcpy(tm->data, mask, ggml_nbytes(tm));
    }
    ggml_tensor * o = ggml_soft_max_ext(ctx, tx, tm, scale, max_bias);
    compute(ctx, o);
    memcpy(y, o->data, ggml_nbytes(o));
    ggml_free(ctx);
    return 0;
}

int refop_rms_norm(const float * x, float * y, int64_t ne0, int64_t nrows, float eps) {
    ggml_context * ctx = ctx_new((size_t) ne0 * nrows * 8);
    if (!ctx) return -1;
    ggml_tensor * tx = ggml_new_tensor_2d(ctx, GGML_TYPE_F32, ne0, nrows);
    memcpy(tx->data, x, ggml_nbytes(tx));
    ggml_tensor * o = ggml_rms_norm(ctx, tx, eps);
    compute(ctx, o);
    memcpy(y, o->data, ggml_nbytes(o));
    ggml_free(ctx);
    return 0;
}

}  // extern "C"
