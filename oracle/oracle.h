/*
 * oracle.h — TEST INFRASTRUCTURE. CPU restatement of the reference's hot-path
 * algorithms (ggml CPU backend / ggml-quants.c). Used only by tests/, by
 * __graft_entry__.smoke() and by bench.py's cpu_baseline leg as the checker;
 * never linked into libggml-mi355x.so.
 *
 * Pinning: the dequantisers are checked byte-for-byte against vectors produced by
 * the reference's own gguf-py quantiser (tests/golden/, tests/test_oracle.py) and
 * the whole oracle against the reference CPU backend built in oracle/_ref.
 */
#pragma once
#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

float    orc_fp16_to_fp32(uint16_t h);
uint16_t orc_fp32_to_fp16(float f);

/* dequantize_row_<type> (ggml-quants.c:307-420, 1352-1374, 1554-1584, 1762-1790) */
int  orc_dequantize_row(int type, const void * x, float * y, int64_t k);
/* quantize_row_q8_0_ref / q8_1_ref / q8_K_ref (ggml-quants.c:199-258, 2555-2592) */
void orc_quantize_row_q8_0(const float * x, void * y, int64_t k);
/* quantize_row_q4_0_ref (ggml-quants.c:36-71) */
void orc_quantize_row_q4_0(const float * x, void * y, int64_t k);
void orc_quantize_row_q8_1(const float * x, void * y, int64_t k);
void orc_quantize_row_q8_K(const float * x, void * y, int64_t k);

/* MUL_MAT as the CPU backend computes it (ggml-cpu.c:1229-1500): src1 rows are
 * quantised to the weight's vec_dot_type (q8_0 for Q4_0/Q8_0..., q8_K for K-quants)
 * and every output is one vec_dot (ggml-cpu/quants.c:115-705 generic paths).
 * w: [K, M] rows of `type`, x: [K, N] f32 row-major, y: [M, N] (y[n*M + m]). */
int  orc_mul_mat(int type, const void * w, size_t w_row_bytes, const float * x, float * y, int64_t K, int64_t M, int64_t N);
/* the same product with exactly dequantised weights and f32 activations (double accumulation) */
int  orc_mul_mat_exact(int type, const void * w, size_t w_row_bytes, const float * x, float * y, int64_t K, int64_t M, int64_t N);

/* ggml_compute_forward_rms_norm_f32 (ops.cpp:3645-3694): Σx² in double */
void orc_rms_norm(const float * x, float * y, int64_t ne0, int64_t nrows, float eps);

/* ggml_compute_forward_rope_flt (ops.cpp:5523-5800), mode 0 (NORMAL) or 2 (NEOX),
 * x: [ne0, ne1 heads, ne2 tokens] contiguous f32, pos[ne2] */
void orc_rope(const float * x, float * y, int64_t ne0, int64_t ne1, int64_t ne2, const int32_t * pos,
              int n_dims, int mode, int n_ctx_orig, float freq_base, float freq_scale, float ext_factor,
              float attn_factor, float beta_fast, float beta_slow, const float * freq_factors);

/* ggml_compute_forward_soft_max_f32 (ops.cpp:5160-5270); mask f16 rows [ne00] per row (nullable) */
void orc_soft_max(const float * x, float * y, int64_t ne00, int64_t ne01, int64_t ne02,
                  const uint16_t * mask_f16, float scale, float max_bias, const float * sinks);

/* ggml_compute_forward_swiglu_f32 (ops.cpp:3062): y = silu(a) * b */
void orc_swiglu(const float * a, const float * b, float * y, int64_t n);

/* f32 → f16 rows (set_rows to an F16 KV cache, ops.cpp:4827-4875) */
void orc_f32_to_f16(const float * x, uint16_t * y, int64_t n);

/* ggml_compute_forward_flash_attn_ext_f16_one_chunk (ops.cpp:8045-8260) for one
 * sequence: q [D, n_q, H] f32, k/v [D, n_kv, Hkv] f16, mask [n_kv, n_q] f16 (nullable),
 * out [D, H, n_q] f32 */
void orc_flash_attn(const float * q, const uint16_t * k, const uint16_t * v, const uint16_t * mask,
                    float * out, int64_t D, int64_t n_q, int64_t n_kv, int64_t H, int64_t Hkv,
                    float scale, float max_bias, float softcap);

/* the same with K/V rows of kv_type (0 f32, 1 f16, 30 bf16, 8 q8_0, 2 q4_0), q in the K
 * type's vec_dot_type (q8_0 blocks for the quantised caches); -1: unsupported */
int orc_flash_attn_t(const float * q, const void * k, const void * v, const uint16_t * mask,
                     float * out, int64_t D, int64_t n_q, int64_t n_kv, int64_t H, int64_t Hkv,
                     float scale, float max_bias, float softcap, int kv_type);
/* the same with K and V of different types (kv_type: K, v_type: V) */
int orc_flash_attn_kv(const float * q, const void * k, const void * v, const uint16_t * mask,
                      float * out, int64_t D, int64_t n_q, int64_t n_kv, int64_t H, int64_t Hkv,
                      float scale, float max_bias, float softcap, int kv_type, int v_type);

#ifdef __cplusplus
}
#endif
