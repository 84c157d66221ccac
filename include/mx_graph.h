/*
 * mx_graph.h — host-side graph construction over the ggml tensor ABI.
 *
 * A minimal re-statement of the reference's graph API (ggml/include/ggml.h:
 * ggml_new_tensor*, ggml_view_*, ggml_reshape_*, ggml_permute, ggml_mul_mat,
 * ggml_rms_norm, ggml_rope_ext, ggml_soft_max_ext, ggml_flash_attn_ext,
 * ggml_get_rows, ggml_set_rows, ggml_glu_split ..., ggml_build_forward_expand)
 * producing byte-identical ggml_tensor nodes, plus allocation into backend
 * buffers (the role of ggml-alloc.c) and ggml_backend_graph_compute. It lets the
 * tests and the bench drive libggml-mi355x.so through the same backend C-ABI the
 * reference scheduler uses, without the reference's libggml.
 * Names mirror ggml with an `mxg_` prefix; argument meaning is unchanged.
 */
#pragma once

#include "ggml_abi.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct mxg_context mxg_context;

mxg_context * mxg_init(void);
void          mxg_free(mxg_context * ctx);   /* frees tensors and the buffers mxg_alloc created */

struct ggml_tensor * mxg_new_tensor(mxg_context * ctx, enum ggml_type type, int n_dims, const int64_t * ne);
struct ggml_tensor * mxg_new_tensor_4d(mxg_context * ctx, enum ggml_type type, int64_t ne0, int64_t ne1, int64_t ne2, int64_t ne3);
void mxg_set_name(struct ggml_tensor * t, const char * name);
void mxg_set_input(struct ggml_tensor * t);
void mxg_set_output(struct ggml_tensor * t);

/* views */
struct ggml_tensor * mxg_reshape_4d(mxg_context * ctx, struct ggml_tensor * a, int64_t ne0, int64_t ne1, int64_t ne2, int64_t ne3);
struct ggml_tensor * mxg_view_4d(mxg_context * ctx, struct ggml_tensor * a, int64_t ne0, int64_t ne1, int64_t ne2, int64_t ne3,
                                 size_t nb1, size_t nb2, size_t nb3, size_t offset);
struct ggml_tensor * mxg_permute(mxg_context * ctx, struct ggml_tensor * a, int ax0, int ax1, int ax2, int ax3);
struct ggml_tensor * mxg_transpose(mxg_context * ctx, struct ggml_tensor * a);

/* ops */
struct ggml_tensor * mxg_cont(mxg_context * ctx, struct ggml_tensor * a);
struct ggml_tensor * mxg_cont_4d(mxg_context * ctx, struct ggml_tensor * a, int64_t ne0, int64_t ne1, int64_t ne2, int64_t ne3);
struct ggml_tensor * mxg_cpy(mxg_context * ctx, struct ggml_tensor * a, struct ggml_tensor * b);
struct ggml_tensor * mxg_cast(mxg_context * ctx, struct ggml_tensor * a, enum ggml_type type);
struct ggml_tensor * mxg_get_rows(mxg_context * ctx, struct ggml_tensor * a, struct ggml_tensor * b);
struct ggml_tensor * mxg_set_rows(mxg_context * ctx, struct ggml_tensor * a, struct ggml_tensor * b, struct ggml_tensor * c);
struct ggml_tensor * mxg_mul_mat(mxg_context * ctx, struct ggml_tensor * a, struct ggml_tensor * b);
struct ggml_tensor * mxg_mul_mat_id(mxg_context * ctx, struct ggml_tensor * as, struct ggml_tensor * b, struct ggml_tensor * ids);
struct ggml_tensor * mxg_binary(mxg_context * ctx, enum ggml_op op, struct ggml_tensor * a, struct ggml_tensor * b); /* ADD/SUB/MUL/DIV */
struct ggml_tensor * mxg_scale(mxg_context * ctx, struct ggml_tensor * a, float s);
struct ggml_tensor * mxg_clamp(mxg_context * ctx, struct ggml_tensor * a, float min, float max);
struct ggml_tensor * mxg_unary(mxg_context * ctx, struct ggml_tensor * a, enum ggml_unary_op op);
struct ggml_tensor * mxg_glu_split(mxg_context * ctx, struct ggml_tensor * a, struct ggml_tensor * b, enum ggml_glu_op op);
struct ggml_tensor * mxg_rms_norm(mxg_context * ctx, struct ggml_tensor * a, float eps);
struct ggml_tensor * mxg_rope_ext(mxg_context * ctx, struct ggml_tensor * a, struct ggml_tensor * pos, struct ggml_tensor * freq_factors,
                                  int n_dims, int mode, int n_ctx_orig, float freq_base, float freq_scale, float ext_factor,
                                  float attn_factor, float beta_fast, float beta_slow);
struct ggml_tensor * mxg_soft_max_ext(mxg_context * ctx, struct ggml_tensor * a, struct ggml_tensor * mask, float scale, float max_bias);
struct ggml_tensor * mxg_flash_attn_ext(mxg_context * ctx, struct ggml_tensor * q, struct ggml_tensor * k, struct ggml_tensor * v,
                                        struct ggml_tensor * mask, float scale, float max_bias, float logit_softcap);
struct ggml_tensor * mxg_argsort(mxg_context * ctx, struct ggml_tensor * a, enum ggml_sort_order order);
struct ggml_tensor * mxg_sum_rows(mxg_context * ctx, struct ggml_tensor * a);

/* graph: forward expansion from `out` (ggml_build_forward_expand order) */
struct ggml_cgraph * mxg_build(mxg_context * ctx, struct ggml_tensor * out);
/* add another output to an existing graph */
void mxg_expand(mxg_context * ctx, struct ggml_cgraph * g, struct ggml_tensor * out);

/* allocate every tensor of ctx that has no data yet into one buffer of `buft` */
int  mxg_alloc(mxg_context * ctx, ggml_backend_buffer_type_t buft);
size_t mxg_alloc_bytes(const mxg_context * ctx);   /* device bytes of the buffers mxg_alloc created */
void mxg_tensor_set(struct ggml_tensor * t, const void * data, size_t offset, size_t size);
void mxg_tensor_get(const struct ggml_tensor * t, void * data, size_t offset, size_t size);
size_t mxg_nbytes(const struct ggml_tensor * t);

enum ggml_status mxg_compute(ggml_backend_t backend, struct ggml_cgraph * g);
void mxg_synchronize(ggml_backend_t backend);
void mxg_backend_free(ggml_backend_t backend);

#ifdef __cplusplus
}
#endif
