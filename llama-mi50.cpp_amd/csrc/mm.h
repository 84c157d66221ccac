// mm.h — internal interface between the MUL_MAT dispatcher and its kernels.
#pragma once
#include "backend.h"
#include "mmvq.cuh"

namespace mx {

static inline int qk_of_type(int t) { return mx_type(t).blck; }

bool mmvq_type_ok(int t);
ActQ quantize_activations(OpCtx & c, const ggml_tensor * src1);
size_t quantize_scratch(const ggml_tensor * src1);
void mmvq_run(OpCtx & c, ggml_tensor * dst);
bool gemv_nc_ok(const ggml_tensor * dst);          // ops_gemv_nc.hip: 2..8 columns, LDS-staged
void gemv_nc_run(OpCtx & c, ggml_tensor * dst);
void mmv_generic_run(OpCtx & c, ggml_tensor * dst);

// prefill GEMM on MFMA (ops_mm.hip)
bool mmq_type_ok(int t);
size_t mmq_scratch(const ggml_tensor * dst);
void mmq_run(OpCtx & c, ggml_tensor * dst);
// f16 activation rows [cols][kp] of x for a prefill GEMM (act cache; ops_mm.hip)
_Float16 * mmq_act_f16(OpCtx & c, const ggml_tensor * x, int64_t kp);

// prefill GEMM v4 (ops_mmq4.hip): false when not eligible (nothing launched)
bool mmq4_on();
size_t mmq4_scratch(const ggml_tensor * dst, bool add_norm = false);   // split-K partial sums
size_t mmq4_moe_scratch(const ggml_tensor * dst);
bool mmq4_moe_glu(OpCtx & c, const ggml_tensor * gate, const ggml_tensor * up, ggml_tensor * glu);   // + SwiGLU, prefill
bool mmq4_moe(OpCtx & c, ggml_tensor * dst);     // MUL_MAT_ID prefill, expert-grouped
bool mmq4_mul_mat(OpCtx & c, const ggml_tensor * w, const ggml_tensor * x, const _Float16 * xa, int64_t kp,
                  ggml_tensor * out, const ggml_tensor * res);
bool mmq4_group(OpCtx & c, ggml_tensor * const * mms, int n, const _Float16 * xa, int64_t kp);
// split-K partials handed to a consumer instead of k_mmq4_reduce (ops_qkv.hip's prefill
// q/k/v epilogue sums them itself): while g_m4_split is set, a split segment-group launch
// without residual / f16 copy fills it (ks > 1) and skips the reduce pass. Partial of
// (plane z, token t, global row r): part[(z N + t) part_ld + r]; segment s starts at row0[s].
struct M4Split { const float * part; int part_ld; int ks; int row0[3]; };
extern thread_local M4Split * g_m4_split;
bool mmq4_glu_ok(const ggml_tensor * wg, const ggml_tensor * wu, const ggml_tensor * x, const ggml_tensor * glu);
void mmq4_glu(OpCtx & c, const ggml_tensor * wg, const ggml_tensor * wu, const ggml_tensor * x, const _Float16 * xa,
              int64_t kp, ggml_tensor * glu, _Float16 * h, int64_t h_col);

}  // namespace mx
