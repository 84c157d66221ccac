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
void mmv_generic_run(OpCtx & c, ggml_tensor * dst);

// prefill GEMM on MFMA (ops_mm.hip)
bool mmq_type_ok(int t);
size_t mmq_scratch(const ggml_tensor * dst);
void mmq_run(OpCtx & c, ggml_tensor * dst);

}  // namespace mx
