// ops_moe.hip — MUL_MAT_ID (MoE expert matmul) on gfx950.
//
// Semantics (ggml_mul_mat_id, ggml.c; CPU ggml-cpu.c:1503): as = [K, M, n_expert],
// b = [K, ne11, n_tok], ids = [n_used, n_tok] i32; for every token t and slot e,
// dst[:, e, t] = as[:, :, ids[e, t]] · b[:, e % ne11, t].
// Reference GPU: ggml_cuda_mul_mat_id (ggml-cuda.cu:2268-2420) — its generic path
// copies ids to the host and synchronises (:2333-2356). Here expert selection is
// resolved on the device inside the kernel (the id is read per block), so the
// whole MoE layer stays capturable in a HIP graph.
#include "backend.h"
#include "mm.h"
#include "gemv.h"

namespace mx {

struct MoeArgs {
    const char * w; size_t w_row, w_exp;
    const char * ids; size_t id0, id1;
    float * dst; size_t d1, d2;           // floats
    int64_t M, K, units, n_used, ne11, n_expert;
};

template <int QT, int LPR>
__global__ __launch_bounds__(256) void k_moe_mmvq(MoeArgs p, ActQ a) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    constexpr int RPW = 64 / LPR;
    const int64_t row = ((int64_t) blockIdx.x * 4 + wave) * RPW + lane / LPR;
    const int sub = lane % LPR;
    const int64_t item = blockIdx.y;   // (e, t)
    const int64_t e = item % p.n_used, t = item / p.n_used;
    const int32_t ex = *(const int32_t *) (p.ids + e * p.id0 + t * p.id1);
    if (ex < 0 || ex >= p.n_expert) return;
    const int64_t col = t * p.ne11 + (e % p.ne11);
    ActQ ac = a;
    ac.q += col * a.kp; ac.d += col * (a.kp / 32); ac.s += col * (a.kp / 32);
    float acc[1] = {0.f};
    if (row < p.M) {
        const char * r = p.w + (size_t) ex * p.w_exp + (size_t) row * p.w_row;
        for (int u = sub; u < p.units; u += LPR) unit_dot<QT, 1>(r, u, ac, acc);
    }
#pragma unroll
    for (int o = LPR / 2; o > 0; o >>= 1) acc[0] += __shfl_xor(acc[0], o, 64);
    if (sub == 0 && row < p.M) p.dst[e * p.d1 + t * p.d2 + row] = acc[0];
}

template <int QT>
__device__ __forceinline__ float moe_w_elem(const char * row, int64_t k) {
    if constexpr (QT == GGML_TYPE_F32) return ((const float *) row)[k];
    else if constexpr (QT == GGML_TYPE_F16) return h2f(((const uint16_t *) row)[k]);
    else return dequant_one<QT>(row + (k / qk_of<QT>()) * qsize_of<QT>(), (int) (k % qk_of<QT>()));
}

// generic: one wave per (row, item), f32 activations, exact dequant
template <int QT>
__global__ __launch_bounds__(256) void k_moe_generic(MoeArgs p, const char * b, size_t b1, size_t b2) {
    const int lane = threadIdx.x & 63;
    const int64_t row = (int64_t) blockIdx.x * 4 + (threadIdx.x >> 6);
    const int64_t item = blockIdx.y;
    const int64_t e = item % p.n_used, t = item / p.n_used;
    const int32_t ex = *(const int32_t *) (p.ids + e * p.id0 + t * p.id1);
    if (row >= p.M || ex < 0 || ex >= p.n_expert) return;
    const char * wr = p.w + (size_t) ex * p.w_exp + (size_t) row * p.w_row;
    const float * x = (const float *) (b + (e % p.ne11) * b1 + t * b2);
    float acc = 0.f;
    for (int64_t k = lane; k < p.K; k += 64) acc += moe_w_elem<QT>(wr, k) * x[k];
    acc = wave_sum(acc);
    if (lane == 0) p.dst[e * p.d1 + t * p.d2 + row] = acc;
}

bool mul_mat_id_supported(const ggml_tensor * dst) {
    const ggml_tensor * as = dst->src[0];
    const ggml_tensor * b = dst->src[1];
    const ggml_tensor * ids = dst->src[2];
    if (dst->type != GGML_TYPE_F32 || b->type != GGML_TYPE_F32 || ids->type != GGML_TYPE_I32) return false;
    if (as->ne[3] != 1 || b->ne[3] != 1) return false;
    if (b->nb[0] != 4 || dst->nb[0] != 4) return false;
    switch (as->type) {
        case GGML_TYPE_F32: case GGML_TYPE_F16:
        case GGML_TYPE_Q4_0: case GGML_TYPE_Q4_1: case GGML_TYPE_Q5_0: case GGML_TYPE_Q5_1: case GGML_TYPE_Q8_0:
        case GGML_TYPE_Q4_K: case GGML_TYPE_Q5_K: case GGML_TYPE_Q6_K:
            return as->nb[0] == (size_t) mx_type(as->type).size;
        default: return false;
    }
}

size_t mul_mat_id_scratch(const ggml_tensor * dst) {
    const ggml_tensor * as = dst->src[0];
    if (const size_t g = mmq4_moe_scratch(dst)) return g;
    if (mmvq_type_ok(as->type) && as->ne[0] % qk_of_type(as->type) == 0) return quantize_scratch(dst->src[1]);
    return 0;
}

template <int QT>
static void moe_launch_q(OpCtx & c, const MoeArgs & p, const ActQ & a, int64_t items) {
    MX_KLOG("moe_mmvq qt=%d K=%d M=%d items=%lld", QT, (int) p.K, (int) p.M, (long long) items);
    if (p.K <= 2048) k_moe_mmvq<QT, 16><<<dim3((unsigned) mx_ceil_div(p.M, 16), (unsigned) items), 256, 0, c.st>>>(p, a);
    else if (p.K <= 8192) k_moe_mmvq<QT, 32><<<dim3((unsigned) mx_ceil_div(p.M, 8), (unsigned) items), 256, 0, c.st>>>(p, a);
    else k_moe_mmvq<QT, 64><<<dim3((unsigned) mx_ceil_div(p.M, 4), (unsigned) items), 256, 0, c.st>>>(p, a);
}

void op_mul_mat_id(OpCtx & c, ggml_tensor * dst) {
    const ggml_tensor * as = dst->src[0];
    const ggml_tensor * b = dst->src[1];
    const ggml_tensor * ids = dst->src[2];
    MoeArgs p{};
    p.w = (const char *) as->data; p.w_row = as->nb[1]; p.w_exp = as->nb[2];
    p.ids = (const char *) ids->data; p.id0 = ids->nb[0]; p.id1 = ids->nb[1];
    p.dst = (float *) dst->data; p.d1 = dst->nb[1] / 4; p.d2 = dst->nb[2] / 4;
    p.M = as->ne[1]; p.K = as->ne[0]; p.units = as->ne[0] / 32;
    p.n_used = ids->ne[0]; p.ne11 = b->ne[1]; p.n_expert = as->ne[2];
    const int64_t items = ids->ne[0] * ids->ne[1];
    if (items == 0) return;
    if (mmq4_moe(c, dst)) return;     // prefill: expert-grouped MFMA GEMM (ops_mmq4.hip)
    if (gemv2_moe(c, dst, nullptr, dst)) return;   // decode: v2 GEMV per (slot, token) item
    if (mmvq_type_ok(as->type) && as->ne[0] % qk_of_type(as->type) == 0) {
        ActQ a = quantize_activations(c, b);
        switch (as->type) {
            case GGML_TYPE_Q4_K: moe_launch_q<GGML_TYPE_Q4_K>(c, p, a, items); break;
            case GGML_TYPE_Q5_K: moe_launch_q<GGML_TYPE_Q5_K>(c, p, a, items); break;
            case GGML_TYPE_Q6_K: moe_launch_q<GGML_TYPE_Q6_K>(c, p, a, items); break;
            case GGML_TYPE_Q4_0: moe_launch_q<GGML_TYPE_Q4_0>(c, p, a, items); break;
            case GGML_TYPE_Q8_0: moe_launch_q<GGML_TYPE_Q8_0>(c, p, a, items); break;
            default: break;
        }
        return;
    }
    dim3 grid((unsigned) mx_ceil_div(p.M, 4), (unsigned) items);
    MX_KLOG("moe_generic type=%d K=%d M=%d items=%lld", (int) as->type, (int) p.K, (int) p.M, (long long) items);
    const char * pb = (const char *) b->data;
    switch (as->type) {
#define MG(T) case T: k_moe_generic<T><<<grid, 256, 0, c.st>>>(p, pb, b->nb[1], b->nb[2]); break;
        MG(GGML_TYPE_F32) MG(GGML_TYPE_F16) MG(GGML_TYPE_Q4_0) MG(GGML_TYPE_Q4_1) MG(GGML_TYPE_Q5_0) MG(GGML_TYPE_Q5_1)
        MG(GGML_TYPE_Q8_0) MG(GGML_TYPE_Q4_K) MG(GGML_TYPE_Q5_K) MG(GGML_TYPE_Q6_K)
#undef MG
        default: MX_ABORT("mul_mat_id type %d", (int) as->type);
    }
}

}  // namespace mx
