// ops_mmvq.hip — decode path of MUL_MAT (≤ 8 activation columns): activation
// quantisation + quantised GEMV, plus the fused gate/up GLU variant.
// Reference dispatch: ggml_cuda_mul_mat (ggml-cuda.cu:2183-2266) routes src1->ne[1]
// <= MMVQ_MAX_BATCH_SIZE (8, mmvq.cuh:3) to mul_mat_vec_q; fused GLU at
// ggml-cuda.cu:2145-2181 / mmvq.cu:195-351.
#include "backend.h"
#include "mmvq.cuh"
#include "mm.h"

namespace mx {

// ---------------------------------------------------------------------------
// activation quantisation: column c (flattened i11,i12,i13) → int8 + per-32 d, d·Σq
// (quantize_q8_1, ggml-cuda/quantize.cu:5-48: d = amax/127, q = round(x/d))
// ---------------------------------------------------------------------------
__global__ void k_quantize_act(const char * __restrict__ x, int64_t K, int64_t ne11, int64_t ne12,
                               size_t nb11, size_t nb12, size_t nb13, int64_t kp,
                               int8_t * __restrict__ q, float * __restrict__ d, float * __restrict__ s) {
    const int64_t col = blockIdx.y;
    const int64_t i11 = col % ne11, i12 = (col / ne11) % ne12, i13 = col / (ne11 * ne12);
    const float * px = (const float *) (x + i11 * nb11 + i12 * nb12 + i13 * nb13);
    const int64_t blk = blockIdx.x * (int64_t) blockDim.x + threadIdx.x;
    if (blk * 32 >= kp) return;
    float v[32];
    const int64_t e0 = blk * 32;
    if (e0 + 32 <= K && ((uintptr_t) (px + e0) % 16) == 0) {
#pragma unroll
        for (int j = 0; j < 32; j += 4) {
            const float4 f = *(const float4 *) (px + e0 + j);
            v[j] = f.x; v[j + 1] = f.y; v[j + 2] = f.z; v[j + 3] = f.w;
        }
    } else {
#pragma unroll
        for (int j = 0; j < 32; ++j) v[j] = e0 + j < K ? px[e0 + j] : 0.0f;
    }
    float amax = 0.f;
#pragma unroll
    for (int j = 0; j < 32; ++j) amax = fmaxf(amax, fabsf(v[j]));
    const float dd = amax / 127.0f;
    const float id = amax == 0.0f ? 0.0f : 1.0f / dd;
    int sum = 0;
    int packed[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        int w = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int qi = (int) roundf(v[4 * j + k] * id);
            sum += qi;
            w |= (qi & 0xFF) << (8 * k);
        }
        packed[j] = w;
    }
    int4 * out = (int4 *) (q + col * kp + e0);
    out[0] = make_int4(packed[0], packed[1], packed[2], packed[3]);
    out[1] = make_int4(packed[4], packed[5], packed[6], packed[7]);
    d[col * (kp / 32) + blk] = dd;
    s[col * (kp / 32) + blk] = dd * (float) sum;
}

ActQ quantize_activations(OpCtx & c, const ggml_tensor * src1) {
    const int64_t K = src1->ne[0];
    const int64_t ncols = src1->ne[1] * src1->ne[2] * src1->ne[3];
    const int64_t kp = (K + 31) / 32 * 32;
    // +8 columns: the GEMV reads NC-padded column groups (NC in {1,2,4,8})
    int8_t * q = (int8_t *) c.scratch->take((ncols + 8) * kp);
    float * d = (float *) c.scratch->take((ncols + 8) * (kp / 32) * sizeof(float));
    float * s = (float *) c.scratch->take((ncols + 8) * (kp / 32) * sizeof(float));
    const int64_t nblk = kp / 32;
    dim3 grid((unsigned) mx_ceil_div(nblk, 128), (unsigned) ncols);
    k_quantize_act<<<grid, 128, 0, c.st>>>((const char *) src1->data, K, src1->ne[1], src1->ne[2],
                                            src1->nb[1], src1->nb[2], src1->nb[3], kp, q, d, s);
    return ActQ{q, d, s, kp};
}

size_t quantize_scratch(const ggml_tensor * src1) {
    const int64_t ncols = src1->ne[1] * src1->ne[2] * src1->ne[3];
    const int64_t kp = (src1->ne[0] + 31) / 32 * 32;
    return (ncols + 8) * kp + 2 * (ncols + 8) * (kp / 32) * sizeof(float) + 3 * 256;
}

// ---------------------------------------------------------------------------
// quantised GEMV. LPR lanes cooperate on one weight row; 4 waves per block.
// Channel c = blockIdx.y spans (i12, i13); src0 broadcast by r2 = ne12/ne02.
// ---------------------------------------------------------------------------
struct MmvArgs {
    const char * w;   size_t w_row, w_c2, w_c3;     // weight base and strides (rows, dim2, dim3)
    const char * w2;                                // second weight (fused GLU up), same geometry
    float * dst;      size_t d_col, d_c2, d_c3;     // dst strides in floats
    int64_t nrows, units;
    int64_t ncols;                                  // activation columns per channel (ne11)
    int64_t ne12, r2, r3;
};

template <int QT, int NC, int LPR, bool GLU>
__global__ __launch_bounds__(256) void k_mmvq(MmvArgs p, ActQ a) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    constexpr int RPW = 64 / LPR;
    const int64_t row = ((int64_t) blockIdx.x * 4 + wave) * RPW + lane / LPR;
    const int sub = lane % LPR;
    const int64_t ch = blockIdx.y;
    const int64_t i12 = ch % p.ne12, i13 = ch / p.ne12;
    ActQ ac = a;
    const int64_t col0 = ch * p.ncols;
    ac.q += col0 * a.kp; ac.d += col0 * (a.kp / 32); ac.s += col0 * (a.kp / 32);
    float acc[NC], acc2[NC];
#pragma unroll
    for (int c = 0; c < NC; ++c) { acc[c] = 0.f; acc2[c] = 0.f; }
    if (row < p.nrows) {
        const size_t off = (size_t) row * p.w_row + (i12 / p.r2) * p.w_c2 + (i13 / p.r3) * p.w_c3;
        const char * r = p.w + off;
        const char * r2 = GLU ? p.w2 + off : nullptr;
        for (int u = sub; u < p.units; u += LPR) {
            unit_dot<QT, NC>(r, u, ac, acc);
            if constexpr (GLU) unit_dot<QT, NC>(r2, u, ac, acc2);
        }
    }
#pragma unroll
    for (int c = 0; c < NC; ++c) {
#pragma unroll
        for (int o = LPR / 2; o > 0; o >>= 1) {
            acc[c] += __shfl_xor(acc[c], o, 64);
            if constexpr (GLU) acc2[c] += __shfl_xor(acc2[c], o, 64);
        }
    }
    if (sub == 0 && row < p.nrows) {
        float * out = p.dst + i12 * p.d_c2 + i13 * p.d_c3 + row;
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            if (c < p.ncols) {
                float v = acc[c];
                if constexpr (GLU) v = (v / (1.0f + expf(-v))) * acc2[c];
                out[c * p.d_col] = v;
            }
        }
    }
}

template <int QT, int NC, bool GLU>
static void launch_mmvq_nc(OpCtx & c, const MmvArgs & p, const ActQ & a, int64_t nch) {
    const int64_t K = p.units * 32;
    // short rows: several rows per wave so every lane has work
    if (K <= 2048) {
        dim3 grid((unsigned) mx_ceil_div(p.nrows, 4 * 4), (unsigned) nch);
        k_mmvq<QT, NC, 16, GLU><<<grid, 256, 0, c.st>>>(p, a);
    } else if (K <= 8192) {
        dim3 grid((unsigned) mx_ceil_div(p.nrows, 4 * 2), (unsigned) nch);
        k_mmvq<QT, NC, 32, GLU><<<grid, 256, 0, c.st>>>(p, a);
    } else {
        dim3 grid((unsigned) mx_ceil_div(p.nrows, 4), (unsigned) nch);
        k_mmvq<QT, NC, 64, GLU><<<grid, 256, 0, c.st>>>(p, a);
    }
}

template <int QT, bool GLU>
static void launch_mmvq(OpCtx & c, const MmvArgs & p, const ActQ & a, int64_t nch) {
    switch (p.ncols) {
        case 1: launch_mmvq_nc<QT, 1, GLU>(c, p, a, nch); break;
        case 2: launch_mmvq_nc<QT, 2, GLU>(c, p, a, nch); break;
        case 3: case 4: launch_mmvq_nc<QT, 4, GLU>(c, p, a, nch); break;
        default: launch_mmvq_nc<QT, 8, GLU>(c, p, a, nch); break;
    }
}

bool mmvq_type_ok(int t) {
    return t == GGML_TYPE_Q4_K || t == GGML_TYPE_Q5_K || t == GGML_TYPE_Q6_K || t == GGML_TYPE_Q4_0 || t == GGML_TYPE_Q8_0;
}

static MmvArgs mmv_args(const ggml_tensor * w, const ggml_tensor * src1, ggml_tensor * dst) {
    MmvArgs p{};
    p.w = (const char *) w->data;
    p.w_row = w->nb[1]; p.w_c2 = w->nb[2]; p.w_c3 = w->nb[3];
    p.dst = (float *) dst->data;
    p.d_col = dst->nb[1] / 4; p.d_c2 = dst->nb[2] / 4; p.d_c3 = dst->nb[3] / 4;
    p.nrows = w->ne[1];
    p.units = w->ne[0] / 32;
    p.ncols = src1->ne[1];
    p.ne12 = src1->ne[2];
    p.r2 = src1->ne[2] / w->ne[2];
    p.r3 = src1->ne[3] / w->ne[3];
    return p;
}

template <bool GLU>
static void mmvq_dispatch(OpCtx & c, int type, const MmvArgs & p, const ActQ & a, int64_t nch) {
    switch (type) {
        case GGML_TYPE_Q4_K: launch_mmvq<GGML_TYPE_Q4_K, GLU>(c, p, a, nch); break;
        case GGML_TYPE_Q5_K: launch_mmvq<GGML_TYPE_Q5_K, GLU>(c, p, a, nch); break;
        case GGML_TYPE_Q6_K: launch_mmvq<GGML_TYPE_Q6_K, GLU>(c, p, a, nch); break;
        case GGML_TYPE_Q4_0: launch_mmvq<GGML_TYPE_Q4_0, GLU>(c, p, a, nch); break;
        case GGML_TYPE_Q8_0: launch_mmvq<GGML_TYPE_Q8_0, GLU>(c, p, a, nch); break;
        default: MX_ABORT("mmvq type %d", type);
    }
}

// dst = src0 · src1 for quantised src0 with ne11 <= 8 (src1 f32, dst f32, contiguous dst rows)
void mmvq_run(OpCtx & c, ggml_tensor * dst) {
    const ggml_tensor * w = dst->src[0];
    const ggml_tensor * x = dst->src[1];
    ActQ a = quantize_activations(c, x);
    MmvArgs p = mmv_args(w, x, dst);
    mmvq_dispatch<false>(c, w->type, p, a, x->ne[2] * x->ne[3]);
}

bool mmvq_fused_glu(OpCtx & c, const ggml_tensor * gate, const ggml_tensor * up, ggml_tensor * glu) {
    const ggml_tensor * wg = gate->src[0], * wu = up->src[0];
    const ggml_tensor * x = gate->src[1];
    if (up->src[1] != x || wg->type != wu->type || !mmvq_type_ok(wg->type)) return false;
    if (mx_op_param<int32_t>(glu, 0) != GGML_GLU_OP_SWIGLU) return false;
    if (x->type != GGML_TYPE_F32 || x->ne[1] > 8 || x->ne[2] != 1 || x->ne[3] != 1) return false;
    for (int i = 0; i < 4; ++i) if (wg->ne[i] != wu->ne[i] || wg->nb[i] != wu->nb[i]) return false;
    if (wg->ne[2] != 1 || wg->ne[3] != 1 || wg->ne[0] % qk_of_type(wg->type) != 0) return false;
    if (glu->type != GGML_TYPE_F32 || glu->nb[0] != 4 || !mx_are_same_shape(glu, gate)) return false;
    ActQ a = quantize_activations(c, x);
    MmvArgs p = mmv_args(wg, x, glu);
    p.w2 = (const char *) wu->data;
    mmvq_dispatch<true>(c, wg->type, p, a, 1);
    return true;
}

// ---------------------------------------------------------------------------
// kernel timing hook for the bench's roofline: quantise x once, then time `iters`
// back-to-back launches of exactly the GEMV kernel the executor would launch for
// MUL_MAT(w, x) (or the fused gate/up GLU when w2 != NULL) with HIP events on the
// backend's own stream. Returns the average µs per launch.
// ---------------------------------------------------------------------------
double time_mmvq(Stream * s, const ggml_tensor * w, const ggml_tensor * w2, const ggml_tensor * x, ggml_tensor * dst, int iters) {
    OpCtx c{s, s->stream, &s->scratch};
    const size_t need = quantize_scratch(x);
    if (need > s->scratch.cap) {
        HIP_CHECK(hipStreamSynchronize(s->stream));
        if (s->scratch.base) HIP_CHECK(hipFree(s->scratch.base));
        HIP_CHECK(hipMalloc((void **) &s->scratch.base, need));
        s->scratch.cap = need;
        s->gcache.key.clear();
    }
    s->scratch.reset();
    ActQ a = quantize_activations(c, x);
    MmvArgs p = mmv_args(w, x, dst);
    if (w2) p.w2 = (const char *) w2->data;
    hipEvent_t e0, e1;
    HIP_CHECK(hipEventCreate(&e0));
    HIP_CHECK(hipEventCreate(&e1));
    for (int i = 0; i < 3; ++i) {
        if (w2) mmvq_dispatch<true>(c, w->type, p, a, 1); else mmvq_dispatch<false>(c, w->type, p, a, 1);
    }
    HIP_CHECK(hipEventRecord(e0, s->stream));
    for (int i = 0; i < iters; ++i) {
        if (w2) mmvq_dispatch<true>(c, w->type, p, a, 1); else mmvq_dispatch<false>(c, w->type, p, a, 1);
    }
    HIP_CHECK(hipEventRecord(e1, s->stream));
    HIP_CHECK(hipEventSynchronize(e1));
    float ms = 0.f;
    HIP_CHECK(hipEventElapsedTime(&ms, e0, e1));
    HIP_CHECK(hipEventDestroy(e0));
    HIP_CHECK(hipEventDestroy(e1));
    return 1000.0 * ms / iters;
}

// ---------------------------------------------------------------------------
// generic GEMV: any dequantisable / float weight type, f32 activations, exact
// dequant (used for types without an sdot4 unit, and as the oracle-shaped path)
// ---------------------------------------------------------------------------
template <int QT>
__device__ __forceinline__ float w_elem(const char * row, int64_t k, size_t nb0) {
    if constexpr (QT == GGML_TYPE_F32) return *(const float *) (row + k * nb0);
    else if constexpr (QT == GGML_TYPE_F16) return h2f(*(const uint16_t *) (row + k * nb0));
    else if constexpr (QT == GGML_TYPE_BF16) return bf2f(*(const uint16_t *) (row + k * nb0));
    else return dequant_one<QT>(row + (k / qk_of<QT>()) * qsize_of<QT>(), (int) (k % qk_of<QT>()));
}

struct MmvGen {
    const char * w; size_t w_nb0, w_row, w_c2, w_c3;
    const char * x; size_t x_nb0, x_col, x_c2, x_c3;
    char * dst; size_t d_row, d_col, d_c2, d_c3;
    int64_t K, M, N, ne12, r2, r3;
};

// one wave per (row, column); K-loop strided over 64 lanes
template <int QT>
__global__ __launch_bounds__(256) void k_mmv_generic(MmvGen p) {
    const int lane = threadIdx.x & 63;
    const int64_t gw = (int64_t) blockIdx.x * 4 + (threadIdx.x >> 6);
    const int64_t row = gw % p.M, col = gw / p.M;
    if (col >= p.N) return;
    const int64_t ch = blockIdx.y;
    const int64_t i12 = ch % p.ne12, i13 = ch / p.ne12;
    const char * wr = p.w + row * p.w_row + (i12 / p.r2) * p.w_c2 + (i13 / p.r3) * p.w_c3;
    const char * xr = p.x + col * p.x_col + i12 * p.x_c2 + i13 * p.x_c3;
    float acc = 0.f;
    for (int64_t k = lane; k < p.K; k += 64) acc += w_elem<QT>(wr, k, p.w_nb0) * *(const float *) (xr + k * p.x_nb0);
    acc = wave_sum(acc);
    if (lane == 0) *(float *) (p.dst + row * p.d_row + col * p.d_col + i12 * p.d_c2 + i13 * p.d_c3) = acc;
}

void mmv_generic_run(OpCtx & c, ggml_tensor * dst) {
    const ggml_tensor * w = dst->src[0];
    const ggml_tensor * x = dst->src[1];
    MmvGen p{};
    p.w = (const char *) w->data; p.w_nb0 = w->nb[0]; p.w_row = w->nb[1]; p.w_c2 = w->nb[2]; p.w_c3 = w->nb[3];
    p.x = (const char *) x->data; p.x_nb0 = x->nb[0]; p.x_col = x->nb[1]; p.x_c2 = x->nb[2]; p.x_c3 = x->nb[3];
    p.dst = (char *) dst->data; p.d_row = dst->nb[0]; p.d_col = dst->nb[1]; p.d_c2 = dst->nb[2]; p.d_c3 = dst->nb[3];
    p.K = w->ne[0]; p.M = w->ne[1]; p.N = x->ne[1]; p.ne12 = x->ne[2];
    p.r2 = x->ne[2] / w->ne[2]; p.r3 = x->ne[3] / w->ne[3];
    dim3 grid((unsigned) mx_ceil_div(p.M * p.N, 4), (unsigned) (x->ne[2] * x->ne[3]));
    switch (w->type) {
#define GEN(T) case T: k_mmv_generic<T><<<grid, 256, 0, c.st>>>(p); break;
        GEN(GGML_TYPE_F32) GEN(GGML_TYPE_F16) GEN(GGML_TYPE_BF16)
        GEN(GGML_TYPE_Q4_0) GEN(GGML_TYPE_Q4_1) GEN(GGML_TYPE_Q5_0) GEN(GGML_TYPE_Q5_1) GEN(GGML_TYPE_Q8_0)
        GEN(GGML_TYPE_Q4_K) GEN(GGML_TYPE_Q5_K) GEN(GGML_TYPE_Q6_K)
#undef GEN
        default: MX_ABORT("mmv_generic type %d", (int) w->type);
    }
}

}  // namespace mx
