// ops_misc.hip — the non-GEMM ops of the decode/prefill graph on gfx950.
//
// Semantics follow the reference CPU backend (ggml/src/ggml-cpu/ops.cpp):
//   get_rows :4755   set_rows :4827-4875   rms_norm :3645-3694   norm :3570
//   rope :5523-5800 (rope_yarn, cache init by repeated multiply)
//   soft_max :5160-5270   swiglu :3062   binary ops binary-ops.cpp   sum_rows, argsort :7961
// Kernels are wave64, vectorised where rows are contiguous; one block per row
// for reductions.
#include "backend.h"
#include "quants.cuh"

#include <cmath>

namespace mx {

// the staged-write flush (backend.cpp stage_flush_locked): workgroup = one kFlushChunk of
// one queued range, copied from the pinned ring (zero-copy reads over PCIe)
__global__ __launch_bounds__(256) void k_stage_flush(StageFlushArgs a) {
    int k = 0;
    while (k + 1 < a.n && blockIdx.x >= a.e[k + 1].chunk0) ++k;   // workgroup-uniform
    const StageEntry e = a.e[k];
    const uint32_t off = (blockIdx.x - e.chunk0) * kFlushChunk;
    const uint32_t n = min(kFlushChunk, e.n - off);
    const char * src = e.src + off;
    char * dst = e.dst + off;
    if ((((uintptr_t) src | (uintptr_t) dst) & 15) == 0) {
        for (uint32_t i = 16 * threadIdx.x; i + 16 <= n; i += 16 * 256) *(uint4 *) (dst + i) = *(const uint4 *) (src + i);
        for (uint32_t i = (n & ~15u) + threadIdx.x; i < n; i += 256) dst[i] = src[i];
    } else {
        for (uint32_t i = threadIdx.x; i < n; i += 256) dst[i] = src[i];
    }
}

void stage_flush_launch(const StageFlushArgs & a, unsigned chunks, hipStream_t st) {
    k_stage_flush<<<chunks, 256, 0, st>>>(a);
}

struct T4 {  // geometry of one operand, passed by value
    int64_t ne[4];
    size_t nb[4];
};
static T4 geo(const ggml_tensor * t) {
    T4 g;
    for (int i = 0; i < 4; ++i) { g.ne[i] = t->ne[i]; g.nb[i] = t->nb[i]; }
    return g;
}

static inline unsigned grid_1d(int64_t n, int bs) {
    int64_t g = (n + bs - 1) / bs;
    return (unsigned) std::min<int64_t>(g, 65535LL * 64);
}

template <typename T> __device__ __forceinline__ float ld(const T * p);
template <> __device__ __forceinline__ float ld<float>(const float * p) { return *p; }
template <> __device__ __forceinline__ float ld<uint16_t>(const uint16_t * p) { return h2f(*p); }
template <typename T> __device__ __forceinline__ void st(T * p, float v);
template <> __device__ __forceinline__ void st<float>(float * p, float v) { *p = v; }
template <> __device__ __forceinline__ void st<uint16_t>(uint16_t * p, float v) { *p = f2h(v); }

// ---------------------------------------------------------------------------
// GET_ROWS: dst[:, i10, i11, i12] = dequant(src0[:, idx[i10,i11,i12], i11, i12])
// ---------------------------------------------------------------------------
// grid (rows, ne0 / 256): one element per thread, so every thread's few block-byte loads
// are in flight at once (a 256-thread block looping over a 4096-wide row paid one
// dependent memory round trip per 256 elements: 12.6 us for the decode's token row)
template <int QT>
__global__ void k_get_rows_q(const char * __restrict__ src0, const int32_t * __restrict__ idx, float * __restrict__ dst,
                             T4 s0, T4 s1, T4 d) {
    const int64_t r = blockIdx.x;  // flat index over (i10, i11, i12)
    const int64_t e = (int64_t) blockIdx.y * blockDim.x + threadIdx.x;
    if (e >= s0.ne[0]) return;
    const int64_t i10 = r % s1.ne[0];
    const int64_t i11 = (r / s1.ne[0]) % s1.ne[1];
    const int64_t i12 = r / (s1.ne[0] * s1.ne[1]);
    const int32_t i01 = *(const int32_t *) ((const char *) idx + i10 * s1.nb[0] + i11 * s1.nb[1] + i12 * s1.nb[2]);
    const char * row = src0 + i01 * s0.nb[1] + i11 * s0.nb[2] + i12 * s0.nb[3];
    float * out = (float *) ((char *) dst + i10 * d.nb[1] + i11 * d.nb[2] + i12 * d.nb[3]);
    out[e] = dequant_one<QT>(row + (e / qk_of<QT>()) * qsize_of<QT>(), (int) (e % qk_of<QT>()));
}

template <typename TS, typename TD>
__global__ void k_get_rows_f(const char * __restrict__ src0, const int32_t * __restrict__ idx, char * __restrict__ dst,
                             T4 s0, T4 s1, T4 d) {
    const int64_t r = blockIdx.x;
    const int64_t i10 = r % s1.ne[0];
    const int64_t i11 = (r / s1.ne[0]) % s1.ne[1];
    const int64_t i12 = r / (s1.ne[0] * s1.ne[1]);
    const int32_t i01 = *(const int32_t *) ((const char *) idx + i10 * s1.nb[0] + i11 * s1.nb[1] + i12 * s1.nb[2]);
    const char * row = src0 + i01 * s0.nb[1] + i11 * s0.nb[2] + i12 * s0.nb[3];
    char * out = dst + i10 * d.nb[1] + i11 * d.nb[2] + i12 * d.nb[3];
    for (int64_t e = threadIdx.x; e < s0.ne[0]; e += blockDim.x) {
        const TS * p = (const TS *) (row + e * s0.nb[0]);
        TD * q = (TD *) (out + e * d.nb[0]);
        if constexpr (std::is_same<TS, TD>::value) *q = *p;
        else st<TD>(q, ld<TS>(p));
    }
}

void op_get_rows(OpCtx & c, ggml_tensor * dst) {
    const ggml_tensor * s0 = dst->src[0];
    const ggml_tensor * s1 = dst->src[1];
    const int64_t nr = s1->ne[0] * s1->ne[1] * s1->ne[2];
    if (nr == 0) return;
    const dim3 grid((unsigned) nr), blk(256);
    T4 g0 = geo(s0), g1 = geo(s1), gd = geo(dst);
    const char * a = (const char *) s0->data;
    const int32_t * ix = (const int32_t *) s1->data;
    switch (s0->type) {
#define GR_Q(T) case T: MX_ASSERT(dst->type == GGML_TYPE_F32 && nr < 65536 * 1024); \
        k_get_rows_q<T><<<dim3((unsigned) nr, (unsigned) mx_ceil_div(s0->ne[0], 256)), blk, 0, c.st>>>(a, ix, (float *) dst->data, g0, g1, gd); break;
        GR_Q(GGML_TYPE_Q4_0) GR_Q(GGML_TYPE_Q4_1) GR_Q(GGML_TYPE_Q5_0) GR_Q(GGML_TYPE_Q5_1) GR_Q(GGML_TYPE_Q8_0)
        GR_Q(GGML_TYPE_Q4_K) GR_Q(GGML_TYPE_Q5_K) GR_Q(GGML_TYPE_Q6_K)
#undef GR_Q
        case GGML_TYPE_F32:
            if (dst->type == GGML_TYPE_F32) k_get_rows_f<float, float><<<grid, blk, 0, c.st>>>(a, ix, (char *) dst->data, g0, g1, gd);
            else k_get_rows_f<float, uint16_t><<<grid, blk, 0, c.st>>>(a, ix, (char *) dst->data, g0, g1, gd);
            break;
        case GGML_TYPE_F16:
            if (dst->type == GGML_TYPE_F32) k_get_rows_f<uint16_t, float><<<grid, blk, 0, c.st>>>(a, ix, (char *) dst->data, g0, g1, gd);
            else k_get_rows_f<uint16_t, uint16_t><<<grid, blk, 0, c.st>>>(a, ix, (char *) dst->data, g0, g1, gd);
            break;
        case GGML_TYPE_I32:
            k_get_rows_f<int32_t, int32_t><<<grid, blk, 0, c.st>>>(a, ix, (char *) dst->data, g0, g1, gd);
            break;
        default: MX_ABORT("get_rows: type %d", (int) s0->type);
    }
}

// ---------------------------------------------------------------------------
// SET_ROWS: dst[:, idx[i, i02%ne11, i03%ne12], i02, i03] = from_float(src0[:, i, i02, i03])
// f32 → f16 uses round-to-nearest-even, bit-identical to the CPU's F16C path.
// ---------------------------------------------------------------------------
template <typename TI, typename TD>
__global__ void k_set_rows(const char * __restrict__ src, const char * __restrict__ idx, char * __restrict__ dst,
                           T4 s0, T4 s1, T4 d) {
    const int64_t r = blockIdx.x;  // over (i, i02, i03)
    const int64_t i = r % s0.ne[1];
    const int64_t i02 = (r / s0.ne[1]) % s0.ne[2];
    const int64_t i03 = r / (s0.ne[1] * s0.ne[2]);
    const int64_t i11 = i02 % s1.ne[1], i12 = i03 % s1.ne[2];
    const int64_t i1 = (int64_t) *(const TI *) (idx + i * s1.nb[0] + i11 * s1.nb[1] + i12 * s1.nb[2]);
    const float * in = (const float *) (src + i * s0.nb[1] + i02 * s0.nb[2] + i03 * s0.nb[3]);
    TD * out = (TD *) (dst + i1 * d.nb[1] + i02 * d.nb[2] + i03 * d.nb[3]);
    for (int64_t e = threadIdx.x; e < s0.ne[0]; e += blockDim.x) {
        if constexpr (std::is_same<TD, float>::value) out[e] = in[e];
        else if constexpr (std::is_same<TD, uint16_t>::value) out[e] = f2h(in[e]);
        else out[e] = f2bf(in[e]);
    }
}
struct bf16_t { uint16_t v; };
template <typename TI>
__global__ void k_set_rows_bf16(const char * __restrict__ src, const char * __restrict__ idx, char * __restrict__ dst,
                                T4 s0, T4 s1, T4 d) {
    const int64_t r = blockIdx.x;
    const int64_t i = r % s0.ne[1];
    const int64_t i02 = (r / s0.ne[1]) % s0.ne[2];
    const int64_t i03 = r / (s0.ne[1] * s0.ne[2]);
    const int64_t i11 = i02 % s1.ne[1], i12 = i03 % s1.ne[2];
    const int64_t i1 = (int64_t) *(const TI *) (idx + i * s1.nb[0] + i11 * s1.nb[1] + i12 * s1.nb[2]);
    const float * in = (const float *) (src + i * s0.nb[1] + i02 * s0.nb[2] + i03 * s0.nb[3]);
    uint16_t * out = (uint16_t *) (dst + i1 * d.nb[1] + i02 * d.nb[2] + i03 * d.nb[3]);
    for (int64_t e = threadIdx.x; e < s0.ne[0]; e += blockDim.x) out[e] = f2bf(in[e]);
}
// f32 → q8_0 rows (quantised KV cache, quantize_row_q8_0_ref ggml-quants.c:199-226)
template <typename TI>
__global__ void k_set_rows_q8_0(const char * __restrict__ src, const char * __restrict__ idx, char * __restrict__ dst,
                                T4 s0, T4 s1, T4 d) {
    const int64_t r = blockIdx.x;
    const int64_t i = r % s0.ne[1];
    const int64_t i02 = (r / s0.ne[1]) % s0.ne[2];
    const int64_t i03 = r / (s0.ne[1] * s0.ne[2]);
    const int64_t i11 = i02 % s1.ne[1], i12 = i03 % s1.ne[2];
    const int64_t i1 = (int64_t) *(const TI *) (idx + i * s1.nb[0] + i11 * s1.nb[1] + i12 * s1.nb[2]);
    const float * in = (const float *) (src + i * s0.nb[1] + i02 * s0.nb[2] + i03 * s0.nb[3]);
    char * out = dst + i1 * d.nb[1] + i02 * d.nb[2] + i03 * d.nb[3];
    const int nblk = (int) (s0.ne[0] / 32);
    for (int b = threadIdx.x; b < nblk; b += blockDim.x) quantize_block_q8_0(in + 32 * b, out + 34 * b);
}

// q4_0 caches (-ctk / -ctv q4_0): the same with quantize_block_q4_0 (18-B blocks)
template <typename TI>
__global__ void k_set_rows_q4_0(const char * __restrict__ src, const char * __restrict__ idx, char * __restrict__ dst,
                                T4 s0, T4 s1, T4 d) {
    const int64_t r = blockIdx.x;
    const int64_t i = r % s0.ne[1];
    const int64_t i02 = (r / s0.ne[1]) % s0.ne[2];
    const int64_t i03 = r / (s0.ne[1] * s0.ne[2]);
    const int64_t i11 = i02 % s1.ne[1], i12 = i03 % s1.ne[2];
    const int64_t i1 = (int64_t) *(const TI *) (idx + i * s1.nb[0] + i11 * s1.nb[1] + i12 * s1.nb[2]);
    const float * in = (const float *) (src + i * s0.nb[1] + i02 * s0.nb[2] + i03 * s0.nb[3]);
    char * out = dst + i1 * d.nb[1] + i02 * d.nb[2] + i03 * d.nb[3];
    const int nblk = (int) (s0.ne[0] / 32);
    for (int b = threadIdx.x; b < nblk; b += blockDim.x) quantize_block_q4_0(in + 32 * b, out + 18 * b);
}

// SET_ROWS of one-element rows: the transposed V cache store of the non-flash-attention
// graph (src/llama-kv-cache.cpp cpy_v with v_trans: v_cur [n_embd_v, n_tokens] reshaped to
// [1, n_embd_v * n_tokens], one index per element, element (d, t) -> row d * kv_size +
// cell(t)). A workgroup per row (the general kernel) made that 524,288 workgroups of one
// 2-byte store at pp512: 92 us per layer. Here a workgroup takes a tile of 32 tokens x 64
// dimensions of the flat index i = t * R + d (R = n_embd_v, the row length before the
// reshape), reads values and indices along d (coalesced), transposes through LDS and
// stores along t, so consecutive lanes write consecutive cache cells. Any index values
// are handled (it only permutes which lane stores which element).
template <typename TI, typename TD>
__global__ __launch_bounds__(256) void k_set_elems(const float * __restrict__ src, const TI * __restrict__ idx, char * __restrict__ dst,
                                                   size_t dnb1, int64_t n, int64_t R) {
    __shared__ float val[32][65];
    __shared__ int64_t ind[32][65];
    const int64_t d0 = (int64_t) blockIdx.x * 64, t0 = (int64_t) blockIdx.y * 32;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        const int l = threadIdx.x + 256 * e, dl = l & 63, tl = l >> 6;
        const int64_t d = d0 + dl, i = (t0 + tl) * R + d;
        const bool ok = d < R && i < n;
        val[tl][dl] = ok ? src[i] : 0.f;
        ind[tl][dl] = ok ? (int64_t) idx[i] : -1;
    }
    __syncthreads();
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        const int l = threadIdx.x + 256 * e, tl = l & 31, dl = l >> 5;
        const int64_t r = ind[tl][dl];
        if (r < 0) continue;
        TD * o = (TD *) (dst + (size_t) r * dnb1);
        if constexpr (std::is_same<TD, float>::value) *o = val[tl][dl];
        else *o = f2h(val[tl][dl]);
    }
}

void op_set_rows(OpCtx & c, ggml_tensor * dst) {
    const ggml_tensor * s0 = dst->src[0];
    const ggml_tensor * s1 = dst->src[1];
    const int64_t nr = s0->ne[1] * s0->ne[2] * s0->ne[3];
    if (nr == 0) return;
    if (s0->ne[0] == 1 && s0->ne[2] == 1 && s0->ne[3] == 1 && s0->type == GGML_TYPE_F32 && s0->nb[1] == 4 && s1->ne[0] == nr &&
        s1->nb[0] == (size_t) mx_type(s1->type).size && (dst->type == GGML_TYPE_F16 || dst->type == GGML_TYPE_F32)) {
        // the row length before libllama's reshape to [1, n] (the transposed V store): the
        // tile shape for coalesced stores; any value is correct
        int64_t R = 64;
        if ((s0->op == GGML_OP_RESHAPE || s0->op == GGML_OP_VIEW) && s0->src[0] && s0->src[0]->ne[0] > 1) R = s0->src[0]->ne[0];
        const dim3 grid((unsigned) mx_ceil_div(R, 64), (unsigned) mx_ceil_div(mx_ceil_div(nr, R), 32));
        MX_KLOG("set_elems n=%lld R=%lld type=%d", (long long) nr, (long long) R, (int) dst->type);
        const float * a = (const float *) s0->data;
        char * o = (char *) dst->data;
#define SE(TI, TD) k_set_elems<TI, TD><<<grid, 256, 0, c.st>>>(a, (const TI *) s1->data, o, dst->nb[1], nr, R)
        if (s1->type == GGML_TYPE_I64) { if (dst->type == GGML_TYPE_F16) SE(int64_t, uint16_t); else SE(int64_t, float); }
        else { if (dst->type == GGML_TYPE_F16) SE(int32_t, uint16_t); else SE(int32_t, float); }
#undef SE
        return;
    }
    const dim3 grid((unsigned) nr), blk(s0->ne[0] >= 256 ? 256 : 64);
    T4 g0 = geo(s0), g1 = geo(s1), gd = geo(dst);
    const char * a = (const char *) s0->data;
    const char * ix = (const char *) s1->data;
    char * o = (char *) dst->data;
    const bool i64 = s1->type == GGML_TYPE_I64;
    switch (dst->type) {
        case GGML_TYPE_F32:
            if (i64) k_set_rows<int64_t, float><<<grid, blk, 0, c.st>>>(a, ix, o, g0, g1, gd);
            else     k_set_rows<int32_t, float><<<grid, blk, 0, c.st>>>(a, ix, o, g0, g1, gd);
            break;
        case GGML_TYPE_F16:
            if (i64) k_set_rows<int64_t, uint16_t><<<grid, blk, 0, c.st>>>(a, ix, o, g0, g1, gd);
            else     k_set_rows<int32_t, uint16_t><<<grid, blk, 0, c.st>>>(a, ix, o, g0, g1, gd);
            break;
        case GGML_TYPE_BF16:
            if (i64) k_set_rows_bf16<int64_t><<<grid, blk, 0, c.st>>>(a, ix, o, g0, g1, gd);
            else     k_set_rows_bf16<int32_t><<<grid, blk, 0, c.st>>>(a, ix, o, g0, g1, gd);
            break;
        case GGML_TYPE_Q8_0:
            if (i64) k_set_rows_q8_0<int64_t><<<grid, dim3(64), 0, c.st>>>(a, ix, o, g0, g1, gd);
            else     k_set_rows_q8_0<int32_t><<<grid, dim3(64), 0, c.st>>>(a, ix, o, g0, g1, gd);
            break;
        case GGML_TYPE_Q4_0:
            if (i64) k_set_rows_q4_0<int64_t><<<grid, dim3(64), 0, c.st>>>(a, ix, o, g0, g1, gd);
            else     k_set_rows_q4_0<int32_t><<<grid, dim3(64), 0, c.st>>>(a, ix, o, g0, g1, gd);
            break;
        default: MX_ABORT("set_rows: dst type %d", (int) dst->type);
    }
}

// ---------------------------------------------------------------------------
// CPY / CONT / DUP: element i of the flattened logical order of src goes to
// element i of dst (shapes may differ, nelements equal — ggml_cpy semantics)
// ---------------------------------------------------------------------------
template <typename TS, typename TD>
__global__ void k_cpy(const char * __restrict__ src, char * __restrict__ dst, T4 s, T4 d, int64_t n) {
    for (int64_t i = blockIdx.x * (int64_t) blockDim.x + threadIdx.x; i < n; i += (int64_t) gridDim.x * blockDim.x) {
        int64_t r = i;
        const int64_t a0 = r % s.ne[0]; r /= s.ne[0];
        const int64_t a1 = r % s.ne[1]; r /= s.ne[1];
        const int64_t a2 = r % s.ne[2]; const int64_t a3 = r / s.ne[2];
        r = i;
        const int64_t b0 = r % d.ne[0]; r /= d.ne[0];
        const int64_t b1 = r % d.ne[1]; r /= d.ne[1];
        const int64_t b2 = r % d.ne[2]; const int64_t b3 = r / d.ne[2];
        const TS * p = (const TS *) (src + a0 * s.nb[0] + a1 * s.nb[1] + a2 * s.nb[2] + a3 * s.nb[3]);
        TD * q = (TD *) (dst + b0 * d.nb[0] + b1 * d.nb[1] + b2 * d.nb[2] + b3 * d.nb[3]);
        if constexpr (std::is_same<TS, TD>::value) *q = *p;
        else if constexpr (std::is_same<TS, float>::value && std::is_same<TD, bf16_t>::value) q->v = f2bf(*p);
        else if constexpr (std::is_same<TS, bf16_t>::value && std::is_same<TD, float>::value) *q = bf2f(p->v);
        else st<TD>(q, ld<TS>(p));
    }
}
// contiguous same-type copy
__global__ void k_copy_bytes(const uint4 * __restrict__ src, uint4 * __restrict__ dst, int64_t n16) {
    for (int64_t i = blockIdx.x * (int64_t) blockDim.x + threadIdx.x; i < n16; i += (int64_t) gridDim.x * blockDim.x) dst[i] = src[i];
}
// f32 rows → q8_0 rows (contiguous), ggml_cpy to a quantised tensor
__global__ void k_cpy_f32_q8_0(const float * __restrict__ src, char * __restrict__ dst, int64_t nblk) {
    for (int64_t b = blockIdx.x * (int64_t) blockDim.x + threadIdx.x; b < nblk; b += (int64_t) gridDim.x * blockDim.x)
        quantize_block_q8_0(src + 32 * b, dst + 34 * b);
}

void op_cpy(OpCtx & c, const ggml_tensor * src, ggml_tensor * dst) {
    const int64_t n = mx_nelements(src);
    if (n == 0) return;
    if (src->type == dst->type && mx_is_contiguous(src) && mx_is_contiguous(dst)) {
        const size_t bytes = mx_nbytes(src);
        if (bytes % 16 == 0 && ((uintptr_t) src->data % 16 == 0) && ((uintptr_t) dst->data % 16 == 0)) {
            const int64_t n16 = bytes / 16;
            k_copy_bytes<<<grid_1d(n16, 256), 256, 0, c.st>>>((const uint4 *) src->data, (uint4 *) dst->data, n16);
        } else {
            HIP_CHECK(hipMemcpyAsync(dst->data, src->data, bytes, hipMemcpyDeviceToDevice, c.st));
        }
        return;
    }
    T4 gs = geo(src), gd = geo(dst);
    const unsigned g = grid_1d(n, 256);
    const char * a = (const char *) src->data;
    char * o = (char *) dst->data;
#define CP(TS, TD) k_cpy<TS, TD><<<g, 256, 0, c.st>>>(a, o, gs, gd, n)
    if (src->type == GGML_TYPE_F32 && dst->type == GGML_TYPE_F32) CP(float, float);
    else if (src->type == GGML_TYPE_F32 && dst->type == GGML_TYPE_F16) CP(float, uint16_t);
    else if (src->type == GGML_TYPE_F16 && dst->type == GGML_TYPE_F32) CP(uint16_t, float);
    else if (src->type == GGML_TYPE_F16 && dst->type == GGML_TYPE_F16) CP(uint16_t, uint16_t);
    else if (src->type == GGML_TYPE_F32 && dst->type == GGML_TYPE_BF16) CP(float, bf16_t);
    else if (src->type == GGML_TYPE_BF16 && dst->type == GGML_TYPE_F32) CP(bf16_t, float);
    else if (src->type == GGML_TYPE_BF16 && dst->type == GGML_TYPE_BF16) CP(uint16_t, uint16_t);
    else if (src->type == GGML_TYPE_I32 && dst->type == GGML_TYPE_I32) CP(int32_t, int32_t);
    else if (src->type == GGML_TYPE_F32 && dst->type == GGML_TYPE_Q8_0 && mx_is_contiguous(src) && mx_is_contiguous(dst)) {
        const int64_t nb = n / 32;
        k_cpy_f32_q8_0<<<grid_1d(nb, 256), 256, 0, c.st>>>((const float *) src->data, o, nb);
    }
    else MX_ABORT("cpy: %d -> %d", (int) src->type, (int) dst->type);
#undef CP
}

// ---------------------------------------------------------------------------
// binary ops with src1 broadcast (ggml_can_repeat(src1, src0))
// ---------------------------------------------------------------------------
template <int OP, typename T0, typename T1, typename TD>
__global__ void k_binary(const char * __restrict__ a, const char * __restrict__ b, char * __restrict__ d,
                         T4 ga, T4 gb, T4 gd) {
    // one block-row per (i1, i2, i3); threads stride over i0
    const int64_t r = blockIdx.x;
    const int64_t i1 = r % gd.ne[1];
    const int64_t i2 = (r / gd.ne[1]) % gd.ne[2];
    const int64_t i3 = r / (gd.ne[1] * gd.ne[2]);
    const char * pa = a + i1 * ga.nb[1] + i2 * ga.nb[2] + i3 * ga.nb[3];
    const char * pb = b + (i1 % gb.ne[1]) * gb.nb[1] + (i2 % gb.ne[2]) * gb.nb[2] + (i3 % gb.ne[3]) * gb.nb[3];
    char * pd = d + i1 * gd.nb[1] + i2 * gd.nb[2] + i3 * gd.nb[3];
    for (int64_t i0 = threadIdx.x; i0 < gd.ne[0]; i0 += blockDim.x) {
        const float x = ld<T0>((const T0 *) (pa + i0 * ga.nb[0]));
        const float y = ld<T1>((const T1 *) (pb + (i0 % gb.ne[0]) * gb.nb[0]));
        float z;
        if constexpr (OP == GGML_OP_ADD) z = x + y;
        else if constexpr (OP == GGML_OP_SUB) z = x - y;
        else if constexpr (OP == GGML_OP_MUL) z = x * y;
        else z = x / y;
        st<TD>((TD *) (pd + i0 * gd.nb[0]), z);
    }
}
// fast path: all f32, contiguous rows, src1 row broadcast only along rows
template <int OP>
__global__ void k_binary_f32_rows(const float * __restrict__ a, const float * __restrict__ b, float * __restrict__ d,
                                  int64_t ne0, int64_t nb_ne0, int64_t n) {
    for (int64_t i = blockIdx.x * (int64_t) blockDim.x + threadIdx.x; i < n; i += (int64_t) gridDim.x * blockDim.x) {
        const float x = a[i];
        const float y = b[i % nb_ne0];
        float z;
        if constexpr (OP == GGML_OP_ADD) z = x + y;
        else if constexpr (OP == GGML_OP_SUB) z = x - y;
        else if constexpr (OP == GGML_OP_MUL) z = x * y;
        else z = x / y;
        d[i] = z;
    }
    (void) ne0;
}

template <int OP>
static void binary_dispatch(OpCtx & c, ggml_tensor * dst) {
    const ggml_tensor * a = dst->src[0];
    const ggml_tensor * b = dst->src[1];
    const int64_t nr = mx_nrows(dst);
    if (nr == 0 || dst->ne[0] == 0) return;
    const bool all32 = a->type == GGML_TYPE_F32 && b->type == GGML_TYPE_F32 && dst->type == GGML_TYPE_F32;
    // b is a contiguous prefix that tiles a (e.g. [ne0] or [ne0, ne1] broadcast over higher dims)
    if (all32 && mx_is_contiguous(a) && mx_is_contiguous(b) && mx_is_contiguous(dst) &&
        ((b->ne[1] == 1 && b->ne[2] == 1 && b->ne[3] == 1 && b->ne[0] == a->ne[0]) || mx_are_same_shape(a, b))) {
        const int64_t n = mx_nelements(dst);
        k_binary_f32_rows<OP><<<grid_1d(n, 256), 256, 0, c.st>>>((const float *) a->data, (const float *) b->data,
                                                                  (float *) dst->data, a->ne[0], mx_nelements(b), n);
        return;
    }
    const dim3 grid((unsigned) nr), blk(dst->ne[0] >= 256 ? 256 : 64);
    T4 ga = geo(a), gb = geo(b), gd = geo(dst);
    const char * pa = (const char *) a->data;
    const char * pb = (const char *) b->data;
    char * pd = (char *) dst->data;
#define BIN(T0, T1, TD) k_binary<OP, T0, T1, TD><<<grid, blk, 0, c.st>>>(pa, pb, pd, ga, gb, gd)
    const int t0 = a->type, t1 = b->type, td = dst->type;
    if (t0 == GGML_TYPE_F32 && t1 == GGML_TYPE_F32 && td == GGML_TYPE_F32) BIN(float, float, float);
    else if (t0 == GGML_TYPE_F16 && t1 == GGML_TYPE_F32 && td == GGML_TYPE_F16) BIN(uint16_t, float, uint16_t);
    else if (t0 == GGML_TYPE_F16 && t1 == GGML_TYPE_F16 && td == GGML_TYPE_F16) BIN(uint16_t, uint16_t, uint16_t);
    else if (t0 == GGML_TYPE_F16 && t1 == GGML_TYPE_F32 && td == GGML_TYPE_F32) BIN(uint16_t, float, float);
    else if (t0 == GGML_TYPE_F32 && t1 == GGML_TYPE_F16 && td == GGML_TYPE_F32) BIN(float, uint16_t, float);
    else MX_ABORT("binary op types %d %d %d", t0, t1, td);
#undef BIN
}

void op_binary(OpCtx & c, ggml_tensor * dst) {
    switch (dst->op) {
        case GGML_OP_ADD: binary_dispatch<GGML_OP_ADD>(c, dst); break;
        case GGML_OP_SUB: binary_dispatch<GGML_OP_SUB>(c, dst); break;
        case GGML_OP_MUL: binary_dispatch<GGML_OP_MUL>(c, dst); break;
        case GGML_OP_DIV: binary_dispatch<GGML_OP_DIV>(c, dst); break;
        default: MX_ABORT("binary op %d", (int) dst->op);
    }
}

// ---------------------------------------------------------------------------
// SCALE / CLAMP / UNARY — f32, strided
// ---------------------------------------------------------------------------
__device__ __forceinline__ float act_silu(float x) { return x / (1.0f + expf(-x)); }
__device__ __forceinline__ float act_gelu(float x) {
    return 0.5f * x * (1.0f + tanhf(0.79788456080286535587989211986876f * x * (1.0f + 0.044715f * x * x)));
}
__device__ __forceinline__ float act_gelu_quick(float x) { return x * (1.0f / (1.0f + expf(-1.702f * x))); }
__device__ __forceinline__ float act_gelu_erf(float x) { return 0.5f * x * (1.0f + erff(x * 0.70710678118654752440f)); }

template <int MODE>  // 0 scale, 1 clamp, 2 unary
__global__ void k_map(const char * __restrict__ a, char * __restrict__ d, T4 ga, T4 gd, float p0, float p1, int uop, int64_t n) {
    for (int64_t i = blockIdx.x * (int64_t) blockDim.x + threadIdx.x; i < n; i += (int64_t) gridDim.x * blockDim.x) {
        int64_t r = i;
        const int64_t i0 = r % gd.ne[0]; r /= gd.ne[0];
        const int64_t i1 = r % gd.ne[1]; r /= gd.ne[1];
        const int64_t i2 = r % gd.ne[2]; const int64_t i3 = r / gd.ne[2];
        const float x = *(const float *) (a + i0 * ga.nb[0] + i1 * ga.nb[1] + i2 * ga.nb[2] + i3 * ga.nb[3]);
        float y;
        if constexpr (MODE == 0) y = x * p0 + p1;
        else if constexpr (MODE == 1) y = fminf(fmaxf(x, p0), p1);
        else {
            switch (uop) {
                case GGML_UNARY_OP_ABS: y = fabsf(x); break;
                case GGML_UNARY_OP_SGN: y = x > 0.f ? 1.f : (x < 0.f ? -1.f : 0.f); break;
                case GGML_UNARY_OP_NEG: y = -x; break;
                case GGML_UNARY_OP_STEP: y = x > 0.f ? 1.f : 0.f; break;
                case GGML_UNARY_OP_TANH: y = tanhf(x); break;
                case GGML_UNARY_OP_ELU: y = x > 0.f ? x : expm1f(x); break;
                case GGML_UNARY_OP_RELU: y = fmaxf(x, 0.f); break;
                case GGML_UNARY_OP_SIGMOID: y = 1.f / (1.f + expf(-x)); break;
                case GGML_UNARY_OP_GELU: y = act_gelu(x); break;
                case GGML_UNARY_OP_GELU_QUICK: y = act_gelu_quick(x); break;
                case GGML_UNARY_OP_SILU: y = act_silu(x); break;
                case GGML_UNARY_OP_HARDSWISH: y = x * fminf(1.0f, fmaxf(0.0f, (x + 3.0f) / 6.0f)); break;
                case GGML_UNARY_OP_HARDSIGMOID: y = fminf(1.0f, fmaxf(0.0f, (x + 3.0f) / 6.0f)); break;
                case GGML_UNARY_OP_EXP: y = expf(x); break;
                case GGML_UNARY_OP_GELU_ERF: y = act_gelu_erf(x); break;
                default: y = x; break;
            }
        }
        *(float *) (d + i0 * gd.nb[0] + i1 * gd.nb[1] + i2 * gd.nb[2] + i3 * gd.nb[3]) = y;
    }
}

static bool unary_supported(int u) {
    switch (u) {
        case GGML_UNARY_OP_ABS: case GGML_UNARY_OP_SGN: case GGML_UNARY_OP_NEG: case GGML_UNARY_OP_STEP:
        case GGML_UNARY_OP_TANH: case GGML_UNARY_OP_ELU: case GGML_UNARY_OP_RELU: case GGML_UNARY_OP_SIGMOID:
        case GGML_UNARY_OP_GELU: case GGML_UNARY_OP_GELU_QUICK: case GGML_UNARY_OP_SILU:
        case GGML_UNARY_OP_HARDSWISH: case GGML_UNARY_OP_HARDSIGMOID: case GGML_UNARY_OP_EXP:
        case GGML_UNARY_OP_GELU_ERF: return true;
        default: return false;
    }
}

void op_scale(OpCtx & c, ggml_tensor * dst) {
    const int64_t n = mx_nelements(dst);
    k_map<0><<<grid_1d(n, 256), 256, 0, c.st>>>((const char *) dst->src[0]->data, (char *) dst->data, geo(dst->src[0]), geo(dst),
                                                 mx_op_param<float>(dst, 0), mx_op_param<float>(dst, 1), 0, n);
}
void op_clamp(OpCtx & c, ggml_tensor * dst) {
    const int64_t n = mx_nelements(dst);
    k_map<1><<<grid_1d(n, 256), 256, 0, c.st>>>((const char *) dst->src[0]->data, (char *) dst->data, geo(dst->src[0]), geo(dst),
                                                 mx_op_param<float>(dst, 0), mx_op_param<float>(dst, 1), 0, n);
}
void op_unary(OpCtx & c, ggml_tensor * dst) {
    const int64_t n = mx_nelements(dst);
    k_map<2><<<grid_1d(n, 256), 256, 0, c.st>>>((const char *) dst->src[0]->data, (char *) dst->data, geo(dst->src[0]), geo(dst),
                                                 0.f, 0.f, mx_op_param<int32_t>(dst, 0), n);
}

// ---------------------------------------------------------------------------
// GLU (swiglu / geglu / reglu), split or fused-halves form
// ---------------------------------------------------------------------------
template <int GOP>
__global__ void k_glu(const char * __restrict__ a, const char * __restrict__ b, float * __restrict__ d,
                      size_t nba, size_t nbb, size_t nbd, int64_t nc, int64_t nrows) {
    const int64_t row = blockIdx.y;
    const float * x = (const float *) (a + row * nba);
    const float * g = (const float *) (b + row * nbb);
    float * o = (float *) ((char *) d + row * nbd);
    for (int64_t i = blockIdx.x * (int64_t) blockDim.x + threadIdx.x; i < nc; i += (int64_t) gridDim.x * blockDim.x) {
        const float v = x[i];
        float act;
        if constexpr (GOP == GGML_GLU_OP_SWIGLU) act = act_silu(v);
        else if constexpr (GOP == GGML_GLU_OP_GEGLU) act = act_gelu(v);
        else if constexpr (GOP == GGML_GLU_OP_REGLU) act = fmaxf(v, 0.f);
        else if constexpr (GOP == GGML_GLU_OP_GEGLU_ERF) act = act_gelu_erf(v);
        else act = act_gelu_quick(v);
        o[i] = act * g[i];
    }
    (void) nrows;
}

void op_glu(OpCtx & c, ggml_tensor * dst) {
    const ggml_tensor * s0 = dst->src[0];
    const ggml_tensor * s1 = dst->src[1];
    const int gop = mx_op_param<int32_t>(dst, 0);
    const bool swapped = mx_op_param<int32_t>(dst, 1) != 0;
    const int64_t nc = s1 ? s0->ne[0] : s0->ne[0] / 2;
    const int64_t nr = mx_nrows(s0);
    const char * pa = (const char *) s0->data;
    const char * pb = s1 ? (const char *) s1->data : (const char *) s0->data;
    if (!s1) {
        if (swapped) pa += nc * sizeof(float); else pb += nc * sizeof(float);
    }
    const size_t nba = s0->nb[1], nbb = s1 ? s1->nb[1] : s0->nb[1];
    dim3 grid((unsigned) std::min<int64_t>(mx_ceil_div(nc, 256), 64), (unsigned) nr);
#define G(OP) k_glu<OP><<<grid, 256, 0, c.st>>>(pa, pb, (float *) dst->data, nba, nbb, dst->nb[1], nc, nr)
    switch (gop) {
        case GGML_GLU_OP_SWIGLU: G(GGML_GLU_OP_SWIGLU); break;
        case GGML_GLU_OP_GEGLU: G(GGML_GLU_OP_GEGLU); break;
        case GGML_GLU_OP_REGLU: G(GGML_GLU_OP_REGLU); break;
        case GGML_GLU_OP_GEGLU_ERF: G(GGML_GLU_OP_GEGLU_ERF); break;
        case GGML_GLU_OP_GEGLU_QUICK: G(GGML_GLU_OP_GEGLU_QUICK); break;
        default: MX_ABORT("glu op %d", gop);
    }
#undef G
}

// ---------------------------------------------------------------------------
// RMS_NORM (+ optional fused MUL by a broadcast weight): one block per row.
// CPU accumulates Σx² in double (ops.cpp:3671); a wave64 tree sum in f32 is
// within the 1e-7 NMSE bound the reference parity harness uses.
// ---------------------------------------------------------------------------
template <bool MUL>
__global__ void k_rms_norm(const char * __restrict__ x, const char * __restrict__ w, char * __restrict__ y,
                           T4 gx, T4 gw, T4 gy, float eps) {
    __shared__ float lds[16];
    const int64_t r = blockIdx.x;
    const int64_t i1 = r % gx.ne[1], i2 = (r / gx.ne[1]) % gx.ne[2], i3 = r / (gx.ne[1] * gx.ne[2]);
    const float * px = (const float *) (x + i1 * gx.nb[1] + i2 * gx.nb[2] + i3 * gx.nb[3]);
    float * py = (float *) (y + i1 * gy.nb[1] + i2 * gy.nb[2] + i3 * gy.nb[3]);
    const int64_t n = gx.ne[0];
    float s = 0.f;
    for (int64_t i = threadIdx.x; i < n; i += blockDim.x) { const float v = px[i]; s += v * v; }
    s = block_sum(s, lds);
    const float scale = 1.0f / sqrtf(s / (float) n + eps);
    if constexpr (MUL) {
        const float * pw = (const float *) (w + (i1 % gw.ne[1]) * gw.nb[1] + (i2 % gw.ne[2]) * gw.nb[2] + (i3 % gw.ne[3]) * gw.nb[3]);
        for (int64_t i = threadIdx.x; i < n; i += blockDim.x) py[i] = (px[i] * scale) * pw[i];
    } else {
        for (int64_t i = threadIdx.x; i < n; i += blockDim.x) py[i] = px[i] * scale;
    }
}

// Rows of n % 4 == 0 floats, 16-byte aligned: each thread holds its VPT float4s in
// registers between the sum and the scale (one read of x instead of two) and moves
// 16 bytes per access (k_rms_norm: 4-byte accesses, x read twice: 9.4 µs per pp512
// norm against ~3 µs of traffic).
template <bool MUL, int VPT>
__global__ __launch_bounds__(256) void k_rms_norm_v4(const char * __restrict__ x, const char * __restrict__ w, char * __restrict__ y,
                                                     T4 gx, T4 gw, T4 gy, float eps, _Float16 * __restrict__ h) {
    __shared__ float lds[16];
    const int64_t r = blockIdx.x;
    const int64_t i1 = r % gx.ne[1], i2 = (r / gx.ne[1]) % gx.ne[2], i3 = r / (gx.ne[1] * gx.ne[2]);
    const float4 * px = (const float4 *) (x + i1 * gx.nb[1] + i2 * gx.nb[2] + i3 * gx.nb[3]);
    float4 * py = (float4 *) (y + i1 * gy.nb[1] + i2 * gy.nb[2] + i3 * gy.nb[3]);
    const int n4 = (int) (gx.ne[0] / 4);
    float4 v[VPT];
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < VPT; ++j) {
        const int i = threadIdx.x + 256 * j;
        v[j] = px[min(i, n4 - 1)];                     // clamped: registers, not a branch
        if (i < n4) s += v[j].x * v[j].x + v[j].y * v[j].y + v[j].z * v[j].z + v[j].w * v[j].w;
    }
    s = block_sum(s, lds);
    const float scale = 1.0f / sqrtf(s / (float) gx.ne[0] + eps);
    const float4 * pw = MUL ? (const float4 *) (w + (i1 % gw.ne[1]) * gw.nb[1] + (i2 % gw.ne[2]) * gw.nb[2] + (i3 % gw.ne[3]) * gw.nb[3]) : nullptr;
#pragma unroll
    for (int j = 0; j < VPT; ++j) {
        const int i = threadIdx.x + 256 * j;
        if (i >= n4) break;
        float4 o = make_float4(v[j].x * scale, v[j].y * scale, v[j].z * scale, v[j].w * scale);
        if constexpr (MUL) { const float4 wv = pw[i]; o.x *= wv.x; o.y *= wv.y; o.z *= wv.z; o.w *= wv.w; }
        py[i] = o;
        if (h) {   // the f16 row a following prefill GEMM reads (act cache, contiguous rows)
            typedef _Float16 h4 __attribute__((ext_vector_type(4)));
            *(h4 *) (h + r * gx.ne[0] + 4 * i) = h4{(_Float16) o.x, (_Float16) o.y, (_Float16) o.z, (_Float16) o.w};
        }
    }
}

void op_rms_norm(OpCtx & c, ggml_tensor * norm, const ggml_tensor * mul, ggml_tensor * out) {
    const ggml_tensor * x = norm->src[0];
    const float eps = mx_op_param<float>(norm, 0);
    const int64_t nr = mx_nrows(x);
    auto al16 = [](const ggml_tensor * t) {
        return ((uintptr_t) t->data % 16) == 0 && t->nb[1] % 16 == 0 && t->nb[2] % 16 == 0 && t->nb[3] % 16 == 0 && t->nb[0] == 4;
    };
    if (x->ne[0] % 4 == 0 && x->ne[0] <= 4 * 256 * 8 && x->ne[0] >= 1024 && al16(x) && al16(out) && (!mul || al16(mul))) {
        const int vpt = (int) mx_ceil_div(x->ne[0] / 4, 256);
        const T4 gw = mul ? geo(mul) : geo(x);
        const char * wp = mul ? (const char *) mul->data : nullptr;
        _Float16 * h = mx_is_contiguous(out) && out->ne[2] == 1 && out->ne[3] == 1 ? mmq_act_claim(c, out->data, out->ne[0], out->ne[1], out->nb[1]) : nullptr;
#define RN(M, V) k_rms_norm_v4<M, V><<<(unsigned) nr, 256, 0, c.st>>>((const char *) x->data, wp, (char *) out->data, geo(x), gw, geo(out), eps, h)
        if (mul) { if (vpt <= 2) RN(true, 2); else if (vpt <= 4) RN(true, 4); else RN(true, 8); }
        else     { if (vpt <= 2) RN(false, 2); else if (vpt <= 4) RN(false, 4); else RN(false, 8); }
#undef RN
        return;
    }
    const int bs = x->ne[0] >= 1024 ? 512 : (x->ne[0] >= 256 ? 256 : 64);
    if (mul) {
        k_rms_norm<true><<<(unsigned) nr, bs, 0, c.st>>>((const char *) x->data, (const char *) mul->data, (char *) out->data,
                                                        geo(x), geo(mul), geo(out), eps);
    } else {
        k_rms_norm<false><<<(unsigned) nr, bs, 0, c.st>>>((const char *) x->data, nullptr, (char *) out->data,
                                                         geo(x), geo(x), geo(out), eps);
    }
}

// RMS_NORM → MUL(w) for decode rows (≤ 8 rows, ne0 % 32 == 0), writing the f32
// output AND its q8 form (int8 + per-32 d, d·Σq) that the following GEMVs consume,
// so no separate activation-quantisation launch is needed (quantize.cu:5-48 semantics).
__global__ void k_rms_norm_q8(const char * __restrict__ x, const char * __restrict__ w, char * __restrict__ y,
                              T4 gx, T4 gw, T4 gy, float eps, int8_t * __restrict__ q, float * __restrict__ qd,
                              float * __restrict__ qs, int64_t kp) {
    __shared__ float lds[16];
    const int64_t r = blockIdx.x;
    const int64_t i1 = r % gx.ne[1], i2 = (r / gx.ne[1]) % gx.ne[2], i3 = r / (gx.ne[1] * gx.ne[2]);
    const float * px = (const float *) (x + i1 * gx.nb[1] + i2 * gx.nb[2] + i3 * gx.nb[3]);
    const float * pw = (const float *) (w + (i1 % gw.ne[1]) * gw.nb[1] + (i2 % gw.ne[2]) * gw.nb[2] + (i3 % gw.ne[3]) * gw.nb[3]);
    float * py = (float *) (y + i1 * gy.nb[1] + i2 * gy.nb[2] + i3 * gy.nb[3]);
    const int64_t n = gx.ne[0];
    const int64_t nchunk = n / 32;
    // one memory round trip: each thread holds its 32-element chunk of x and w in
    // registers across the reduction (n <= 32*blockDim; larger rows loop below)
    const int64_t b0 = threadIdx.x;
    float xr[32], wr[32];
    float s = 0.f;
    if (b0 < nchunk) {
#pragma unroll
        for (int j = 0; j < 32; j += 4) {
            const float4 xv = *(const float4 *) (px + 32 * b0 + j);
            const float4 wv = *(const float4 *) (pw + 32 * b0 + j);
            xr[j] = xv.x; xr[j + 1] = xv.y; xr[j + 2] = xv.z; xr[j + 3] = xv.w;
            wr[j] = wv.x; wr[j + 1] = wv.y; wr[j + 2] = wv.z; wr[j + 3] = wv.w;
        }
#pragma unroll
        for (int j = 0; j < 32; ++j) s += xr[j] * xr[j];
    }
    for (int64_t i = 32 * (b0 + blockDim.x); i < n; i += 32 * blockDim.x)
        for (int j = 0; j < 32; ++j) s += px[i + j] * px[i + j];
    s = block_sum(s, lds);
    const float scale = 1.0f / sqrtf(s / (float) n + eps);
    for (int64_t b = b0; b < nchunk; b += blockDim.x) {
        float v[32];
        if (b != b0) {
            for (int j = 0; j < 32; ++j) { xr[j] = px[32 * b + j]; wr[j] = pw[32 * b + j]; }
        }
#pragma unroll
        for (int j = 0; j < 32; j += 4) {
            v[j] = (xr[j] * scale) * wr[j]; v[j + 1] = (xr[j + 1] * scale) * wr[j + 1];
            v[j + 2] = (xr[j + 2] * scale) * wr[j + 2]; v[j + 3] = (xr[j + 3] * scale) * wr[j + 3];
            *(float4 *) (py + 32 * b + j) = make_float4(v[j], v[j + 1], v[j + 2], v[j + 3]);
        }
        float amax = 0.f;
#pragma unroll
        for (int j = 0; j < 32; ++j) amax = fmaxf(amax, fabsf(v[j]));
        const Q8Scale qsc = q8_scale(amax);
        const float dd = qsc.d, id = qsc.id;
        int sum = 0, packed[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            int wq = 0;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int qi = q8_round(v[4 * j + k], id);
                sum += qi;
                wq |= (qi & 0xFF) << (8 * k);
            }
            packed[j] = wq;
        }
        int4 * out = (int4 *) (q + r * kp + 32 * b);
        out[0] = make_int4(packed[0], packed[1], packed[2], packed[3]);
        out[1] = make_int4(packed[4], packed[5], packed[6], packed[7]);
        qd[r * (kp / 32) + b] = dd;
        qs[r * (kp / 32) + b] = dd * (float) sum;
    }
}

bool rms_norm_mul_q8(OpCtx & c, ggml_tensor * norm, const ggml_tensor * w, ggml_tensor * out) {
    const ggml_tensor * x = norm->src[0];
    const int64_t nr = mx_nrows(x);
    if (nr > 8 || x->ne[0] % 32 != 0 || x->nb[0] != 4 || w->nb[0] != 4 || out->nb[0] != 4) return false;
    if ((uintptr_t) x->data % 16 || (uintptr_t) w->data % 16 || (uintptr_t) out->data % 16) return false;
    for (int i = 1; i < 4; ++i) if (x->nb[i] % 16 || w->nb[i] % 16 || out->nb[i] % 16) return false;
    ActQ * a = act_cache_alloc(c.s, out);
    if (!a) return false;
    k_rms_norm_q8<<<(unsigned) nr, 256, 0, c.st>>>((const char *) x->data, (const char *) w->data, (char *) out->data,
                                                  geo(x), geo(w), geo(out), mx_op_param<float>(norm, 0),
                                                  (int8_t *) a->q, (float *) a->d, (float *) a->s, a->kp);
    return true;
}

__global__ void k_norm(const char * __restrict__ x, char * __restrict__ y, T4 gx, T4 gy, float eps) {
    __shared__ float lds[16];
    const int64_t r = blockIdx.x;
    const int64_t i1 = r % gx.ne[1], i2 = (r / gx.ne[1]) % gx.ne[2], i3 = r / (gx.ne[1] * gx.ne[2]);
    const float * px = (const float *) (x + i1 * gx.nb[1] + i2 * gx.nb[2] + i3 * gx.nb[3]);
    float * py = (float *) (y + i1 * gy.nb[1] + i2 * gy.nb[2] + i3 * gy.nb[3]);
    const int64_t n = gx.ne[0];
    float s = 0.f;
    for (int64_t i = threadIdx.x; i < n; i += blockDim.x) s += px[i];
    const float mean = block_sum(s, lds) / (float) n;
    float v = 0.f;
    for (int64_t i = threadIdx.x; i < n; i += blockDim.x) { const float d = px[i] - mean; v += d * d; }
    const float var = block_sum(v, lds) / (float) n;
    const float scale = 1.0f / sqrtf(var + eps);
    for (int64_t i = threadIdx.x; i < n; i += blockDim.x) py[i] = (px[i] - mean) * scale;
}

void op_norm(OpCtx & c, ggml_tensor * dst) {
    const ggml_tensor * x = dst->src[0];
    const int64_t nr = mx_nrows(x);
    const int bs = x->ne[0] >= 1024 ? 512 : (x->ne[0] >= 256 ? 256 : 64);
    k_norm<<<(unsigned) nr, bs, 0, c.st>>>((const char *) x->data, (char *) dst->data, geo(x), geo(dst), mx_op_param<float>(dst, 0));
}

// ---------------------------------------------------------------------------
// ROPE (NORMAL and NEOX), YaRN-corrected. theta follows the CPU cache order:
// θ_i = p · scale^i accumulated by repeated f32 multiplication, with the host
// computing scale = powf(base, -2/n_dims) exactly as the CPU does.
// ---------------------------------------------------------------------------
struct RopeP {
    int n_dims, mode;
    float freq_scale, ext_factor, attn_factor, theta_scale;
    float corr0, corr1;
};

__device__ __forceinline__ void rope_cs(float theta_extrap, const RopeP & p, int i0, float * c, float * s) {
    const float theta_interp = p.freq_scale * theta_extrap;
    float theta = theta_interp;
    float mscale = p.attn_factor;
    if (p.ext_factor != 0.0f) {
        const float y = (i0 / 2 - p.corr0) / fmaxf(0.001f, p.corr1 - p.corr0);
        const float ramp_mix = (1.0f - fminf(1.0f, fmaxf(0.0f, y))) * p.ext_factor;
        theta = theta_interp * (1 - ramp_mix) + theta_extrap * ramp_mix;
        mscale *= 1.0f + 0.1f * logf(1.0f / p.freq_scale);
    }
    *c = cosf(theta) * mscale;
    *s = sinf(theta) * mscale;
}

template <typename T, bool NEOX>
__global__ void k_rope(const char * __restrict__ x, const int32_t * __restrict__ pos, const float * __restrict__ ff,
                       char * __restrict__ y, T4 gx, T4 gy, RopeP p) {
    // block = one row (i1, i2, i3); threads over pairs
    const int64_t r = blockIdx.x;
    const int64_t i1 = r % gx.ne[1], i2 = (r / gx.ne[1]) % gx.ne[2], i3 = r / (gx.ne[1] * gx.ne[2]);
    const T * px = (const T *) (x + i1 * gx.nb[1] + i2 * gx.nb[2] + i3 * gx.nb[3]);
    T * py = (T *) (y + i1 * gy.nb[1] + i2 * gy.nb[2] + i3 * gy.nb[3]);
    const float pf = (float) pos[i2];
    const int64_t ne0 = gx.ne[0];
    for (int64_t i0 = 2 * threadIdx.x; i0 < ne0; i0 += 2 * blockDim.x) {
        if (i0 < p.n_dims) {
            float theta = pf;
            for (int k = 0; k < i0 / 2; ++k) theta *= p.theta_scale;
            const float f = ff ? ff[i0 / 2] : 1.0f;
            float cs, sn;
            rope_cs(theta / f, p, (int) i0, &cs, &sn);
            const int64_t a = NEOX ? i0 / 2 : i0;
            const int64_t b = NEOX ? a + p.n_dims / 2 : a + 1;
            const float x0 = ld<T>(px + a), x1 = ld<T>(px + b);
            st<T>(py + a, x0 * cs - x1 * sn);
            st<T>(py + b, x0 * sn + x1 * cs);
        } else {
            py[i0] = px[i0];
            py[i0 + 1] = px[i0 + 1];
        }
    }
}

// Prefill form: one workgroup per token (i2, i3) rotates every head of it. The token's
// cos/sin table (same θ recurrence and YaRN ramp as k_rope, so bit-identical) is built
// once into LDS — k_rope recomputed it per head: an up-to-63-step θ loop plus libm
// sincos per pair, ~11.5 µs per pp512 ROPE against ~3 µs of memory traffic.
constexpr int MX_ROPE2_MAXP = 512;    // n_dims / 2 limit of the LDS table
static const bool g_rope1 = getenv("GGML_MI355X_ROPE1") != nullptr;   // A/B: the per-row kernel
template <typename T, bool NEOX>
__global__ __launch_bounds__(256) void k_rope2(const char * __restrict__ x, const int32_t * __restrict__ pos, const float * __restrict__ ff,
                                               char * __restrict__ y, T4 gx, T4 gy, RopeP p) {
    __shared__ float2 tab[MX_ROPE2_MAXP];
    const int64_t i2 = blockIdx.x % gx.ne[2], i3 = blockIdx.x / gx.ne[2];
    const float pf = (float) pos[i2];
    const int np = p.n_dims / 2;
    for (int i = threadIdx.x; i < np; i += blockDim.x) {
        float theta = pf;
        for (int k = 0; k < i; ++k) theta *= p.theta_scale;
        const float f = ff ? ff[i] : 1.0f;
        float cs, sn;
        rope_cs(theta / f, p, 2 * i, &cs, &sn);
        tab[i] = make_float2(cs, sn);
    }
    __syncthreads();
    const int64_t ne0 = gx.ne[0], hp = ne0 / 2;
    for (int64_t idx = threadIdx.x; idx < gx.ne[1] * hp; idx += blockDim.x) {
        const int64_t i1 = idx / hp, i0 = 2 * (idx % hp);
        const T * px = (const T *) (x + i1 * gx.nb[1] + i2 * gx.nb[2] + i3 * gx.nb[3]);
        T * py = (T *) (y + i1 * gy.nb[1] + i2 * gy.nb[2] + i3 * gy.nb[3]);
        if (i0 < p.n_dims) {
            const float2 t = tab[i0 / 2];
            const int64_t a = NEOX ? i0 / 2 : i0;
            const int64_t b = NEOX ? a + p.n_dims / 2 : a + 1;
            const float x0 = ld<T>(px + a), x1 = ld<T>(px + b);
            st<T>(py + a, x0 * t.x - x1 * t.y);
            st<T>(py + b, x0 * t.y + x1 * t.x);
        } else {
            py[i0] = px[i0];
            py[i0 + 1] = px[i0 + 1];
        }
    }
}

static float yarn_corr_dim(int n_dims, int n_ctx_orig, float n_rot, float base) {
    return n_dims * logf(n_ctx_orig / (n_rot * 2 * (float) M_PI)) / (2 * logf(base));
}

void op_rope(OpCtx & c, ggml_tensor * dst) {
    const ggml_tensor * x = dst->src[0];
    const ggml_tensor * pos = dst->src[1];
    const ggml_tensor * ff = dst->src[2];
    RopeP p;
    p.n_dims = mx_op_param<int32_t>(dst, 1);
    p.mode = mx_op_param<int32_t>(dst, 2);
    const int n_ctx_orig = mx_op_param<int32_t>(dst, 4);
    const float freq_base = mx_op_param<float>(dst, 5);
    p.freq_scale = mx_op_param<float>(dst, 6);
    p.ext_factor = mx_op_param<float>(dst, 7);
    p.attn_factor = mx_op_param<float>(dst, 8);
    const float beta_fast = mx_op_param<float>(dst, 9), beta_slow = mx_op_param<float>(dst, 10);
    p.theta_scale = powf(freq_base, -2.0f / p.n_dims);
    const float start = floorf(yarn_corr_dim(p.n_dims, n_ctx_orig, beta_fast, freq_base));
    const float end = ceilf(yarn_corr_dim(p.n_dims, n_ctx_orig, beta_slow, freq_base));
    p.corr0 = std::max(0.0f, start);
    p.corr1 = std::min((float) (p.n_dims - 1), end);
    const int64_t nr = mx_nrows(x);
    const int bs = 64;
    const float * pff = ff ? (const float *) ff->data : nullptr;
    const bool neox = (p.mode & GGML_ROPE_TYPE_NEOX) != 0;
    if (x->ne[2] * x->ne[3] > 1 && x->ne[1] > 1 && p.n_dims / 2 <= MX_ROPE2_MAXP && x->ne[0] % 2 == 0 && !g_rope1) {
        const unsigned g = (unsigned) (x->ne[2] * x->ne[3]);
#define R2(T, NX) k_rope2<T, NX><<<g, 256, 0, c.st>>>((const char *) x->data, (const int32_t *) pos->data, pff, (char *) dst->data, geo(x), geo(dst), p)
        if (x->type == GGML_TYPE_F32) { if (neox) R2(float, true); else R2(float, false); }
        else { if (neox) R2(uint16_t, true); else R2(uint16_t, false); }
#undef R2
        return;
    }
    if (x->type == GGML_TYPE_F32) {
        if (neox) k_rope<float, true><<<(unsigned) nr, bs, 0, c.st>>>((const char *) x->data, (const int32_t *) pos->data, pff, (char *) dst->data, geo(x), geo(dst), p);
        else      k_rope<float, false><<<(unsigned) nr, bs, 0, c.st>>>((const char *) x->data, (const int32_t *) pos->data, pff, (char *) dst->data, geo(x), geo(dst), p);
    } else {
        if (neox) k_rope<uint16_t, true><<<(unsigned) nr, bs, 0, c.st>>>((const char *) x->data, (const int32_t *) pos->data, pff, (char *) dst->data, geo(x), geo(dst), p);
        else      k_rope<uint16_t, false><<<(unsigned) nr, bs, 0, c.st>>>((const char *) x->data, (const int32_t *) pos->data, pff, (char *) dst->data, geo(x), geo(dst), p);
    }
}

// ---------------------------------------------------------------------------
// SOFT_MAX: softmax(x*scale + slope*mask) (+ sinks), one block per row
// ---------------------------------------------------------------------------
template <typename TM>
__global__ void k_soft_max(const char * __restrict__ x, const char * __restrict__ mask, const float * __restrict__ sinks,
                           char * __restrict__ y, T4 gx, T4 gm, T4 gy, float scale, float max_bias, float m0, float m1,
                           uint32_t n_head_log2) {
    __shared__ float lds[16];
    const int64_t r = blockIdx.x;
    const int64_t i1 = r % gx.ne[1], i2 = (r / gx.ne[1]) % gx.ne[2], i3 = r / (gx.ne[1] * gx.ne[2]);
    const float * px = (const float *) (x + i1 * gx.nb[1] + i2 * gx.nb[2] + i3 * gx.nb[3]);
    float * py = (float *) (y + i1 * gy.nb[1] + i2 * gy.nb[2] + i3 * gy.nb[3]);
    const TM * pm = mask ? (const TM *) (mask + i1 * gm.nb[1] + (i2 % gm.ne[2]) * gm.nb[2] + (i3 % gm.ne[3]) * gm.nb[3]) : nullptr;
    const uint32_t h = (uint32_t) i2;
    const float slope = max_bias > 0.0f ? (h < n_head_log2 ? powf(m0, h + 1) : powf(m1, 2 * (h - n_head_log2) + 1)) : 1.0f;
    const int64_t n = gx.ne[0];
    float mx = -INFINITY;
    for (int64_t i = threadIdx.x; i < n; i += blockDim.x) {
        float v = px[i] * scale;
        if (pm) v += slope * ld<TM>(pm + i);
        py[i] = v;
        mx = fmaxf(mx, v);
    }
    mx = block_max(mx, lds);
    if (sinks) mx = fmaxf(mx, sinks[i2]);
    float s = 0.f;
    for (int64_t i = threadIdx.x; i < n; i += blockDim.x) {
        const float e = expf(py[i] - mx);
        py[i] = e;
        s += e;
    }
    s = block_sum(s, lds);
    if (sinks) s += expf(sinks[i2] - mx);
    const float inv = 1.0f / s;
    for (int64_t i = threadIdx.x; i < n; i += blockDim.x) py[i] *= inv;
}

void op_soft_max(OpCtx & c, ggml_tensor * dst) {
    const ggml_tensor * x = dst->src[0];
    const ggml_tensor * m = dst->src[1];
    const ggml_tensor * sk = dst->src[2];
    const float scale = mx_op_param<float>(dst, 0), max_bias = mx_op_param<float>(dst, 1);
    const uint32_t n_head = (uint32_t) x->ne[2];
    const uint32_t n_head_log2 = 1u << (uint32_t) floor(log2((double) n_head));
    const float m0 = powf(2.0f, -(max_bias) / n_head_log2);
    const float m1 = powf(2.0f, -(max_bias / 2.0f) / n_head_log2);
    const int64_t nr = mx_nrows(x);
    const int bs = x->ne[0] >= 1024 ? 512 : (x->ne[0] >= 256 ? 256 : 64);
    const float * psk = sk ? (const float *) sk->data : nullptr;
    T4 gm = m ? geo(m) : geo(x);
    if (!m || m->type == GGML_TYPE_F32) {
        k_soft_max<float><<<(unsigned) nr, bs, 0, c.st>>>((const char *) x->data, m ? (const char *) m->data : nullptr, psk,
                                                          (char *) dst->data, geo(x), gm, geo(dst), scale, max_bias, m0, m1, n_head_log2);
    } else {
        k_soft_max<uint16_t><<<(unsigned) nr, bs, 0, c.st>>>((const char *) x->data, (const char *) m->data, psk,
                                                             (char *) dst->data, geo(x), gm, geo(dst), scale, max_bias, m0, m1, n_head_log2);
    }
}

// ---------------------------------------------------------------------------
// SUM_ROWS, ARGSORT (bitonic in LDS, one block per row)
// ---------------------------------------------------------------------------
__global__ void k_sum_rows(const char * __restrict__ x, char * __restrict__ y, T4 gx, T4 gy) {
    __shared__ float lds[16];
    const int64_t r = blockIdx.x;
    const int64_t i1 = r % gx.ne[1], i2 = (r / gx.ne[1]) % gx.ne[2], i3 = r / (gx.ne[1] * gx.ne[2]);
    const char * px = x + i1 * gx.nb[1] + i2 * gx.nb[2] + i3 * gx.nb[3];
    float s = 0.f;
    for (int64_t i = threadIdx.x; i < gx.ne[0]; i += blockDim.x) s += *(const float *) (px + i * gx.nb[0]);
    s = block_sum(s, lds);
    if (threadIdx.x == 0) *(float *) (y + i1 * gy.nb[1] + i2 * gy.nb[2] + i3 * gy.nb[3]) = s;
}
void op_sum_rows(OpCtx & c, ggml_tensor * dst) {
    const ggml_tensor * x = dst->src[0];
    k_sum_rows<<<(unsigned) mx_nrows(x), 64, 0, c.st>>>((const char *) x->data, (char *) dst->data, geo(x), geo(dst));
}

// order: 0 asc, 1 desc; ties keep the lower index first (stable like std::sort on (value, idx) pairs)
__global__ void k_argsort(const float * __restrict__ x, int32_t * __restrict__ y, int64_t ncols, size_t nbx, size_t nby,
                          int npad, int order) {
    extern __shared__ int idx[];
    const int64_t row = blockIdx.x;
    const float * px = (const float *) ((const char *) x + row * nbx);
    for (int i = threadIdx.x; i < npad; i += blockDim.x) idx[i] = i;
    __syncthreads();
    for (int k = 2; k <= npad; k <<= 1) {
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int i = threadIdx.x; i < npad; i += blockDim.x) {
                const int ixj = i ^ j;
                if (ixj > i) {
                    const int a = idx[i], b = idx[ixj];
                    // padded slots sort last
                    bool a_gt_b;
                    if (a >= ncols) a_gt_b = true;
                    else if (b >= ncols) a_gt_b = false;
                    else {
                        const float va = px[a], vb = px[b];
                        a_gt_b = order == 0 ? (va > vb || (va == vb && a > b)) : (va < vb || (va == vb && a > b));
                    }
                    const bool up = (i & k) == 0;
                    if (a_gt_b == up) { idx[i] = b; idx[ixj] = a; }
                }
            }
            __syncthreads();
        }
    }
    int32_t * py = (int32_t *) ((char *) y + row * nby);
    for (int i = threadIdx.x; i < ncols; i += blockDim.x) py[i] = idx[i];
}
void op_argsort(OpCtx & c, ggml_tensor * dst) {
    const ggml_tensor * x = dst->src[0];
    const int order = mx_op_param<int32_t>(dst, 0);
    int npad = 1;
    while (npad < x->ne[0]) npad <<= 1;
    k_argsort<<<(unsigned) mx_nrows(x), 256, npad * sizeof(int), c.st>>>((const float *) x->data, (int32_t *) dst->data,
                                                                        x->ne[0], x->nb[1], dst->nb[1], npad, order);
}

// ---------------------------------------------------------------------------
// supports_op — truthful, the scheduler relies on it (ggml-backend.cpp:896-923)
// ---------------------------------------------------------------------------
static bool is_f(int t) { return t == GGML_TYPE_F32 || t == GGML_TYPE_F16; }

bool supports_op(const ggml_tensor * op) {
    const ggml_tensor * s0 = op->src[0];
    const ggml_tensor * s1 = op->src[1];
    switch (op->op) {
        case GGML_OP_NONE: case GGML_OP_RESHAPE: case GGML_OP_VIEW: case GGML_OP_PERMUTE: case GGML_OP_TRANSPOSE:
            return true;
        case GGML_OP_GET_ROWS:
            if (s1->type != GGML_TYPE_I32) return false;
            switch (s0->type) {
                case GGML_TYPE_F32: case GGML_TYPE_F16: return op->type == GGML_TYPE_F32 || op->type == s0->type;
                case GGML_TYPE_I32: return op->type == GGML_TYPE_I32;
                case GGML_TYPE_Q4_0: case GGML_TYPE_Q4_1: case GGML_TYPE_Q5_0: case GGML_TYPE_Q5_1: case GGML_TYPE_Q8_0:
                case GGML_TYPE_Q4_K: case GGML_TYPE_Q5_K: case GGML_TYPE_Q6_K:
                    return op->type == GGML_TYPE_F32;
                default: return false;
            }
        case GGML_OP_SET_ROWS:
            return s0->type == GGML_TYPE_F32 && (s1->type == GGML_TYPE_I64 || s1->type == GGML_TYPE_I32) &&
                   (op->type == GGML_TYPE_F32 || op->type == GGML_TYPE_F16 || op->type == GGML_TYPE_BF16 ||
                    ((op->type == GGML_TYPE_Q8_0 || op->type == GGML_TYPE_Q4_0) && s0->ne[0] % 32 == 0));
        case GGML_OP_DUP: case GGML_OP_CONT: case GGML_OP_CPY: {
            const int ts = s0->type, td = op->type;
            if (ts == td && mx_is_contiguous(s0) && mx_is_contiguous(op)) return true;
            if ((ts == GGML_TYPE_F32 || ts == GGML_TYPE_F16 || ts == GGML_TYPE_BF16) &&
                (td == GGML_TYPE_F32 || td == GGML_TYPE_F16 || td == GGML_TYPE_BF16)) {
                return !(ts == GGML_TYPE_F16 && td == GGML_TYPE_BF16) && !(ts == GGML_TYPE_BF16 && td == GGML_TYPE_F16);
            }
            if (ts == GGML_TYPE_I32 && td == GGML_TYPE_I32) return true;
            if (ts == GGML_TYPE_F32 && td == GGML_TYPE_Q8_0) return mx_is_contiguous(s0) && mx_is_contiguous(op) && s0->ne[0] % 32 == 0;
            return false;
        }
        case GGML_OP_ADD: case GGML_OP_SUB: case GGML_OP_MUL: case GGML_OP_DIV: {
            const int t0 = s0->type, t1 = s1->type, td = op->type;
            for (int i = 0; i < 4; ++i) if (s1->ne[i] == 0 || s0->ne[i] % s1->ne[i] != 0) return false;
            if (t0 == GGML_TYPE_F32 && t1 == GGML_TYPE_F32 && td == GGML_TYPE_F32) return true;
            if (t0 == GGML_TYPE_F16 && is_f(t1) && is_f(td)) return true;
            if (t0 == GGML_TYPE_F32 && t1 == GGML_TYPE_F16 && td == GGML_TYPE_F32) return true;
            return false;
        }
        case GGML_OP_SCALE: case GGML_OP_CLAMP:
            return s0->type == GGML_TYPE_F32 && op->type == GGML_TYPE_F32;
        case GGML_OP_UNARY:
            return s0->type == GGML_TYPE_F32 && op->type == GGML_TYPE_F32 && unary_supported(mx_op_param<int32_t>(op, 0));
        case GGML_OP_GLU: {
            const int g = mx_op_param<int32_t>(op, 0);
            if (g == GGML_GLU_OP_SWIGLU_OAI) return false;
            if (s0->type != GGML_TYPE_F32 || op->type != GGML_TYPE_F32) return false;
            if (!mx_is_contiguous_n(s0, 1) || !mx_is_contiguous_n(op, 1)) return false;
            if (s1 && (s1->type != GGML_TYPE_F32 || !mx_is_contiguous_n(s1, 1))) return false;
            return true;
        }
        case GGML_OP_RMS_NORM: case GGML_OP_NORM:
            return s0->type == GGML_TYPE_F32 && op->type == GGML_TYPE_F32 && s0->nb[0] == 4;
        case GGML_OP_ROPE: {
            const int mode = mx_op_param<int32_t>(op, 2);
            if (mode != GGML_ROPE_TYPE_NORMAL && mode != GGML_ROPE_TYPE_NEOX) return false;
            if (!is_f(s0->type) || s0->type != op->type || s0->nb[0] != (size_t) mx_type(s0->type).size) return false;
            if (op->src[2] && op->src[2]->type != GGML_TYPE_F32) return false;
            return s1->type == GGML_TYPE_I32 && s0->ne[0] % 2 == 0;
        }
        case GGML_OP_SOFT_MAX:
            if (s0->type != GGML_TYPE_F32 || op->type != GGML_TYPE_F32 || s0->nb[0] != 4) return false;
            if (s1 && !(s1->type == GGML_TYPE_F32 || s1->type == GGML_TYPE_F16)) return false;
            if (op->src[2] && op->src[2]->type != GGML_TYPE_F32) return false;
            return true;
        case GGML_OP_SUM_ROWS:
            return s0->type == GGML_TYPE_F32 && op->type == GGML_TYPE_F32;
        case GGML_OP_ARGSORT:
            return s0->type == GGML_TYPE_F32 && mx_is_contiguous_rows(s0) && s0->ne[0] <= 8192;
        case GGML_OP_MUL_MAT:        return mul_mat_supported(op);
        case GGML_OP_MUL_MAT_ID:     return mul_mat_id_supported(op);
        case GGML_OP_FLASH_ATTN_EXT: return flash_attn_supported(op);
        default: return false;
    }
}

}  // namespace mx
