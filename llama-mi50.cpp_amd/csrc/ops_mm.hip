// ops_mm.hip — MUL_MAT dispatcher and the prefill GEMM on CDNA4 matrix cores.
//
// Reference: ggml_cuda_mul_mat (ggml-cuda.cu:2183-2266) chooses mmvq for
// src1->ne[1] <= 8 and mmq (mmq.cuh:3364-3700, int8 MMA over q8_1 tiles) above.
// MI355X design for the GEMM ("dequant-into-LDS → MFMA"):
//   * activations are converted once to f16 rows padded to the K tile (scratch);
//   * per 128-deep K step a 256-thread block dequantises a 128-row weight tile
//     straight from the ggml super-blocks (16-byte qs chunks per lane) into f16 LDS,
//     and stages a 128-token activation tile with 16-byte loads;
//   * 4 waves (2×2) each own a 64×64 output tile = 2×2 v_mfma_f32_32x32x16_f16,
//     A operand = tokens, B operand = weight rows, so the epilogue's 32 lanes
//     write 32 consecutive output rows (128-byte coalesced stores);
//   * LDS rows are 256 B; 16-byte chunks are XOR-swizzled by (row & 15) so every
//     ds_read_b128 lane group hits 16 distinct bank slots.
#include "backend.h"
#include "mm.h"
#include "gemv.h"

namespace mx {

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float float16v __attribute__((ext_vector_type(16)));

constexpr int MM_BT = 128;   // tokens per block
constexpr int MM_BW = 128;   // weight rows per block
constexpr int MM_BK = 128;   // K per step

struct MmqArgs {
    const char * w; size_t w_row, w_c2, w_c3;
    const char * w2;                         // k_mmq3g: the up matrix (same layout as w)
    _Float16 * h; int64_t h_col;             // k_mmq3g: also the f16 copy of the output (act cache)
    const float * res; size_t r_col;         // k_mmq2/k_mmq3: + residual (MUL_MAT -> ADD), in floats
    const _Float16 * x; int64_t kp;          // activations f16 [cols][kp]
    float * dst; size_t d_col, d_c2, d_c3;   // in floats
    int64_t M, N, K, ne12, r2, r3;
    int dbg;                                 // timing experiments (g_tune[13], k_mmq3): 1 weight loads
                                             // from one L2-resident block, 2 no MFMAs, 4 activation
                                             // loads from one 256-B row, 8 no dequantisation, 16 two K steps
};

// ---- f32 → f16 activation rows, zero padded to kp (8 values per thread) ------
__global__ void k_act_f16(const char * __restrict__ x, int64_t K, int64_t ne11, int64_t ne12,
                          size_t nb10, size_t nb11, size_t nb12, size_t nb13, int64_t kp, _Float16 * __restrict__ out) {
    const int64_t col = blockIdx.y;
    const int64_t i11 = col % ne11, i12 = (col / ne11) % ne12, i13 = col / (ne11 * ne12);
    const char * px = x + i11 * nb11 + i12 * nb12 + i13 * nb13;
    const int64_t k = 8 * (blockIdx.x * (int64_t) blockDim.x + threadIdx.x);
    if (k >= kp) return;
    half8 h;
    if (nb10 == 4 && k + 8 <= K && ((uintptr_t) (px + 4 * k) % 16) == 0) {
        const float4 a = *(const float4 *) (px + 4 * k), b = *(const float4 *) (px + 4 * k + 16);
        h[0] = (_Float16) a.x; h[1] = (_Float16) a.y; h[2] = (_Float16) a.z; h[3] = (_Float16) a.w;
        h[4] = (_Float16) b.x; h[5] = (_Float16) b.y; h[6] = (_Float16) b.z; h[7] = (_Float16) b.w;
    } else {
#pragma unroll
        for (int i = 0; i < 8; ++i) h[i] = (_Float16) (k + i < K ? *(const float *) (px + (k + i) * nb10) : 0.0f);
    }
    *(half8 *) (out + col * kp + k) = h;
}

__device__ __forceinline__ int swz(int row, int chunk) { return row * 16 + (chunk ^ (row & 15)); }  // in 16-byte units

template <int CPR>   // CPR 16-byte chunks per row (power of two)
__device__ __forceinline__ int swzn(int row, int chunk) { return row * CPR + (chunk ^ (row & (CPR - 1))); }

template <int CPR>
__device__ __forceinline__ void st_h8n(uint4 * lds, int row, int chunk, const float (&v)[8]) {
    half8 h;
#pragma unroll
    for (int i = 0; i < 8; ++i) h[i] = (_Float16) v[i];
    lds[swzn<CPR>(row, chunk)] = *(uint4 *) &h;
}

__device__ __forceinline__ void st_h8(uint4 * lds, int row, int chunk, const float (&v)[8]) {
    half8 h;
#pragma unroll
    for (int i = 0; i < 8; ++i) h[i] = (_Float16) v[i];
    lds[swz(row, chunk)] = *(uint4 *) &h;
}

// Dequantise the weight tile [MM_BW rows][MM_BK k] starting at k0 into LDS.
template <int QT>
__device__ __forceinline__ void load_w_tile(const MmqArgs & p, const char * wbase, int64_t row0, int64_t k0, uint4 * lds) {
    const int tid = threadIdx.x;
    if constexpr (QT == GGML_TYPE_Q4_K || QT == GGML_TYPE_Q5_K) {
        // 128 rows × 4 qs chunks (half a super-block) = 512 units, 2 per thread
#pragma unroll
        for (int it = 0; it < 2; ++it) {
            const int unit = tid + 256 * it;
            const int r = unit >> 2, c = unit & 3;
            const int64_t row = row0 + r;
            float lo[16], hi[16];
            if (row < p.M) {
                const int64_t sb = k0 >> 8;
                const int hf = (int) ((k0 >> 7) & 1);
                const char * b = wbase + row * p.w_row + sb * qsize_of<QT>();
                const int g = 2 * hf + (c >> 1), h = c & 1;
                const int4 hd = *(const int4 *) b;
                const int4 w = *(const int4 *) (b + (QT == GGML_TYPE_Q4_K ? 16 : 48) + 16 * (4 * hf + c));
                const uint8_t * sc = (const uint8_t *) b + 4;
                int s0, m0, s1, m1;
                scale_min_k4(2 * g, sc, s0, m0);
                scale_min_k4(2 * g + 1, sc, s1, m1);
                const float d = h2f((uint16_t) (hd.x & 0xFFFF)), dmin = h2f((uint16_t) ((uint32_t) hd.x >> 16));
                const float d0 = d * s0, mm0 = dmin * m0, d1 = d * s1, mm1 = dmin * m1;
                const uint32_t wv[4] = {(uint32_t) w.x, (uint32_t) w.y, (uint32_t) w.z, (uint32_t) w.w};
                uint32_t hv[4] = {0, 0, 0, 0};
                if constexpr (QT == GGML_TYPE_Q5_K) {
                    const int4 qh = *(const int4 *) (b + 16 + 16 * h);
                    hv[0] = qh.x; hv[1] = qh.y; hv[2] = qh.z; hv[3] = qh.w;
                }
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    const uint32_t byte = (wv[i >> 2] >> (8 * (i & 3))) & 0xFF;
                    int ql = byte & 0xF, qhh = byte >> 4;
                    if constexpr (QT == GGML_TYPE_Q5_K) {
                        const uint32_t hb = (hv[i >> 2] >> (8 * (i & 3))) & 0xFF;
                        ql += ((hb >> (2 * g)) & 1) << 4;
                        qhh += ((hb >> (2 * g + 1)) & 1) << 4;
                    }
                    lo[i] = d0 * ql - mm0;
                    hi[i] = d1 * qhh - mm1;
                }
            } else {
#pragma unroll
                for (int i = 0; i < 16; ++i) { lo[i] = 0.f; hi[i] = 0.f; }
            }
            // k_local of lo run = 64*(c>>1) + 16*h ; hi run = +32 ; 16-byte chunk = k_local/8
            const int kl = 64 * (c >> 1) + 16 * (c & 1);
            float t[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) t[i] = lo[i];
            st_h8(lds, r, kl / 8, t);
#pragma unroll
            for (int i = 0; i < 8; ++i) t[i] = lo[8 + i];
            st_h8(lds, r, kl / 8 + 1, t);
#pragma unroll
            for (int i = 0; i < 8; ++i) t[i] = hi[i];
            st_h8(lds, r, (kl + 32) / 8, t);
#pragma unroll
            for (int i = 0; i < 8; ++i) t[i] = hi[8 + i];
            st_h8(lds, r, (kl + 32) / 8 + 1, t);
        }
    } else if constexpr (QT == GGML_TYPE_Q6_K) {
        // 128 rows × 4 l-runs (t) of half n = k0/128 % 2 : 512 units, 2 per thread
#pragma unroll
        for (int it = 0; it < 2; ++it) {
            const int unit = tid + 256 * it;
            const int r = unit >> 2, t = unit & 3;
            const int64_t row = row0 + r;
            float v[4][8];
            if (row < p.M) {
                const int64_t sb = k0 >> 8;
                const int n = (int) ((k0 >> 7) & 1);
                const char * b = wbase + row * p.w_row + sb * 210;
                const float d = h2f(ld_u16(b + 208));
                const char * qlp = b + 64 * n + 8 * t;
                const char * qhp = b + 128 + 32 * n + 8 * t;
                const int8_t * scp = (const int8_t *) (b + 192 + 8 * n + (t >> 1));
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    const uint8_t la = (uint8_t) qlp[i], lb = (uint8_t) qlp[32 + i], hb = (uint8_t) qhp[i];
                    v[0][i] = (float) (((la & 0xF) | (((hb >> 0) & 3) << 4)) - 32);
                    v[1][i] = (float) (((lb & 0xF) | (((hb >> 2) & 3) << 4)) - 32);
                    v[2][i] = (float) (((la >> 4) | (((hb >> 4) & 3) << 4)) - 32);
                    v[3][i] = (float) (((lb >> 4) | (((hb >> 6) & 3) << 4)) - 32);
                }
#pragma unroll
                for (int qq = 0; qq < 4; ++qq) {
                    const float s = d * (float) scp[2 * qq];
#pragma unroll
                    for (int i = 0; i < 8; ++i) v[qq][i] *= s;
                }
            } else {
#pragma unroll
                for (int qq = 0; qq < 4; ++qq)
#pragma unroll
                    for (int i = 0; i < 8; ++i) v[qq][i] = 0.f;
            }
#pragma unroll
            for (int qq = 0; qq < 4; ++qq) st_h8(lds, r, (32 * qq + 8 * t) / 8, v[qq]);
        }
    } else if constexpr (QT == GGML_TYPE_F16) {
        // 128 rows × 16 chunks of 8 halves
#pragma unroll
        for (int it = 0; it < 8; ++it) {
            const int unit = tid + 256 * it;
            const int r = unit >> 4, ch = unit & 15;
            const int64_t row = row0 + r;
            const int64_t k = k0 + 8 * ch;
            uint4 val = make_uint4(0, 0, 0, 0);
            if (row < p.M) {
                const uint16_t * src = (const uint16_t *) (wbase + row * p.w_row) + k;
                if (k + 8 <= p.K && ((uintptr_t) src % 16) == 0) val = *(const uint4 *) src;
                else {
                    uint16_t tmp[8];
#pragma unroll
                    for (int i = 0; i < 8; ++i) tmp[i] = k + i < p.K ? src[i] : 0;
                    val = *(uint4 *) tmp;
                }
            }
            lds[swz(r, ch)] = val;
        }
    } else {
        // generic: 8 consecutive k per unit via exact per-element dequant
#pragma unroll 2
        for (int it = 0; it < 8; ++it) {
            const int unit = tid + 256 * it;
            const int r = unit >> 4, ch = unit & 15;
            const int64_t row = row0 + r;
            const int64_t k = k0 + 8 * ch;
            float v[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const int64_t kk = k + i;
                if (row < p.M && kk < p.K) {
                    const char * rb = wbase + row * p.w_row;
                    if constexpr (QT == GGML_TYPE_F32) v[i] = ((const float *) rb)[kk];
                    else if constexpr (QT == GGML_TYPE_BF16) v[i] = bf2f(((const uint16_t *) rb)[kk]);
                    else v[i] = dequant_one<QT>(rb + (kk / qk_of<QT>()) * qsize_of<QT>(), (int) (kk % qk_of<QT>()));
                } else {
                    v[i] = 0.f;
                }
            }
            st_h8(lds, r, ch, v);
        }
    }
}

template <int QT>
__global__ __launch_bounds__(256, 2) void k_mmq(MmqArgs p) {
    __shared__ uint4 lds_a[MM_BT * MM_BK / 8];   // tokens × K (f16)
    __shared__ uint4 lds_b[MM_BW * MM_BK / 8];   // weight rows × K (f16)
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave >> 1, wn = wave & 1;     // wave's 64-token × 64-row quadrant
    const int64_t tok0 = (int64_t) blockIdx.x * MM_BT;
    const int64_t row0 = (int64_t) blockIdx.y * MM_BW;
    const int64_t ch = blockIdx.z;
    const int64_t i12 = ch % p.ne12, i13 = ch / p.ne12;
    const char * wbase = p.w + (i12 / p.r2) * p.w_c2 + (i13 / p.r3) * p.w_c3;
    const _Float16 * xbase = p.x + ch * p.N * p.kp;

    float16v acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

    const int r = lane & 31, hsel = lane >> 5;
    for (int64_t k0 = 0; k0 < p.K; k0 += MM_BK) {
        // activation tile: 128 tokens × 16 chunks, 8 per thread
#pragma unroll
        for (int it = 0; it < 8; ++it) {
            const int unit = tid + 256 * it;
            const int t = unit >> 4, chn = unit & 15;
            const int64_t tok = tok0 + t;
            uint4 v = make_uint4(0, 0, 0, 0);
            if (tok < p.N) v = *(const uint4 *) (xbase + tok * p.kp + k0 + 8 * chn);
            lds_a[swz(t, chn)] = v;
        }
        load_w_tile<QT>(p, wbase, row0, k0, lds_b);
        __syncthreads();
#pragma unroll
        for (int kk = 0; kk < MM_BK; kk += 16) {
            const int chn = kk / 8 + hsel;
            half8 a[2], b[2];
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const uint4 va = lds_a[swz(wm * 64 + i * 32 + r, chn)];
                a[i] = *(const half8 *) &va;
                const uint4 vb = lds_b[swz(wn * 64 + i * 32 + r, chn)];
                b[i] = *(const half8 *) &vb;
            }
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[i], b[j], acc[i][j], 0, 0, 0);
        }
        __syncthreads();
    }
    // epilogue: C[token][row]; col = lane&31 → weight row, row formula → token
    float * dbase = p.dst + i12 * p.d_c2 + i13 * p.d_c3;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int64_t wrow = row0 + wn * 64 + j * 32 + (lane & 31);
#pragma unroll
            for (int e = 0; e < 16; ++e) {
                const int64_t tok = tok0 + wm * 64 + i * 32 + (e & 3) + 8 * (e >> 2) + 4 * hsel;
                if (tok < p.N && wrow < p.M) dbase[tok * p.d_col + wrow] = acc[i][j][e];
            }
        }
    }
}

// ---------------------------------------------------------------------------
// Pipelined K-quant GEMM (Q4_K / Q5_K / Q6_K, K % 256 == 0): the tile loop of k_mmq with
// the next K step's global loads (activation chunks + raw super-block bytes) issued
// into registers before the current step's MFMAs, dequantised into LDS after them, so
// HBM latency hides behind matrix work. BM weight rows (128, or 64 for small grids so
// the chip stays filled) × 128 tokens per block, 4 waves 2 × 2.
// ---------------------------------------------------------------------------
template <int QT> struct RawW;
template <> struct RawW<GGML_TYPE_Q4_K> { int4 hd, w; };
template <> struct RawW<GGML_TYPE_Q5_K> { int4 hd, w, qh; };
template <> struct RawW<GGML_TYPE_Q6_K> { uint2 la, lb, qh, sc; uint16_t d; };

__device__ __forceinline__ uint2 ldu8(const char * p) {
    uint2 v;
    __builtin_memcpy(&v, __builtin_assume_aligned(p, 2), 8);
    return v;
}

// unit u of the tile: Q4_K/Q5_K (row r = u>>2, 16-byte qs chunk c = u&3 of the half
// super-block), Q6_K (row r = u>>2, 8-wide l-run t = u&3 of the half n)
template <int QT>
__device__ __forceinline__ void raw_load(const MmqArgs & p, const char * wbase, int64_t row, int64_t k0, int c, RawW<QT> & r) {
    const int64_t rr = row < p.M ? row : p.M - 1;   // clamped: the loads stay branch-free
    const int64_t sb = k0 >> 8;
    const int hf = (int) ((k0 >> 7) & 1);
    if constexpr (QT == GGML_TYPE_Q4_K || QT == GGML_TYPE_Q5_K) {
        const char * b = wbase + rr * p.w_row + sb * qsize_of<QT>();
        r.hd = *(const int4 *) b;
        r.w = *(const int4 *) (b + (QT == GGML_TYPE_Q4_K ? 16 : 48) + 16 * (4 * hf + c));
        if constexpr (QT == GGML_TYPE_Q5_K) r.qh = *(const int4 *) (b + 16 + 16 * (c & 1));
    } else {
        const char * b = wbase + rr * p.w_row + sb * 210;
        r.la = ldu8(b + 64 * hf + 8 * c);
        r.lb = ldu8(b + 64 * hf + 32 + 8 * c);
        r.qh = ldu8(b + 128 + 32 * hf + 8 * c);
        r.sc = ldu8(b + 192 + 8 * hf + (c >> 1));
        r.d = ld_u16(b + 208);
    }
}

template <int QT, int CPR = 16>
__device__ __forceinline__ void raw_store(const RawW<QT> & r, int k0, bool valid, int rl, int c, uint4 * lds, int choff = 0) {
    if constexpr (QT == GGML_TYPE_Q4_K || QT == GGML_TYPE_Q5_K) {
        const int hf = (k0 >> 7) & 1;
        const int g = 2 * hf + (c >> 1), h = c & 1;
        // get_scale_min_k4 (ggml-quants.c:703) for all eight sub-blocks at once, four 6-bit
        // values per dword, then this unit's pair (2g, 2g+1) by one select and one shift
        // (as the decode dot, gemv.cuh); value selects only — a runtime-indexed byte pick
        // out of the struct made the raw-weight stages an LDS-promoted alloca
        const uint32_t q0 = (uint32_t) r.hd.y, q1 = (uint32_t) r.hd.z, q2 = (uint32_t) r.hd.w;
        const uint32_t scw = g < 2 ? (q0 & 0x3F3F3F3Fu) : ((q2 & 0x0F0F0F0Fu) | ((q0 >> 2) & 0x30303030u));
        const uint32_t mnw = g < 2 ? (q1 & 0x3F3F3F3Fu) : (((q2 >> 4) & 0x0F0F0F0Fu) | ((q1 >> 2) & 0x30303030u));
        const uint32_t scp = scw >> (16 * (g & 1)), mnp = mnw >> (16 * (g & 1));
        const int s0 = (int) (scp & 0xFF), s1 = (int) ((scp >> 8) & 0xFF);
        const int m0 = (int) (mnp & 0xFF), m1 = (int) ((mnp >> 8) & 0xFF);
        const float d = h2f((uint16_t) (r.hd.x & 0xFFFF)), dmin = h2f((uint16_t) ((uint32_t) r.hd.x >> 16));
        const float d0 = valid ? d * s0 : 0.f, mm0 = valid ? dmin * m0 : 0.f;
        const float d1 = valid ? d * s1 : 0.f, mm1 = valid ? dmin * m1 : 0.f;
        const uint32_t wv[4] = {(uint32_t) r.w.x, (uint32_t) r.w.y, (uint32_t) r.w.z, (uint32_t) r.w.w};
        float lo[16], hi[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const uint32_t byte = (wv[i >> 2] >> (8 * (i & 3))) & 0xFF;
            int ql = byte & 0xF, qhh = byte >> 4;
            if constexpr (QT == GGML_TYPE_Q5_K) {
                const uint32_t hv[4] = {(uint32_t) r.qh.x, (uint32_t) r.qh.y, (uint32_t) r.qh.z, (uint32_t) r.qh.w};
                const uint32_t hb = (hv[i >> 2] >> (8 * (i & 3))) & 0xFF;
                ql += ((hb >> (2 * g)) & 1) << 4;
                qhh += ((hb >> (2 * g + 1)) & 1) << 4;
            }
            lo[i] = d0 * ql - mm0;
            hi[i] = d1 * qhh - mm1;
        }
        const int kl = 64 * (c >> 1) + 16 * h;
        float t[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) t[i] = lo[i];
        st_h8n<CPR>(lds, rl, choff + kl / 8, t);
#pragma unroll
        for (int i = 0; i < 8; ++i) t[i] = lo[8 + i];
        st_h8n<CPR>(lds, rl, choff + kl / 8 + 1, t);
#pragma unroll
        for (int i = 0; i < 8; ++i) t[i] = hi[i];
        st_h8n<CPR>(lds, rl, choff + (kl + 32) / 8, t);
#pragma unroll
        for (int i = 0; i < 8; ++i) t[i] = hi[8 + i];
        st_h8n<CPR>(lds, rl, choff + (kl + 32) / 8 + 1, t);
    } else {
        const float d = valid ? h2f(r.d) : 0.f;
        const uint8_t * la = (const uint8_t *) &r.la, * lb = (const uint8_t *) &r.lb, * hb = (const uint8_t *) &r.qh;
        const int8_t * scp = (const int8_t *) &r.sc;
        float v[4][8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            v[0][i] = (float) (((la[i] & 0xF) | (((hb[i] >> 0) & 3) << 4)) - 32);
            v[1][i] = (float) (((lb[i] & 0xF) | (((hb[i] >> 2) & 3) << 4)) - 32);
            v[2][i] = (float) (((la[i] >> 4) | (((hb[i] >> 4) & 3) << 4)) - 32);
            v[3][i] = (float) (((lb[i] >> 4) | (((hb[i] >> 6) & 3) << 4)) - 32);
        }
#pragma unroll
        for (int qq = 0; qq < 4; ++qq) {
            const float sc = d * (float) scp[2 * qq];
#pragma unroll
            for (int i = 0; i < 8; ++i) v[qq][i] *= sc;
            st_h8n<CPR>(lds, rl, choff + (32 * qq + 8 * c) / 8, v[qq]);
        }
    }
}

template <int QT, int BM>
__global__ __launch_bounds__(256, 2) void k_mmq2(MmqArgs p) {
    constexpr int UPT = BM * 4 / 256;           // weight units per thread per K step
    constexpr int WM = BM / 2;                  // weight rows per wave
    constexpr int TM = WM / 32;                 // 32-row MFMA tiles per wave (1 or 2)
    __shared__ uint4 lds_a[MM_BT * MM_BK / 8];
    __shared__ uint4 lds_b[BM * MM_BK / 8];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave >> 1, wn = wave & 1;    // wave: 64 tokens (wm) x WM weight rows (wn)
    const int64_t tok0 = (int64_t) blockIdx.x * MM_BT;
    const int64_t row0 = (int64_t) blockIdx.y * BM;
    const int64_t ch = blockIdx.z;
    const int64_t i12 = ch % p.ne12, i13 = ch / p.ne12;
    const char * wbase = p.w + (i12 / p.r2) * p.w_c2 + (i13 / p.r3) * p.w_c3;
    const _Float16 * xbase = p.x + ch * p.N * p.kp;
    const int64_t nk = p.K / MM_BK;

    float16v acc[2][TM];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < TM; ++j)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

    uint4 ra[8];
    RawW<QT> rw[UPT];
    auto load = [&](int64_t k0) {
#pragma unroll
        for (int it = 0; it < 8; ++it) {
            const int unit = tid + 256 * it;
            const int t = unit >> 4, chn = unit & 15;
            const int64_t tok = min(tok0 + t, p.N - 1);
            ra[it] = *(const uint4 *) (xbase + tok * p.kp + k0 + 8 * chn);
        }
#pragma unroll
        for (int it = 0; it < UPT; ++it) {
            const int unit = tid + 256 * it;
            raw_load<QT>(p, wbase, row0 + (unit >> 2), k0, unit & 3, rw[it]);
        }
    };
    auto store = [&](int64_t k0) {
#pragma unroll
        for (int it = 0; it < 8; ++it) {
            const int unit = tid + 256 * it;
            const int t = unit >> 4, chn = unit & 15;
            lds_a[swz(t, chn)] = tok0 + t < p.N ? ra[it] : make_uint4(0, 0, 0, 0);
        }
#pragma unroll
        for (int it = 0; it < UPT; ++it) {
            const int unit = tid + 256 * it;
            raw_store<QT>(rw[it], (int) k0, row0 + (unit >> 2) < p.M, unit >> 2, unit & 3, lds_b);
        }
    };

    const int r = lane & 31, hsel = lane >> 5;
    load(0);
    store(0);
    __syncthreads();
    for (int64_t kt = 0; kt < nk; ++kt) {
        if (kt + 1 < nk) load((kt + 1) * MM_BK);       // next step's bytes in flight during the MFMAs
#pragma unroll
        for (int kk = 0; kk < MM_BK; kk += 16) {
            const int chn = kk / 8 + hsel;
            half8 a[2], b[TM];
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const uint4 va = lds_a[swz(wm * 64 + i * 32 + r, chn)];
                a[i] = *(const half8 *) &va;
            }
#pragma unroll
            for (int j = 0; j < TM; ++j) {
                const uint4 vb = lds_b[swz(wn * WM + j * 32 + r, chn)];
                b[j] = *(const half8 *) &vb;
            }
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < TM; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[i], b[j], acc[i][j], 0, 0, 0);
        }
        __syncthreads();
        if (kt + 1 < nk) {
            store((kt + 1) * MM_BK);
            __syncthreads();
        }
    }
    float * dbase = p.dst + i12 * p.d_c2 + i13 * p.d_c3;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
#pragma unroll
        for (int j = 0; j < TM; ++j) {
            const int64_t wrow = row0 + wn * WM + j * 32 + (lane & 31);
#pragma unroll
            for (int e = 0; e < 16; ++e) {
                const int64_t tok = tok0 + wm * 64 + i * 32 + (e & 3) + 8 * (e >> 2) + 4 * hsel;
                if (tok < p.N && wrow < p.M) dbase[tok * p.d_col + wrow] = acc[i][j][e] + (p.res ? p.res[tok * p.r_col + wrow] : 0.f);
            }
        }
    }
}

// 8 waves, K step 256 (a whole super-block per row): waves 0-3 and 4-7 cover the same
// 128-token x 64-row tile over the two 128-wide halves of every K step (kh), so each SIMD
// holds two waves that hide each other's LDS-read / MFMA / dequantisation latencies, and
// every thread stages exactly one 32-weight unit (half kh of the super-block). With four
// waves (one per SIMD) and 128-wide steps, removing the MFMAs, the HBM weight stream and
// the activation loads (g_tune[13]) still left ~75 % of the time: the per-step skeleton
// (staging, dequantisation, barriers) set the pace, so the step is as wide as LDS allows
// (96 KB). Two register stages: step k+2 loads while k computes and k+1 is in flight.
// The halves' accumulators are summed through LDS once, at the end.
constexpr int MM3_BK = 256;
constexpr int MM3_CPR = MM3_BK / 8;             // 16-byte chunks per LDS row

// XCD-aware tile order (workgroup i runs on XCD i % 8): the tiles of one XCD are a
// contiguous run of (token block fastest, row block) tiles, so the token blocks that
// share a weight tile read it through one L2. On when p.dbg & 32 (A/B) or g_xcd_tiles.
__device__ __forceinline__ void mmq_tile_xy(const MmqArgs & p, int & bx, int & by) {
    const int gx = (int) gridDim.x, n = gx * (int) gridDim.y;
    int id = (int) blockIdx.x + gx * (int) blockIdx.y;
    if (MX_DBG(p.dbg & 32) && n % 8 == 0) id = (id % 8) * (n / 8) + id / 8;
    bx = id % gx; by = id / gx;
}

// one 128-token x BM-row output tile (blocks x: tokens, z: batch; the rows are row0..)
template <int QT, int BM>
__device__ __forceinline__ void mmq3_tile(const MmqArgs & p, int64_t row0, int64_t tok0, uint4 * lds) {
    constexpr int NT = 512;
    static_assert(BM * 8 == NT, "one weight unit per thread");
    constexpr int WM = BM / 2;                  // weight rows per wave
    constexpr int TM = WM / 32;                 // 32-row MFMA tiles per wave
    constexpr int NA = MM_BT * MM3_BK / 8 / NT; // activation 16-byte chunks per thread per K step
    static_assert(2 * 4 * TM * 16 * 64 * 4 <= (MM_BT + BM) * MM3_BK * 2, "accumulator exchange fits the tiles");
    uint4 * lds_a = lds;
    uint4 * lds_b = lds + MM_BT * MM3_BK / 8;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int kh = wave >> 2, wq = wave & 3;    // K half of the step; place in the 2 x 2 wave grid
    const int wm = wq >> 1, wn = wq & 1;        // wave: 64 tokens (wm) x WM weight rows (wn)
    const int64_t ch = blockIdx.z;
    const int64_t i12 = ch % p.ne12, i13 = ch / p.ne12;
    const char * wbase = p.w + (i12 / p.r2) * p.w_c2 + (i13 / p.r3) * p.w_c3;
    const _Float16 * xbase = p.x + ch * p.N * p.kp;
    const int64_t nk = MX_DBG(p.dbg & 16) ? 2 : p.K / MM3_BK;
    // this thread's weight unit: half kh (wave-uniform) of row ur's super-block, chunk uc
    const int ur = (tid & 255) >> 2, uc = tid & 3;

    float16v acc[2][TM];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < TM; ++j)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

    uint4 raA[NA], raB[NA];
    RawW<QT> rwA[1], rwB[1];
    auto load = [&](uint4 (&ra)[NA], RawW<QT> (&rw)[1], int64_t kt) {   // unconditional, clamped
        const int64_t k0 = min(kt, nk - 1) * MM3_BK;
#pragma unroll
        for (int it = 0; it < NA; ++it) {
            const int unit = tid + NT * it;
            const int t = unit / MM3_CPR, chn = unit % MM3_CPR;
            const int64_t tok = min(tok0 + t, p.N - 1);
            ra[it] = *(const uint4 *) (xbase + (MX_DBG(p.dbg & 4) ? 8 * chn : tok * p.kp + k0 + 8 * chn));
        }
        raw_load<QT>(p, wbase, MX_DBG(p.dbg & 1) ? row0 : row0 + ur, MX_DBG(p.dbg & 1) ? 0 : k0 + 128 * kh, uc, rw[0]);
    };
    auto store = [&](const uint4 (&ra)[NA], const RawW<QT> (&rw)[1], int64_t kt) {
        const int64_t k0 = min(kt, nk - 1) * MM3_BK;
#pragma unroll
        for (int it = 0; it < NA; ++it) {
            const int unit = tid + NT * it;
            const int t = unit / MM3_CPR, chn = unit % MM3_CPR;
            lds_a[swzn<MM3_CPR>(t, chn)] = tok0 + t < p.N ? ra[it] : make_uint4(0, 0, 0, 0);
        }
        if (!MX_DBG(p.dbg & 8)) raw_store<QT, MM3_CPR>(rw[0], (int) (k0 + 128 * kh), row0 + ur < p.M, ur, uc, lds_b, 16 * kh);
    };

    const int r = lane & 31, hsel = lane >> 5;
    auto mfma_step = [&]() {
#pragma unroll
        for (int kq = 0; kq < MM3_BK / 2; kq += 16) {
            if (MX_DBG(p.dbg & 2)) break;
            const int chn = (kh * (MM3_BK / 2) + kq) / 8 + hsel;
            half8 a[2], b[TM];
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const uint4 va = lds_a[swzn<MM3_CPR>(wm * 64 + i * 32 + r, chn)];
                a[i] = *(const half8 *) &va;
            }
#pragma unroll
            for (int j = 0; j < TM; ++j) {
                const uint4 vb = lds_b[swzn<MM3_CPR>(wn * WM + j * 32 + r, chn)];
                b[j] = *(const half8 *) &vb;
            }
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < TM; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[i], b[j], acc[i][j], 0, 0, 0);
        }
    };
    load(raA, rwA, 0);
    load(raB, rwB, 1);
    store(raA, rwA, 0);
    __syncthreads();
    // straight-line pairs (early exits made the waitcnt pass drain the prefetch at the
    // loop head); an odd last step skips only its MFMAs
    for (int64_t kt = 0; kt < nk; kt += 2) {
        // LDS: step kt; B: step kt+1 in flight; A: free -> step kt+2
        load(raA, rwA, kt + 2);
        mfma_step();
        __syncthreads();
        store(raB, rwB, kt + 1);
        __syncthreads();
        load(raB, rwB, kt + 3);
        if (kt + 1 < nk) mfma_step();                         // workgroup-uniform
        __syncthreads();
        store(raA, rwA, kt + 2);
        __syncthreads();
    }
    // K halves: waves 4-7 hand their accumulators to waves 0-3 (the loop ended on a barrier)
    float * red = (float *) lds;
    if (kh == 1) {
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < TM; ++j)
#pragma unroll
                for (int e = 0; e < 16; ++e) red[(((wq * 2 + i) * TM + j) * 16 + e) * 64 + lane] = acc[i][j][e];
    }
    __syncthreads();
    if (kh == 1) return;
    float * dbase = p.dst + i12 * p.d_c2 + i13 * p.d_c3;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
#pragma unroll
        for (int j = 0; j < TM; ++j) {
            const int64_t wrow = row0 + wn * WM + j * 32 + (lane & 31);
#pragma unroll
            for (int e = 0; e < 16; ++e) {
                const float v = acc[i][j][e] + red[(((wq * 2 + i) * TM + j) * 16 + e) * 64 + lane];
                const int64_t tok = tok0 + wm * 64 + i * 32 + (e & 3) + 8 * (e >> 2) + 4 * hsel;
                if (tok < p.N && wrow < p.M) dbase[tok * p.d_col + wrow] = v + (p.res ? p.res[tok * p.r_col + wrow] : 0.f);
            }
        }
    }
}

template <int QT, int BM>
__global__ __launch_bounds__(512, 2) void k_mmq3(MmqArgs p) {
    __shared__ uint4 lds[(MM_BT + BM) * MM3_BK / 8];
    int bx, by;
    mmq_tile_xy(p, bx, by);
    mmq3_tile<QT, BM>(p, (int64_t) by * BM, (int64_t) bx * MM_BT, lds);
}

// Up to three GEMMs that share the activation (the q/k/v projections of a prefill
// ubatch) in one launch: blockIdx.y runs over the row tiles of all of them, so the
// small k/v grids (64 workgroups each at pp512) fill the CUs beside q's. Segments of
// type QTB (Q4_K_M's Q6_K attn_v) take the second instantiation of the tile.
constexpr int MQ3M_MAX = 3;
struct MmqSegs {
    const char * w[MQ3M_MAX]; size_t w_row[MQ3M_MAX];
    float * dst[MQ3M_MAX]; size_t d_col[MQ3M_MAX];
    int64_t M[MQ3M_MAX];
    int tb0[MQ3M_MAX + 1];                     // first row tile of each segment (prefix sums)
    int isb[MQ3M_MAX];                         // segment of type QTB
    int n;
};

template <int QTA, int QTB>
__global__ __launch_bounds__(512, 2) void k_mmq3m(MmqArgs p, MmqSegs sg) {
    __shared__ uint4 lds[(MM_BT + 64) * MM3_BK / 8];
    int bx, by;
    mmq_tile_xy(p, bx, by);
    int seg = 0;
#pragma unroll
    for (int k = 1; k < MQ3M_MAX; ++k) if (k < sg.n && by >= sg.tb0[k]) seg = k;
    MmqArgs q = p;
    q.w = sg.w[seg]; q.w_row = sg.w_row[seg]; q.dst = sg.dst[seg]; q.d_col = sg.d_col[seg]; q.M = sg.M[seg];
    const int64_t row0 = (int64_t) (by - sg.tb0[seg]) * 64;
    if (sg.isb[seg]) mmq3_tile<QTB, 64>(q, row0, (int64_t) bx * MM_BT, lds);
    else mmq3_tile<QTA, 64>(q, row0, (int64_t) bx * MM_BT, lds);
}

// FFN gate/up/SwiGLU of a prefill ubatch in one pass (MUL_MAT(gate), MUL_MAT(up),
// GLU(SWIGLU) — the decode form is gemv2 EPI 1): the k_mmq3 tile with two weight
// matrices. Waves 0-3 multiply the shared 128-token activation tile by the gate rows,
// waves 4-7 by the up rows, each over the whole 256-wide K step; the up half hands its
// accumulators over through LDS and the gate half writes silu(g)·u. The activation tile
// is staged once for both products, gate and up are never written, and the separate GLU
// pass (a 88 MB read-write at pp512) disappears.
template <int QT>
__global__ __launch_bounds__(512, 2) void k_mmq3g(MmqArgs p) {
    constexpr int NT = 512, BM = 64;
    constexpr int WM = BM / 2, TM = WM / 32;
    constexpr int NA = MM_BT * MM3_BK / 8 / NT;
    constexpr int LB = BM * MM3_BK / 8;          // uint4 per weight tile
    static_assert(2 * 4 * TM * 16 * 64 * 4 <= (MM_BT + 2 * BM) * MM3_BK * 2, "accumulator exchange fits the tiles");
    __shared__ uint4 lds[(MM_BT + 2 * BM) * MM3_BK / 8];
    uint4 * lds_a = lds;
    uint4 * lds_b = lds + MM_BT * MM3_BK / 8;    // [gate | up]
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int mh = wave >> 2, wq = wave & 3;     // matrix (0 gate, 1 up); place in the 2 x 2 wave grid
    const int wm = wq >> 1, wn = wq & 1;
    int bx, by;
    mmq_tile_xy(p, bx, by);
    const int64_t tok0 = (int64_t) bx * MM_BT;
    const int64_t row0 = (int64_t) by * BM;
    const _Float16 * xbase = p.x;
    const int64_t nk = p.K / MM3_BK;
    // this thread's two weight units: half hh of row ur's super-block, chunk uc, of gate and of up
    const int hh = tid >> 8, ur = (tid & 255) >> 2, uc = tid & 3;

    float16v acc[2][TM];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < TM; ++j)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

    uint4 raA[NA], raB[NA];
    RawW<QT> rwA[2], rwB[2];
    auto load = [&](uint4 (&ra)[NA], RawW<QT> (&rw)[2], int64_t kt) {   // unconditional, clamped
        const int64_t k0 = min(kt, nk - 1) * MM3_BK;
#pragma unroll
        for (int it = 0; it < NA; ++it) {
            const int unit = tid + NT * it;
            const int t = unit / MM3_CPR, chn = unit % MM3_CPR;
            const int64_t tok = min(tok0 + t, p.N - 1);
            ra[it] = *(const uint4 *) (xbase + tok * p.kp + k0 + 8 * chn);
        }
        raw_load<QT>(p, p.w, row0 + ur, k0 + 128 * hh, uc, rw[0]);
        raw_load<QT>(p, p.w2, row0 + ur, k0 + 128 * hh, uc, rw[1]);
    };
    auto store = [&](const uint4 (&ra)[NA], const RawW<QT> (&rw)[2], int64_t kt) {
        const int64_t k0 = min(kt, nk - 1) * MM3_BK;
#pragma unroll
        for (int it = 0; it < NA; ++it) {
            const int unit = tid + NT * it;
            const int t = unit / MM3_CPR, chn = unit % MM3_CPR;
            lds_a[swzn<MM3_CPR>(t, chn)] = tok0 + t < p.N ? ra[it] : make_uint4(0, 0, 0, 0);
        }
        raw_store<QT, MM3_CPR>(rw[0], (int) (k0 + 128 * hh), row0 + ur < p.M, ur, uc, lds_b, 16 * hh);
        raw_store<QT, MM3_CPR>(rw[1], (int) (k0 + 128 * hh), row0 + ur < p.M, ur, uc, lds_b + LB, 16 * hh);
    };

    const int r = lane & 31, hsel = lane >> 5;
    const uint4 * lbm = lds_b + mh * LB;
    auto mfma_step = [&]() {
#pragma unroll
        for (int kk = 0; kk < MM3_BK; kk += 16) {
            const int chn = kk / 8 + hsel;
            half8 a[2], b[TM];
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const uint4 va = lds_a[swzn<MM3_CPR>(wm * 64 + i * 32 + r, chn)];
                a[i] = *(const half8 *) &va;
            }
#pragma unroll
            for (int j = 0; j < TM; ++j) {
                const uint4 vb = lbm[swzn<MM3_CPR>(wn * WM + j * 32 + r, chn)];
                b[j] = *(const half8 *) &vb;
            }
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < TM; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[i], b[j], acc[i][j], 0, 0, 0);
        }
    };
    load(raA, rwA, 0);
    load(raB, rwB, 1);
    store(raA, rwA, 0);
    __syncthreads();
    for (int64_t kt = 0; kt < nk; kt += 2) {
        load(raA, rwA, kt + 2);
        mfma_step();
        __syncthreads();
        store(raB, rwB, kt + 1);
        __syncthreads();
        load(raB, rwB, kt + 3);
        if (kt + 1 < nk) mfma_step();                          // workgroup-uniform
        __syncthreads();
        store(raA, rwA, kt + 2);
        __syncthreads();
    }
    float * red = (float *) lds;
    if (mh == 1) {
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < TM; ++j)
#pragma unroll
                for (int e = 0; e < 16; ++e) red[(((wq * 2 + i) * TM + j) * 16 + e) * 64 + lane] = acc[i][j][e];
    }
    __syncthreads();
    if (mh == 1) return;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
#pragma unroll
        for (int j = 0; j < TM; ++j) {
            const int64_t wrow = row0 + wn * WM + j * 32 + (lane & 31);
#pragma unroll
            for (int e = 0; e < 16; ++e) {
                const float g = acc[i][j][e], u = red[(((wq * 2 + i) * TM + j) * 16 + e) * 64 + lane];
                const int64_t tok = tok0 + wm * 64 + i * 32 + (e & 3) + 8 * (e >> 2) + 4 * hsel;
                const float v = (g / (1.0f + expf(-g))) * u;
                if (tok < p.N && wrow < p.M) {
                    p.dst[tok * p.d_col + wrow] = v;
                    if (p.h) p.h[tok * p.h_col + wrow] = (_Float16) v;
                }
            }
        }
    }
}

static bool g_mmq_v1 = getenv("GGML_MI355X_MMQ_V1") != nullptr;
static const bool g_act_claim_off = getenv("GGML_MI355X_NO_ACT_CLAIM") != nullptr;   // A/B

bool mmq_type_ok(int t) {
    switch (t) {
        case GGML_TYPE_Q4_0: case GGML_TYPE_Q4_1: case GGML_TYPE_Q5_0: case GGML_TYPE_Q5_1: case GGML_TYPE_Q8_0:
        case GGML_TYPE_Q4_K: case GGML_TYPE_Q5_K: case GGML_TYPE_Q6_K:
        case GGML_TYPE_F16: case GGML_TYPE_F32: case GGML_TYPE_BF16:
            return true;
        default: return false;
    }
}

static int64_t mmq_kp(const ggml_tensor * dst) { return mx_ceil_div(dst->src[0]->ne[0], MM_BK) * MM_BK; }

size_t mmq_scratch(const ggml_tensor * dst) {
    const ggml_tensor * x = dst->src[1];
    const int64_t ncols = x->ne[1] * x->ne[2] * x->ne[3];
    return ncols * mmq_kp(dst) * 2 + 256;
}

// A producer of a prefill GEMM's input (RMS norm, attention, fused SwiGLU) writes the f16
// copy itself: it claims the cache slot for its f32 output rows (data, K, ncols, row
// stride) and the GEMM's mmq_act finds it — no separate conversion pass. Rows of K %
// 128 == 0 only (kp == K, no padding to write); null when the slot does not fit.
_Float16 * mmq_act_claim(OpCtx & c, const void * data, int64_t K, int64_t ncols, size_t row_bytes) {
    Stream * s = c.s;
    if (g_act_claim_off || K % MM_BK || ncols <= 8 || !s->f16.base || (size_t) K * ncols * 2 > s->f16.cap) return nullptr;
    const int64_t key[4] = {K, ncols, (int64_t) row_bytes, K};
    const int k = 1 - s->f16_last;             // not the slot the running kernel may be reading
    s->f16_src[k] = data;
    memcpy(s->f16_key[k], key, sizeof key);
    s->f16_last = k;
    return (_Float16 *) s->f16.base + (size_t) k * (s->f16.cap / 2);
}

// f32 activation -> f16 rows padded to kp, cached by (tensor, K, ncols) so GEMMs that
// share their input (q/k/v, gate/up) convert it once
static _Float16 * mmq_act(OpCtx & c, const ggml_tensor * x, int64_t kp) {
    const int64_t ncols = x->ne[1] * x->ne[2] * x->ne[3];
    const size_t abytes = (size_t) ncols * kp * 2;
    Stream * s = c.s;
    _Float16 * xa;
    const int64_t key[4] = {x->ne[0], ncols, (int64_t) x->nb[1], kp};
    const bool cacheable = s->f16.base && abytes <= s->f16.cap && mx_is_contiguous(x);
    auto slot = [&](int k) { return (_Float16 *) s->f16.base + (size_t) k * (s->f16.cap / 2); };
    for (int k = 0; k < 2 && cacheable; ++k)
        if (s->f16_src[k] == x->data && !memcmp(s->f16_key[k], key, sizeof key)) {
            s->f16_last = k;                // same activation as an earlier GEMM / its producer
            return slot(k);
        }
    const int k = 1 - s->f16_last;
    xa = cacheable ? slot(k) : (_Float16 *) c.scratch->take(abytes);
    dim3 grid((unsigned) mx_ceil_div(kp, 8 * 256), (unsigned) ncols);
    k_act_f16<<<grid, 256, 0, c.st>>>((const char *) x->data, x->ne[0], x->ne[1], x->ne[2],
                                      x->nb[0], x->nb[1], x->nb[2], x->nb[3], kp, xa);
    if (cacheable) { s->f16_src[k] = x->data; memcpy(s->f16_key[k], key, sizeof key); s->f16_last = k; }
    return xa;
}
_Float16 * mmq_act_f16(OpCtx & c, const ggml_tensor * x, int64_t kp) { return mmq_act(c, x, kp); }

// out (default dst) receives the product, + res when given (K-quant MFMA kernels only:
// the caller checks mmq_kq_ok)
static void mmq_run_ex(OpCtx & c, ggml_tensor * dst, ggml_tensor * out, const ggml_tensor * res) {
    const ggml_tensor * w = dst->src[0];
    const ggml_tensor * x = dst->src[1];
    const int64_t kp = mmq_kp(dst);
    _Float16 * xa = mmq_act(c, x, kp);
    MmqArgs p{};
    p.w = (const char *) w->data; p.w_row = w->nb[1]; p.w_c2 = w->nb[2]; p.w_c3 = w->nb[3];
    p.x = xa; p.kp = kp;
    p.dst = (float *) out->data; p.d_col = out->nb[1] / 4; p.d_c2 = out->nb[2] / 4; p.d_c3 = out->nb[3] / 4;
    if (res) { p.res = (const float *) res->data; p.r_col = res->nb[1] / 4; }
    p.M = w->ne[1]; p.N = x->ne[1]; p.K = w->ne[0]; p.ne12 = x->ne[2];
    p.r2 = x->ne[2] / w->ne[2]; p.r3 = x->ne[3] / w->ne[3];
    p.dbg = MX_AB_VARIANTS ? g_tune[13] : 0;
    const bool kq = w->type == GGML_TYPE_Q4_K || w->type == GGML_TYPE_Q5_K || w->type == GGML_TYPE_Q6_K;
    // (round 5: Q8_0 too — k_mmq4's Q8_0 B operand; the k_mmq2/3 paths below are K-quant only)
    if ((kq || w->type == GGML_TYPE_Q8_0) && !g_mmq_v1 && p.K % 256 == 0 && mmq4_mul_mat(c, w, x, xa, kp, out, res)) return;
    if (kq && !g_mmq_v1 && p.K % 256 == 0) {
        const int64_t tiles128 = mx_ceil_div(p.N, MM_BT) * mx_ceil_div(p.M, 128) * (x->ne[2] * x->ne[3]);
        int bm = tiles128 < 512 ? 64 : 128;
        if (g_tune[8]) bm = g_tune[8];   // sweeps
        dim3 g2((unsigned) mx_ceil_div(p.N, MM_BT), (unsigned) mx_ceil_div(p.M, bm), (unsigned) (x->ne[2] * x->ne[3]));
        // one round of 64-row tiles on the CUs: the 8-wave kernel (two waves per SIMD, K
        // step split between the wave halves) — pp512 q/k/v/o 51 -> 44 us, down 203 -> 189;
        // larger grids keep the 4-wave kernel, two of whose workgroups share a CU
        // (gate/up 131 vs 163 us, profiles/r01/opbench_mmq_dbg.txt)
        const bool w8 = g_tune[5] == 1 || (g_tune[5] == 0 && bm == 64 && (int64_t) g2.x * g2.y * g2.z <= 256);
        MX_KLOG("mmq%d qt=%d bm=%d M=%lld N=%lld K=%lld res=%d", w8 && bm == 64 ? 3 : 2, (int) w->type, bm,
                (long long) p.M, (long long) p.N, (long long) p.K, res != nullptr);
        if (w8 && bm == 64) {
#define MQ3(T) case T: k_mmq3<T, 64><<<g2, 512, 0, c.st>>>(p); return;
            switch (w->type) { MQ3(GGML_TYPE_Q4_K) MQ3(GGML_TYPE_Q5_K) MQ3(GGML_TYPE_Q6_K) default: break; }
#undef MQ3
        }
#define MQ2(T) case T: if (bm == 64) k_mmq2<T, 64><<<g2, 256, 0, c.st>>>(p); else k_mmq2<T, 128><<<g2, 256, 0, c.st>>>(p); return;
        switch (w->type) { MQ2(GGML_TYPE_Q4_K) MQ2(GGML_TYPE_Q5_K) MQ2(GGML_TYPE_Q6_K) default: break; }
#undef MQ2
    }
    MX_ASSERT(!res && out == dst);
    dim3 grid((unsigned) mx_ceil_div(p.N, MM_BT), (unsigned) mx_ceil_div(p.M, MM_BW), (unsigned) (x->ne[2] * x->ne[3]));
    MX_KLOG("mmq1 qt=%d M=%lld N=%lld K=%lld", (int) w->type, (long long) p.M, (long long) p.N, (long long) p.K);
    switch (w->type) {
#define MQ(T) case T: k_mmq<T><<<grid, 256, 0, c.st>>>(p); break;
        MQ(GGML_TYPE_Q4_0) MQ(GGML_TYPE_Q4_1) MQ(GGML_TYPE_Q5_0) MQ(GGML_TYPE_Q5_1) MQ(GGML_TYPE_Q8_0)
        MQ(GGML_TYPE_Q4_K) MQ(GGML_TYPE_Q5_K) MQ(GGML_TYPE_Q6_K)
        MQ(GGML_TYPE_F16) MQ(GGML_TYPE_F32) MQ(GGML_TYPE_BF16)
#undef MQ
        default: MX_ABORT("mmq type %d", (int) w->type);
    }
}

void mmq_run(OpCtx & c, ggml_tensor * dst) { mmq_run_ex(c, dst, dst, nullptr); }

static bool mmq_ok(const ggml_tensor * dst);
// A/B: GGML_MI355X_NO_MMQ_GLU=1 turns off the prefill GEMM fusions (gate/up/SwiGLU, + residual)
static const bool g_mmq_glu_off = getenv("GGML_MI355X_NO_MMQ_GLU") != nullptr;

// MUL_MAT -> ADD(mm, residual) of a prefill ubatch: the residual is added in the GEMM
// epilogue (attention output and FFN down projections: no product round trip, no ADD pass)
bool mmq_fused_add(OpCtx & c, const ggml_tensor * mm, const ggml_tensor * res, ggml_tensor * add) {
    const ggml_tensor * w = mm->src[0], * x = mm->src[1];
    const bool kq = w->type == GGML_TYPE_Q4_K || w->type == GGML_TYPE_Q5_K || w->type == GGML_TYPE_Q6_K;
    if (!kq || g_mmq_v1 || g_mmq_glu_off || w->ne[0] % 256 || x->ne[1] <= 8 || !mmq_ok(mm)) return false;
    if (x->ne[2] != 1 || x->ne[3] != 1 || w->ne[2] != 1 || w->ne[3] != 1) return false;
    if (res->type != GGML_TYPE_F32 || add->type != GGML_TYPE_F32 || !mx_are_same_shape(res, mm) || !mx_are_same_shape(add, mm)) return false;
    if (res->nb[0] != 4 || add->nb[0] != 4 || res->nb[1] % 4 || add->nb[1] % 4) return false;
    deferred_guard_read(c, x);
    deferred_guard_read(c, res);
    deferred_guard_write(c, add);
    mmq_run_ex(c, const_cast<ggml_tensor *>(mm), add, res);
    return true;
}


// MUL_MAT -> ADD(residual) -> RMS_NORM -> MUL(w) of a prefill ubatch (round 3): the output
// projection + ffn_norm and the FFN down projection + the next layer's attn_norm. After
// the GEMM, ONE pass per token row sums its split-K partial planes (or reads the plain
// product), adds the residual, stores the sum (the next residual) and writes the norm·w
// rows with their f16 copy for the next GEMM — instead of k_mmq4_reduce (+ residual) and
// k_rms_norm_v4, which re-read the sum. The arithmetic is the two kernels' own: planes in
// order, then the residual; k_rms_norm_v4's per-thread float4 sums and block_sum.
template <int VPT, bool SPLIT>
__global__ __launch_bounds__(256) void k_add_rms_norm(const float * __restrict__ part, int part_ld, int ks, int N,
                                                      const float * prod, size_t p_col,
                                                      const float * res, size_t r_col, float * add, size_t a_col,
                                                      const float * __restrict__ w, float * __restrict__ y, size_t y_col,
                                                      float eps, int n, _Float16 * __restrict__ h) {
    __shared__ float lds[16];
    const int t = blockIdx.x, n4 = n / 4;
    const float4 * pr = (const float4 *) (res + (size_t) t * r_col);
    float4 * pa = (float4 *) (add + (size_t) t * a_col);
    float4 v[VPT];
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < VPT; ++j) {
        const int i = threadIdx.x + 256 * j, ii = min(i, n4 - 1);
        float4 a;
        if constexpr (SPLIT) {
            const float4 * pp = (const float4 *) (part + (size_t) t * part_ld) + ii;
            a = pp[0];
            for (int z = 1; z < ks; ++z) {
                const float4 b = pp[(size_t) z * N * part_ld / 4];
                a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
            }
        } else a = ((const float4 *) (prod + (size_t) t * p_col))[ii];
        const float4 r = pr[ii];
        a.x += r.x; a.y += r.y; a.z += r.z; a.w += r.w;
        v[j] = a;
        if (i < n4) s += a.x * a.x + a.y * a.y + a.z * a.z + a.w * a.w;
    }
    s = block_sum(s, lds);                  // (its barriers also order every read of res before the stores)
    const float scale = 1.0f / sqrtf(s / (float) n + eps);
    const float4 * pw = (const float4 *) w;
    float4 * py = (float4 *) (y + (size_t) t * y_col);
#pragma unroll
    for (int j = 0; j < VPT; ++j) {
        const int i = threadIdx.x + 256 * j;
        if (i >= n4) break;
        pa[i] = v[j];
        float4 o = make_float4(v[j].x * scale, v[j].y * scale, v[j].z * scale, v[j].w * scale);
        const float4 wv = pw[i];
        o.x *= wv.x; o.y *= wv.y; o.z *= wv.z; o.w *= wv.w;
        py[i] = o;
        if (h) {
            typedef _Float16 h4 __attribute__((ext_vector_type(4)));
            *(h4 *) (h + (size_t) t * n + 4 * i) = h4{(_Float16) o.x, (_Float16) o.y, (_Float16) o.z, (_Float16) o.w};
        }
    }
}

static const bool g_no_add_norm = getenv("GGML_MI355X_NO_ADD_NORM_FUSION") != nullptr;   // A/B
bool mm_add_rms_norm(OpCtx & c, ggml_tensor * mm, const ggml_tensor * res, ggml_tensor * add, const ggml_tensor * norm,
                     const ggml_tensor * w, ggml_tensor * mul) {
    if (g_no_add_norm || (g_tune[27] & 512)) return false;
    const ggml_tensor * wt = mm->src[0], * x = mm->src[1];
    const bool kq = wt->type == GGML_TYPE_Q4_K || wt->type == GGML_TYPE_Q5_K || wt->type == GGML_TYPE_Q6_K;
    if (!kq || g_mmq_v1 || g_mmq_glu_off || wt->ne[0] % 256 || x->ne[1] <= 8 || !mmq_ok(mm)) return false;
    if (x->ne[2] != 1 || x->ne[3] != 1 || wt->ne[2] != 1 || wt->ne[3] != 1) return false;
    const int64_t n = add->ne[0], N = add->ne[1];
    auto rows16 = [&](const ggml_tensor * t) {
        return t->type == GGML_TYPE_F32 && t->ne[0] == n && t->ne[1] == N && t->ne[2] == 1 && t->ne[3] == 1 && t->nb[0] == 4 &&
               t->nb[1] % 16 == 0 && (uintptr_t) t->data % 16 == 0;
    };
    if (!rows16(add) || !rows16(res) || !rows16(mul) || !mx_are_same_shape(add, mm) || N > INT32_MAX) return false;
    if (n % 4 || n < 128 || n > 4 * 256 * 8) return false;
    if (w->type != GGML_TYPE_F32 || mx_nelements(w) != n || !mx_is_contiguous(w) || (uintptr_t) w->data % 16) return false;
    // The norm rows are written while other rows' sums are still being read: mul must not
    // overlap add or w, and res only exactly (the workgroup of row t reads res row t before
    // it writes mul row t — block_sum's barriers). x is consumed by the GEMM (through its f16
    // copy) before this pass starts, so mul may reuse x's memory: libllama's allocator places
    // the norm there (x, the SwiGLU or attention output, dies at the GEMM) — refusing that
    // overlap had kept the fusion off in every drop-in prefill (r03 drop-in pp512 profile:
    // 62 k_mmq4_reduce + 62 k_rms_norm_v4 launches per ubatch, profiles/r04/).
    const bool mul_on_res = mul->data == res->data && mul->nb[1] == res->nb[1];
    if (t_overlaps_ext(mul, add) || (!mul_on_res && t_overlaps_ext(mul, res)) || t_overlaps_ext(mul, w)) return false;
    if (add->data != res->data && t_overlaps_ext(add, res)) return false;
    // every refusal comes before the deferred-norm guards act (mmq4_scratch sizes the arena
    // for this product and the split-K planes together)
    if (add->data == res->data && c.scratch->avail() < (size_t) n * N * 4 + 256) return false;
    deferred_guard_read(c, x);
    deferred_guard_read(c, res);
    deferred_guard_write(c, add);
    deferred_guard_write(c, mul);
    // the product alone (the residual is added below), into add — or, when the ADD runs in
    // place over the residual, into scratch (unless the GEMM splits: then only partials)
    ggml_tensor prod = *add;
    if (add->data == res->data) {
        prod.data = c.scratch->take((size_t) n * N * 4);
        prod.nb[1] = (size_t) n * 4; prod.nb[2] = prod.nb[3] = (size_t) n * N * 4;
    }
    M4Split sp{};
    g_m4_split = &sp;
    mmq_run_ex(c, mm, &prod, nullptr);
    g_m4_split = nullptr;
    act_cache_invalidate(c.s, mul);   // (after the GEMM: mul may lie over x, whose f16 copy it read)
    const float eps = mx_op_param<float>(norm, 0);
    _Float16 * h = mmq_act_claim(c, mul->data, n, N, mul->nb[1]);
    const int vpt = (int) mx_ceil_div(n / 4, 256);
    MX_KLOG("add_rms_norm n=%lld N=%lld ks=%d", (long long) n, (long long) N, sp.ks);
#define AN(V, S) k_add_rms_norm<V, S><<<(unsigned) N, 256, 0, c.st>>>(sp.part, sp.part_ld, sp.ks, (int) N, (const float *) prod.data, \
        prod.nb[1] / 4, (const float *) res->data, \
        res->nb[1] / 4, (float *) add->data, add->nb[1] / 4, (const float *) w->data, (float *) mul->data, mul->nb[1] / 4, eps, (int) n, h)
    if (sp.ks > 1) { if (vpt <= 2) AN(2, true); else if (vpt <= 4) AN(4, true); else AN(8, true); }
    else { if (vpt <= 2) AN(2, false); else if (vpt <= 4) AN(4, false); else AN(8, false); }
#undef AN
    return true;
}

bool mmq_fused_glu(OpCtx & c, const ggml_tensor * gate, const ggml_tensor * up, ggml_tensor * glu) {
    const ggml_tensor * wg = gate->src[0], * wu = up->src[0];
    const ggml_tensor * x = gate->src[1];
    if (g_mmq_glu_off || g_mmq_v1 || up->src[1] != x || wg->type != wu->type) return false;
    if (wg->type != GGML_TYPE_Q4_K && wg->type != GGML_TYPE_Q5_K && wg->type != GGML_TYPE_Q6_K && wg->type != GGML_TYPE_Q8_0) return false;
    if (wg->type == GGML_TYPE_Q8_0 && !mmq4_glu_ok(wg, wu, x, glu)) return false;   // k_mmq4 only (round 5)
    if (mx_op_param<int32_t>(glu, 0) != GGML_GLU_OP_SWIGLU || mx_op_param<int32_t>(glu, 1) != 0) return false;
    if (x->type != GGML_TYPE_F32 || x->ne[1] <= 8 || x->ne[2] != 1 || x->ne[3] != 1) return false;
    for (int i = 0; i < 4; ++i) if (wg->ne[i] != wu->ne[i] || wg->nb[i] != wu->nb[i]) return false;
    if (wg->ne[2] != 1 || wg->ne[3] != 1 || wg->ne[0] % 256 || x->ne[0] != wg->ne[0]) return false;
    if (!mmq_ok(gate) || !mmq_ok(up)) return false;
    if (glu->type != GGML_TYPE_F32 || glu->nb[0] != 4 || glu->ne[0] != wg->ne[1] || glu->ne[1] != x->ne[1]) return false;
    deferred_guard_read(c, x);
    deferred_guard_write(c, glu);
    const int64_t kp = mmq_kp(gate);
    MmqArgs p{};
    p.w = (const char *) wg->data; p.w2 = (const char *) wu->data; p.w_row = wg->nb[1];
    p.x = mmq_act(c, x, kp); p.kp = kp;
    if (mmq4_glu_ok(wg, wu, x, glu)) {
        _Float16 * h = mmq_act_claim(c, glu->data, glu->ne[0], glu->ne[1], glu->nb[1]);
        mmq4_glu(c, wg, wu, x, p.x, kp, glu, h, glu->ne[0]);
        return true;
    }
    p.dst = (float *) glu->data; p.d_col = glu->nb[1] / 4;
    p.M = wg->ne[1]; p.N = x->ne[1]; p.K = wg->ne[0]; p.ne12 = 1; p.r2 = 1; p.r3 = 1; p.dbg = MX_AB_VARIANTS ? g_tune[13] : 0;
    // the down projection reads this output: write its f16 copy too (claimed after the
    // input conversion above, which used the same slot)
    p.h = mmq_act_claim(c, glu->data, glu->ne[0], glu->ne[1], glu->nb[1]);
    p.h_col = glu->ne[0];
    const dim3 g((unsigned) mx_ceil_div(p.N, MM_BT), (unsigned) mx_ceil_div(p.M, 64), 1);
    MX_KLOG("mmq3g qt=%d M=%lld N=%lld K=%lld", (int) wg->type, (long long) p.M, (long long) p.N, (long long) p.K);
    switch (wg->type) {
        case GGML_TYPE_Q4_K: k_mmq3g<GGML_TYPE_Q4_K><<<g, 512, 0, c.st>>>(p); break;
        case GGML_TYPE_Q5_K: k_mmq3g<GGML_TYPE_Q5_K><<<g, 512, 0, c.st>>>(p); break;
        default:             k_mmq3g<GGML_TYPE_Q6_K><<<g, 512, 0, c.st>>>(p); break;
    }
    return true;
}

// q/k/v of a prefill ubatch in one launch (k_mmq3m): members share src1, K-quant weights
// of at most two types (the first member's, and one other), K % 256 == 0
static bool kq_type(int t) { return t == GGML_TYPE_Q4_K || t == GGML_TYPE_Q5_K || t == GGML_TYPE_Q6_K; }

bool mmq_group_run(OpCtx & c, ggml_tensor * const * mms, int n) {
    if (n < 2 || n > MQ3M_MAX || g_mmq_v1 || g_mmq_glu_off || g_tune[5] == 2) return false;
    const ggml_tensor * x = mms[0]->src[1];
    const int ta = mms[0]->src[0]->type;
    int tb = ta;
    for (int k = 0; k < n; ++k) {
        const ggml_tensor * m = mms[k], * w = m->src[0];
        if (m->src[1] != x || !(kq_type(w->type) || w->type == GGML_TYPE_Q8_0) || !mmq_ok(m)) return false;
        if (w->ne[0] != x->ne[0] || w->ne[0] % 256 || w->ne[2] != 1 || w->ne[3] != 1) return false;
        if (m->type != GGML_TYPE_F32 || m->nb[0] != 4 || m->ne[2] != 1 || m->ne[3] != 1) return false;
        if (w->type != ta) { if (tb != ta && tb != w->type) return false; tb = w->type; }
    }
    if (x->type != GGML_TYPE_F32 || x->ne[1] <= 8 || x->ne[2] != 1 || x->ne[3] != 1) return false;
    if (ta == GGML_TYPE_Q8_0 || tb == GGML_TYPE_Q8_0) {   // round 5: k_mmq4 only (the 8-expert recipe's q8_0 k / v)
        const int64_t kp8 = mmq_kp(mms[0]);
        return mmq4_group(c, mms, n, mmq_act(c, x, kp8), kp8);
    }
    const bool combo = (ta == GGML_TYPE_Q6_K || tb == GGML_TYPE_Q6_K || ta == tb) && !(ta == GGML_TYPE_Q5_K && tb == GGML_TYPE_Q4_K) &&
                       !(ta == GGML_TYPE_Q4_K && tb == GGML_TYPE_Q5_K);
    if (!combo || (ta == GGML_TYPE_Q6_K && tb == GGML_TYPE_Q5_K)) return false;
    const int64_t kp = mmq_kp(mms[0]);
    MmqArgs p{};
    p.x = mmq_act(c, x, kp); p.kp = kp;
    if (mmq4_group(c, mms, n, p.x, kp)) return true;
    p.N = x->ne[1]; p.K = x->ne[0]; p.ne12 = 1; p.r2 = 1; p.r3 = 1; p.dbg = MX_AB_VARIANTS ? g_tune[13] : 0;
    MmqSegs sg{};
    sg.n = n;
    sg.tb0[0] = 0;
    for (int k = 0; k < n; ++k) {
        const ggml_tensor * m = mms[k], * w = m->src[0];
        sg.w[k] = (const char *) w->data; sg.w_row[k] = w->nb[1];
        sg.dst[k] = (float *) m->data; sg.d_col[k] = m->nb[1] / 4; sg.M[k] = w->ne[1];
        sg.isb[k] = w->type != ta;
        sg.tb0[k + 1] = sg.tb0[k] + (int) mx_ceil_div(w->ne[1], 64);
    }
    const dim3 g((unsigned) mx_ceil_div(p.N, MM_BT), (unsigned) sg.tb0[n], 1);
    MX_KLOG("mmq3m n=%d qta=%d qtb=%d N=%lld K=%lld", n, ta, tb, (long long) p.N, (long long) p.K);
#define M3M(A, B) if (ta == A && tb == B) { k_mmq3m<A, B><<<g, 512, 0, c.st>>>(p, sg); return true; }
    M3M(GGML_TYPE_Q4_K, GGML_TYPE_Q4_K) M3M(GGML_TYPE_Q4_K, GGML_TYPE_Q6_K) M3M(GGML_TYPE_Q6_K, GGML_TYPE_Q4_K)
    M3M(GGML_TYPE_Q5_K, GGML_TYPE_Q5_K) M3M(GGML_TYPE_Q5_K, GGML_TYPE_Q6_K) M3M(GGML_TYPE_Q6_K, GGML_TYPE_Q6_K)
#undef M3M
    return false;
}

// ---------------------------------------------------------------------------
// MUL_MAT dispatch
// ---------------------------------------------------------------------------
static bool quant_fast_path_ok(const ggml_tensor * dst) {
    const ggml_tensor * w = dst->src[0];
    const ggml_tensor * x = dst->src[1];
    if (!mmvq_type_ok(w->type)) return false;
    if (x->type != GGML_TYPE_F32 || dst->nb[0] != 4) return false;
    if (w->nb[0] != (size_t) mx_type(w->type).size) return false;    // rows of whole blocks
    if (w->ne[0] % qk_of_type(w->type) != 0) return false;
    if (x->nb[0] != 4) return false;
    return true;
}

static bool mmq_ok(const ggml_tensor * dst) {
    const ggml_tensor * w = dst->src[0];
    const ggml_tensor * x = dst->src[1];
    if (!mmq_type_ok(w->type) || x->type != GGML_TYPE_F32 || dst->nb[0] != 4) return false;
    if (w->nb[0] != (size_t) mx_type(w->type).size) return false;
    if (mx_type(w->type).quant && w->ne[0] % qk_of_type(w->type) != 0) return false;
    // K-quant tile loaders step through whole 128-wide halves of super-blocks
    if ((w->type == GGML_TYPE_Q4_K || w->type == GGML_TYPE_Q5_K || w->type == GGML_TYPE_Q6_K) && w->ne[0] % 256 != 0) return false;
    if ((w->type == GGML_TYPE_F16) && (w->nb[1] % 16 != 0)) return false;
    return true;
}

bool mul_mat_supported(const ggml_tensor * dst) {
    const ggml_tensor * w = dst->src[0];
    const ggml_tensor * x = dst->src[1];
    if (dst->type != GGML_TYPE_F32 || x->type != GGML_TYPE_F32) return false;
    if (x->ne[2] % w->ne[2] != 0 || x->ne[3] % w->ne[3] != 0) return false;
    switch (w->type) {
        case GGML_TYPE_F32: case GGML_TYPE_F16: case GGML_TYPE_BF16:
        case GGML_TYPE_Q4_0: case GGML_TYPE_Q4_1: case GGML_TYPE_Q5_0: case GGML_TYPE_Q5_1: case GGML_TYPE_Q8_0:
        case GGML_TYPE_Q4_K: case GGML_TYPE_Q5_K: case GGML_TYPE_Q6_K:
            break;
        default: return false;
    }
    if (mx_type(w->type).quant && w->nb[0] != (size_t) mx_type(w->type).size) return false;
    return true;
}

bool mm_skinny_run(OpCtx & c, ggml_tensor * dst);   // ops_mmvq.hip

size_t mmq_act_bytes(const ggml_tensor * dst) {
    const ggml_tensor * x = dst->src[1];
    // MoE prefill (round 5): the expert GEMMs' input, and the fused gate/up SwiGLU's f16
    // output claimed for the down projection (ne0 x n_used x n_tok, ~29 MB for Mixtral pp512)
    if (dst->op == GGML_OP_MUL_MAT_ID) return mmq4_moe_scratch(dst) ? (size_t) x->ne[0] * x->ne[1] * x->ne[2] * 2 : 0;
    if (dst->op != GGML_OP_MUL_MAT || x->ne[1] <= 8 || !mmq_ok(dst)) return 0;
    return (size_t) x->ne[1] * x->ne[2] * x->ne[3] * mmq_kp(dst) * 2;
}

size_t mul_mat_scratch(const ggml_tensor * dst, bool add_norm) {
    const ggml_tensor * x = dst->src[1];
    size_t s = 0;
    if (x->ne[1] <= 8 && quant_fast_path_ok(dst)) s = quantize_scratch(x);
    else if (mmq_ok(dst)) s = mmq_scratch(dst) + mmq4_scratch(dst, add_norm);
    return s;
}

void op_mul_mat(OpCtx & c, ggml_tensor * dst) {
    const ggml_tensor * x = dst->src[1];
    if (g_gemv2 && gemv2_ok(dst->src[0], x, dst)) {
        gemv2_launch(c, dst->src[0], nullptr, xstage_of(c.s, x), (float *) dst->data, nullptr);
        return;
    }
    if (x->ne[1] <= 8 && gemv_nc_ok(dst)) { gemv_nc_run(c, dst); return; }
    if (x->ne[1] <= 8 && quant_fast_path_ok(dst)) { mmvq_run(c, dst); return; }
    if (x->ne[1] > 8 && mm_skinny_run(c, dst)) return;   // few f32/f16 rows (the MoE router in prefill)
    if (x->ne[1] > 8 && mmq_ok(dst)) { mmq_run(c, dst); return; }
    mmv_generic_run(c, dst);
}

}  // namespace mx
