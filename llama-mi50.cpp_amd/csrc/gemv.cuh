// gemv.cuh — building blocks of the single-column decode GEMV (y = W·x, one token),
// the hot loop of llama-bench tg (reference: mul_mat_vec_q, ggml-cuda/mmvq.cu:142-356,
// vec_dot_q*_K_q8_1 vecdotq.cuh:461-867).
//
// MI355X design (v2)
//  * prologue: every workgroup reads the f32 activation x (L2-resident, written by the
//    previous kernel), optionally applies the RMS norm · weight that precedes it in the
//    graph (build_norm, src/llama-graph.cpp), and quantises it into LDS: int8 q[K],
//    f32 d[K/32] and d·Σq [K/32] (quantize_q8_1 semantics, ggml-cuda/quantize.cu:5-48,
//    with the CPU's s = d·Σq, ggml-quants.c:270-300). No separate quantise or norm
//    launch, no global round trip of the quantised activation;
//  * the weight loads of all a lane's units are issued before the prologue runs, so the
//    HBM latency overlaps the x read and the LDS fill;
//  * a "unit" is 64 weights of a K-quant super-block (Q4_K/Q5_K: one 6-bit scale pair,
//    Q6_K: four 16-wide runs) or one 32-weight block (Q4_0/Q8_0); loads are 16-byte
//    (dwordx4) even where the block is only 2-byte aligned (gfx950 global loads need no
//    natural alignment: the compiler itself emits dwordx4 for 2-aligned memcpy);
//  * int8 dot products with v_dot4_i32_i8, scales in f32, wave64 shuffle reductions.
#pragma once

#include "common.h"
#include "quants.cuh"
#include "gemv.h"

namespace mx {

// ---------------------------------------------------------------------------
// activation staging
// ---------------------------------------------------------------------------
struct LdsAct {
    int8_t * q;
    float * d;
    float * s;
};

// activation source of a GEMV, compile-time (each mode keeps only its own registers).
// *_LDS modes stage the f32 x (and norm weight) into LDS by LDS-DMA before the weight
// loads are issued and quantise from LDS afterwards: no registers, no wait on x.
// *_H2 modes hold two 16-value halves per thread (K up to 32 * threads); the plain modes
// one (K <= 16 * threads, e.g. n_embd 4096 on 256 threads) and so half the registers,
// which is occupancy on the large grids.
// XS_FAP2/4/8 (round 5): the attention's split partials (up to 2/4/8 splits) merged into x
enum { XS_F32 = 0, XS_NORM = 1, XS_Q8 = 2, XS_F32_LDS = 3, XS_NORM_LDS = 4, XS_F32_H2 = 5, XS_NORM_H2 = 6,
       XS_FAP2 = 7, XS_FAP4 = 8, XS_FAP8 = 9 };
__host__ __device__ constexpr bool xs_norm(int m) { return m == XS_NORM || m == XS_NORM_H2; }
__host__ __device__ constexpr bool xs_f32reg(int m) { return m == XS_F32 || m == XS_F32_H2; }
__host__ __device__ constexpr int xs_fap(int m) { return m == XS_FAP2 ? 2 : m == XS_FAP4 ? 4 : m == XS_FAP8 ? 8 : 0; }

__host__ __device__ inline size_t gemv_lds_base(int64_t K) { return ((size_t) K + (size_t) (K / 32) * 8 + 64 + 15) & ~(size_t) 15; }
__host__ __device__ inline size_t gemv_lds_bytes(int64_t K, int mode = XS_Q8) {
    return gemv_lds_base(K) + (mode == XS_F32_LDS || mode == XS_NORM_LDS ? 4 * (size_t) K : 0) + (mode == XS_NORM_LDS ? 4 * (size_t) K : 0);
}
__host__ __device__ inline float * gemv_lds_red(char * smem, int64_t K) { return (float *) (smem + K + (K / 32) * 8); }
// Staging mode for a source. Register staging keeps x (and the norm weight) in VGPRs,
// LDS-DMA staging (~25 GB/s per CU) keeps them out of the register file. Measured on
// MI355X (tools/opbench.py ffn_block / q_q4k, profiles/r01): grids of one block per CU
// (the 4096-row projections) are latency-bound and win with registers; grids of several
// waves' worth per SIMD (SwiGLU, lm_head) win with the occupancy LDS staging buys.
extern int g_tune[48];
inline int gemv_mode(const XStage & xs, int64_t K, int64_t n_waves = 0, int nt = 256) {
    if (xs.fap) return xs.fap_ns <= 4 ? XS_FAP4 : XS_FAP8;   // (XS_FAP2 not instantiated)
    if (xs.q8) return XS_Q8;
    bool lds = n_waves >= 2048;
    if (g_tune[9] == 1) lds = true;    // sweeps
    if (g_tune[9] == 2) lds = false;
    const bool h2 = K > 16 * nt;
    if (xs.norm) return lds && gemv_lds_bytes(K, XS_NORM_LDS) <= 65536 ? XS_NORM_LDS : (h2 ? XS_NORM_H2 : XS_NORM);
    return lds && gemv_lds_bytes(K, XS_F32_LDS) <= 65536 ? XS_F32_LDS : (h2 ? XS_F32_H2 : XS_F32);
}

__device__ __forceinline__ LdsAct lds_act(char * smem, int64_t K) {
    LdsAct a;
    a.q = (int8_t *) smem;
    a.d = (float *) (smem + K);
    a.s = a.d + K / 32;
    return a;
}

// LDS accesses of the LDS-DMA-staged prologues (XS_F32_LDS / XS_NORM_LDS) as inline
// asm: for an ordinary LDS access issued while an LDS-DMA may be pending, the compiler's
// waitcnt pass waits for EVERY vector-memory op in flight (vmcnt(0)) — the first batch
// of weight loads included — so the prologue ran only after the weights had landed
// instead of under their latency. Each read and its lgkmcnt(0) wait are one asm
// statement (outputs exist only once the data has landed); writes are waited for by the
// next lds_barrier.
// Round 3: default OFF. Same-box A/B at HEAD (profiles/r03/ab_noasm): the decode SwiGLU
// 17.52 -> 16.76 us and tg128 594.4 / 595.2 -> 597.1 / 597.6 tok/s without the asm
// accesses; the bisect put the whole round-2 SwiGLU regression (15.25 -> 17.3 us,
// profiles/r03/bisect_swiglu_roofline.txt) on the commit that introduced them.
// MX_PROLOGUE_ONE=1: each thread reads its 16-value half (and norm weight) once and keeps
// it in registers (round 2, 0d87f1f). Default 0 (round 1's loop, each half read per use):
// with the dense/EXT split of k_gemv2 the same-box decode ran 620 / 619 tok/s against
// 602 / 615 with it (profiles/r03/ab_gemv_variants.txt)
#ifndef MX_PROLOGUE_ONE
#define MX_PROLOGUE_ONE 0
#endif
#ifndef MX_PROLOGUE_ASM
#define MX_PROLOGUE_ASM 0
#endif
#if MX_PROLOGUE_ASM
__device__ __forceinline__ uint32_t lds_off(const void * p) {
    return (uint32_t) (uintptr_t) (const __attribute__((address_space(3))) char *) p;
}
typedef float v4f_t __attribute__((ext_vector_type(4)));
typedef int v4i_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void lds_rd16(const float * p, float (&d)[16]) {
    v4f_t a, b, c, e;
    asm volatile("ds_read_b128 %0, %4\n\tds_read_b128 %1, %4 offset:16\n\tds_read_b128 %2, %4 offset:32\n\t"
                 "ds_read_b128 %3, %4 offset:48\n\ts_waitcnt lgkmcnt(0)"
                 : "=&v"(a), "=&v"(b), "=&v"(c), "=&v"(e) : "v"(lds_off(p)));
#pragma unroll
    for (int j = 0; j < 4; ++j) { d[j] = a[j]; d[4 + j] = b[j]; d[8 + j] = c[j]; d[12 + j] = e[j]; }
}
// x and the norm weight of one 16-value half in one round trip
__device__ __forceinline__ void lds_rd16x2(const float * p, const float * q, float (&d)[16], float (&e)[16]) {
    v4f_t a, b, c, f, g, h, i, j;
    asm volatile("ds_read_b128 %0, %8\n\tds_read_b128 %1, %8 offset:16\n\tds_read_b128 %2, %8 offset:32\n\t"
                 "ds_read_b128 %3, %8 offset:48\n\tds_read_b128 %4, %9\n\tds_read_b128 %5, %9 offset:16\n\t"
                 "ds_read_b128 %6, %9 offset:32\n\tds_read_b128 %7, %9 offset:48\n\ts_waitcnt lgkmcnt(0)"
                 : "=&v"(a), "=&v"(b), "=&v"(c), "=&v"(f), "=&v"(g), "=&v"(h), "=&v"(i), "=&v"(j)
                 : "v"(lds_off(p)), "v"(lds_off(q)));
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        d[k] = a[k]; d[4 + k] = b[k]; d[8 + k] = c[k]; d[12 + k] = f[k];
        e[k] = g[k]; e[4 + k] = h[k]; e[8 + k] = i[k]; e[12 + k] = j[k];
    }
}
// sum of N (4, 8 or 16) consecutive floats, one round trip
template <int N>
__device__ __forceinline__ float lds_sum(const float * p) {
    static_assert(N == 4 || N == 8 || N == 16, "lds_sum");
    v4f_t a, b, c, d;
    if constexpr (N == 4) {
        asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=&v"(a) : "v"(lds_off(p)));
        return (a[0] + a[1]) + (a[2] + a[3]);
    } else if constexpr (N == 8) {
        asm volatile("ds_read_b128 %0, %2\n\tds_read_b128 %1, %2 offset:16\n\ts_waitcnt lgkmcnt(0)" : "=&v"(a), "=&v"(b) : "v"(lds_off(p)));
        float s = 0.f;
#pragma unroll
        for (int k = 0; k < 4; ++k) s += a[k];
#pragma unroll
        for (int k = 0; k < 4; ++k) s += b[k];
        return s;
    } else {
        asm volatile("ds_read_b128 %0, %4\n\tds_read_b128 %1, %4 offset:16\n\tds_read_b128 %2, %4 offset:32\n\t"
                     "ds_read_b128 %3, %4 offset:48\n\ts_waitcnt lgkmcnt(0)" : "=&v"(a), "=&v"(b), "=&v"(c), "=&v"(d) : "v"(lds_off(p)));
        float s = 0.f;
#pragma unroll
        for (int k = 0; k < 4; ++k) s += a[k];
#pragma unroll
        for (int k = 0; k < 4; ++k) s += b[k];
#pragma unroll
        for (int k = 0; k < 4; ++k) s += c[k];
#pragma unroll
        for (int k = 0; k < 4; ++k) s += d[k];
        return s;
    }
}
__device__ __forceinline__ float4 lds_rd4(const float * p) {
    v4f_t a;
    asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=&v"(a) : "v"(lds_off(p)));
    return make_float4(a[0], a[1], a[2], a[3]);
}
__device__ __forceinline__ float lds_rd1(const float * p) {
    float a;
    asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=&v"(a) : "v"(lds_off(p)));
    return a;
}
__device__ __forceinline__ void lds_wr1(float * p, float v) {
    asm volatile("ds_write_b32 %0, %1" :: "v"(lds_off(p)), "v"(v) : "memory");
}
__device__ __forceinline__ void lds_wr4i(void * p, int4 v) {
    v4i_t w = {v.x, v.y, v.z, v.w};
    asm volatile("ds_write_b128 %0, %1" :: "v"(lds_off(p)), "v"(w) : "memory");
}

#else   // A/B build (EXTRA=-DMX_PROLOGUE_ASM=0): ordinary LDS accesses
typedef float v4f_t __attribute__((ext_vector_type(4)));
typedef int v4i_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void lds_rd16(const float * p, float (&d)[16]) { for (int j = 0; j < 16; ++j) d[j] = p[j]; }
__device__ __forceinline__ void lds_rd16x2(const float * p, const float * q, float (&d)[16], float (&e)[16]) {
    for (int j = 0; j < 16; ++j) { d[j] = p[j]; e[j] = q[j]; }
}
template <int N> __device__ __forceinline__ float lds_sum(const float * p) { float s = 0.f; for (int j = 0; j < N; ++j) s += p[j]; return s; }
__device__ __forceinline__ float4 lds_rd4(const float * p) { return *(const float4 *) p; }
__device__ __forceinline__ float lds_rd1(const float * p) { return *p; }
__device__ __forceinline__ void lds_wr1(float * p, float v) { *p = v; }
__device__ __forceinline__ void lds_wr4i(void * p, int4 v) { *(int4 *) p = v; }
#endif

// quantise 16 values held by this thread; the partner thread (tid ^ 1) holds the other
// half of the 32-block (k_quantize_act semantics up to the rounding noted below).
// ASMW: LDS writes by inline asm (the LDS-DMA-staged prologues, see lds_rd16)
template <bool ASMW = false>
__device__ __forceinline__ void q8_half(const float (&v)[16], int hg, LdsAct a) {
    float amax = 0.f;
#pragma unroll
    for (int j = 0; j < 16; ++j) amax = fmaxf(amax, fabsf(v[j]));
    amax = fmaxf(amax, dpp_f<0xB1>(-INFINITY, amax));   // partner lane tid ^ 1
    const Q8Scale qs = q8_scale(amax);   // common.h: the backend's one q8 quantiser
    const float dd = qs.d, id = qs.id;
    int sum = 0, pk[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        int w = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int qi = q8_round(v[4 * j + k], id);
            sum += qi;
            w |= (qi & 0xFF) << (8 * k);
        }
        pk[j] = w;
    }
    sum += dpp_i<0xB1>(0, sum);
    if constexpr (ASMW) {
        lds_wr4i(a.q + 16 * hg, make_int4(pk[0], pk[1], pk[2], pk[3]));
        if ((hg & 1) == 0) { lds_wr1(a.d + (hg >> 1), dd); lds_wr1(a.s + (hg >> 1), dd * (float) sum); }
        return;
    }
    *(int4 *) (a.q + 16 * hg) = make_int4(pk[0], pk[1], pk[2], pk[3]);
    if ((hg & 1) == 0) {
        a.d[hg >> 1] = dd;
        a.s[hg >> 1] = dd * (float) sum;
    }
}

// Fill LDS with the quantised activation. Block = NT threads, K % 32 == 0.
// Three sources: a q8 activation already in memory (copied), f32 x (quantised), or
// f32 x through RMS norm · nw (K <= 2*16*NT: two 16-value halves per thread held
// across the block reduction).
// Split in two because vector-memory loads retire in issue order: issue() starts the
// activation loads BEFORE the weight stream is issued, finish() (after the weight loads
// are in flight) waits only for them, quantises into LDS and ends with a barrier.
template <int NT, int MODE>
struct StageRegs {
    static constexpr int HPT = (MODE == XS_F32_H2 || MODE == XS_NORM_H2) ? 2 : 1;   // f32 halves per thread
    static constexpr int NSP = xs_fap(MODE) ? xs_fap(MODE) : 1;                      // attention splits
    float v[xs_fap(MODE) ? NSP : HPT][16];       // XS_FAP*: split s's O of the thread's half
    float w[xs_norm(MODE) ? HPT : 1][16];
    float ml[NSP][2];                            // XS_FAP*: split s's (max, sum) of the half's head
};

typedef __attribute__((address_space(3))) void * lds_ptr_t;

// q8 source: global -> LDS by LDS-DMA (global_load_lds), no registers held; each wave
// moves 64 lanes x `B` bytes per instruction to a wave-uniform LDS address
template <int NT, int B>
__device__ __forceinline__ void dma_to_lds(const void * src, void * dst, int nbytes) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int n = nbytes / B;
    for (int c = wave * 64; c < n; c += NT) {
        if (c + lane < n) {
            const void * g = (const char *) src + (size_t) (c + lane) * B;
            const lds_ptr_t l = (lds_ptr_t) ((char *) dst + c * B);
            if constexpr (B == 16) __builtin_amdgcn_global_load_lds(g, l, 16, 0, 0);
            else __builtin_amdgcn_global_load_lds(g, l, 4, 0, 0);
        }
    }
}

__device__ __forceinline__ void load_half(int hg, float (&dst)[16], const float * src) {
#pragma unroll
    for (int j = 0; j < 16; j += 4) {
        const float4 f = *(const float4 *) (src + 16 * hg + j);
        dst[j] = f.x; dst[j + 1] = f.y; dst[j + 2] = f.z; dst[j + 3] = f.w;
    }
}

// unconditional loads at clamped indices (no partially initialised arrays: the registers
// must stay registers); out-of-range entries are ignored by stage_finish
template <int NT, int MODE>
__device__ __forceinline__ void stage_issue(const XStage & xs, int K, const LdsAct & a, StageRegs<NT, MODE> & r) {
    if constexpr (MODE == XS_Q8) {
        dma_to_lds<NT, 16>(xs.q8, a.q, K);
        dma_to_lds<NT, 4>(xs.q8d, a.d, K / 32 * 4);
        dma_to_lds<NT, 4>(xs.q8s, a.s, K / 32 * 4);
    } else if constexpr (MODE == XS_F32_LDS || MODE == XS_NORM_LDS) {
        char * stg = (char *) a.q + gemv_lds_base(K);
        dma_to_lds<NT, 16>(xs.x, stg, 4 * K);
        if constexpr (MODE == XS_NORM_LDS) dma_to_lds<NT, 16>(xs.nw, stg + 4 * K, 4 * K);
    } else if constexpr (xs_fap(MODE)) {
        // the thread's 16 values lie in one head (fap_d % 16 == 0): its O run and the
        // (max, sum) pair of every split, all loads in flight together (K <= 16 NT)
        const int t = threadIdx.x, hg = min(t, K / 16 - 1);
        const int hh = (16 * hg) / xs.fap_d, d0 = 16 * hg - hh * xs.fap_d;
#pragma unroll
        for (int s = 0; s < xs_fap(MODE); ++s) {
            const float * b = xs.fap + ((size_t) hh * xs.fap_ns + min(s, xs.fap_ns - 1)) * (xs.fap_d + 2);
            // rows of fap_d + 2 floats: 8-byte aligned only
#pragma unroll
            for (int j = 0; j < 16; j += 4) {
                float4 f;
                __builtin_memcpy(&f, __builtin_assume_aligned(b + d0 + j, 8), 16);
                r.v[s][j] = f.x; r.v[s][j + 1] = f.y; r.v[s][j + 2] = f.z; r.v[s][j + 3] = f.w;
            }
            const float2 m = *(const float2 *) (b + xs.fap_d);
            r.ml[s][0] = m.x; r.ml[s][1] = m.y;
        }
    } else {
        const int t = threadIdx.x, nhg = K / 16;
#pragma unroll
        for (int h = 0; h < StageRegs<NT, MODE>::HPT; ++h) {
            const int hg = min(t + NT * h, nhg - 1);
            load_half(hg, r.v[h], xs.x);
            if constexpr (xs_norm(MODE)) load_half(hg, r.w[h], xs.nw);
        }
    }
}

// Raw workgroup barrier for LDS data: waits for this wave's LDS writes (lgkmcnt) and
// nothing else. __syncthreads() would also drain the vector-memory counter whenever an
// LDS-DMA is pending, i.e. wait for every weight load in flight (the whole HBM latency)
// before the prologue could finish (cdna_hip_programming.md, pipelining across barriers).
__device__ __forceinline__ void lds_barrier() {
    __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0) alone
    __builtin_amdgcn_s_barrier();
}
// s_waitcnt vmcnt(N) alone (gfx9 encoding: vmcnt bits [3:0] + [15:14], expcnt and
// lgkmcnt at their maxima)
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
    static_assert(N >= 0 && N < 64, "vmcnt range");
    __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}

// NW = vector-memory instructions this wave issued after its LDS-DMA (the weight loads
// of the first batch): the DMA modes wait for the staged activation with vmcnt(NW) —
// loads retire in issue order — and leave the weight stream in flight.
template <int NT, int MODE, int NW = 0>
__device__ __forceinline__ void stage_finish(const XStage & xs, int K, const LdsAct & a, float * red, StageRegs<NT, MODE> & r) {
    constexpr int HPT = StageRegs<NT, MODE>::HPT;
    const int t = threadIdx.x, nhg = K / 16;
    if constexpr (MODE == XS_Q8) {
        wait_vmcnt<NW>();                     // the LDS-DMA of stage_issue has landed
    } else if constexpr (MODE == XS_F32_LDS || MODE == XS_NORM_LDS) {
        const float * xf = (const float *) ((const char *) a.q + gemv_lds_base(K));
        if (xs.drain) wait_vmcnt<0>();       // A/B (g_tune[14]): prologue after the whole stream
        else wait_vmcnt<NW>();
        lds_barrier();                        // staged x (and norm weight) visible
        // K <= 16 NT (every SwiGLU / lm_head grid): each thread reads its one 16-value half
        // (and norm weight) once, in one round trip, and keeps it for Σx² and quantisation
        const bool one = MX_PROLOGUE_ONE && nhg <= NT;
        float v1[16], w1[16];
        if (one && t < nhg) {
            if constexpr (MODE == XS_NORM_LDS) lds_rd16x2(xf + 16 * t, xf + K + 16 * t, v1, w1);
            else lds_rd16(xf + 16 * t, v1);
        }
        float scale = 1.0f;
        if constexpr (MODE == XS_NORM_LDS) {
            float ss = 0.f;
            if (one) {
                if (t < nhg) {
#pragma unroll
                    for (int j = 0; j < 16; ++j) ss += v1[j] * v1[j];
                }
            } else {
                for (int i = 4 * t; i < K; i += 4 * NT) {
                    const float4 f = lds_rd4(xf + i);
                    ss += f.x * f.x + f.y * f.y + f.z * f.z + f.w * f.w;
                }
            }
            ss = wave_sum(ss);
            if ((t & 63) == 0) lds_wr1(red + (t >> 6), ss);
            lds_barrier();
            ss = lds_sum<NT / 64>(red);
            scale = __builtin_amdgcn_rsqf(ss / (float) K + xs.eps);
        }
        if (one) {
            if (t < nhg) {                           // nhg is even: partner lanes stay paired
                if constexpr (MODE == XS_NORM_LDS) {
#pragma unroll
                    for (int j = 0; j < 16; ++j) v1[j] = (v1[j] * scale) * w1[j];
                }
                q8_half<true>(v1, t, a);
            }
        } else for (int hg = t; hg < nhg; hg += NT) {   // nhg is even: partner lanes stay paired
            float v2[16];
            lds_rd16(xf + 16 * hg, v2);
            if constexpr (MODE == XS_NORM_LDS) {
                float w2[16];
                lds_rd16(xf + K + 16 * hg, w2);
#pragma unroll
                for (int j = 0; j < 16; ++j) v2[j] = (v2[j] * scale) * w2[j];
            }
            q8_half<true>(v2, hg, a);
        }
    } else if constexpr (xs_fap(MODE)) {
        // merge of the splits (k_fattn_dec2_combine's arithmetic): weights 2^(m_s - max),
        // x = sum_s w_s O_s / sum_s w_s l_s
        constexpr int NS = xs_fap(MODE);
        if (t < nhg) {                               // nhg is even: partner lanes stay paired
            float mx = -INFINITY;
#pragma unroll
            for (int s = 0; s < NS; ++s) if (s < xs.fap_ns) mx = fmaxf(mx, r.ml[s][0]);
            float wt[NS], l = 0.f;
#pragma unroll
            for (int s = 0; s < NS; ++s) {
                wt[s] = s < xs.fap_ns && r.ml[s][0] != -INFINITY ? __builtin_amdgcn_exp2f(r.ml[s][0] - mx) : 0.f;
                l += wt[s] * r.ml[s][1];
            }
            float v[16];
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                float o = 0.f;
#pragma unroll
                for (int s = 0; s < NS; ++s) o += wt[s] * r.v[s][j];
                v[j] = l == 0.f ? 0.f : o / l;
            }
            q8_half(v, t, a);
        }
    } else if constexpr (xs_norm(MODE)) {
        // K <= 16 * HPT * NT (GEMV2_MAX_NORM_K checks it for the 256-thread kernels)
        float ss = 0.f;
#pragma unroll
        for (int h = 0; h < HPT; ++h) {
            float sh = 0.f;
#pragma unroll
            for (int j = 0; j < 16; ++j) sh += r.v[h][j] * r.v[h][j];
            ss += t + NT * h < nhg ? sh : 0.f;
        }
        ss = wave_sum(ss);
        if ((t & 63) == 0) red[t >> 6] = ss;
        if (xs.postscale) {   // block-uniform: quantise x * nw now, s after the dots (XStage)
#pragma unroll
            for (int h = 0; h < HPT; ++h) {
                const int hg = t + NT * h;
                if (hg < nhg) {
#pragma unroll
                    for (int j = 0; j < 16; ++j) r.v[h][j] *= r.w[h][j];
                    q8_half(r.v[h], hg, a);
                }
            }
            lds_barrier();    // the q8 image and the per-wave sums of squares
            return;
        }
        lds_barrier();
        ss = 0.f;
#pragma unroll
        for (int wv = 0; wv < NT / 64; ++wv) ss += red[wv];
        const float scale = __builtin_amdgcn_rsqf(ss / (float) K + xs.eps);
#pragma unroll
        for (int h = 0; h < HPT; ++h) {
            const int hg = t + NT * h;
            if (hg < nhg) {
#pragma unroll
                for (int j = 0; j < 16; ++j) r.v[h][j] = (r.v[h][j] * scale) * r.w[h][j];
                q8_half(r.v[h], hg, a);
            }
        }
    } else {
#pragma unroll
        for (int h = 0; h < HPT; ++h) if (t + NT * h < nhg) q8_half(r.v[h], t + NT * h, a);
        for (int hg = t + HPT * NT; hg < nhg; hg += NT) {
            float v2[16];
            load_half(hg, v2, xs.x);
            q8_half(v2, hg, a);
        }
    }
    lds_barrier();
}

// XCD-aware block order: workgroups are dispatched round-robin over the 8 XCDs
// (block b -> XCD b % 8), so consecutive blocks — adjacent output rows — land on
// different XCDs and every 128-B line of the output (and of the KV-cache rows the QKV
// kernel stores) is written partially by several L2s, each writing back a partial
// line at the kernel boundary. Remapped, XCD x owns one contiguous run of logical
// blocks: its outputs are whole lines in one L2 (and its weight rows one contiguous
// HBM range). `on` = 0 keeps the dispatch order (A/B).
__device__ __forceinline__ int xcd_block(int b, int G, bool on) {
    const int G8 = G & ~7;
    if (!on || b >= G8) return b;
    return (b & 7) * (G8 >> 3) + (b >> 3);
}

// ---------------------------------------------------------------------------
// weight units (v2)
// ---------------------------------------------------------------------------
template <int QT> struct W2;
template <> struct W2<GGML_TYPE_Q4_K> { int4 hd, w0, w1; };
template <> struct W2<GGML_TYPE_Q5_K> { int4 hd, w0, w1, h0, h1; };
template <> struct W2<GGML_TYPE_Q6_K> { int4 la, lb, qh, sc; uint16_t d; };
template <> struct W2<GGML_TYPE_Q4_0> { int4 w; uint16_t d; };
template <> struct W2<GGML_TYPE_Q8_0> { int4 w0, w1; uint16_t d; };

template <int QT> __host__ __device__ constexpr int unit_w() {   // weights per unit
    return (QT == GGML_TYPE_Q4_0 || QT == GGML_TYPE_Q8_0) ? 32 : 64;
}

// MX_GEMV_NT=1 at build time makes the weight loads non-temporal (`nt`). Measured on
// MI355X: tg128 593 -> 495 tok/s. A lane's unit spans two or three 16-B loads of one
// 128-B line issued by different instructions (Q4_K: header, low, high quants), and nt
// lets the line leave the cache between them: the stream is re-fetched. Default policy.
#ifndef MX_GEMV_NT
#define MX_GEMV_NT 0
#endif
typedef int v4i_a2 __attribute__((ext_vector_type(4), aligned(2)));
__device__ __forceinline__ int4 v4_int4(v4i_t v) { return make_int4(v.x, v.y, v.z, v.w); }
__device__ __forceinline__ int4 ld_a4(const void * p) {
    if constexpr (MX_GEMV_NT) return v4_int4(__builtin_nontemporal_load((const v4i_t *) p));
    return *(const int4 *) p;
}
__device__ __forceinline__ int4 ldu4(const char * p) {   // 16-byte load, any 2-byte alignment
    if constexpr (MX_GEMV_NT) return v4_int4(__builtin_nontemporal_load((const v4i_a2 *) p));
    int4 v;
    __builtin_memcpy(&v, __builtin_assume_aligned(p, 2), 16);
    return v;
}
__device__ __forceinline__ uint16_t ldw_u16(const char * p) {
    if constexpr (MX_GEMV_NT) return __builtin_nontemporal_load((const uint16_t *) p);
    return *(const uint16_t *) p;
}

template <int QT>
__device__ __forceinline__ void w2_load(const char * __restrict__ row, int u, W2<QT> & r) {
    if constexpr (QT == GGML_TYPE_Q4_K) {
        const char * b = row + (int64_t) (u >> 2) * 144;
        const int g = u & 3;
        r.hd = ld_a4(b);
        r.w0 = ld_a4(b + 16 + 32 * g);
        r.w1 = ld_a4(b + 32 + 32 * g);
    } else if constexpr (QT == GGML_TYPE_Q5_K) {
        const char * b = row + (int64_t) (u >> 2) * 176;
        const int g = u & 3;
        r.hd = ld_a4(b);
        r.h0 = ld_a4(b + 16);
        r.h1 = ld_a4(b + 32);
        r.w0 = ld_a4(b + 48 + 32 * g);
        r.w1 = ld_a4(b + 64 + 32 * g);
    } else if constexpr (QT == GGML_TYPE_Q6_K) {
        const char * b = row + (int64_t) (u >> 2) * 210;
        const int n = (u >> 1) & 1, hl = u & 1;
        r.la = ldu4(b + 64 * n + 16 * hl);
        r.lb = ldu4(b + 64 * n + 32 + 16 * hl);
        r.qh = ldu4(b + 128 + 32 * n + 16 * hl);
        r.sc = ldu4(b + 192);
        r.d = ldw_u16(b + 208);
    } else if constexpr (QT == GGML_TYPE_Q4_0) {
        const char * b = row + (int64_t) u * 18;
        r.d = ldw_u16(b);
        r.w = ldu4(b + 2);
    } else if constexpr (QT == GGML_TYPE_Q8_0) {
        const char * b = row + (int64_t) u * 34;
        r.d = ldw_u16(b);
        r.w0 = ldu4(b + 2);
        r.w1 = ldu4(b + 18);
    }
}

__device__ __forceinline__ int dot16(const int (&w)[4], int4 a, int acc) {
    acc = dot4_i8(w[0], a.x, acc); acc = dot4_i8(w[1], a.y, acc);
    acc = dot4_i8(w[2], a.z, acc); acc = dot4_i8(w[3], a.w, acc);
    return acc;
}

template <int QT>
__device__ __forceinline__ float w2_dot(const W2<QT> & r, int u, const LdsAct & a) {
    if constexpr (QT == GGML_TYPE_Q4_K || QT == GGML_TYPE_Q5_K) {
        const int sb = u >> 2, g = u & 3;
        const uint32_t s0 = (uint32_t) r.hd.y, s1 = (uint32_t) r.hd.z, s2 = (uint32_t) r.hd.w;
        // get_scale_min_k4 (ggml-quants.c:703) for all eight sub-blocks at once, four 6-bit
        // values per dword (j < 4: low 6 bits of bytes j / j+4; j >= 4: low nibble of byte
        // j+4 with the top two bits of byte j-4 / j), then this unit's pair (2g, 2g+1) by one
        // select and one shift: ~10 VALU instead of ~25 for per-scale byte selects
        const uint32_t scw = g < 2 ? (s0 & 0x3F3F3F3Fu) : ((s2 & 0x0F0F0F0Fu) | ((s0 >> 2) & 0x30303030u));
        const uint32_t mnw = g < 2 ? (s1 & 0x3F3F3F3Fu) : (((s2 >> 4) & 0x0F0F0F0Fu) | ((s1 >> 2) & 0x30303030u));
        const uint32_t scp = scw >> (16 * (g & 1)), mnp = mnw >> (16 * (g & 1));
        const int sc[2] = {(int) (scp & 0xFF), (int) ((scp >> 8) & 0xFF)};
        const int mn[2] = {(int) (mnp & 0xFF), (int) ((mnp >> 8) & 0xFF)};
        const float d = h2f((uint16_t) (r.hd.x & 0xFFFF)), dmin = h2f((uint16_t) ((uint32_t) r.hd.x >> 16));
        const int wv[8] = {r.w0.x, r.w0.y, r.w0.z, r.w0.w, r.w1.x, r.w1.y, r.w1.z, r.w1.w};
        int lo[2][4], hi[2][4];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            lo[k >> 2][k & 3] = wv[k] & 0x0F0F0F0F;
            hi[k >> 2][k & 3] = (wv[k] >> 4) & 0x0F0F0F0F;
        }
        if constexpr (QT == GGML_TYPE_Q5_K) {
            const int hv[8] = {r.h0.x, r.h0.y, r.h0.z, r.h0.w, r.h1.x, r.h1.y, r.h1.z, r.h1.w};
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                lo[k >> 2][k & 3] |= ((hv[k] >> (2 * g)) & 0x01010101) << 4;
                hi[k >> 2][k & 3] |= ((hv[k] >> (2 * g + 1)) & 0x01010101) << 4;
            }
        }
        const int e0 = sb * 256 + 64 * g;
        const int4 * aq = (const int4 *) (a.q + e0);
        int d0 = 0, d1 = 0;
        d0 = dot16(lo[0], aq[0], d0); d0 = dot16(lo[1], aq[1], d0);
        d1 = dot16(hi[0], aq[2], d1); d1 = dot16(hi[1], aq[3], d1);
        const int b0 = e0 >> 5;
        const float2 ad = *(const float2 *) (a.d + b0);
        const float2 as = *(const float2 *) (a.s + b0);
        return d * ((float) sc[0] * ad.x * (float) d0 + (float) sc[1] * ad.y * (float) d1)
             - dmin * ((float) mn[0] * as.x + (float) mn[1] * as.y);
    } else if constexpr (QT == GGML_TYPE_Q6_K) {
        const int sb = u >> 2, n = (u >> 1) & 1, hl = u & 1;
        const int la[4] = {r.la.x, r.la.y, r.la.z, r.la.w};
        const int lb[4] = {r.lb.x, r.lb.y, r.lb.z, r.lb.w};
        const int qh[4] = {r.qh.x, r.qh.y, r.qh.z, r.qh.w};
        int q[4][4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            q[0][k] = (la[k] & 0x0F0F0F0F) | (((qh[k] >> 0) & 0x03030303) << 4);
            q[1][k] = (lb[k] & 0x0F0F0F0F) | (((qh[k] >> 2) & 0x03030303) << 4);
            q[2][k] = ((la[k] >> 4) & 0x0F0F0F0F) | (((qh[k] >> 4) & 0x03030303) << 4);
            q[3][k] = ((lb[k] >> 4) & 0x0F0F0F0F) | (((qh[k] >> 6) & 0x03030303) << 4);
        }
        // scales sc[8n + hl + 2qq]: byte (8n + hl + 2qq) of the 16 scale bytes
        const int scw[4] = {r.sc.x, r.sc.y, r.sc.z, r.sc.w};
        const int e0 = sb * 256 + 128 * n + 16 * hl;
        float v = 0.f;
#pragma unroll
        for (int qq = 0; qq < 4; ++qq) {
            const int si = 8 * n + hl + 2 * qq;
            const int scv = (int) (int8_t) ((scw[si >> 2] >> (8 * (si & 3))) & 0xFF);
            const int4 av = *(const int4 *) (a.q + e0 + 32 * qq);
            int dt = dot16(q[qq], av, 0);
            int sm = 0;
            sm = dot4_i8(0x20202020, av.x, sm); sm = dot4_i8(0x20202020, av.y, sm);
            sm = dot4_i8(0x20202020, av.z, sm); sm = dot4_i8(0x20202020, av.w, sm);
            v += (float) scv * a.d[(e0 >> 5) + qq] * (float) (dt - sm);
        }
        return h2f(r.d) * v;
    } else if constexpr (QT == GGML_TYPE_Q4_0) {
        const int w[4] = {r.w.x, r.w.y, r.w.z, r.w.w};
        int lo[4], hi[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) { lo[k] = w[k] & 0x0F0F0F0F; hi[k] = (w[k] >> 4) & 0x0F0F0F0F; }
        const int4 * aq = (const int4 *) (a.q + 32 * u);
        int dt = dot16(lo, aq[0], 0);
        dt = dot16(hi, aq[1], dt);
        return h2f(r.d) * (a.d[u] * (float) dt - 8.0f * a.s[u]);
    } else if constexpr (QT == GGML_TYPE_Q8_0) {
        const int w0[4] = {r.w0.x, r.w0.y, r.w0.z, r.w0.w};
        const int w1[4] = {r.w1.x, r.w1.y, r.w1.z, r.w1.w};
        const int4 * aq = (const int4 *) (a.q + 32 * u);
        int dt = dot16(w0, aq[0], 0);
        dt = dot16(w1, aq[1], dt);
        return h2f(r.d) * a.d[u] * (float) dt;
    }
    return 0.f;
}

// vector-memory instructions w2_load issues per unit (a lower bound is safe for
// stage_finish's counted wait: it can only wait longer)
template <int QT> __host__ __device__ constexpr int w2_loads() {
    return QT == GGML_TYPE_Q4_K ? 3 : QT == GGML_TYPE_Q5_K ? 5 : QT == GGML_TYPE_Q6_K ? 5 : QT == GGML_TYPE_Q4_0 ? 2 : 3;
}

template <int QT> __host__ __device__ constexpr bool gemv2_type_ok() {
    return QT == GGML_TYPE_Q4_K || QT == GGML_TYPE_Q5_K || QT == GGML_TYPE_Q6_K || QT == GGML_TYPE_Q4_0 || QT == GGML_TYPE_Q8_0;
}

// One row's partial dot over its units, LPR lanes per row, UPL units per lane in
// flight. Order: activation loads (stager.issue), weight loads of the first batch,
// activation quantisation into LDS (stager.finish, waits only for its own loads),
// dot products.
template <int QT, int UPL, int NM>
__device__ __forceinline__ void w2_load_batch(const char * const (&rows)[NM], int u0, int lpr, int units, W2<QT> (&r)[NM][UPL]) {
#pragma unroll
    for (int j = 0; j < UPL; ++j)
#pragma unroll
        for (int m = 0; m < NM; ++m) w2_load<QT>(rows[m], min(u0 + j * lpr, units - 1), r[m][j]);
}

template <int QT, int UPL, int NM>
__device__ __forceinline__ void w2_dot_batch(const W2<QT> (&r)[NM][UPL], int u0, int lpr, int units, const LdsAct & a, float (&acc)[NM]) {
#pragma unroll
    for (int j = 0; j < UPL; ++j) {
        if (u0 + j * lpr < units) {
#pragma unroll
            for (int m = 0; m < NM; ++m) acc[m] += w2_dot<QT>(r[m][j], u0 + j * lpr, a);
        }
        // keep the scheduler from hoisting every unit's LDS activation reads at once
        // (that costs ~16 VGPRs per unit, i.e. occupancy)
        __builtin_amdgcn_sched_barrier(0);
    }
}

// One row's partial dot over its units, LPR lanes per row, UPL units per lane per batch.
// Order: activation loads (stage_issue), weight batch 0, activation quantisation into
// LDS (stage_finish, waits only for its own loads), dot products; later batches load and
// compute in turn (a two-deep register pipeline measured slower: it costs occupancy).
// The caller issues the activation loads (stage_issue) so that a kernel with several
// block-uniform weight-type branches (QKV) issues them once, ahead of the branch: when
// each arm began with the same activation code, SimplifyCFG hoisted it (and the
// sum-of-squares waiting on it) above the arms, i.e. above the weight loads.
// `fence` runs after the prologue's wait for the staged activation: kernels pass the
// values they loaded (before stage_issue) for their epilogue — residual, KV-cache row
// index, position — through it, pinning those loads ahead of the weight stream instead
// of a round trip at the end (the opaque asm keeps the compiler from sinking them).
struct NoFence { __device__ void operator()() const {} };
template <int QT, int LPR, int UPL, int NM, int NT, int MODE, typename F = NoFence>
__device__ __forceinline__ void gemv_rows_staged(const char * const (&rows)[NM], int units, int sub, const LdsAct & a,
                                                 const XStage & xs, int K, float * red, StageRegs<NT, MODE> & sr, float (&acc)[NM],
                                                 F fence = F()) {
    W2<QT> r[NM][UPL];
#pragma unroll
    for (int m = 0; m < NM; ++m) acc[m] = 0.f;
    // block-uniform trip count: stage_finish holds a barrier. Batch 0 is peeled so the
    // prologue sits after the first weight loads in straight-line code: inside the loop
    // (under it == 0) LICM hoisted the activation amax above the loads, making every
    // block wait for x (an L2 round trip) before its HBM stream started.
    constexpr int STEP = LPR * UPL;
    const int n_iter = (units + STEP - 1) / STEP;
    __builtin_amdgcn_sched_barrier(0);       // the DMA of stage_issue stays ahead of the weights
    w2_load_batch<QT, UPL, NM>(rows, sub, LPR, units, r);
    __builtin_amdgcn_sched_barrier(0);
    // opaque redefinition of the staged activation registers: nothing computed from them
    // can move above this point (i.e. above the weight loads), whatever the IR passes do
    if constexpr (xs_f32reg(MODE) || xs_norm(MODE)) {
#pragma unroll
        for (int h = 0; h < StageRegs<NT, MODE>::HPT; ++h)
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                asm volatile("" : "+v"(sr.v[h][j]));
                if constexpr (xs_norm(MODE)) asm volatile("" : "+v"(sr.w[h][j]));
            }
    }
    if constexpr (xs_fap(MODE) != 0) {
#pragma unroll
        for (int s = 0; s < StageRegs<NT, MODE>::NSP; ++s) {
#pragma unroll
            for (int j = 0; j < 16; ++j) asm volatile("" : "+v"(sr.v[s][j]));
            asm volatile("" : "+v"(sr.ml[s][0]), "+v"(sr.ml[s][1]));
        }
    }
    if (!MX_DBG(xs.dbg & 1)) stage_finish<NT, MODE, UPL * NM * w2_loads<QT>()>(xs, K, a, red, sr);
    fence();                                  // older than the staged x: already landed
    if (MX_DBG(xs.dbg & 2)) {                         // timing experiment: consume the loads only
        for (int it = 0; it < n_iter; ++it) {
            if (it) w2_load_batch<QT, UPL, NM>(rows, it * STEP + sub, LPR, units, r);
            const int * wv = (const int *) &r[0][0];
            int x = 0;
#pragma unroll
            for (int j = 0; j < (int) (sizeof(r) / 4); ++j) x ^= wv[j];
            acc[0] += (float) x;
        }
    } else {
        if (n_iter > 0) w2_dot_batch<QT, UPL, NM>(r, sub, LPR, units, a, acc);
        for (int it = 1; it < n_iter; ++it) {
            w2_load_batch<QT, UPL, NM>(rows, it * STEP + sub, LPR, units, r);
            w2_dot_batch<QT, UPL, NM>(r, it * STEP + sub, LPR, units, a, acc);
        }
    }
    // row sum over the LPR lanes: in every lane for LPR <= 16, in the group's last lane
    // (sub == LPR - 1) for LPR = 32, 64
#pragma unroll
    for (int m = 0; m < NM; ++m) acc[m] = dpp_sum_group<LPR>(acc[m]);
    if constexpr (xs_norm(MODE)) {
        if (xs.postscale && !MX_DBG(xs.dbg & 1)) {   // the RMS scale of the prologue's quantisation (stage_finish)
            float ss = 0.f;
#pragma unroll
            for (int wv = 0; wv < NT / 64; ++wv) ss += red[wv];
            const float scale = __builtin_amdgcn_rsqf(ss / (float) K + xs.eps);
#pragma unroll
            for (int m = 0; m < NM; ++m) acc[m] *= scale;
        }
    }
}

template <int QT, int LPR, int UPL, int NM, int NT, int MODE, typename F = NoFence>
__device__ __forceinline__ void gemv_rows(const char * const (&rows)[NM], int units, int sub, const LdsAct & a,
                                          const XStage & xs, int K, float * red, float (&acc)[NM], F fence = F()) {
    StageRegs<NT, MODE> sr;
    stage_issue<NT, MODE>(xs, K, a, sr);
    gemv_rows_staged<QT, LPR, UPL, NM, NT, MODE>(rows, units, sub, a, xs, K, red, sr, acc, fence);
}

}  // namespace mx
