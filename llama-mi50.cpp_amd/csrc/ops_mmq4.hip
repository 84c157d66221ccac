// ops_mmq4.hip — prefill GEMM v4: K-quant weights dequantised in registers straight into
// the MFMA operand, activations staged by LDS-DMA. Replaces mul_mat_q for batched
// prefill (ggml-cuda/mmq.cuh:3364-3700, mmq.cu:262-366) on gfx950.
//
// Why a new skeleton (profiles/r01/pmc_prefill_sq.json): the v2/v3 kernels
// dequantised weight tiles into LDS and read them back as MFMA operands — LDS writes,
// reads, bank conflicts and two barriers per K step for data each wave then used alone;
// MFMA was ~20 % busy. Here:
//   * a wave owns 32 weight rows x 128 tokens (4 v_mfma_f32_32x32x16_f16 tiles); its
//     lanes load their rows' quantised bytes (16-byte qs chunks) into registers one K
//     chunk ahead and dequantise them just in time into the B operand — weights never
//     touch LDS. Lane (r, h) holds row r, and k-slice h of every 16-deep MFMA step; the
//     MFMA's k order is permuted to follow the super-block layout (a 16-byte qs chunk =
//     16 low nibbles of one sub-block + 16 high nibbles of the next), the activation
//     fragments are read in the same order;
//   * the f16 activation tile (128 tokens x 128 k, 32 KB) is double-buffered in LDS and
//     filled by LDS-DMA (global_load_lds, no registers, counted vmcnt + raw s_barrier:
//     the weight stream stays in flight); 16-byte chunks XOR-swizzled by (token & 15);
//   * dequantisation is packed f16 math on bit-assembled values: the nibble OR 0x6400
//     is the f16 1024 + q (low nibbles), the high nibble in place OR 0x5400 is 64 + q;
//     one v_pk_add removes the bias exactly, one v_pk_fma applies d*sc and -dmin*m —
//     ~1.75 VALU per weight, hidden behind the MFMAs of the partner wave on the SIMD.
//     Weights are scaled by ws = 2^10 so d*sc stays a normal f16; the epilogue undoes it.
//     A row whose super-block scales would push a scaled weight past 2^15 (|w| > 32 at
//     2^10: outlier rows of real checkpoints) lowers its lane's ws to a smaller power of two
//     and rescales its accumulators once (m4_range, wave-uniform branch, never taken for
//     ordinary weights);
//   * epilogues: store (+ residual), SwiGLU of a gate/up pair (waves 0-1 gate rows,
//     2-3 up rows of the same 64; combined through LDS), the f16 copy of the output for
//     the next GEMM (act cache), and the MoE gather/scatter of grouped expert tiles.
#include "backend.h"
#include "mm.h"
#include "gemv.h"

#include <type_traits>

namespace mx {

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef _Float16 h2 __attribute__((ext_vector_type(2)));
typedef float f16v __attribute__((ext_vector_type(16)));

constexpr int M4_KC = 128;        // K per chunk (half a super-block)
// timing experiments only (variant builds, results wrong): 1 no per-chunk vmcnt wait and
// barrier, 2 no dequantisation (raw weight bits as the B operand), 4 LDS activation
// fragments read once per chunk
// X (template) bits: 8 = the short Q6_K dequantisation (MX_M4_Q6V2 sets it by default);
// timing experiments only (g_tune[31], results wrong): 1 no per-chunk wait and barrier,
// 2 no dequantisation (raw weight bits as the B operand), 4 LDS activation fragments read
// once per chunk
// Defaults measured on MI355X (opbench after a warm-up arm, profiles/r03/ab_mmq4_x.txt):
// glu 185.7 -> 173.5 us, down Q4_K 83.8 -> 77.4 us (X 0 -> 24)
#ifndef MX_M4_Q6V2
#define MX_M4_Q6V2 1
#endif
#ifndef MX_M4_PIPE
#define MX_M4_PIPE 1
#endif
#ifndef MX_M4_2STAGE      // two-chunk stages (round 4): glu 181 -> 159, down Q6_K 114 -> 100 us
#define MX_M4_2STAGE 1    // (same-box opbench, profiles/r04/mmq4_two_chunk_stages_ab.txt)
#endif
#ifndef MX_M4_5SLOT       // five-slot (160 KB) ring with two-chunk stages: glu 164.8 -> 159.0,
#define MX_M4_5SLOT 1     // down Q6_K 105 -> 102 us (profiles/r04/mmq4_five_slot_ab.txt)
#endif
constexpr int M4_XDEF = (MX_M4_Q6V2 ? 8 : 0) | (MX_M4_PIPE ? 16 : 0) | (MX_M4_2STAGE ? 32 : 0) |
                        (MX_M4_2STAGE && MX_M4_5SLOT ? 64 : 0);
#ifndef MX_M4_LDA
#define MX_M4_LDA 1               // MFMA steps the LDS activation reads run ahead (1 or 2)
#endif
constexpr int M4_MAXSEG = 3;
constexpr float M4_WSCALE = 1024.0f;

struct M4Seg {
    const char * w; size_t w_row;
    float * dst; size_t d_col;       // in floats
    const float * res; size_t r_col; // + residual (nullable)
    int M;
    int isb;                         // weight type QTB (else QTA)
    int tile0;                       // first row tile of the segment in grid.y
};

struct M4Args {
    M4Seg seg[M4_MAXSEG];
    int nseg;
    const char * w2;                 // GLU: the up matrix (layout and type of seg[0])
    const _Float16 * x; int64_t kp;  // activations f16 [cols][kp]
    const int32_t * gather;          // MoE: activation column of token slot t (null: t)
    const int32_t * scatter;         // MoE: output column of token slot t (null: t)
    const int32_t * tile_tab;        // MoE: per-expert (token-slot start, count) pairs, grid.z = expert
    size_t w_exp;                    // MoE: expert stride of the weights (bytes)
    int N, K;
    _Float16 * h; int64_t h_col;     // f16 copy of the output (next GEMM's input), nullable
    int ksplit;                      // EPI 0: K shares over grid.z (1: no split)
    float * part; int part_ld;       // split-K partial sums [ksplit][N][part_ld] (part_ld = padded rows)
    unsigned long long * trace;      // debug (opbench --trace, slot 3): phase stamps of workgroup 0
    unsigned long long * trace_blk;  // debug (opbench --trace-blocks): {start, end} of every workgroup
    int dbg;                         // timing experiments (g_tune[19]): 4 no activation DMA, 8 weights of
                                     // chunk 0 only
};

// ---------------------------------------------------------------------------
// weight registers of one lane for one K chunk (its row, k-slice h = lane >> 5)
// ---------------------------------------------------------------------------
template <int QT> struct M4W;
template <> struct M4W<GGML_TYPE_Q4_K> { int4 hd, q0, q1; };
template <> struct M4W<GGML_TYPE_Q5_K> { int4 hd, q0, q1, h0, h1; };
template <> struct M4W<GGML_TYPE_Q6_K> { int4 l0, l1, h0, h1, sc; uint32_t d; };
// round 5: Q8_0 (the 8-expert recipe's attn_k / attn_v, llama-quant.cpp:311-321; q8_0
// models): the lane's two 32-weight blocks of the chunk (k 64h .. 64h + 63), each 34 B =
// f16 d + 32 int8; unit j = block 2h + j
template <> struct M4W<GGML_TYPE_Q8_0> { int4 a0, a1, b0, b1; uint32_t d; };

template <int QT> __host__ __device__ constexpr int m4_loads() {   // vector loads per chunk (lower bound)
    return QT == GGML_TYPE_Q4_K ? 3 : QT == GGML_TYPE_Q8_0 ? 6 : 5;
}

__device__ __forceinline__ int4 ldu16(const char * p) {   // 16 bytes at any 2-byte alignment
    int4 v;
    __builtin_memcpy(&v, __builtin_assume_aligned(p, 2), 16);
    return v;
}

template <int QT>
__device__ __forceinline__ void m4_load(const char * row, int kc, int h, M4W<QT> & r) {
    const int sb = kc >> 1, hf = kc & 1;
    if constexpr (QT == GGML_TYPE_Q4_K) {
        const char * b = row + (size_t) sb * 144;
        r.hd = *(const int4 *) b;
        r.q0 = *(const int4 *) (b + 16 + 16 * (4 * hf + 2 * h));
        r.q1 = *(const int4 *) (b + 32 + 16 * (4 * hf + 2 * h));
    } else if constexpr (QT == GGML_TYPE_Q5_K) {
        const char * b = row + (size_t) sb * 176;
        r.hd = *(const int4 *) b;
        r.h0 = *(const int4 *) (b + 16);
        r.h1 = *(const int4 *) (b + 32);
        r.q0 = *(const int4 *) (b + 48 + 16 * (4 * hf + 2 * h));
        r.q1 = *(const int4 *) (b + 64 + 16 * (4 * hf + 2 * h));
    } else if constexpr (QT == GGML_TYPE_Q8_0) {
        const char * b = row + (size_t) (4 * kc + 2 * h) * 34;       // blocks 4kc + 2h, + 1
        r.a0 = ldu16(b + 2);
        r.a1 = ldu16(b + 18);
        r.b0 = ldu16(b + 36);
        r.b1 = ldu16(b + 52);
        r.d = (uint32_t) *(const uint16_t *) b | ((uint32_t) *(const uint16_t *) (b + 34) << 16);
    } else {
        const char * b = row + (size_t) sb * 210;
        r.l0 = ldu16(b + 64 * hf + 32 * h);
        r.l1 = ldu16(b + 64 * hf + 32 * h + 16);
        r.h0 = ldu16(b + 128 + 32 * hf);
        r.h1 = ldu16(b + 128 + 32 * hf + 16);
        r.sc = ldu16(b + 192);
        r.d = *(const uint16_t *) (b + 208);
    }
}

__device__ __forceinline__ uint32_t dw(const int4 & v, int i) {
    return (uint32_t) (i == 0 ? v.x : i == 1 ? v.y : i == 2 ? v.z : v.w);
}
// bytes 0,1 (sel01) or 2,3 (sel23) of w into the low bytes of the two halfwords
__device__ __forceinline__ uint32_t pair_bytes(uint32_t w, int hi_pair) {
    return __builtin_amdgcn_perm(0u, w, hi_pair ? 0x0c030c02u : 0x0c010c00u);
}
__device__ __forceinline__ h2 as_h2(uint32_t u) { h2 v; __builtin_memcpy(&v, &u, 4); return v; }
// (x & m) | b as one v_and_or_b32 (mask from an SGPR, bias from a VGPR: GFX9 VOP3 reads
// one constant-bus operand and no literal; the compiler otherwise emits v_and + v_or)
#ifndef MX_M4_ANDOR      // same box: glu 210.4 -> 205.9 us, down Q4_K 97.4 -> 93.5 (profiles/r03/ab_mmq4.txt)
#define MX_M4_ANDOR 1
#endif
__device__ __forceinline__ uint32_t m4_and_or(uint32_t x, uint32_t m, uint32_t b) {
#if MX_M4_ANDOR
    uint32_t r;
    asm("v_and_or_b32 %0, %1, %2, %3" : "=v"(r) : "v"(x), "s"(m), "v"(b));
    return r;
#else
    return (x & m) | b;
#endif
}

// dequantised scales of one lane's unit: lo / hi sub-block (d*sc, -dmin*m) x ws, f16;
// Q5_K also the qh bit index of the two sub-blocks
struct M4Scale { h2 slo, mlo, shi, mhi; int gb; };

template <int QT>
__device__ __forceinline__ M4Scale m4_scales(const M4W<QT> & r, int kc, int h, int j, float ws) {
    M4Scale s;
    const int hf = kc & 1, U = 2 * h + j;
    if constexpr (QT == GGML_TYPE_Q4_K || QT == GGML_TYPE_Q5_K) {
        const int g = 2 * hf + h;                              // sub-block pair (2g, 2g+1) of unit U
        const uint32_t s0 = dw(r.hd, 1), s1 = dw(r.hd, 2), s2 = dw(r.hd, 3);
        // get_scale_min_k4 (ggml-quants.c:703) of sub-blocks 2g, 2g+1, packed extraction.
        // g < 2 <=> hf == 0 (h is 0 or 1): written on the wave-uniform hf, so the select is
        // scalar — as `g < 2` the compiler branched on the lane's h (exec-mask branches in
        // every MFMA step)
        const uint32_t scw = hf == 0 ? (s0 & 0x3F3F3F3Fu) : ((s2 & 0x0F0F0F0Fu) | ((s0 >> 2) & 0x30303030u));
        const uint32_t mnw = hf == 0 ? (s1 & 0x3F3F3F3Fu) : (((s2 >> 4) & 0x0F0F0F0Fu) | ((s1 >> 2) & 0x30303030u));
        const uint32_t scp = scw >> (16 * (g & 1)), mnp = mnw >> (16 * (g & 1));
        const float d = h2f((uint16_t) (dw(r.hd, 0) & 0xFFFF)) * ws;
        const float dm = h2f((uint16_t) (dw(r.hd, 0) >> 16)) * ws;
        const _Float16 a = (_Float16) (d * (float) (scp & 0xFF)), b = (_Float16) (d * (float) ((scp >> 8) & 0xFF));
        const _Float16 c = (_Float16) (-dm * (float) (mnp & 0xFF)), e = (_Float16) (-dm * (float) ((mnp >> 8) & 0xFF));
        s.slo = h2{a, a}; s.shi = h2{b, b}; s.mlo = h2{c, c}; s.mhi = h2{e, e};
        s.gb = 2 * g;
    } else if constexpr (QT == GGML_TYPE_Q8_0) {
        const _Float16 a = (_Float16) (h2f((uint16_t) (j ? r.d >> 16 : r.d & 0xFFFF)) * ws);
        s.slo = h2{a, a}; s.shi = s.slo;
        s.mlo = h2{0, 0}; s.mhi = h2{0, 0};
        s.gb = 0;
    } else {
        // 16-wide groups: lo k = 128hf + 16U + i -> scale 8hf + U, hi (+64) -> 8hf + 4 + U
        const int slo = 8 * hf + U, shi = slo + 4;
        const float d = h2f((uint16_t) r.d) * ws;
        const int8_t vlo = (int8_t) (dw(r.sc, slo >> 2) >> (8 * (slo & 3)));
        const int8_t vhi = (int8_t) (dw(r.sc, shi >> 2) >> (8 * (shi & 3)));
        const _Float16 a = (_Float16) (d * (float) vlo), b = (_Float16) (d * (float) vhi);
        s.slo = h2{a, a}; s.shi = h2{b, b};
        s.mlo = h2{0, 0}; s.mhi = h2{0, 0};
        s.gb = 0;
    }
    return s;
}

// Range guard of one chunk: the largest scaled weight magnitude the chunk can produce is
// ws x (Q4_K 15*63 d | 63 dmin, Q5_K 31*63 d | 63 dmin, Q6_K 32*128 d); it must stay below
// 2^15 (f16 max 65504). A lane whose chunk exceeds it takes the largest power of two that
// fits and rescales its accumulators by the ratio (its accumulators are all of its own
// row, and the row's other lane (r + 32) reads the same super-block header, so both pick
// the same ws). Scales only ever shrink, so a row rescales at most a few times.
template <int QT, int TT>
__device__ __forceinline__ void m4_range(const M4W<QT> & r, float & ws, f16v (&acc)[TT]) {
    float need;
    if constexpr (QT == GGML_TYPE_Q6_K) {
        need = __builtin_fabsf(h2f((uint16_t) r.d)) * 4096.0f;
    } else if constexpr (QT == GGML_TYPE_Q8_0) {
        // the row's two lanes (h = 0, 1) hold different blocks (K-quant lanes share the
        // super-block header): the largest of all four, so both pick the same scale — the
        // MFMA sums both halves' B values into one output
        need = __builtin_fmaxf(__builtin_fabsf(h2f((uint16_t) (r.d & 0xFFFF))), __builtin_fabsf(h2f((uint16_t) (r.d >> 16)))) * 128.0f;
        need = __builtin_fmaxf(need, __shfl_xor(need, 32, 64));
    } else {
        const float d = __builtin_fabsf(h2f((uint16_t) (dw(r.hd, 0) & 0xFFFF)));
        const float dm = __builtin_fabsf(h2f((uint16_t) (dw(r.hd, 0) >> 16)));
        need = __builtin_fmaxf(d * (QT == GGML_TYPE_Q4_K ? 945.0f : 1953.0f), dm * 63.0f);
    }
    const bool over = need * ws >= 32768.0f;
    if (__builtin_amdgcn_ballot_w64(over)) {          // wave-uniform; ordinary weights never enter
        int e;
        (void) __builtin_frexpf(32768.0f / need, &e);
        const float wn = over ? __builtin_ldexpf(1.0f, e - 1) : ws;
        const float f = wn / ws;
#pragma unroll
        for (int t = 0; t < TT; ++t)
#pragma unroll
            for (int k = 0; k < 16; ++k) acc[t][k] *= f;
        ws = wn;
    }
}

// B operand of MFMA step q of unit j (q 0,1: the low sub-block's positions 8q..8q+7 of
// the 16-byte chunk; q 2,3: the high one's 8(q-2)..), element e = position + e
template <int QT, int X>
__device__ __forceinline__ h8 m4_deq(const M4W<QT> & r, const M4Scale & s, int h, int j, int q) {
    const bool hi = q >= 2;
    const int pd = 2 * (q & 1);                                // first of the chunk's two dwords
    h8 out;
    if constexpr (QT == GGML_TYPE_Q4_K || QT == GGML_TYPE_Q5_K) {
        const int4 & qs = j ? r.q1 : r.q0;
#pragma unroll
        for (int dd = 0; dd < 2; ++dd) {
            const uint32_t w = dw(qs, pd + dd);
            uint32_t qh = 0;
            if constexpr (QT == GGML_TYPE_Q5_K) qh = dw(j ? r.h1 : r.h0, pd + dd);   // qh byte = position
#pragma unroll
            for (int pp = 0; pp < 2; ++pp) {
                const uint32_t x = pair_bytes(w, pp);
                uint32_t v = hi ? m4_and_or(x, 0x00F000F0u, 0x54005400u)     // 64 + q (high nibble in place)
                                : m4_and_or(x, 0x000F000Fu, 0x64006400u);    // 1024 + q
                if constexpr (QT == GGML_TYPE_Q5_K) {
                    const uint32_t y = pair_bytes(qh, pp);
                    v |= hi ? (((y >> (s.gb + 1)) & 0x00010001u) << 8) : (((y >> s.gb) & 0x00010001u) << 4);
                }
                h2 f = as_h2(v) - (hi ? h2{64, 64} : h2{1024, 1024});
                f = hi ? (f * s.shi + s.mhi) : (f * s.slo + s.mlo);
                out[4 * dd + 2 * pp] = f[0];
                out[4 * dd + 2 * pp + 1] = f[1];
            }
        }
    } else if constexpr (QT == GGML_TYPE_Q8_0) {
        // bytes 8q .. 8q + 7 of block j: int8 -> f16 by the exponent trick, (q + 128) | 0x6400
        // = 1024 + 128 + q as one v_xor (the pair's high bytes are zero), minus 1152 exactly,
        // times d ws
        const int4 & qs = (q < 2) ? (j ? r.b0 : r.a0) : (j ? r.b1 : r.a1);
#pragma unroll
        for (int dd = 0; dd < 2; ++dd) {
            const uint32_t w = dw(qs, pd + dd);
#pragma unroll
            for (int pp = 0; pp < 2; ++pp) {
                const uint32_t v = pair_bytes(w, pp) ^ 0x64806480u;
                const h2 f = (as_h2(v) - h2{1152, 1152}) * s.slo;
                out[4 * dd + 2 * pp] = f[0];
                out[4 * dd + 2 * pp + 1] = f[1];
            }
        }
    } else {
        const int4 & ql = j ? r.l1 : r.l0;
        const int4 & qhv = j ? r.h1 : r.h0;
        const int sh = (hi ? 4 : 0) + 2 * h;                   // qh bit pair: position < 32 (h 0) or not
#pragma unroll
        for (int dd = 0; dd < 2; ++dd) {
            if constexpr (X & 8) {
            // per dword: the four 2-bit qh fields OR'd into the f16 exponent byte 0x54 (one
            // v_and_or), then per value pair one perm puts them in the high bytes, one
            // v_and_or adds the nibbles (pre-shifted for the low half): ~6.5 VALU per pair
            // instead of ~10.5
            uint32_t w = dw(ql, pd + dd);
            if (!hi) w <<= 4;
            const uint32_t t = m4_and_or(dw(qhv, pd + dd) >> sh, 0x03030303u, 0x54545454u);
#pragma unroll
            for (int pp = 0; pp < 2; ++pp) {
                const uint32_t hb = __builtin_amdgcn_perm(0u, t, pp ? 0x030c020cu : 0x010c000cu);
                const uint32_t v = m4_and_or(pair_bytes(w, pp), 0x00F000F0u, hb);          // 64 + q6
                const h2 f = (as_h2(v) - h2{96, 96}) * (hi ? s.shi : s.slo);            // (q6 - 32) d sc
                out[4 * dd + 2 * pp] = f[0];
                out[4 * dd + 2 * pp + 1] = f[1];
            }
            } else {
            const uint32_t w = dw(ql, pd + dd), qh = dw(qhv, pd + dd);
#pragma unroll
            for (int pp = 0; pp < 2; ++pp) {
                const uint32_t x = pair_bytes(w, pp), y = pair_bytes(qh, pp);
                const uint32_t nib = hi ? (x & 0x00F000F0u) : ((x << 4) & 0x00F000F0u);
                const uint32_t v = nib | (((y >> sh) & 0x00030003u) << 8) | 0x54005400u;   // 64 + q6
                const h2 f = (as_h2(v) - h2{96, 96}) * (hi ? s.shi : s.slo);            // (q6 - 32) d sc
                out[4 * dd + 2 * pp] = f[0];
                out[4 * dd + 2 * pp + 1] = f[1];
            }
            }
        }
    }
    return out;
}

// 16-byte chunk (8 k) of the 128-k activation tile that MFMA step q of unit j reads
template <int QT>
__device__ __forceinline__ int m4_ci(int h, int j, int q) {
    if constexpr (QT == GGML_TYPE_Q6_K) return 4 * h + 2 * j + (q < 2 ? q : 6 + q);   // lo 16U, hi 64 + 16U
    else if constexpr (QT == GGML_TYPE_Q8_0) return 8 * h + 4 * j + q;               // k 64h + 32j + 8q
    else return 8 * h + 2 * j + (q < 2 ? q : 2 + q);                                 // lo 64h + 16j, hi + 32
}

typedef __attribute__((address_space(3))) void * m4_lds_t;

template <int N>
__device__ __forceinline__ void m4_wait_vm() {   // s_waitcnt vmcnt(N), expcnt / lgkmcnt untouched
    static_assert(N >= 0 && N < 64, "vmcnt range");
    __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}
__device__ __forceinline__ void m4_barrier() {   // LDS reads/writes of this wave done, then s_barrier
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_s_barrier();
}

constexpr int M4_WAVES = 8;        // waves per workgroup (two per SIMD)
constexpr int M4_S = 4;            // activation ring stages (prefetch distance M4_S - 1 chunks)
template <int X> __host__ __device__ constexpr int m4_slots() { return (X & 64) ? 5 : M4_S; }   // X 64: 160 KB ring

// The K loop of one wave over chunks [c0, c0 + nc): its lane's row `wrow`, tokens
// [tok0, tok0 + 32 TT) of the workgroup's activation ring (cols: activation column of
// each of this wave's DMA pieces). Weight registers rotate over three sets (loads two
// chunks ahead), the activation ring runs M4_S - 1 chunks ahead; one barrier per chunk
// (it also retires the stage the previous chunk read, which the DMA then refills).
template <int QT, int TT, int X>
__device__ __forceinline__ void m4_kloop(const M4Args & p, const char * wrow, const int (&cols)[TT],
                                         uint4 * lds, int c0, int nc, f16v (&acc)[TT], float & ws,
                                         unsigned long long * tr) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, r = lane & 31, h = lane >> 5;
    constexpr int NDMA = TT;                     // 1-KB LDS-DMA pieces per wave per chunk (32 TT rows / 8 waves / 4 rows)
    constexpr int TILE = 32 * TT * 16;           // uint4 per stage
    constexpr int NW = m4_loads<QT>();
#pragma unroll
    for (int t = 0; t < TT; ++t)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[t][e] = 0.f;
    auto dma = [&](int i) {
        if (MX_DBG(p.dbg & 4)) return;
        const int st = (i % m4_slots<X>()) * TILE, kc = c0 + i;
#pragma unroll
        for (int d = 0; d < NDMA; ++d) {
            const int trow = (wave * NDMA + d) * 4 + (lane >> 4);
            const int slot = (lane & 15) ^ (trow & 15);
            const _Float16 * g = p.x + (size_t) cols[d] * p.kp + (size_t) kc * M4_KC + 8 * slot;
            __builtin_amdgcn_global_load_lds(g, (m4_lds_t) (lds + st + (wave * NDMA + d) * 64), 16, 0, 0);
        }
    };
    // activation fragments of step (j, q) for every token tile, read one step ahead so
    // the LDS latency overlaps the previous step's MFMAs and this step's dequantisation.
    // (No runtime switches in here: even a never-taken branch costs the loop its MFMA
    // schedule — branches around every MFMA and accumulator copies at the joins.)
    auto lda = [&](const uint4 * L, int j, int q, h8 (&a)[TT]) {
        const int ci = m4_ci<QT>(h, j, q) ^ (r & 15);
#pragma unroll
        for (int t = 0; t < TT; ++t) {
            const uint4 av = L[(32 * t + r) * 16 + ci];
            __builtin_memcpy(&a[t], &av, 16);
        }
    };
    auto compute = [&](const M4W<QT> & rw, int i) {
        const uint4 * L = lds + (i % m4_slots<X>()) * TILE;
        const int kc = c0 + i;
        // activation fragments MX_M4_LDA steps ahead (ring of MX_M4_LDA + 1 register sets)
        constexpr int D = (X & 16) ? 2 : MX_M4_LDA;
        h8 af[D + 1][TT];
#pragma unroll
        for (int st = 0; st < D; ++st) lda(L, st >> 2, st & 3, af[st]);
        if constexpr (!(X & 2)) m4_range<QT, TT>(rw, ws, acc);
        // the two units' scales once per chunk (they depend on j only, not on the step)
        const M4Scale sj[2] = {m4_scales<QT>(rw, kc, h, 0, ws), m4_scales<QT>(rw, kc, h, 1, ws)};
        if constexpr (X & 16) {
            // software-pipelined: step st+1's B operand is dequantised while step st's MFMAs
            // run, the schedule interleaving one MFMA, one LDS read and NV VALU instructions
            // (a block of 4 MFMAs followed by the dequantisation left the matrix pipe idle
            // while the VALU ran, with both waves of a SIMD in the same phase)
            constexpr int NV = QT == GGML_TYPE_Q6_K ? 7 : 6;
            h8 bq[2];
            bq[0] = m4_deq<QT, X>(rw, sj[0], h, 0, 0);
#pragma unroll
            for (int st = 0; st < 8; ++st) {
                h8 (&cur)[TT] = af[st % (D + 1)];
                if (st + D < 8) lda(L, (st + D) >> 2, (st + D) & 3, af[(st + D) % (D + 1)]);
                if (st + 1 < 8) bq[(st + 1) & 1] = m4_deq<QT, X>(rw, sj[(st + 1) >> 2], h, (st + 1) >> 2, (st + 1) & 3);
#pragma unroll
                for (int t = 0; t < TT; ++t) acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(cur[t], bq[st & 1], acc[t], 0, 0, 0);
#pragma unroll
                for (int t = 0; t < TT; ++t) {
                    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                    __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
                    __builtin_amdgcn_sched_group_barrier(0x002, NV, 0);
                }
                __builtin_amdgcn_sched_barrier(0);   // one scheduling region per step
            }
            return;
        }
#pragma unroll
        for (int st = 0; st < 8; ++st) {
            const int j = st >> 2, q = st & 3;
            const M4Scale & s = sj[j];
            h8 (&cur)[TT] = af[(X & 4) ? 0 : st % (D + 1)];
            if (!(X & 4) && st + D < 8) lda(L, (st + D) >> 2, (st + D) & 3, af[(st + D) % (D + 1)]);
            h8 b;
            if constexpr (X & 2) {   // timing only
                int4 w;
                if constexpr (QT == GGML_TYPE_Q6_K) w = j ? rw.l1 : rw.l0; else w = j ? rw.q1 : rw.q0;
                __builtin_memcpy(&b, &w, 16);
            }
            else b = m4_deq<QT, X>(rw, s, h, j, q);
#pragma unroll
            for (int t = 0; t < TT; ++t) acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(cur[t], b, acc[t], 0, 0, 0);
        }
    };
    auto wl = [&](int i, M4W<QT> & rw) { m4_load<QT>(wrow, MX_DBG(p.dbg & 8) ? c0 : c0 + i, h, rw); };
    M4W<QT> r0, r1, r2;
    // prologue: ring stages 0 .. S-2 (two-chunk stages: chunks 0 and 1), weights of chunks 0 and 1
#pragma unroll
    for (int i = 0; i < ((X & 64) ? 3 : (X & 32) ? 2 : M4_S - 1); ++i) if (i < nc) dma(i);
    __builtin_amdgcn_sched_barrier(0);
    wl(0, r0);
    if (nc > 1) wl(1, r1);
    __builtin_amdgcn_sched_barrier(0);
    MX_TRACE(tr, 1);
    if constexpr (X & 32) {
        // round 4 (X bit 32, the default; g_tune[3] = 2 restores one-chunk stages): two-chunk
        // stages — the ring's four chunk slots
        // are filled two at a time, one counted wait + barrier per PAIR of chunks (the
        // per-chunk wait + barrier was 44 of 203 us of the glu, profiles/r03/
        // mmq4_decomposition.txt); prefetch distance two chunks instead of three. Loop
        // unrolled by six (weight register sets rotate by three, stages by two).
        auto iter2 = [&](int i, bool even, const M4W<QT> & rc, M4W<QT> & rn) {
            if (even && (X & 64)) {
                // five slots: chunks i+3, i+4 go into the slots of i-2, i-1 (done before this
                // barrier); issued after DMA(i+1) (at i - 2): DMA(i+2) and the weights of
                // chunks i and i+1
                if (i + 2 < nc) m4_wait_vm<NDMA + 2 * NW>();
                else m4_wait_vm<0>();
                m4_barrier();
                __builtin_amdgcn_sched_barrier(0);
                if (i + 3 < nc) dma(i + 3);
                if (i + 4 < nc) dma(i + 4);
            } else if (even) {
                // issued after DMA(i), DMA(i+1) (at i - 2): the weights of chunks i and i+1
                if (i + 3 < nc) m4_wait_vm<2 * NW>();
                else m4_wait_vm<0>();
                m4_barrier();
                __builtin_amdgcn_sched_barrier(0);
                if (i + 2 < nc) dma(i + 2);
                if (i + 3 < nc) dma(i + 3);
            }
            __builtin_amdgcn_sched_barrier(0);
            if (i + 2 < nc) wl(i + 2, rn);
            __builtin_amdgcn_sched_barrier(0);
            compute(rc, i);
        };
        for (int i = 0; i < nc; i += 6) {
            iter2(i, true, r0, r2);
            if (i + 1 < nc) iter2(i + 1, false, r1, r0);
            if (i + 2 < nc) iter2(i + 2, true, r2, r1);
            if (i + 3 < nc) iter2(i + 3, false, r0, r2);
            if (i + 4 < nc) iter2(i + 4, true, r1, r0);
            if (i + 5 < nc) iter2(i + 5, false, r2, r1);
        }
        MX_TRACE(tr, 6);
        return;
    }
    auto iter = [&](int i, const M4W<QT> & rc, M4W<QT> & rn) {
        // instructions issued after DMA(i): >= DMA(i+1), DMA(i+2) and two chunks of weight
        // loads in steady state; the last chunks drain everything
        if constexpr (!(X & 1)) {
            if (i + 2 < nc) m4_wait_vm<2 * NDMA + 2 * NW>();
            else m4_wait_vm<0>();
        }
        if (i == 2) MX_TRACE(tr, 2);
        if constexpr (!(X & 1)) m4_barrier();
        if (i == 2) MX_TRACE(tr, 3);
        __builtin_amdgcn_sched_barrier(0);
        if (i + M4_S - 1 < nc) dma(i + M4_S - 1);
        __builtin_amdgcn_sched_barrier(0);
        if (i + 2 < nc) wl(i + 2, rn);
        __builtin_amdgcn_sched_barrier(0);
        compute(rc, i);
        if (i == 2) MX_TRACE(tr, 4);
        if (i == 5) MX_TRACE(tr, 5);
    };
    for (int i = 0; i < nc; i += 3) {
        iter(i, r0, r2);
        if (i + 1 < nc) iter(i + 1, r1, r0);
        if (i + 2 < nc) iter(i + 2, r2, r1);
    }
    MX_TRACE(tr, 6);
}

// EPI 0: store (+ residual) to the segment; 1: SwiGLU of a gate/up pair (waves 0-3 gate
// rows, 4-7 up rows of the same 128); 2: MoE expert tile — grid.z = expert, token slots
// gathered through p.gather, outputs scattered through p.scatter; 3 (round 5): both — the
// MoE gate/up/SwiGLU of an expert's tokens in one launch (w / w2 = gate / up experts).
// Split K (EPI 0, grid.z = p.ksplit > 1): each workgroup sums its share of the K chunks
// into p.part[z][token][global row]; k_mmq4_reduce adds the shares in order.
template <int QTA, int QTB, int TT, int EPI, int X = M4_XDEF>
__global__ __launch_bounds__(512, 1) void k_mmq4(M4Args p) {
    extern __shared__ __align__(16) uint4 lds[];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, r = lane & 31, h = lane >> 5;
    constexpr int BT = 32 * TT;
    constexpr bool MOE = EPI == 2 || EPI == 3, GLU = EPI == 1 || EPI == 3;
    // MoE (EPI 2, 3): grid.x = row tile, grid.y = token tile. Workgroups go to the XCDs
    // round-robin by linear index, and most token tiles of an expert are empty: with the
    // token tile fastest every busy workgroup (token tile 0) landed on XCD 0 (measured:
    // 1.8 ms instead of ~0.3 for a Mixtral pp512 gate projection)
    const int by = MOE ? (int) blockIdx.x : (int) blockIdx.y;
    const int bx = MOE ? (int) blockIdx.y : (int) blockIdx.x;
    int si = 0;
#pragma unroll
    for (int i = 1; i < M4_MAXSEG; ++i) if (i < p.nseg && by >= p.seg[i].tile0) si = i;
    const M4Seg & sg = p.seg[si];
    const int tile = by - sg.tile0;
    int tok0 = bx * BT, ntok = p.N, slot0 = 0;
    const char * wb = sg.w, * wb2 = p.w2;
    const int nk = p.K / M4_KC;
    int c0 = 0, nc = nk;
    const size_t bid = blockIdx.x + (size_t) gridDim.x * (blockIdx.y + (size_t) gridDim.y * blockIdx.z);
    if (p.trace_blk && tid == 0 && bid < 65536) p.trace_blk[2 * bid] = __builtin_amdgcn_s_memrealtime();
    if constexpr (MOE) {
        const int e = (int) blockIdx.z;
        slot0 = p.tile_tab[2 * e];
        ntok = p.tile_tab[2 * e + 1];
        if (tok0 >= ntok) {                           // block-uniform, before any barrier
            if (p.trace_blk && tid == 0 && bid < 65536) p.trace_blk[2 * bid + 1] = __builtin_amdgcn_s_memrealtime();
            return;
        }
        wb += (size_t) e * p.w_exp;
        if constexpr (GLU) wb2 += (size_t) e * p.w_exp;
    } else if (p.ksplit > 1) {
        c0 = (int) blockIdx.z * nk / p.ksplit;
        nc = ((int) blockIdx.z + 1) * nk / p.ksplit - c0;
    }
    // rows of this wave
    constexpr int RPT = GLU ? 32 * M4_WAVES / 2 : 32 * M4_WAVES;   // output rows per tile
    const int wr = GLU ? (wave & (M4_WAVES / 2 - 1)) : wave;
    const int row = tile * RPT + wr * 32 + r;
    const int rr = row < sg.M ? row : sg.M - 1;
    const char * wrow = (GLU && wave >= M4_WAVES / 2 ? wb2 : wb) + (size_t) rr * sg.w_row;
    // activation columns of this wave's DMA pieces (token row clamped into range)
    int cols[TT];
#pragma unroll
    for (int i = 0; i < TT; ++i) {
        int t = tok0 + (wave * TT + i) * 4 + (lane >> 4);
        t = t < ntok ? t : ntok - 1;
        cols[i] = MOE ? p.gather[slot0 + t] : t;
    }
    f16v acc[TT];
    float ws = M4_WSCALE;                             // this lane's weight scale (m4_range)
    unsigned long long * tr = (blockIdx.x | blockIdx.y | blockIdx.z) == 0 ? p.trace : nullptr;
    MX_TRACE(tr, 0);
    if (!sg.isb || QTA == QTB) m4_kloop<QTA, TT, X>(p, wrow, cols, lds, c0, nc, acc, ws, tr);
    else m4_kloop<QTB, TT, X>(p, wrow, cols, lds, c0, nc, acc, ws, tr);

    if (p.trace_blk && tid == 0 && bid < 65536) p.trace_blk[2 * bid + 1] = __builtin_amdgcn_s_memrealtime();
    const float inv = 1.0f / ws;
    if constexpr (GLU) {
        float * red = (float *) lds;                  // 4 waves x TT x 16 x 64 floats (<= the ring)
        m4_barrier();                                 // every wave is done with the ring
        if (wave >= M4_WAVES / 2) {
#pragma unroll
            for (int t = 0; t < TT; ++t)
#pragma unroll
                for (int e = 0; e < 16; ++e) red[(((wave - M4_WAVES / 2) * TT + t) * 16 + e) * 64 + lane] = acc[t][e] * inv;
        }
        m4_barrier();
        if (wave >= M4_WAVES / 2) return;
#pragma unroll
        for (int t = 0; t < TT; ++t)
#pragma unroll
            for (int e = 0; e < 16; ++e) {
                const int tok = tok0 + 32 * t + (e & 3) + 8 * (e >> 2) + 4 * h;
                const float g = acc[t][e] * inv, u = red[((wave * TT + t) * 16 + e) * 64 + lane];
                const float v = g * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(-g * 1.4426950408889634f)) * u;
                if (tok < ntok && row < sg.M) {
                    const size_t oc = MOE ? (size_t) p.scatter[slot0 + tok] : (size_t) tok;
                    sg.dst[oc * sg.d_col + row] = v;
                    if (p.h) p.h[oc * p.h_col + row] = (_Float16) v;
                }
            }
    } else if (EPI == 0 && p.ksplit > 1) {
        float * part = p.part + (size_t) blockIdx.z * p.N * p.part_ld + sg.tile0 * RPT;
#pragma unroll
        for (int t = 0; t < TT; ++t)
#pragma unroll
            for (int e = 0; e < 16; ++e) {
                const int tok = tok0 + 32 * t + (e & 3) + 8 * (e >> 2) + 4 * h;
                if (tok < ntok && row < sg.M) part[(size_t) tok * p.part_ld + row] = acc[t][e] * inv;
            }
    } else {
#pragma unroll
        for (int t = 0; t < TT; ++t)
#pragma unroll
            for (int e = 0; e < 16; ++e) {
                const int tok = tok0 + 32 * t + (e & 3) + 8 * (e >> 2) + 4 * h;
                if (tok < ntok && row < sg.M) {
                    float v = acc[t][e] * inv;
                    const size_t oc = EPI == 2 ? (size_t) p.scatter[slot0 + tok] : (size_t) tok;
                    if (EPI == 0 && sg.res) v += sg.res[oc * sg.r_col + row];
                    sg.dst[oc * sg.d_col + row] = v;
                    if (p.h) p.h[oc * p.h_col + row] = (_Float16) v;
                }
            }
    }
}

// split-K reduction: out = sum over shares z (in order) + residual, per segment
__global__ void k_mmq4_reduce(M4Args p) {
    const int tok = (int) blockIdx.y;
    const int row = (int) (blockIdx.x * blockDim.x + threadIdx.x);   // global row over segments
    if (row >= p.part_ld) return;
    int si = 0;
    for (int i = 1; i < p.nseg; ++i) if (row >= p.seg[i].tile0 * 32 * M4_WAVES) si = i;
    const M4Seg & sg = p.seg[si];
    const int lr = row - sg.tile0 * 32 * M4_WAVES;
    if (lr >= sg.M) return;
    float v = 0.f;
    for (int z = 0; z < p.ksplit; ++z) v += p.part[((size_t) z * p.N + tok) * p.part_ld + row];
    if (sg.res) v += sg.res[(size_t) tok * sg.r_col + lr];
    sg.dst[(size_t) tok * sg.d_col + lr] = v;
    if (p.h) p.h[(size_t) tok * p.h_col + lr] = (_Float16) v;
}

// ---------------------------------------------------------------------------
// k_mmq5: the gate/up/SwiGLU GEMM on 256-token tiles, one wave per SIMD (round 4).
// In k_mmq4 a wave multiplies one dequantised 32-row B fragment into 4 token tiles: ~6
// VALU per MFMA, which with the partner wave's share overfills the MFMA's issue gaps (at
// most ~5 single-issue fillers hide per v_mfma_f32_32x32x16, MI355X_MICROARCH.md constants
// table), and every MFMA reads its own activation fragment from LDS. Here a wave holds 32
// gate rows AND the same 32 up rows (two B fragments) x 256 tokens (eight token tiles):
// per 16-deep step 16 MFMAs on 8 LDS reads and 2 dequantisations (~2-3 VALU per MFMA);
// 256 accumulators (512-register wave), and the SwiGLU pairs gate and up inside the lane
// that holds both (no LDS exchange). Four waves = 128 row pairs x 256 tokens per
// workgroup; a 2 x 64 KB activation ring (one wait + barrier per 128-deep chunk, DMA one
// chunk ahead), weights two chunks ahead in three register sets. Token tiles of one row
// tile go to one XCD (they read the same weight rows: one HBM read per L2).
// ---------------------------------------------------------------------------
#ifndef M5TT_
#define M5TT_ 8
#endif
#ifndef M5_SCHED
#define M5_SCHED 1
#endif
constexpr int M5_WAVES = 4, M5_TT = M5TT_, M5_BT = 32 * M5_TT;
typedef uint32_t v4u __attribute__((ext_vector_type(4)));
typedef uint32_t v2u __attribute__((ext_vector_type(2)));
constexpr int M5_TILE = M5_BT * 16;                  // uint4 per ring slot (64 KB)
constexpr int M5_NDMA = M5_BT / 4 / M5_WAVES;        // 1-KB LDS-DMA pieces per wave per chunk
constexpr int M5_LDS = 2 * M5_TILE * 16;
constexpr int M5_XDEF = M4_XDEF;   // (| 128: interleaved issue, g_tune[3] = 16; measured slower)

// m4_load with the chunk-dependent part of every address uniform (base + kc offsets) and
// the lane's part a 32-bit offset (row, k-slice h)
template <int QT>
__device__ __forceinline__ void m5_load(const char * base, uint32_t wo, int kc, int h, M4W<QT> & r) {
    const int sb = kc >> 1, hf = kc & 1;
    const uint32_t qo = wo + 32u * (uint32_t) h;
    if constexpr (QT == GGML_TYPE_Q4_K) {
        const char * b = base + (size_t) sb * 144;
        r.hd = *(const int4 *) (b + wo);
        r.q0 = *(const int4 *) (b + 16 + 64 * hf + qo);
        r.q1 = *(const int4 *) (b + 32 + 64 * hf + qo);
    } else {
        static_assert(QT == GGML_TYPE_Q5_K, "k_mmq5: Q4_K / Q5_K");
        const char * b = base + (size_t) sb * 176;
        r.hd = *(const int4 *) (b + wo);
        r.h0 = *(const int4 *) (b + 16 + wo);
        r.h1 = *(const int4 *) (b + 32 + wo);
        r.q0 = *(const int4 *) (b + 48 + 64 * hf + qo);
        r.q1 = *(const int4 *) (b + 64 + 64 * hf + qo);
    }
}

// largest scaled weight magnitude of a Q4_K / Q5_K super-block per unit of scale (its
// d / dmin header dword), and the weight scale a row whose maximum is `need` takes
template <int QT>
__device__ __forceinline__ float m5_need(uint32_t dd) {
    const float d = __builtin_fabsf(h2f((uint16_t) (dd & 0xFFFF)));
    const float dm = __builtin_fabsf(h2f((uint16_t) (dd >> 16)));
    return __builtin_fmaxf(d * (QT == GGML_TYPE_Q4_K ? 945.0f : 1953.0f), dm * 63.0f);
}
__device__ __forceinline__ float m5_ws(float need) {
    if (need * M4_WSCALE < 32768.0f) return M4_WSCALE;
    int e;
    (void) __builtin_frexpf(32768.0f / need, &e);
    return __builtin_ldexpf(1.0f, e - 1);
}

template <int QT, int X = M5_XDEF>
__global__ __attribute__((amdgpu_flat_work_group_size(256, 256), amdgpu_waves_per_eu(1, 1)))
void k_mmq5_glu(M4Args p) {
    extern __shared__ __align__(16) uint4 lds[];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, r = lane & 31, h = lane >> 5;
    const M4Seg & sg = p.seg[0];
    const int T = (p.N + M5_BT - 1) / M5_BT, R = (sg.M + 127) / 128, L = (int) blockIdx.x;
    int rt, tt;
    if ((R & 7) == 0) { const int k = L >> 3; rt = (k / T) * 8 + (L & 7); tt = k % T; }   // XCD = L mod 8
    else { rt = L / T; tt = L % T; }
    const int tok0 = tt * M5_BT, ntok = p.N;
    const int row = rt * 128 + wave * 32 + r;
    const int rr = row < sg.M ? row : sg.M - 1;
    // 32-bit lane offsets from uniform bases (global loads in saddr form: no 64-bit
    // address arithmetic per load; x < 4 GiB and a weight matrix < 4 GiB by the host check)
    uint32_t xo[M5_NDMA];
#pragma unroll
    for (int d = 0; d < M5_NDMA; ++d) {
        const int trow = (wave * M5_NDMA + d) * 4 + (lane >> 4);
        const int t = tok0 + trow < ntok ? tok0 + trow : ntok - 1;
        xo[d] = (uint32_t) t * (uint32_t) p.kp * 2u + 16u * (uint32_t) ((lane & 15) ^ (trow & 15));
    }
    const uint32_t wo = (uint32_t) rr * (uint32_t) sg.w_row;
    f16v acc[2][M5_TT];
#pragma unroll
    for (int f = 0; f < 2; ++f)
#pragma unroll
        for (int t = 0; t < M5_TT; ++t)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[f][t][e] = 0.f;
    const int nc = p.K / M4_KC;
    // weight scales of the row pair, fixed for the whole K loop: the largest power of two
    // <= 2^10 that keeps every scaled weight of the row below 2^15 (the lane pair of a row
    // scans alternate super-blocks' d / dmin; k_mmq4's m4_range reaches the same scale
    // chunk by chunk, rescaling its accumulators — 256 accumulators do not leave registers
    // for that)
    float ng = 0.f, nu = 0.f;
    {
        constexpr int BS = QT == GGML_TYPE_Q4_K ? 144 : 176;
        const int nsb = p.K / 256;
        for (int s0 = 0; s0 < nsb; s0 += 16) {
            uint32_t vg[8], vu[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const int sb = s0 + 2 * k + h;
                vg[k] = sb < nsb ? *(const uint32_t *) (sg.w + (size_t) sb * BS + wo) : 0u;
                vu[k] = sb < nsb ? *(const uint32_t *) (p.w2 + (size_t) sb * BS + wo) : 0u;
            }
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                ng = __builtin_fmaxf(ng, m5_need<QT>(vg[k]));
                nu = __builtin_fmaxf(nu, m5_need<QT>(vu[k]));
            }
        }
        ng = __builtin_fmaxf(ng, __shfl_xor(ng, 32));
        nu = __builtin_fmaxf(nu, __shfl_xor(nu, 32));
    }
    const float ws0 = m5_ws(ng), ws1 = m5_ws(nu);
    // X bit 256 (diagnostic builds): cycle sums per wave of workgroup 0 — prologue, chunk-head
    // wait + barrier, chunk compute, epilogue (s_memtime; opbench --trace)
    unsigned long long t_k0 = 0, t_loop = 0, t_wait = 0, t_comp = 0, t_a = 0;
    const bool trw = (X & 256) && p.trace && L == 0;
    if constexpr (X & 256) t_k0 = __builtin_amdgcn_s_memtime();
    constexpr int NW = m4_loads<QT>();
    constexpr int NV = QT == GGML_TYPE_Q4_K ? 2 : 3;   // VALU per MFMA in the step schedule
    auto dma_part = [&](int i, int d0, int nd) {
        const int st = (i & 1) * M5_TILE;
        const char * xb = (const char *) p.x + (size_t) i * (2 * M4_KC);
#pragma unroll
        for (int d = d0; d < d0 + nd; ++d)
            __builtin_amdgcn_global_load_lds((const void *) (xb + xo[d]), (m4_lds_t) (lds + st + (wave * M5_NDMA + d) * 64), 16, 0, 0);
    };
    auto dma = [&](int i) {
        if (MX_DBG(p.dbg & 4)) return;
        dma_part(i, 0, M5_NDMA);
    };
    auto lda = [&](const uint4 * Ls, int j, int q, h8 (&a)[M5_TT]) {
        const int ci = m4_ci<QT>(h, j, q) ^ (r & 15);
#pragma unroll
        for (int t = 0; t < M5_TT; ++t) {
            const uint4 av = Ls[(32 * t + r) * 16 + ci];
            __builtin_memcpy(&a[t], &av, 16);
        }
    };
    // X bit 128 (g_tune[3] = 16; glu 151 -> 159 us, so not the default): chunk i + 1's activation DMA (4 pieces in each of steps 0-3)
    // and chunk i + 2's weights (step 4) are issued between the MFMAs of chunk i — with one
    // wave per SIMD a burst of them at the chunk head left the matrix pipe idle while they
    // issued (~60-185 cycles per LDS-DMA piece, MI355X_MICROARCH.md). Past the end the
    // loads are clamped to the last chunk (into the free slot / register set: no branch in
    // the MFMA loop).
    auto compute = [&](int i, const M4W<QT> & wg, const M4W<QT> & wu, M4W<QT> & ng, M4W<QT> & nu) {
        const uint4 * Ls = lds + (i & 1) * M5_TILE;
        h8 af[2][M5_TT];
        lda(Ls, 0, 0, af[0]);
        const M4Scale sg_[2] = {m4_scales<QT>(wg, i, h, 0, ws0), m4_scales<QT>(wg, i, h, 1, ws0)};
        const M4Scale su_[2] = {m4_scales<QT>(wu, i, h, 0, ws1), m4_scales<QT>(wu, i, h, 1, ws1)};
        h8 bg[2], bu[2];
        bg[0] = m4_deq<QT, X>(wg, sg_[0], h, 0, 0);
        bu[0] = m4_deq<QT, X>(wu, su_[0], h, 0, 0);
#pragma unroll
        for (int st = 0; st < 8; ++st) {
            h8 (&cur)[M5_TT] = af[st & 1];
            if constexpr (X & 128) {
                if (st < 4) dma_part(i + 1 < nc ? i + 1 : nc - 1, 4 * st, 4);
                if (st == 4) {
                    const int kw = i + 2 < nc ? i + 2 : nc - 1;
                    m5_load<QT>(sg.w, wo, kw, h, ng); m5_load<QT>(p.w2, wo, kw, h, nu);
                }
            }
            if (st + 1 < 8) {
                const int j = (st + 1) >> 2, q = (st + 1) & 3;
                lda(Ls, j, q, af[(st + 1) & 1]);
                if constexpr (X & 2) {   // timing only: raw weight bits as the B operand
                    const int4 a = j ? wg.q1 : wg.q0, b = j ? wu.q1 : wu.q0;
                    __builtin_memcpy(&bg[(st + 1) & 1], &a, 16);
                    __builtin_memcpy(&bu[(st + 1) & 1], &b, 16);
                } else {
                    bg[(st + 1) & 1] = m4_deq<QT, X>(wg, sg_[j], h, j, q);
                    bu[(st + 1) & 1] = m4_deq<QT, X>(wu, su_[j], h, j, q);
                }
            }
#pragma unroll
            for (int t = 0; t < M5_TT; ++t)
                acc[0][t] = (X & 512) ? __builtin_amdgcn_mfma_f32_32x32x16_f16(bg[st & 1], cur[t], acc[0][t], 0, 0, 0)
                                      : __builtin_amdgcn_mfma_f32_32x32x16_f16(cur[t], bg[st & 1], acc[0][t], 0, 0, 0);
#pragma unroll
            for (int t = 0; t < M5_TT; ++t)
                acc[1][t] = (X & 512) ? __builtin_amdgcn_mfma_f32_32x32x16_f16(bu[st & 1], cur[t], acc[1][t], 0, 0, 0)
                                      : __builtin_amdgcn_mfma_f32_32x32x16_f16(cur[t], bu[st & 1], acc[1][t], 0, 0, 0);
#if M5_SCHED
#pragma unroll
            for (int t = 0; t < M5_TT; ++t) {
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                if ((X & 128) && ((st < 4 && t < 4) || (st == 4 && t < 2 * NW)))
                    __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
                __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
                __builtin_amdgcn_sched_group_barrier(0x002, NV, 0);
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                __builtin_amdgcn_sched_group_barrier(0x002, NV, 0);
            }
            __builtin_amdgcn_sched_barrier(0);
#endif
        }
    };
    M4W<QT> ga, ua, gb, ub, gc, uc;
    dma(0);
    __builtin_amdgcn_sched_barrier(0);
    m5_load<QT>(sg.w, wo, 0, h, ga); m5_load<QT>(p.w2, wo, 0, h, ua);
    if (nc > 1) { m5_load<QT>(sg.w, wo, 1, h, gb); m5_load<QT>(p.w2, wo, 1, h, ub); }
    __builtin_amdgcn_sched_barrier(0);
    // issued after DMA(i): the weights of chunk i + 1 (2 NW loads, at least); the wait also
    // retires the weights of chunk i (issued before DMA(i))
    auto iter = [&](int i, const M4W<QT> & cg, const M4W<QT> & cu, M4W<QT> & ng, M4W<QT> & nu) {
        if constexpr (X & 256) { __builtin_amdgcn_sched_barrier(0); t_a = __builtin_amdgcn_s_memtime(); if (i == 0) t_loop = t_a; }
        if constexpr (!(X & 1)) {
            if (i + 1 < nc) m4_wait_vm<2 * NW>();
            else m4_wait_vm<0>();
            m4_barrier();   // DMA(i) of every wave landed; chunk i - 1's slot is free
        }
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (!(X & 128)) {
            if (i + 1 < nc) dma(i + 1);
            __builtin_amdgcn_sched_barrier(0);
            if (i + 2 < nc) {
                const int kw = MX_DBG(p.dbg & 8) ? 0 : i + 2;
                m5_load<QT>(sg.w, wo, kw, h, ng); m5_load<QT>(p.w2, wo, kw, h, nu);
            }
            __builtin_amdgcn_sched_barrier(0);
        }
        if constexpr (X & 256) { __builtin_amdgcn_sched_barrier(0); const unsigned long long t = __builtin_amdgcn_s_memtime(); t_wait += t - t_a; t_a = t; }
        compute(i, cg, cu, ng, nu);
        if constexpr (X & 256) { __builtin_amdgcn_sched_barrier(0); t_comp += __builtin_amdgcn_s_memtime() - t_a; }
    };
    for (int i = 0; i < nc; i += 3) {
        iter(i, ga, ua, gc, uc);
        if (i + 1 < nc) iter(i + 1, gb, ub, ga, ua);
        if (i + 2 < nc) iter(i + 2, gc, uc, gb, ub);
    }
    m4_wait_vm<0>();   // (the clamped loads past the end)
    if constexpr (X & 512) {
        // weights as the A operand (X bit 512): the accumulators are D[row][token] — lane
        // (r, h) holds token 32t + r and rows 8g + 4h + 0..3 of the wave's 32 (g = e >> 2),
        // i.e. four consecutive output floats: one 16-byte store (and one 8-byte f16 store)
        // per four values instead of four 4-byte (and four 2-byte) ones. The rows' weight
        // scales come from the lanes that scanned them.
        float ig[4][4], iu[4][4];
#pragma unroll
        for (int g = 0; g < 4; ++g)
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                ig[g][c] = 1.0f / __shfl(ws0, 8 * g + 4 * h + c);
                iu[g][c] = 1.0f / __shfl(ws1, 8 * g + 4 * h + c);
            }
        const int rbase = rt * 128 + wave * 32 + 4 * h;          // + 8 g
        const bool rows_full = rt * 128 + 128 <= sg.M;
        const __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc(sg.dst, 0, (int) ((uint32_t) ntok * (uint32_t) sg.d_col * 4u), 0x00020000);
        const uint32_t lo = ((uint32_t) (tok0 + r) * (uint32_t) sg.d_col + (uint32_t) rbase) * 4u;
        const uint32_t lh = ((uint32_t) (tok0 + r) * (uint32_t) p.h_col + (uint32_t) rbase) * 2u;
        auto store = [&](auto with_h) {
            const __amdgpu_buffer_rsrc_t rh = with_h ? __builtin_amdgcn_make_buffer_rsrc(p.h, 0, (int) ((uint32_t) ntok * (uint32_t) p.h_col * 2u), 0x00020000) : rd;
#pragma unroll
            for (int t = 0; t < M5_TT; ++t)
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    float v[4];
#pragma unroll
                    for (int c = 0; c < 4; ++c) {
                        const float a = acc[0][t][4 * g + c] * ig[g][c], b = acc[1][t][4 * g + c] * iu[g][c];
                        v[c] = a * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(-a * 1.4426950408889634f)) * b;
                    }
                    if (!rows_full && rbase + 8 * g >= sg.M) continue;   // (M % 4 == 0: whole groups)
                    const uint32_t ot = 32u * t;
                    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u, v), rd, (int) (lo + (ot * (uint32_t) sg.d_col + 8u * g) * 4u), 0, 0);
                    if constexpr (decltype(with_h)::value) {
                        const h2 p0 = {(_Float16) v[0], (_Float16) v[1]}, p1 = {(_Float16) v[2], (_Float16) v[3]};
                        v2u hv = {__builtin_bit_cast(uint32_t, p0), __builtin_bit_cast(uint32_t, p1)};
                        __builtin_amdgcn_raw_buffer_store_b64(hv, rh, (int) (lh + (ot * (uint32_t) p.h_col + 8u * g) * 2u), 0, 0);
                    }
                }
        };
        if (p.h) store(std::true_type{});
        else store(std::false_type{});
        return;
    }
    const float inv0 = 1.0f / ws0, inv1 = 1.0f / ws1;
    if (row >= sg.M) return;
    // raw buffer stores: the lane's 32-bit byte offset (the host checks both outputs
    // < 4 GiB), no address arithmetic beyond one add per store, and the tokens past N
    // dropped by the descriptor's range (num_records = N rows of the output) instead of a
    // branch per store
    const uint32_t lo = ((uint32_t) (tok0 + 4 * h) * (uint32_t) sg.d_col + (uint32_t) row) * 4u;
    const uint32_t lh = ((uint32_t) (tok0 + 4 * h) * (uint32_t) p.h_col + (uint32_t) row) * 2u;
    const __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc(sg.dst, 0, (int) ((uint32_t) ntok * (uint32_t) sg.d_col * 4u), 0x00020000);
    auto store = [&](auto with_h) {
        const __amdgpu_buffer_rsrc_t rh = with_h ? __builtin_amdgcn_make_buffer_rsrc(p.h, 0, (int) ((uint32_t) ntok * (uint32_t) p.h_col * 2u), 0x00020000) : rd;
#pragma unroll
        for (int t = 0; t < M5_TT; ++t)
#pragma unroll
            for (int e = 0; e < 16; ++e) {
                const uint32_t tu = 32 * t + (e & 3) + 8 * (e >> 2);
                const float g = acc[0][t][e] * inv0, u = acc[1][t][e] * inv1;
                const float v = g * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(-g * 1.4426950408889634f)) * u;
                __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v), rd, (int) (lo + tu * (uint32_t) sg.d_col * 4u), 0, 0);
                if constexpr (decltype(with_h)::value) {
                    const _Float16 hv = (_Float16) v;
                    __builtin_amdgcn_raw_buffer_store_b16(__builtin_bit_cast(uint16_t, hv), rh, (int) (lh + tu * (uint32_t) p.h_col * 2u), 0, 0);
                }
            }
    };
    if (p.h) store(std::true_type{});
    else store(std::false_type{});
    if constexpr (X & 256) {
        const unsigned long long t_end = __builtin_amdgcn_s_memtime();
        if (trw && lane == 0) {
            unsigned long long * tr = p.trace + wave * 8;
            tr[0] = 1; tr[1] = 1 + t_loop - t_k0; tr[2] = 1 + t_wait; tr[3] = 1 + t_comp;
            tr[4] = 1 + t_end - t_loop - t_wait - t_comp; tr[5] = 1 + nc;
        }
    }
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
static bool m4_kq(int t) { return t == GGML_TYPE_Q4_K || t == GGML_TYPE_Q5_K || t == GGML_TYPE_Q6_K || t == GGML_TYPE_Q8_0; }

// g_tune[17]: 0 = v4 for every K-quant prefill GEMM it takes (round 3: with the pipelined
// loop and the cost-model split, also the q/k/v group and the K = 4096 projections),
// 5 = round 2's choice (v4 for the gate/up/SwiGLU pair and K >= 8192 only), 1 = v4 off,
// 3 = v4 everywhere, 2 / 4 = v4 everywhere at 64 / 128 tokens per tile
thread_local M4Split * g_m4_split = nullptr;

bool mmq4_on() { return g_tune[17] != 1 && getenv("GGML_MI355X_MMQ4_OFF") == nullptr; }
static bool m4_all() { return g_tune[17] != 5; }
static bool m4_plain_ok(int64_t K) { return m4_all() || K >= 8192; }

template <int QTA, int QTB, int TT, int EPI, int X = M4_XDEF>
static void m4_kernel_x(hipStream_t st, const M4Args & a, dim3 g) {
    constexpr int lds = m4_slots<X>() * 32 * TT * 256;
    MX_LDS_OPTIN((k_mmq4<QTA, QTB, TT, EPI, X>), lds);
    k_mmq4<QTA, QTB, TT, EPI, X><<<g, 64 * M4_WAVES, lds, st>>>(a);
}

template <int QTA, int QTB, int TT, int EPI>
static void m4_kernel(hipStream_t st, const M4Args & a, dim3 g) {
    // A/B: g_tune[3] = 2 the round-3 loop (one wait + barrier per chunk, four slots), 4 the
    // four-slot two-chunk stages
    if constexpr (QTA == QTB && TT == 4 && EPI < 2) {
        if (g_tune[3] == 2) return m4_kernel_x<QTA, QTB, TT, EPI, M4_XDEF & ~(32 | 64)>(st, a, g);
        if (g_tune[3] == 4) return m4_kernel_x<QTA, QTB, TT, EPI, (M4_XDEF & ~64) | 32>(st, a, g);
    }
    if constexpr (MX_AB_VARIANTS && QTA == QTB && TT == 4 && EPI < 2 && QTA != GGML_TYPE_Q5_K) {
        switch (g_tune[31]) {   // timing experiments (X bits above), the prefill GEMM shapes only
            case 1: return m4_kernel_x<QTA, QTB, TT, EPI, 1 | M4_XDEF>(st, a, g);
            case 2: return m4_kernel_x<QTA, QTB, TT, EPI, 2 | (M4_XDEF & 8)>(st, a, g);
            case 4: return m4_kernel_x<QTA, QTB, TT, EPI, 4 | (M4_XDEF & 8)>(st, a, g);   // (no pipelining)
            case 7: return m4_kernel_x<QTA, QTB, TT, EPI, 7 | (M4_XDEF & 8)>(st, a, g);
            case 32: return m4_kernel_x<QTA, QTB, TT, EPI, 0>(st, a, g);                  // round-2 form
            default: break;
        }
    }
    m4_kernel_x<QTA, QTB, TT, EPI>(st, a, g);
}

template <int EPI, int TT>
static bool m4_go(hipStream_t st, const M4Args & a, int ta, int tb, dim3 g) {
#define M4K(A, B) if (ta == A && tb == B) { m4_kernel<A, B, TT, EPI>(st, a, g); return true; }
    constexpr int Q4 = GGML_TYPE_Q4_K, Q5 = GGML_TYPE_Q5_K, Q6 = GGML_TYPE_Q6_K, Q8 = GGML_TYPE_Q8_0;
    if constexpr (EPI == 0) {
        M4K(Q4, Q4) M4K(Q4, Q6) M4K(Q6, Q4) M4K(Q5, Q5) M4K(Q5, Q6) M4K(Q6, Q5) M4K(Q6, Q6)
        M4K(Q4, Q8) M4K(Q5, Q8) M4K(Q6, Q8) M4K(Q8, Q8)    // round 5: Q8_0 (8-expert k/v, q8_0 models)
    } else {
        M4K(Q4, Q4) M4K(Q5, Q5) M4K(Q6, Q6) M4K(Q8, Q8)
    }
#undef M4K
    return false;
}

// tokens per tile: 128 (g_tune[18] = 2 forces 64)
static int m4_tt() {
    if (g_tune[17] == 2 || g_tune[17] == 4) return g_tune[17];
    if (g_tune[18] == 2 || g_tune[18] == 4) return g_tune[18];
    return 4;
}

// K shares: the k_mmq4 workgroup takes a whole CU (128 KB ring), so a grid of G
// workgroups runs in ceil(G / 256) rounds of ceil(nk / ks) chunks each (~2.7 us per chunk
// at 128 tokens, profiles/r03/ab_mmq4_x.txt); a split adds the k_mmq4_reduce pass (launch
// + (ks + 1) partial planes of N x M floats at ~5 TB/s). Pick the cheapest ks <= 8 with
// >= 4 chunks per share. g_tune[20] forces it.
static int m4_ksplit(int64_t wgs, int nk, int64_t n, int64_t m) {
    if (g_tune[20] > 0) return std::min(g_tune[20], nk);
    int best = 1;
    double bt = 1e30;
    for (int ks = 1; ks <= 8 && nk / ks >= 4; ++ks) {
        const double t = (double) mx_ceil_div(wgs * ks, 256) * (double) mx_ceil_div(nk, ks) * 2.7 +
                         (ks > 1 ? 2.0 + (double) (ks + 1) * (double) (n * m * 4) / 5e6 : 0.0);
        if (t < bt) { bt = t; best = ks; }
    }
    return best;
}

size_t mmq4_scratch(const ggml_tensor * dst, bool add_norm) {
    const ggml_tensor * w = dst->src[0], * x = dst->src[1];
    if (!m4_kq(w->type) || x->ne[1] <= 8) return 0;
    const int64_t rows = mx_ceil_div(w->ne[1] + w->ne[1] / 2, 256) * 256;   // room for a q/k/v group
    const int ks = m4_ksplit(mx_ceil_div(x->ne[1], 128) * mx_ceil_div(rows, 256), (int) (w->ne[0] / M4_KC), x->ne[1], rows);
    // + the product itself where an ADD -> RMS_NORM follows (add_norm, exec.cpp's sizing
    // pass): mm_add_rms_norm keeps an unsplit product in scratch when the ADD runs in place
    // over its residual, and must not squeeze the split-K planes out (only there)
    return (ks > 1 ? (size_t) ks * x->ne[1] * rows * 4 + 256 : 0) + (add_norm ? (size_t) w->ne[1] * x->ne[1] * 4 + 256 : 0);
}

template <int EPI>
static bool m4_dispatch(OpCtx & c, M4Args & a, int ta, int tb, int tiles_y, int nz, int tt) {
    a.dbg = MX_AB_VARIANTS ? g_tune[19] : 0;
    a.trace = mx_trace_slot(3);
    a.trace_blk = mx_trace_blocks();
    const int nk = a.K / M4_KC;
    const int64_t gx = mx_ceil_div(a.N, 32 * tt);
    a.ksplit = 1;
    if (EPI == 0) {
        int ks = m4_ksplit(gx * tiles_y, nk, a.N, (int64_t) tiles_y * 32 * M4_WAVES);
        const size_t need = (size_t) ks * a.N * tiles_y * 32 * M4_WAVES * 4;
        if (ks > 1 && c.scratch->avail() >= need + 256) {
            a.ksplit = ks;
            a.part_ld = tiles_y * 32 * M4_WAVES;
            a.part = (float *) c.scratch->take(need);
            nz = ks;
        }
    }
    const dim3 g = EPI >= 2 ? dim3((unsigned) tiles_y, (unsigned) gx, (unsigned) nz) : dim3((unsigned) gx, (unsigned) tiles_y, (unsigned) nz);
    const bool ok = tt == 4 ? m4_go<EPI, 4>(c.st, a, ta, tb, g) : m4_go<EPI, 2>(c.st, a, ta, tb, g);
    bool taken = false;
    if (ok && a.ksplit > 1 && g_m4_split && !a.h) {
        taken = true;
        for (int s = 0; s < a.nseg; ++s) taken = taken && a.seg[s].res == nullptr;
        if (taken) {
            g_m4_split->part = a.part; g_m4_split->part_ld = a.part_ld; g_m4_split->ks = a.ksplit;
            for (int s = 0; s < 3; ++s) g_m4_split->row0[s] = s < a.nseg ? a.seg[s].tile0 * 32 * M4_WAVES : 0;
        }
    }
    if (ok && a.ksplit > 1 && !taken) {
        const dim3 gr((unsigned) mx_ceil_div(a.part_ld, 256), (unsigned) a.N);
        k_mmq4_reduce<<<gr, 256, 0, c.st>>>(a);
    }
    MX_KLOG("mmq4 launch epi=%d ks=%d planes=%d tiles=%d gx=%lld", EPI, a.ksplit, (int) taken, tiles_y, (long long) gx);
    return ok;
}

static bool m4_weight_ok(const ggml_tensor * w, int64_t K) {
    return m4_kq(w->type) && w->ne[0] == K && K % 256 == 0 && w->ne[2] == 1 && w->ne[3] == 1 &&
           w->nb[0] == (size_t) mx_type(w->type).size && ((uintptr_t) w->data % 16) == 0 && w->nb[1] % 16 == 0;
}

// out = W·x (+ res): one K-quant weight, x already in the f16 act cache (xa, kp)
bool mmq4_mul_mat(OpCtx & c, const ggml_tensor * w, const ggml_tensor * x, const _Float16 * xa, int64_t kp,
                  ggml_tensor * out, const ggml_tensor * res) {
    if (!mmq4_on() || !m4_plain_ok(x->ne[0]) || !m4_weight_ok(w, x->ne[0]) || x->ne[2] * x->ne[3] != 1 || x->ne[1] > INT32_MAX) return false;
    if (out->nb[0] != 4 || out->nb[1] % 4 || (res && (res->nb[0] != 4 || res->nb[1] % 4))) return false;
    M4Args a{};
    a.nseg = 1;
    a.seg[0] = M4Seg{(const char *) w->data, w->nb[1], (float *) out->data, out->nb[1] / 4,
                     res ? (const float *) res->data : nullptr, res ? res->nb[1] / 4 : 0, (int) w->ne[1], 0, 0};
    a.x = xa; a.kp = kp; a.N = (int) x->ne[1]; a.K = (int) x->ne[0];
    const int tiles = (int) mx_ceil_div(w->ne[1], 32 * M4_WAVES), tt = m4_tt();
    MX_KLOG("mmq4 qt=%d tt=%d M=%lld N=%d K=%d res=%d", (int) w->type, tt, (long long) w->ne[1], a.N, a.K, res != nullptr);
    return m4_dispatch<0>(c, a, w->type, w->type, tiles, 1, tt);
}

// 2-3 MUL_MATs sharing x (q/k/v) in one launch; weights of at most two K-quant types
bool mmq4_group(OpCtx & c, ggml_tensor * const * mms, int n, const _Float16 * xa, int64_t kp) {
    if (!mmq4_on() || !m4_all() || n < 1 || n > M4_MAXSEG) return false;
    const ggml_tensor * x = mms[0]->src[1];
    const int ta = mms[0]->src[0]->type;
    int tb = ta;
    M4Args a{};
    a.nseg = n;
    int tiles = 0;
    for (int k = 0; k < n; ++k) {
        const ggml_tensor * m = mms[k], * w = m->src[0];
        if (m->src[1] != x || !m4_weight_ok(w, x->ne[0]) || m->nb[0] != 4 || m->nb[1] % 4) return false;
        if (w->type != ta) { if (tb != ta && tb != w->type) return false; tb = w->type; }
        a.seg[k] = M4Seg{(const char *) w->data, w->nb[1], (float *) m->data, m->nb[1] / 4, nullptr, 0, (int) w->ne[1],
                         w->type != ta, tiles};
        tiles += (int) mx_ceil_div(w->ne[1], 32 * M4_WAVES);
    }
    a.x = xa; a.kp = kp; a.N = (int) x->ne[1]; a.K = (int) x->ne[0];
    const int tt = m4_tt();
    MX_KLOG("mmq4 group n=%d qta=%d qtb=%d tt=%d N=%d K=%d", n, ta, tb, tt, a.N, a.K);
    return m4_dispatch<0>(c, a, ta, tb, tiles, 1, tt);
}

template <int QT, int X>
static void m5_launch(hipStream_t st, const M4Args & a, dim3 g) {
    MX_LDS_OPTIN((k_mmq5_glu<QT, X>), M5_LDS);
    k_mmq5_glu<QT, X><<<g, 64 * M5_WAVES, M5_LDS, st>>>(a);
}

// silu(Wg·x) * (Wu·x) into glu (+ its f16 copy h for the down projection)
bool mmq4_glu_ok(const ggml_tensor * wg, const ggml_tensor * wu, const ggml_tensor * x, const ggml_tensor * glu) {
    if (!mmq4_on() || !m4_weight_ok(wg, x->ne[0]) || !m4_weight_ok(wu, x->ne[0]) || wg->type != wu->type) return false;
    return wg->nb[1] == wu->nb[1] && wg->ne[1] == wu->ne[1] && glu->nb[0] == 4 && glu->nb[1] % 4 == 0;
}

void mmq4_glu(OpCtx & c, const ggml_tensor * wg, const ggml_tensor * wu, const ggml_tensor * x, const _Float16 * xa,
              int64_t kp, ggml_tensor * glu, _Float16 * h, int64_t h_col) {
    M4Args a{};
    a.nseg = 1;
    a.seg[0] = M4Seg{(const char *) wg->data, wg->nb[1], (float *) glu->data, glu->nb[1] / 4, nullptr, 0, (int) wg->ne[1], 0, 0};
    a.w2 = (const char *) wu->data;
    a.x = xa; a.kp = kp; a.N = (int) x->ne[1]; a.K = (int) x->ne[0];
    a.h = h; a.h_col = h_col;
    const int tiles = (int) mx_ceil_div(wg->ne[1], 16 * M4_WAVES), tt = m4_tt();
    MX_KLOG("mmq4 glu qt=%d tt=%d M=%lld N=%d K=%d", (int) wg->type, tt, (long long) wg->ne[1], a.N, a.K);
    // k_mmq5 (256-token tiles) from 256 tokens on; g_tune[3] = 8 keeps k_mmq4
    if (a.N >= M5_BT && g_tune[3] != 8 && wg->type == GGML_TYPE_Q4_K &&
        (size_t) a.N * a.kp * 2 < (1ull << 32) && (size_t) wg->ne[1] * wg->nb[1] < (1ull << 32) &&
        (size_t) a.N * glu->nb[1] < (1ull << 32) && (size_t) a.N * (size_t) h_col * 2 < (1ull << 32)) {
        const int R = (int) mx_ceil_div(wg->ne[1], 128), T = (int) mx_ceil_div(a.N, M5_BT);
        a.ksplit = 1;
        const dim3 g((unsigned) (R * T));
        // 16-byte row-vector stores: rows in whole groups of four, 16- / 8-byte aligned
        const bool vec_ok = wg->ne[1] % 4 == 0 && (a.seg[0].d_col % 4) == 0 && ((uintptr_t) glu->data % 16) == 0 &&
                            (!h || (h_col % 4 == 0 && (uintptr_t) h % 8 == 0));
        if constexpr (MX_AB_VARIANTS) {
            // timing experiments (results wrong): g_tune[31] 1 no wait + barrier, 2 no
            // dequantisation; g_tune[19] 4 no activation DMA, 8 weights of chunk 0 only
            a.dbg = g_tune[19];
            a.trace = mx_trace_slot(3);
            if (a.trace && g_tune[3] == 32 && vec_ok) { m5_launch<GGML_TYPE_Q4_K, M5_XDEF | 256 | 512>(c.st, a, g); goto m5_done; }
            if (a.trace) { m5_launch<GGML_TYPE_Q4_K, M5_XDEF | 256>(c.st, a, g); goto m5_done; }
            switch (g_tune[31]) {
                case 1: m5_launch<GGML_TYPE_Q4_K, M5_XDEF | 1>(c.st, a, g); break;
                case 2: m5_launch<GGML_TYPE_Q4_K, M5_XDEF | 2>(c.st, a, g); break;
                case 3: m5_launch<GGML_TYPE_Q4_K, M5_XDEF | 3>(c.st, a, g); break;
                default: m5_launch<GGML_TYPE_Q4_K, M5_XDEF>(c.st, a, g);
            }
        } else if (g_tune[3] == 16) {   // A/B: the next chunks' loads interleaved with the MFMAs
            m5_launch<GGML_TYPE_Q4_K, M5_XDEF | 128>(c.st, a, g);
        } else if (g_tune[3] == 32 && vec_ok) {   // A/B: weights as the A operand, 16-byte stores
            m5_launch<GGML_TYPE_Q4_K, M5_XDEF | 512>(c.st, a, g);
        } else {
            m5_launch<GGML_TYPE_Q4_K, M5_XDEF>(c.st, a, g);
        }
    m5_done:
        MX_KLOG("mmq4 launch epi=1 ks=1 planes=0 tiles=%d gx=%d wide=1", R, T);
        return;
    }
    MX_ASSERT(m4_dispatch<1>(c, a, wg->type, wg->type, tiles, 1, tt));
}


// ---------------------------------------------------------------------------
// MUL_MAT_ID (MoE) prefill: expert-grouped GEMM. The (token, slot) items are sorted by
// expert on the device (no host sync, graph-capturable — reference: mm_ids_helper,
// ggml-cuda/mmid.cu:28-160, and mul_mat_id's per-expert mmq, mmq.cu:160-217); each
// expert's items then run as k_mmq4 tiles (grid.z = expert), the activation rows gathered
// and the outputs scattered through the sorted lists.
// ---------------------------------------------------------------------------
constexpr int M4_MAXEXP = 1024;

__global__ __launch_bounds__(1024) void k_moe_sort(const char * ids, size_t id0, size_t id1, int n_used, int n_tok,
                                                  int n_expert, int ne11, int32_t * gather, int32_t * scatter,
                                                  int32_t * tile_tab) {
    __shared__ int cnt[M4_MAXEXP], cur[M4_MAXEXP];
    const int tid = threadIdx.x, n = n_used * n_tok;
    for (int e = tid; e < n_expert; e += blockDim.x) cnt[e] = 0;
    __syncthreads();
    for (int i = tid; i < n; i += blockDim.x) {
        const int t = i / n_used, sl = i % n_used;
        const int ex = *(const int32_t *) (ids + (size_t) sl * id0 + (size_t) t * id1);
        if (ex >= 0 && ex < n_expert) atomicAdd(&cnt[ex], 1);
    }
    __syncthreads();
    if (tid == 0) {
        int acc = 0;
        for (int e = 0; e < n_expert; ++e) {
            tile_tab[2 * e] = acc;
            tile_tab[2 * e + 1] = cnt[e];
            cur[e] = acc;
            acc += cnt[e];
        }
    }
    __syncthreads();
    // positions inside an expert's list depend on arrival order; each item's result does not
    for (int i = tid; i < n; i += blockDim.x) {
        const int t = i / n_used, sl = i % n_used;
        const int ex = *(const int32_t *) (ids + (size_t) sl * id0 + (size_t) t * id1);
        if (ex < 0 || ex >= n_expert) continue;
        const int pos = atomicAdd(&cur[ex], 1);
        gather[pos] = t * ne11 + sl % ne11;     // activation column of b [K, ne11, n_tok]
        scatter[pos] = t * n_used + sl;         // output column of dst [M, n_used, n_tok]
    }
}

static bool m4_moe_ok(const ggml_tensor * dst) {
    const ggml_tensor * as = dst->src[0], * b = dst->src[1], * ids = dst->src[2];
    if (!mmq4_on() || !m4_kq(as->type) || as->ne[0] % 256 || as->ne[3] != 1 || as->ne[2] > M4_MAXEXP) return false;
    if (as->nb[0] != (size_t) mx_type(as->type).size || ((uintptr_t) as->data % 16) || as->nb[1] % 16 || as->nb[2] % 16) return false;
    if (b->type != GGML_TYPE_F32 || b->ne[0] != as->ne[0] || b->ne[3] != 1 || b->nb[0] != 4) return false;
    if (ids->type != GGML_TYPE_I32 || dst->type != GGML_TYPE_F32 || dst->nb[0] != 4) return false;
    if (dst->nb[2] != dst->nb[1] * dst->ne[1] || dst->nb[1] % 4) return false;     // [M, n_used, n_tok] rows
    const int64_t items = ids->ne[0] * ids->ne[1];
    return items >= 32 && ids->ne[1] == b->ne[2] && dst->ne[1] == ids->ne[0];
}

size_t mmq4_moe_scratch(const ggml_tensor * dst) {
    if (!m4_moe_ok(dst)) return 0;
    const ggml_tensor * b = dst->src[1], * ids = dst->src[2];
    const size_t items = ids->ne[0] * ids->ne[1];
    return (size_t) b->ne[1] * b->ne[2] * b->ne[0] * 2 + 2 * items * 4 + 2 * M4_MAXEXP * 4 + 1024;
}

bool mmq4_moe(OpCtx & c, ggml_tensor * dst) {
    if (!m4_moe_ok(dst)) return false;
    const ggml_tensor * as = dst->src[0], * b = dst->src[1], * ids = dst->src[2];
    const int n_used = (int) ids->ne[0], n_tok = (int) ids->ne[1], n_exp = (int) as->ne[2];
    const int items = n_used * n_tok;
    int32_t * gather = (int32_t *) c.scratch->take((size_t) items * 4);
    int32_t * scatter = (int32_t *) c.scratch->take((size_t) items * 4);
    int32_t * tab = (int32_t *) c.scratch->take((size_t) 2 * M4_MAXEXP * 4);
    k_moe_sort<<<1, 1024, 0, c.st>>>((const char *) ids->data, ids->nb[0], ids->nb[1], n_used, n_tok, n_exp,
                                     (int) b->ne[1], gather, scatter, tab);
    const int64_t kp = as->ne[0];
    const _Float16 * xa = mmq_act_f16(c, b, kp);
    M4Args a{};
    a.nseg = 1;
    a.seg[0] = M4Seg{(const char *) as->data, as->nb[1], (float *) dst->data, dst->nb[1] / 4, nullptr, 0, (int) as->ne[1], 0, 0};
    a.x = xa; a.kp = kp; a.N = items; a.K = (int) as->ne[0];
    a.gather = gather; a.scatter = scatter; a.tile_tab = tab; a.w_exp = as->nb[2];
    const int tt = m4_tt(), tiles = (int) mx_ceil_div(as->ne[1], 32 * M4_WAVES);
    MX_KLOG("mmq4 moe qt=%d tt=%d M=%lld items=%d experts=%d K=%d", (int) as->type, tt, (long long) as->ne[1], items, n_exp, a.K);
    // grid.x covers the worst case (every item on one expert); the tiles past an expert's
    // count exit at once
    MX_ASSERT(m4_dispatch<2>(c, a, as->type, as->type, tiles, n_exp, tt));
    return true;
}

// Round 5: MUL_MAT_ID(gate) , MUL_MAT_ID(up) , GLU(swiglu) of a prefill ubatch in ONE k_mmq4
// launch (EPI 3): one expert sort, each expert's token tile multiplied by its gate rows
// (waves 0-3) and up rows (waves 4-7) over the same activation tile, silu(g) * u written
// to the GLU output and its f16 copy for the down projection's GEMM (claimed in the
// activation cache, as the dense SwiGLU does). Before: two EPI 2 launches (each gathering
// the activations) + a GLU pass + an f16 conversion pass.
bool mmq4_moe_glu(OpCtx & c, const ggml_tensor * gate, const ggml_tensor * up, ggml_tensor * glu) {
    if (!m4_moe_ok(gate) || !m4_moe_ok(up)) return false;
    const ggml_tensor * wg = gate->src[0], * wu = up->src[0], * b = gate->src[1], * ids = gate->src[2];
    if (up->src[1] != b || up->src[2] != ids || wg->type != wu->type) return false;
    for (int i = 0; i < 4; ++i) if (wg->ne[i] != wu->ne[i] || wg->nb[i] != wu->nb[i]) return false;
    if (!mx_are_same_shape(glu, gate) || glu->type != GGML_TYPE_F32 || glu->nb[0] != 4 || glu->nb[1] != gate->nb[1] ||
        glu->nb[2] != gate->nb[2]) return false;
    const int n_used = (int) ids->ne[0], n_tok = (int) ids->ne[1], n_exp = (int) wg->ne[2];
    const int items = n_used * n_tok;
    int32_t * gather = (int32_t *) c.scratch->take((size_t) items * 4);
    int32_t * scatter = (int32_t *) c.scratch->take((size_t) items * 4);
    int32_t * tab = (int32_t *) c.scratch->take((size_t) 2 * M4_MAXEXP * 4);
    k_moe_sort<<<1, 1024, 0, c.st>>>((const char *) ids->data, ids->nb[0], ids->nb[1], n_used, n_tok, n_exp,
                                     (int) b->ne[1], gather, scatter, tab);
    const int64_t kp = wg->ne[0];
    const _Float16 * xa = mmq_act_f16(c, b, kp);
    M4Args a{};
    a.nseg = 1;
    a.seg[0] = M4Seg{(const char *) wg->data, wg->nb[1], (float *) glu->data, glu->nb[1] / 4, nullptr, 0, (int) wg->ne[1], 0, 0};
    a.w2 = (const char *) wu->data;
    a.x = xa; a.kp = kp; a.N = items; a.K = (int) wg->ne[0];
    a.gather = gather; a.scatter = scatter; a.tile_tab = tab; a.w_exp = wg->nb[2];
    // the down projection's f16 input, rows of glu->nb[1] bytes = one (slot, token) column each
    a.h = mmq_act_claim(c, glu->data, glu->ne[0], (int64_t) glu->ne[1] * glu->ne[2], glu->nb[1]);
    a.h_col = glu->ne[0];
    const int tt = m4_tt(), tiles = (int) mx_ceil_div(wg->ne[1], 16 * M4_WAVES);
    MX_KLOG("mmq4 moe_glu qt=%d tt=%d M=%lld items=%d experts=%d K=%d h=%d", (int) wg->type, tt, (long long) wg->ne[1], items, n_exp,
            a.K, a.h != nullptr);
    return m4_dispatch<3>(c, a, wg->type, wg->type, tiles, n_exp, tt);
}

}  // namespace mx
