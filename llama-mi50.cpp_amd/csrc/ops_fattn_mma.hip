// ops_fattn_mma.hip — FLASH_ATTN_EXT for prefill (many query rows) on CDNA4 matrix cores.
//
// Semantics as ops_fattn.hip (ggml-cpu/ops.cpp:8045-8260: q rounded to f16, masked keys
// skipped, online softmax); the reference GPU path is fattn-mma / fattn-tile
// (fattn.cu:280-482). Scope: f16 K/V, D in {64, 128}, no softcap / ALiBi / sinks (those
// keep the tile kernel).
//
// MI355X design: one workgroup = 64 query rows of one head, 2 waves x 32 rows. Per tile
// of 64 keys the workgroup stages K [key][d] and V^T [d][key] (f16) and the mask tile in
// LDS; each wave computes S = Q K^T with v_mfma_f32_32x32x16_f16 (Q fragments stay in
// registers for the whole key loop), writes S to LDS, runs the online softmax with two
// lanes per query row, writes P (f16) back, rescales O and accumulates O += P V with
// the same MFMA. Key tiles the mask removes entirely (the causal upper triangle) are
// skipped.
#include "backend.h"
#include "gemv.h"

namespace mx {

typedef _Float16 fhalf8 __attribute__((ext_vector_type(8)));
typedef float ffloat16v __attribute__((ext_vector_type(16)));

struct FaMmaArgs {
    const char * q; size_t q1, q2;        // f32 [D, n_q, H]
    const char * k; size_t k1, k2;        // f16 [D, n_kv, Hkv]
    const char * v; size_t v1, v2;
    const char * mask; size_t m1;         // f16 [n_kv, n_q] or null
    char * dst; size_t d1, d2;            // f32 [D, H, n_q]
    _Float16 * h;                         // k_fa_mma2: also f16 [n_q][H * D] (act cache) or null
    int n_q, n_kv, H, Hkv;
    float scale;
    int qround;                           // q in K's vec-dot type before f16 (fa_q_round): 0 f16, 1 q8_0, 2 bf16
};

// Round 6: q as the CPU backend rounds it for the K cache's vec-dot type
// (type_traits_cpu[k->type].vec_dot_type, ggml-cpu/ops.cpp:8045-8130): q8_0 blocks for q8_0 /
// q4_0 caches (d = amax/127 as f16, q = round(x/d): the value d·q, then f16), bf16 for bf16.
// x[s][0..7] = dims 16 s + 8 hl .. + 7 of the lane's query; a 32-dim block is steps 2b, 2b+1
// of this lane and of its partner lane^32 (the other hl).
template <int NKS>
__device__ __forceinline__ void fa_q_round(float (&x)[NKS][8], int mode) {
    if (mode == 1) {
#pragma unroll
        for (int b = 0; b < NKS / 2; ++b) {
            float m = 0.f;
#pragma unroll
            for (int j = 0; j < 8; ++j) m = fmaxf(m, fmaxf(fabsf(x[2 * b][j]), fabsf(x[2 * b + 1][j])));
            m = fmaxf(m, __shfl_xor(m, 32, 64));
            const float d = m / 127.0f, id = d != 0.0f ? 1.0f / d : 0.0f;
            const float dh = (float) (_Float16) d;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                x[2 * b][j] = dh * roundf(x[2 * b][j] * id);
                x[2 * b + 1][j] = dh * roundf(x[2 * b + 1][j] * id);
            }
        }
    } else if (mode == 2) {
#pragma unroll
        for (int s = 0; s < NKS; ++s)
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                uint32_t u = __float_as_uint(x[s][j]);
                u = (u + 0x7fff + ((u >> 16) & 1)) & 0xffff0000u;
                x[s][j] = __uint_as_float(u);
            }
    }
}

static const bool g_fa_mma1 = getenv("GGML_MI355X_FA_MMA1") != nullptr;   // A/B: the first kernel

constexpr int FM_QT = 64;    // query rows per workgroup
constexpr int FM_KT = 64;    // keys per tile

template <int D>
__device__ __forceinline__ int kswz(int row, int chunk) {   // K tile: D/8 16-byte chunks per row
    constexpr int C = D / 8;
    return row * C + (chunk ^ (row & (C - 1)));
}
__device__ __forceinline__ int vswz(int row, int chunk) {   // V^T tile: 8 chunks (64 keys) per row
    return row * 8 + (chunk ^ (row & 7));
}

template <int D>
__global__ __launch_bounds__(128, 2) void k_fa_mma(FaMmaArgs p) {
    constexpr int C = D / 8;                 // 16-byte chunks per K row
    constexpr int NKS = D / 16;              // MFMA k-steps over the head dim
    constexpr int NDT = D / 32;              // 32-wide output tiles over the head dim
    __shared__ uint4 ks[FM_KT * C];
    __shared__ uint4 vts[D * 8];
    __shared__ uint16_t mk[FM_QT][FM_KT];
    __shared__ float sbuf[2][32][FM_KT + 1];
    __shared__ __align__(16) _Float16 pbuf[2][32][FM_KT];
    __shared__ float arow[2][32], lrow[2][32];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int h = blockIdx.y, hk = h / (p.H / p.Hkv);
    const int q0 = blockIdx.x * FM_QT;
    const int qw = q0 + 32 * wave;           // this wave's first query row
    const int r32 = lane & 31, hsel = lane >> 5;
    const char * kb = p.k + (size_t) hk * p.k2;
    const char * vb = p.v + (size_t) hk * p.v2;

    // Q fragments (A operand: row = query r32, k = 8 dims at 8*hsel within each 16-dim step)
    fhalf8 qa[NKS];
    {
        const int qr = min(qw + r32, p.n_q - 1);
        const float * qp = (const float *) (p.q + (size_t) qr * p.q1 + (size_t) h * p.q2);
        float x[NKS][8];
#pragma unroll
        for (int s = 0; s < NKS; ++s) {
            const float4 f0 = *(const float4 *) (qp + 16 * s + 8 * hsel);
            const float4 f1 = *(const float4 *) (qp + 16 * s + 8 * hsel + 4);
            x[s][0] = f0.x; x[s][1] = f0.y; x[s][2] = f0.z; x[s][3] = f0.w; x[s][4] = f1.x; x[s][5] = f1.y; x[s][6] = f1.z; x[s][7] = f1.w;
        }
        if (p.qround) fa_q_round<NKS>(x, p.qround);
#pragma unroll
        for (int s = 0; s < NKS; ++s)
#pragma unroll
            for (int j = 0; j < 8; ++j) qa[s][j] = (_Float16) x[s][j];
    }
    ffloat16v acc_o[NDT];
#pragma unroll
    for (int t = 0; t < NDT; ++t)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc_o[t][e] = 0.f;
    // softmax state: lane pair (2*row, 2*row+1) owns query row `lane >> 1` of this wave
    float m_run = -INFINITY, l_run = 0.f;
    const int srow = lane >> 1, shalf = lane & 1;

    const int n_tiles = (p.n_kv + FM_KT - 1) / FM_KT;
    for (int kt = 0; kt < n_tiles; ++kt) {
        const int key0 = kt * FM_KT;
        // ---- stage the mask tile, K tile and V^T tile
        int live = 0;
#pragma unroll
        for (int j = 0; j < FM_QT * FM_KT / 8 / 128; ++j) {          // 16-byte mask chunks
            const int u = tid + 128 * j;
            const int qr = u >> 3, c8 = u & 7;
            const int qg = q0 + qr, kg = key0 + 8 * c8;
            uint4 mv;
            if (p.mask && qg < p.n_q && kg + 8 <= p.n_kv) {
                mv = *(const uint4 *) (p.mask + (size_t) qg * p.m1 + (size_t) kg * 2);
            } else {
                uint16_t tmp[8];
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    const bool in = qg < p.n_q && kg + i < p.n_kv;
                    tmp[i] = !in ? (uint16_t) 0xFC00 : (p.mask ? ((const uint16_t *) (p.mask + (size_t) qg * p.m1))[kg + i] : (uint16_t) 0);
                }
                mv = *(uint4 *) tmp;
            }
            *(uint4 *) &mk[qr][8 * c8] = mv;
            // a tile is live if any entry is not -inf (0xFC00)
            const uint32_t w4[4] = {mv.x, mv.y, mv.z, mv.w};
#pragma unroll
            for (int i = 0; i < 4; ++i) live |= ((w4[i] & 0xFFFF) != 0xFC00) | ((w4[i] >> 16) != 0xFC00);
        }
        if (!__syncthreads_or(live)) continue;   // the whole tile is masked out for these rows
#pragma unroll
        for (int j = 0; j < FM_KT * C / 128; ++j) {
            const int u = tid + 128 * j;
            const int kr = u / C, c = u % C;
            const int kg = min(key0 + kr, p.n_kv - 1);
            ks[kswz<D>(kr, c)] = *(const uint4 *) (kb + (size_t) kg * p.k1 + 16 * c);
            const uint4 vv = *(const uint4 *) (vb + (size_t) kg * p.v1 + 16 * c);
            const uint16_t * vh = (const uint16_t *) &vv;
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const int d = 8 * c + i;
                ((uint16_t *) &vts[vswz(d, kr >> 3)])[kr & 7] = vh[i];
            }
        }
        __syncthreads();
        // ---- S = Q K^T for this wave's 32 rows x 64 keys
        ffloat16v acc_s[2];
#pragma unroll
        for (int n = 0; n < 2; ++n)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc_s[n][e] = 0.f;
#pragma unroll
        for (int s = 0; s < NKS; ++s) {
#pragma unroll
            for (int n = 0; n < 2; ++n) {
                const uint4 kv = ks[kswz<D>(32 * n + r32, 2 * s + hsel)];
                acc_s[n] = __builtin_amdgcn_mfma_f32_32x32x16_f16(qa[s], *(const fhalf8 *) &kv, acc_s[n], 0, 0, 0);
            }
        }
        // scale + mask -> LDS (C layout: row = (e&3) + 8(e>>2) + 4 hsel, col = key r32)
#pragma unroll
        for (int n = 0; n < 2; ++n)
#pragma unroll
            for (int e = 0; e < 16; ++e) {
                const int row = (e & 3) + 8 * (e >> 2) + 4 * hsel;
                const int col = 32 * n + r32;
                const float mval = h2f(mk[32 * wave + row][col]);
                sbuf[wave][row][col] = mval == -INFINITY ? -INFINITY : acc_s[n][e] * p.scale + mval;
            }
        __syncthreads();
        // ---- online softmax: two lanes per row, 32 keys each
        {
            float sv[32];
            float mt = -INFINITY;
#pragma unroll
            for (int i = 0; i < 32; ++i) { sv[i] = sbuf[wave][srow][32 * shalf + i]; mt = fmaxf(mt, sv[i]); }
            mt = fmaxf(mt, dpp_f<0xB1>(-INFINITY, mt));
            const float m_new = fmaxf(m_run, mt);
            const float alpha = m_run == m_new ? 1.0f : expf(m_run - m_new);
            float lt = 0.f;
#pragma unroll
            for (int i = 0; i < 32; i += 8) {
                fhalf8 ph;
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const float pv = m_new == -INFINITY ? 0.f : expf(sv[i + j] - m_new);
                    lt += pv;
                    ph[j] = (_Float16) pv;
                }
                *(fhalf8 *) &pbuf[wave][srow][32 * shalf + i] = ph;
            }
            lt += dpp_f<0xB1>(0.f, lt);
            l_run = l_run * alpha + lt;
            m_run = m_new;
            if (shalf == 0) arow[wave][srow] = alpha;
        }
        __syncthreads();
        // ---- O = O * alpha + P V
#pragma unroll
        for (int e = 0; e < 16; ++e) {
            const float al = arow[wave][(e & 3) + 8 * (e >> 2) + 4 * hsel];
#pragma unroll
            for (int t = 0; t < NDT; ++t) acc_o[t][e] *= al;
        }
#pragma unroll
        for (int s = 0; s < FM_KT / 16; ++s) {
            const fhalf8 pa = *(const fhalf8 *) &pbuf[wave][r32][16 * s + 8 * hsel];
#pragma unroll
            for (int t = 0; t < NDT; ++t) {
                const uint4 vv = vts[vswz(32 * t + r32, 2 * s + hsel)];
                acc_o[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(pa, *(const fhalf8 *) &vv, acc_o[t], 0, 0, 0);
            }
        }
        __syncthreads();   // K/V/mask/P buffers are rewritten by the next tile
    }
    // ---- normalise and store
    if (shalf == 0) lrow[wave][srow] = l_run;
    __syncthreads();
#pragma unroll
    for (int e = 0; e < 16; ++e) {
        const int row = (e & 3) + 8 * (e >> 2) + 4 * hsel;
        const int qg = qw + row;
        if (qg >= p.n_q) continue;
        const float l = lrow[wave][row];
        const float inv = l == 0.f ? 0.f : 1.0f / l;
        float * out = (float *) (p.dst + (size_t) h * p.d1 + (size_t) qg * p.d2);
#pragma unroll
        for (int t = 0; t < NDT; ++t) out[32 * t + r32] = acc_o[t][e] * inv;
    }
}

// ---------------------------------------------------------------------------------------
// v2 (D = 128): the first kernel spent ~11 µs per 64-key tile (profiles/r01: 90 µs per
// layer at pp512) on a 16-way bank-conflicted V transpose in LDS, S and P round trips
// through LDS and un-overlapped tile loads. v2:
//  * S^T = K·Q^T (A = K rows from LDS, B = the wave's Q fragments in registers): a lane
//    holds 32 of the 64 scores of ITS query (lane & 31), the other 32 in lane ^ 32 —
//    the softmax max is one cross-half shuffle, no LDS;
//  * O^T = V^T·P^T: B = P^T straight from those registers (the MFMA k index is mapped to
//    the keys the lane already holds; V's rows follow the same map), A = V^T read from the
//    plain row-major V tile with ds_read_b64_tr_b16 (gfx950 transposing LDS read) — no
//    transposed staging; O^T's columns are queries, so the rescale by alpha is lane-local;
//  * K and V tiles in one swizzled [key][128 x f16] image each (256-B rows, chunk XOR
//    ((row&3)<<2 | (row>>2)&3): conflict-free for both the b128 row reads and the
//    transposed reads); the next live tile's K/V and the mask two tiles ahead are in
//    flight while the current tile computes; tiles the mask removes are not loaded;
//  * 4 waves = the HG query heads of a GQA group that share the K/V tile x 32 queries
//    (HG = 4: K/V staged once for four heads).
typedef _Float16 fhalf4 __attribute__((ext_vector_type(4)));
typedef __fp16 fp16x4_t __attribute__((vector_size(8)));
typedef __attribute__((address_space(3))) fp16x4_t * lds_h4_t;
__device__ __forceinline__ fhalf4 lds_tr16(const char * a) {   // ds_read_b64_tr_b16
    return __builtin_bit_cast(fhalf4, __builtin_amdgcn_ds_read_tr16_b64_v4f16((lds_h4_t) a));
}

__device__ __forceinline__ int fm2_off(int row, int ch) {     // byte offset in a 256-B-row tile
    return 256 * row + 16 * (ch ^ (((row & 3) << 2) | ((row >> 2) & 3)));
}
// V^T tile (VT: the non-flash-attention path's transposed V cache, src/llama-kv-cache.cpp
// cpy_v with v_trans): 128 dimension rows x 64 keys (128 B), 8-byte chunks of 4 keys
// XOR-swizzled by (row >> 1) & 15, so the 32 rows one half-wave reads with ds_read_b64 at
// one key chunk fall on 32 distinct bank pairs
__device__ __forceinline__ int vt_off(int row, int q) { return 128 * row + 8 * (q ^ ((row >> 1) & 15)); }

// KS (key split, round 4): the four waves are 2 heads x 2 key halves of 32 queries — waves
// 0-1 take the even 64-key tiles, 2-3 the odd ones (two tiles staged per iteration), and
// the halves' (O, m, l) are merged through LDS at the end. At pp512 the HG = 4 grid was
// n_q / 32 x Hkv = 128 workgroups of 4 waves = 512 waves for 1,024 SIMDs, and the causal
// last query block walked all 8 tiles alone; split, 256 workgroups, 4 tiles at most per wave.
template <int HG, bool VT = false, bool KS = false>
__global__ __launch_bounds__(256) void k_fa_mma2(FaMmaArgs p) {
    constexpr int D = 128, NKS = D / 16, NDT = D / 32;
    static_assert(!KS || HG == 2, "key split: 2 heads x 2 key halves");
    constexpr int QB = KS ? 32 : 32 * (4 / HG);                // queries per workgroup
    constexpr int NB = KS ? 2 : 1;                             // K/V tiles staged per iteration
    __shared__ __align__(16) char ks[NB * FM_KT * 256];
    __shared__ __align__(16) char vs[NB * FM_KT * 256];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int l32 = lane & 31, hl = lane >> 5;
    const int Gt = p.H / p.Hkv, NGB = Gt / HG;
    const int hk = blockIdx.y / NGB;
    const int h = hk * Gt + (blockIdx.y % NGB) * HG + wave % HG;
    const int khalf = KS ? wave >> 1 : 0;                       // KS: this wave's tile parity
    const int qw = blockIdx.x * QB + (KS ? 0 : 32 * (wave / HG));   // this wave's first query
    const int qr = min(qw + l32, p.n_q - 1);                   // this lane's query (clamped)
    const char * kb = p.k + (size_t) hk * p.k2;
    const char * vb = p.v + (size_t) hk * p.v2;
    const uint16_t * mrow = p.mask ? (const uint16_t *) (p.mask + (size_t) qr * p.m1) : nullptr;

    // Q fragments, B operand of S^T: column = query l32, k = 8 dims at 16 s + 8 hl
    fhalf8 qa[NKS];
    {
        const float * qp = (const float *) (p.q + (size_t) qr * p.q1 + (size_t) h * p.q2);
        float x[NKS][8];
#pragma unroll
        for (int s = 0; s < NKS; ++s) {
            const float4 f0 = *(const float4 *) (qp + 16 * s + 8 * hl);
            const float4 f1 = *(const float4 *) (qp + 16 * s + 8 * hl + 4);
            x[s][0] = f0.x; x[s][1] = f0.y; x[s][2] = f0.z; x[s][3] = f0.w; x[s][4] = f1.x; x[s][5] = f1.y; x[s][6] = f1.z; x[s][7] = f1.w;
        }
        if (!VT && p.qround) fa_q_round<NKS>(x, p.qround);
#pragma unroll
        for (int s = 0; s < NKS; ++s)
#pragma unroll
            for (int j = 0; j < 8; ++j) qa[s][j] = (_Float16) x[s][j];
    }
    // the lane's 32 keys of a tile: 32 n + 8 m + 4 hl + (0..3), n < 2, m < 4 (S^T's C layout).
    // load_mask only issues (8-byte loads at clamped keys, unconditional: a load under a
    // branch makes the join wait for every load in flight, the K/V prefetch included);
    // fix_mask, one iteration later, shifts clamped groups into place and sets keys past
    // n_kv (and a missing mask) to -inf / 0
    const uint16_t * mp = mrow ? mrow : (const uint16_t *) p.k;
    auto load_mask = [&](int kt, uint2 (&mk)[8]) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int base = kt * FM_KT + 32 * (i >> 2) + 8 * (i & 3) + 4 * hl;
            mk[i] = *(const uint2 *) (mp + min(base, p.n_kv - 4));
        }
    };
    auto fix_mask = [&](int kt, uint2 (&mk)[8]) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int base = kt * FM_KT + 32 * (i >> 2) + 8 * (i & 3) + 4 * hl;
            const int sh = base - min(base, p.n_kv - 4);
            uint64_t v = mrow ? ((uint64_t) mk[i].y << 32 | mk[i].x) : 0;
            v = sh >= 4 ? 0 : v >> (16 * sh);
#pragma unroll
            for (int j = 0; j < 4; ++j)
                if (base + j >= p.n_kv) v = (v & ~(0xFFFFull << (16 * j))) | (0xFC00ull << (16 * j));
            mk[i] = make_uint2((uint32_t) v, (uint32_t) (v >> 32));
        }
    };
    auto any_live = [](const uint2 (&mk)[8]) {
        int live = 0;
#pragma unroll
        for (int i = 0; i < 8; ++i)
            live |= ((mk[i].x & 0xFFFF) != 0xFC00) | ((mk[i].x >> 16) != 0xFC00) | ((mk[i].y & 0xFFFF) != 0xFC00) | ((mk[i].y >> 16) != 0xFC00);
        return live;
    };
    // K/V tile rows, 16 B per thread per instruction: 16 threads read one 256-B row
    // (unconditional: a load under a branch would make the loop-carried registers a
    // scratch array; a dead tile reads one 16-B chunk for the whole workgroup instead).
    // VT: V^T rows (one per dimension, 64 keys = 128 B, p.v1 = the dimension stride): thread
    // tid + 256 j loads keys 8 (u & 7) .. +7 of dimension u >> 3 (n_kv % 64 == 0: no clamp)
    uint4 kr0, kr1, kr2, kr3, vr0, vr1, vr2, vr3;
    uint4 kq0, kq1, kq2, kq3, vq0, vq1, vq2, vq3;               // KS: the odd tile
#define FM2_VT_SRC(KT, J) (vb + ((size_t) ((tid + 256 * (J)) >> 3) * p.v1 + (size_t) (2 * ((KT) * FM_KT + 8 * ((tid + 256 * (J)) & 7)))))
#define FM2_LOAD_KV(KT, LIVE) FM2_LOAD_KV_INTO(KT, LIVE, kr0, kr1, kr2, kr3, vr0, vr1, vr2, vr3)
#define FM2_LOAD_KV_INTO(KT, LIVE, kr0, kr1, kr2, kr3, vr0, vr1, vr2, vr3) do { \
        const int kt_ = (KT); const bool lv_ = (LIVE); \
        const size_t r0_ = (size_t) min(kt_ * FM_KT + (tid >> 4), p.n_kv - 1), r1_ = (size_t) min(kt_ * FM_KT + 16 + (tid >> 4), p.n_kv - 1); \
        const size_t r2_ = (size_t) min(kt_ * FM_KT + 32 + (tid >> 4), p.n_kv - 1), r3_ = (size_t) min(kt_ * FM_KT + 48 + (tid >> 4), p.n_kv - 1); \
        const int c_ = 16 * (tid & 15); \
        kr0 = *(const uint4 *) (kb + (lv_ ? r0_ * p.k1 + c_ : 0)); \
        kr1 = *(const uint4 *) (kb + (lv_ ? r1_ * p.k1 + c_ : 0)); \
        kr2 = *(const uint4 *) (kb + (lv_ ? r2_ * p.k1 + c_ : 0)); \
        kr3 = *(const uint4 *) (kb + (lv_ ? r3_ * p.k1 + c_ : 0)); \
        if constexpr (VT) { \
            vr0 = *(const uint4 *) (lv_ ? FM2_VT_SRC(kt_, 0) : vb); vr1 = *(const uint4 *) (lv_ ? FM2_VT_SRC(kt_, 1) : vb); \
            vr2 = *(const uint4 *) (lv_ ? FM2_VT_SRC(kt_, 2) : vb); vr3 = *(const uint4 *) (lv_ ? FM2_VT_SRC(kt_, 3) : vb); \
        } else { \
            vr0 = *(const uint4 *) (vb + (lv_ ? r0_ * p.v1 + c_ : 0)); vr1 = *(const uint4 *) (vb + (lv_ ? r1_ * p.v1 + c_ : 0)); \
            vr2 = *(const uint4 *) (vb + (lv_ ? r2_ * p.v1 + c_ : 0)); vr3 = *(const uint4 *) (vb + (lv_ ? r3_ * p.v1 + c_ : 0)); \
        } \
    } while (0)

    ffloat16v acc_o[NDT];                                       // O^T: column = query l32
#pragma unroll
    for (int t = 0; t < NDT; ++t)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc_o[t][e] = 0.f;
    float m_run = -INFINITY, l_run = 0.f;                       // l_run: this half's keys only

    const int n_tiles = (p.n_kv + FM_KT - 1) / FM_KT;
    const int n_it = KS ? (n_tiles + 1) / 2 : n_tiles;
    // software pipeline, one tile deep: tile kt+1's K/V rows and mask words are loaded
    // while tile kt computes. The load destinations are consumed (mask fixed into mA,
    // K/V stored to LDS) before they are reloaded, so no register copy waits on them.
    // KS: iteration it stages tiles 2 it (buffer 0) and 2 it + 1 (buffer 1, clamped for the
    // load; its mask index is not clamped, so a tile past the end is dead for waves 2-3)
    uint2 mreg[8], mA[8];
    auto my_tile = [&](int it) { return KS ? 2 * it + khalf : it; };
    FM2_LOAD_KV(0, true);
    if constexpr (KS) FM2_LOAD_KV_INTO(min(1, n_tiles - 1), true, kq0, kq1, kq2, kq3, vq0, vq1, vq2, vq3);
    load_mask(min(my_tile(0), n_tiles - 1), mreg);
    auto store_kv = [&](char * kd, char * vd, const uint4 & k0, const uint4 & k1, const uint4 & k2, const uint4 & k3,
                        const uint4 & v0, const uint4 & v1, const uint4 & v2, const uint4 & v3) {
        const int row = tid >> 4, ch = tid & 15;
        *(uint4 *) (kd + fm2_off(row, ch)) = k0;
        *(uint4 *) (kd + fm2_off(row + 16, ch)) = k1;
        *(uint4 *) (kd + fm2_off(row + 32, ch)) = k2;
        *(uint4 *) (kd + fm2_off(row + 48, ch)) = k3;
        if constexpr (VT) {
            const uint4 vv[4] = {v0, v1, v2, v3};
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int u = tid + 256 * j, d = u >> 3, c = u & 7;
                *(uint2 *) (vd + vt_off(d, 2 * c)) = make_uint2(vv[j].x, vv[j].y);
                *(uint2 *) (vd + vt_off(d, 2 * c + 1)) = make_uint2(vv[j].z, vv[j].w);
            }
        } else {
            *(uint4 *) (vd + fm2_off(row, ch)) = v0;
            *(uint4 *) (vd + fm2_off(row + 16, ch)) = v1;
            *(uint4 *) (vd + fm2_off(row + 32, ch)) = v2;
            *(uint4 *) (vd + fm2_off(row + 48, ch)) = v3;
        }
    };
    const char * const ksw = ks + khalf * FM_KT * 256;          // this wave's tile buffer
    const char * const vsw = vs + khalf * FM_KT * 256;
    for (int it = 0; it < n_it; ++it) {
        const int kt = my_tile(it);
#pragma unroll
        for (int i = 0; i < 8; ++i) mA[i] = mreg[i];
        fix_mask(kt, mA);
        store_kv(ks, vs, kr0, kr1, kr2, kr3, vr0, vr1, vr2, vr3);
        if constexpr (KS) store_kv(ks + FM_KT * 256, vs + FM_KT * 256, kq0, kq1, kq2, kq3, vq0, vq1, vq2, vq3);
        bool live_cur;
        if constexpr (KS) { __syncthreads(); live_cur = __any(any_live(mA)); }   // per wave (its own tile)
        else live_cur = __syncthreads_or(any_live(mA));          // + the tiles are visible
        if constexpr (KS) {
            FM2_LOAD_KV(min(2 * it + 2, n_tiles - 1), true);
            FM2_LOAD_KV_INTO(min(2 * it + 3, n_tiles - 1), true, kq0, kq1, kq2, kq3, vq0, vq1, vq2, vq3);
        } else {
            FM2_LOAD_KV(min(kt + 1, n_tiles - 1), true);
        }
        load_mask(min(my_tile(it + 1), n_tiles - 1), mreg);
        if (live_cur) {
            // ---- S^T = K Q^T: 64 keys (2 blocks of 32) x this wave's 32 queries
            ffloat16v acc_s[2];
#pragma unroll
            for (int n = 0; n < 2; ++n)
#pragma unroll
                for (int e = 0; e < 16; ++e) acc_s[n][e] = 0.f;
#pragma unroll
            for (int s = 0; s < NKS; ++s)
#pragma unroll
                for (int n = 0; n < 2; ++n) {
                    const fhalf8 kf = *(const fhalf8 *) (ksw + fm2_off(32 * n + l32, 2 * s + hl));
                    acc_s[n] = __builtin_amdgcn_mfma_f32_32x32x16_f16(kf, qa[s], acc_s[n], 0, 0, 0);
                }
            // ---- online softmax of this lane's query over its 32 keys + the partner half's,
            // in the log2 domain (v_exp_f32), with a lazily raised reference max: O and l are
            // rescaled only when a query's max grows by more than 2^8 (P <= 256 stays exact
            // enough in f16), i.e. on the first tiles, not on every tile
            constexpr float LOG2E = 1.4426950408889634f;
            const float sl = p.scale * LOG2E;
            float mt = -INFINITY;
#pragma unroll
            for (int n = 0; n < 2; ++n)
#pragma unroll
                for (int e = 0; e < 16; ++e) {
                    const uint2 mv = mA[4 * n + (e >> 2)];
                    const uint32_t w = (e & 2) ? mv.y : mv.x;
                    const float mval = h2f((uint16_t) ((e & 1) ? (w >> 16) : (w & 0xFFFF)));
                    acc_s[n][e] = acc_s[n][e] * sl + mval * LOG2E;
                    mt = fmaxf(mt, acc_s[n][e]);
                }
            mt = fmaxf(mt, __shfl_xor(mt, 32, 64));
            const bool raise = mt > m_run + 8.0f;               // false while mt = -inf
            if (__any(raise)) {                                 // wave-uniform
                const float m_new = raise ? mt : m_run;
                const float alpha = raise ? __builtin_amdgcn_exp2f(m_run - m_new) : 1.f;   // m_run = -inf: 0
                l_run *= alpha;
                m_run = m_new;
#pragma unroll
                for (int t = 0; t < NDT; ++t)
#pragma unroll
                    for (int e = 0; e < 16; ++e) acc_o[t][e] *= alpha;
            }
            fhalf8 pb[4];                                       // P^T fragments, k-step s
            float lt = 0.f;
#pragma unroll
            for (int s = 0; s < 4; ++s)
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const float pv = m_run == -INFINITY ? 0.f : __builtin_amdgcn_exp2f(acc_s[s >> 1][8 * (s & 1) + j] - m_run);
                    lt += pv;
                    pb[s][j] = (_Float16) pv;
                }
            l_run += lt;
            // ---- O^T += V^T P^T; A = V^T by transposing reads: the 16-lane group g reads
            // keys r0 + (0..3) [+ 8] x dims 32 t + 16 (g & 1) + (0..15); lane 4q + pp of the
            // group addresses row r0 + q, dims +4 pp .. +4 pp + 3
            const int g = lane >> 4, iq = (lane >> 2) & 3, ip = lane & 3;
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                const int r0 = 32 * (s >> 1) + 16 * (s & 1) + 4 * (g >> 1) + iq;
#pragma unroll
                for (int t = 0; t < NDT; ++t) {
                    fhalf4 lo, hi;
                    if constexpr (VT) {   // A row = dimension 32 t + l32; its keys 4 hl + (0..3) and 8 + 4 hl + (0..3)
                        const int d = 32 * t + l32, q = 8 * (s >> 1) + 4 * (s & 1) + hl;
                        lo = *(const fhalf4 *) (vsw + vt_off(d, q));
                        hi = *(const fhalf4 *) (vsw + vt_off(d, q + 2));
                    } else {
                        const int c0 = 4 * t + 2 * (g & 1) + (ip >> 1);
                        lo = lds_tr16(vsw + fm2_off(r0, c0) + 8 * (ip & 1));
                        hi = lds_tr16(vsw + fm2_off(r0 + 8, c0) + 8 * (ip & 1));
                    }
                    const fhalf8 vf = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
                    acc_o[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(vf, pb[s], acc_o[t], 0, 0, 0);
                }
            }
        }
        __syncthreads();                                        // K/V tiles are rewritten next
    }
    if constexpr (KS) {
        // merge the odd-tile half into the even one: waves 2-3 leave (O, m, l) in LDS (the
        // tile buffers are free after the loop's last barrier), waves 0-1 rescale both to
        // the larger reference max and add
        float * xo = (float *) ks;                              // [2 heads][NDT * 16][64 lanes]
        float * xm = (float *) vs;                              // [2 heads][2][64 lanes]
        if (khalf) {
#pragma unroll
            for (int t = 0; t < NDT; ++t)
#pragma unroll
                for (int e = 0; e < 16; ++e) xo[((wave & 1) * NDT * 16 + t * 16 + e) * 64 + lane] = acc_o[t][e];
            xm[((wave & 1) * 2 + 0) * 64 + lane] = m_run;
            xm[((wave & 1) * 2 + 1) * 64 + lane] = l_run;
        }
        __syncthreads();
        if (khalf) return;
        const float m1 = xm[((wave & 1) * 2 + 0) * 64 + lane], l1 = xm[((wave & 1) * 2 + 1) * 64 + lane];
        const float mm = fmaxf(m_run, m1);
        const float a0 = m_run == -INFINITY ? 0.f : __builtin_amdgcn_exp2f(m_run - mm);
        const float a1 = m1 == -INFINITY ? 0.f : __builtin_amdgcn_exp2f(m1 - mm);
        l_run = l_run * a0 + l1 * a1;
#pragma unroll
        for (int t = 0; t < NDT; ++t)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc_o[t][e] = acc_o[t][e] * a0 + xo[((wave & 1) * NDT * 16 + t * 16 + e) * 64 + lane] * a1;
    }
    // ---- normalise and store: lane = query l32, rows d = 32 t + 8 g + 4 hl + (0..3)
    const float l_tot = l_run + __shfl_xor(l_run, 32, 64);
    const float inv = l_tot == 0.f ? 0.f : 1.0f / l_tot;
    if (qw + l32 < p.n_q) {
        float * out = (float *) (p.dst + (size_t) h * p.d1 + (size_t) (qw + l32) * p.d2);
#pragma unroll
        for (int t = 0; t < NDT; ++t)
#pragma unroll
            for (int g = 0; g < 4; ++g)
                *(float4 *) (out + 32 * t + 8 * g + 4 * hl) = make_float4(acc_o[t][4 * g] * inv, acc_o[t][4 * g + 1] * inv,
                                                                         acc_o[t][4 * g + 2] * inv, acc_o[t][4 * g + 3] * inv);
        if (p.h) {      // the output projection's f16 input row (act cache)
            typedef _Float16 h4 __attribute__((ext_vector_type(4)));
            _Float16 * ho = p.h + (size_t) (qw + l32) * p.H * D + (size_t) h * D;
#pragma unroll
            for (int t = 0; t < NDT; ++t)
#pragma unroll
                for (int g = 0; g < 4; ++g)
                    *(h4 *) (ho + 32 * t + 8 * g + 4 * hl) = h4{(_Float16) (acc_o[t][4 * g] * inv), (_Float16) (acc_o[t][4 * g + 1] * inv),
                                                               (_Float16) (acc_o[t][4 * g + 2] * inv), (_Float16) (acc_o[t][4 * g + 3] * inv)};
        }
    }
#undef FM2_LOAD_KV
#undef FM2_LOAD_KV_INTO
#undef FM2_VT_SRC
}

// the key-split form (KS above) for GQA groups of an even size; g_tune[0] = 1 keeps HG = 4
static bool fa_key_split(int Gt) { return Gt % 2 == 0 && g_tune[0] != 1; }

bool fa_mma_ok(const ggml_tensor * dst) {
    const ggml_tensor * q = dst->src[0];
    const ggml_tensor * k = dst->src[1];
    const ggml_tensor * v = dst->src[2];
    const ggml_tensor * m = dst->src[3];
    if (dst->src[4]) return false;                                        // sinks
    if (mx_op_param<float>(dst, 1) != 0.0f || mx_op_param<float>(dst, 2) != 0.0f) return false;   // ALiBi, softcap
    if (q->type != GGML_TYPE_F32) return false;
    // bf16 / q8_0 / q4_0 caches run on f16 copies (fa_kv_to_f16), K and V each (round 6: the
    // types may differ — -ctk q8_0 -ctv f16 converts K only)
    auto cv = [](ggml_type t) { return t == GGML_TYPE_BF16 || t == GGML_TYPE_Q8_0 || t == GGML_TYPE_Q4_0; };
    const bool convk = cv(k->type), convv = cv(v->type);
    if ((k->type != GGML_TYPE_F16 && !convk) || (v->type != GGML_TYPE_F16 && !convv)) return false;
    const int64_t D = k->ne[0];
    if ((D != 64 && D != 128) || v->ne[0] != D) return false;
    if (q->ne[1] < 16 || q->ne[3] != 1 || k->ne[3] != 1 || q->ne[2] % k->ne[2]) return false;
    if (m && (m->type != GGML_TYPE_F16 || m->ne[2] != 1 || m->ne[3] != 1 || m->nb[1] % 16 || (uintptr_t) m->data % 16)) return false;
    if (q->nb[1] % 16 || q->nb[0] != 4 || (uintptr_t) q->data % 16) return false;
    if (!convk && (k->nb[1] % 16 || (uintptr_t) k->data % 16)) return false;
    if (!convv && (v->nb[1] % 16 || (uintptr_t) v->data % 16)) return false;
    if (dst->nb[0] != 4 || k->ne[1] > INT32_MAX / 2 || q->ne[1] > INT32_MAX / 2) return false;
    return true;
}

void fa_kv_to_f16(OpCtx & c, const ggml_tensor * t, uint16_t * dst);

void fa_mma_run(OpCtx & c, ggml_tensor * dst) {
    const ggml_tensor * q = dst->src[0];
    const ggml_tensor * k = dst->src[1];
    const ggml_tensor * v = dst->src[2];
    const ggml_tensor * m = dst->src[3];
    FaMmaArgs p{};
    p.q = (const char *) q->data; p.q1 = q->nb[1]; p.q2 = q->nb[2];
    p.k = (const char *) k->data; p.k1 = k->nb[1]; p.k2 = k->nb[2];
    p.v = (const char *) v->data; p.v1 = v->nb[1]; p.v2 = v->nb[2];
    if (k->type != GGML_TYPE_F16) {
        uint16_t * kh = (uint16_t *) c.scratch->take((size_t) k->ne[0] * k->ne[1] * k->ne[2] * 2);
        fa_kv_to_f16(c, k, kh);
        p.k = (const char *) kh; p.k1 = k->ne[0] * 2; p.k2 = k->ne[0] * k->ne[1] * 2;
    }
    if (v->type != GGML_TYPE_F16) {
        uint16_t * vh = (uint16_t *) c.scratch->take((size_t) v->ne[0] * v->ne[1] * v->ne[2] * 2);
        fa_kv_to_f16(c, v, vh);
        p.v = (const char *) vh; p.v1 = v->ne[0] * 2; p.v2 = v->ne[0] * v->ne[1] * 2;
    }
    if (m) { p.mask = (const char *) m->data; p.m1 = m->nb[1]; }
    p.dst = (char *) dst->data; p.d1 = dst->nb[1]; p.d2 = dst->nb[2];
    p.n_q = (int) q->ne[1]; p.n_kv = (int) k->ne[1]; p.H = (int) q->ne[2]; p.Hkv = (int) k->ne[2];
    p.scale = mx_op_param<float>(dst, 0);
    p.qround = k->type == GGML_TYPE_Q8_0 || k->type == GGML_TYPE_Q4_0 ? 1 : (k->type == GGML_TYPE_BF16 ? 2 : 0);
    if (k->ne[0] == 128 && k->ne[1] >= 4 && !g_fa_mma1 && (dst->nb[1] % 16) == 0 && ((uintptr_t) dst->data % 16) == 0) {
        const int Gt = p.H / p.Hkv, HG = Gt % 4 == 0 ? 4 : (Gt % 2 == 0 ? 2 : 1);
        // contiguous [D, H, n_q] output: the output projection reads it as [H*D, n_q] rows
        if (dst->nb[1] == 4 * (size_t) k->ne[0] && dst->nb[2] == (size_t) 4 * k->ne[0] * p.H && dst->ne[3] == 1)
            p.h = mmq_act_claim(c, dst->data, k->ne[0] * p.H, p.n_q, dst->nb[2]);
        if (fa_key_split(Gt)) {   // 2 heads x 2 key halves per workgroup (g_tune[0] = 1: off)
            const dim3 g2((unsigned) mx_ceil_div(p.n_q, 32), (unsigned) (p.Hkv * (Gt / 2)));
            MX_KLOG("fa_mma2 HG=2 ks=2 n_q=%d n_kv=%d H=%d Hkv=%d", p.n_q, p.n_kv, p.H, p.Hkv);
            k_fa_mma2<2, false, true><<<g2, 256, 0, c.st>>>(p);
            return;
        }
        const dim3 g2((unsigned) mx_ceil_div(p.n_q, 32 * (4 / HG)), (unsigned) (p.Hkv * (Gt / HG)));
        MX_KLOG("fa_mma2 HG=%d n_q=%d n_kv=%d H=%d Hkv=%d", HG, p.n_q, p.n_kv, p.H, p.Hkv);
        if (HG == 4) k_fa_mma2<4><<<g2, 256, 0, c.st>>>(p);
        else if (HG == 2) k_fa_mma2<2><<<g2, 256, 0, c.st>>>(p);
        else k_fa_mma2<1><<<g2, 256, 0, c.st>>>(p);
        return;
    }
    dim3 grid((unsigned) mx_ceil_div(p.n_q, FM_QT), (unsigned) p.H);
    MX_KLOG("fa_mma D=%d n_q=%d n_kv=%d", (int) k->ne[0], p.n_q, p.n_kv);
    if (k->ne[0] == 64) k_fa_mma<64><<<grid, 128, 0, c.st>>>(p);
    else k_fa_mma<128><<<grid, 128, 0, c.st>>>(p);
}

// llama-bench's default -fa 0 prefill: the node chain MUL_MAT(k, q) -> SOFT_MAX(mask, scale)
// -> MUL_MAT(v^T, kq) -> PERMUTE -> CONT (src/llama-graph.cpp:1740-1796) for n_q >= 16 query
// rows in one k_fa_mma2<HG, VT = true> launch (exec: fuse_attn_nofa). Semantics per node:
// kq = K·f16(q) with f32 accumulation (the first mul_mat's vec_dot_type conversion), the
// softmax of kq·scale + mask, kqv = V^T·f16(p). The kernel's softmax is the online form of
// the flash-attention path (exp in the log2 domain, P rounded to f16 before normalisation
// instead of after: both round each probability once to f16, NMSE ~1e-7 against the chain).
// The f32 mask of the non-FA graph is converted to the f16 mask the kernel reads — what
// libllama's flash-attention graph does with ggml_cast(kq_mask, F16) (llama-graph.cpp);
// exact for llama's 0 / -inf masks. dst: [D, H, n_q] contiguous (the CONT's output).
__global__ void k_mask_to_f16(const char * m, size_t m1, int n_kv, int n_q, uint16_t * out) {
    const int q = blockIdx.y, i = (blockIdx.x * blockDim.x + threadIdx.x) * 4;
    if (i >= n_kv) return;
    const float4 v = *(const float4 *) (m + (size_t) q * m1 + (size_t) i * 4);
    uint2 h;
    h.x = (uint32_t) f2h(v.x) | ((uint32_t) f2h(v.y) << 16);
    h.y = (uint32_t) f2h(v.z) | ((uint32_t) f2h(v.w) << 16);
    *(uint2 *) (out + (size_t) q * n_kv + i) = h;
}

void fa_mma_nofa_launch(OpCtx & c, const ggml_tensor * q, const ggml_tensor * k, const ggml_tensor * v, const ggml_tensor * m,
                        float scale, ggml_tensor * out) {
    FaMmaArgs p{};
    const int D = (int) k->ne[0];
    p.q = (const char *) q->data; p.q1 = q->nb[1]; p.q2 = q->nb[2];
    p.k = (const char *) k->data; p.k1 = k->nb[1]; p.k2 = k->nb[2];
    p.v = (const char *) v->data; p.v1 = v->nb[1]; p.v2 = v->nb[2];   // v: [n_kv, D, Hkv], keys contiguous
    p.n_q = (int) q->ne[1]; p.n_kv = (int) k->ne[1]; p.H = (int) q->ne[2]; p.Hkv = (int) k->ne[2];
    p.scale = scale;
    if (m) {
        if (m->type == GGML_TYPE_F32) {
            // round 6: converted once per graph pass — every layer's chain reads the same input
            // mask (the per-layer conversion was 32 x 4.8 us per pp2048 ubatch, profiles/r06/)
            Stream * s = c.s;
            const size_t bytes = (size_t) p.n_kv * p.n_q * 2;
            const int64_t key[3] = {(int64_t) p.n_kv, (int64_t) p.n_q, (int64_t) m->nb[1]};
            uint16_t * m16 = nullptr;
            static const bool no_cache = getenv("GGML_MI355X_NO_MASK_CACHE") != nullptr;   // A/B: per layer
            if (!no_cache && s->mask16_src == m->data && !memcmp(s->mask16_key, key, sizeof(key))) {
                m16 = s->mask16;
            } else {
                hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
                HIP_CHECK(hipStreamIsCapturing(c.st, &cs));
                if (!no_cache && bytes > s->mask16_cap && cs == hipStreamCaptureStatusNone) {   // (grown in an eager pass only)
                    HIP_CHECK(hipStreamSynchronize(c.st));
                    if (s->mask16) { HIP_CHECK(hipFree(s->mask16)); exec_bump_buf_gen(); }   // (captures hold the old one)
                    HIP_CHECK(hipMalloc((void **) &s->mask16, bytes));
                    s->mask16_cap = bytes;
                }
                const bool keep = !no_cache && bytes <= s->mask16_cap;
                m16 = keep ? s->mask16 : (uint16_t *) c.scratch->take(bytes);
                k_mask_to_f16<<<dim3((unsigned) mx_ceil_div(p.n_kv / 4, 256), (unsigned) p.n_q), 256, 0, c.st>>>(
                    (const char *) m->data, m->nb[1], p.n_kv, p.n_q, m16);
                s->mask16_src = keep ? m->data : nullptr;
                memcpy(s->mask16_key, key, sizeof(key));
            }
            p.mask = (const char *) m16; p.m1 = (size_t) p.n_kv * 2;
        } else {
            p.mask = (const char *) m->data; p.m1 = m->nb[1];
        }
    }
    p.dst = (char *) out->data; p.d1 = (size_t) D * 4; p.d2 = (size_t) D * 4 * p.H;
    p.h = mmq_act_claim(c, out->data, (int64_t) D * p.H, p.n_q, p.d2);
    const int Gt = p.H / p.Hkv, HG = Gt % 4 == 0 ? 4 : (Gt % 2 == 0 ? 2 : 1);
    if (fa_key_split(Gt)) {
        const dim3 g2((unsigned) mx_ceil_div(p.n_q, 32), (unsigned) (p.Hkv * (Gt / 2)));
        MX_KLOG("attn_nofa_mma HG=2 ks=2 n_q=%d n_kv=%d H=%d Hkv=%d mask=%d", p.n_q, p.n_kv, p.H, p.Hkv, m ? (int) m->type : -1);
        k_fa_mma2<2, true, true><<<g2, 256, 0, c.st>>>(p);
        return;
    }
    const dim3 g2((unsigned) mx_ceil_div(p.n_q, 32 * (4 / HG)), (unsigned) (p.Hkv * (Gt / HG)));
    MX_KLOG("attn_nofa_mma HG=%d n_q=%d n_kv=%d H=%d Hkv=%d mask=%d", HG, p.n_q, p.n_kv, p.H, p.Hkv, m ? (int) m->type : -1);
    if (HG == 4) k_fa_mma2<4, true><<<g2, 256, 0, c.st>>>(p);
    else if (HG == 2) k_fa_mma2<2, true><<<g2, 256, 0, c.st>>>(p);
    else k_fa_mma2<1, true><<<g2, 256, 0, c.st>>>(p);
}

}  // namespace mx
