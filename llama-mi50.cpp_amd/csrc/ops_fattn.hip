// ops_fattn.hip — FLASH_ATTN_EXT on gfx950.
//
// Semantics: ggml_compute_forward_flash_attn_ext_f16_one_chunk
// (ggml-cpu/ops.cpp:8045-8260): Q is rounded to the K vec-dot type (f16),
// s = (q·k)·scale [softcap·tanh(s)] + slope·mask, keys whose mask is −inf are
// skipped, online softmax over keys, sinks enter once, empty rows give 0.
// Reference GPU: fattn.cu:280-482 (vec/tile kernels + split-KV combine).
//
// MI355X design: one block = (query row, KV head, KV split). The G = H/Hkv query
// heads that share a KV head are processed together, so each K/V byte is read
// once per query row (GQA 32/8 → 4× less KV traffic than per-head kernels).
// Per 256-key tile: lane-per-key scores for the G heads (q in LDS, broadcast
// reads), block softmax update, then threads over (head, dim) accumulate P·V with
// coalesced V row reads. Splits are merged by a combine kernel.
#include "backend.h"
#include "quants.cuh"
#include <type_traits>

namespace mx {

// e^x as v_exp_f32(x · log2 e): the libm expf's range reduction sat on the softmax's
// critical path (decode FA v2: 6.95 -> 5.56 us at 256 keys with the same change)
__device__ __forceinline__ float fa_exp(float x) { return __builtin_amdgcn_exp2f(x * 1.4426950408889634f); }

extern int g_tune[48];

constexpr int FA_TILE = 256;
constexpr int FA_MAXG = 8;

struct FaArgs {
    const char * q; size_t q1, q2, q3;     // q strides (row, head, seq)
    const char * k; size_t k1, k2, k3;
    const char * v; size_t v1, v2, v3;
    const char * mask; size_t m1, m2, m3; int64_t mne2, mne3;
    float * opart; float * mpart; float * lpart;
    int64_t n_q, n_kv, H, Hkv, ns, nsplit, chunk;
    float scale, softcap, max_bias, m0, m1f;
    uint32_t n_head_log2;
    int k_aligned;                          // K rows 16-byte aligned → vector loads
    unsigned long long * trace;             // debug: phase timestamps (MX_TRACE)
    unsigned long long * trace_blk;
};

#define FA_TRACE(ph) MX_TRACE((blockIdx.x == 0 && blockIdx.y == 0) ? p.trace : nullptr, ph)

// K/V element types of the tile kernel: f16 (uint16_t), f32 (float) and the tags below.
// Element i of a row: the quantised caches store 32-element blocks, an f16 scale first
// (block_q8_0 / block_q4_0, ggml-common.h), dequantised as the CPU's v_to_float does.
struct KvBF16 {};
struct KvQ8 {};
struct KvQ4 {};
template <typename T> __device__ __forceinline__ float kv_get(const char * row, int i);
template <> __device__ __forceinline__ float kv_get<uint16_t>(const char * row, int i) { return h2f(((const uint16_t *) row)[i]); }
template <> __device__ __forceinline__ float kv_get<float>(const char * row, int i) { return ((const float *) row)[i]; }
template <> __device__ __forceinline__ float kv_get<KvBF16>(const char * row, int i) {
    return __uint_as_float((uint32_t) ((const uint16_t *) row)[i] << 16);
}
template <> __device__ __forceinline__ float kv_get<KvQ8>(const char * row, int i) {
    const char * b = row + (i >> 5) * 34;
    return h2f(ld_u16(b)) * (float) (int8_t) b[2 + (i & 31)];
}
template <> __device__ __forceinline__ float kv_get<KvQ4>(const char * row, int i) {
    const char * b = row + (i >> 5) * 18;
    const int j = i & 31;
    const int x = (uint8_t) b[2 + (j & 15)];
    return h2f(ld_u16(b)) * (float) ((j < 16 ? x & 15 : x >> 4) - 8);
}
// q in the K type's vec-dot type (type_traits_cpu[k->type].vec_dot_type): f16 / bf16
// rounding; the quantised K types dot against q8_0 blocks (quantize_row_q8_0_ref,
// ggml-quants.c: d = amax/127 stored as f16, q = round(x/d)) — applied per 32-block
// after the row is in LDS (fa_q8_blocks)
template <typename TK> __device__ __forceinline__ float q_round(float x) {
    if constexpr (std::is_same<TK, uint16_t>::value) return (float) (_Float16) x;
    else if constexpr (std::is_same<TK, KvBF16>::value) {
        uint32_t u = __float_as_uint(x);
        if ((u & 0x7fffffff) > 0x7f800000) return __uint_as_float((u | 0x00400000u) & 0xffff0000u);   // quiet NaN
        u += 0x7fff + ((u >> 16) & 1);
        return __uint_as_float(u & 0xffff0000u);
    } else return x;
}
template <typename TK> __host__ __device__ constexpr bool kv_q8dot() { return std::is_same<TK, KvQ8>::value || std::is_same<TK, KvQ4>::value; }

template <typename TK, typename TV, int D>
__global__ __launch_bounds__(256) void k_fattn(FaArgs p) {
    __shared__ float qs[FA_MAXG][D];
    __shared__ float sc[FA_MAXG][FA_TILE];
    __shared__ float red[FA_MAXG][4];
    __shared__ float mrun[FA_MAXG], lrun[FA_MAXG], alpha[FA_MAXG];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int64_t bx = blockIdx.x;
    const int64_t hk = bx % p.Hkv;
    const int64_t iq1 = (bx / p.Hkv) % p.n_q;
    const int64_t iq3 = bx / (p.Hkv * p.n_q);
    const int64_t split = blockIdx.y;
    const int G = (int) (p.H / p.Hkv);
    const int64_t kbeg = split * p.chunk, kend = min(p.n_kv, kbeg + p.chunk);

    // q rows of the G heads, rounded to f16 like the CPU vec-dot conversion
    for (int i = tid; i < G * D; i += blockDim.x) {
        const int g = i / D, d = i % D;
        const int64_t h = hk * G + g;
        const float x = *(const float *) (p.q + iq1 * p.q1 + h * p.q2 + iq3 * p.q3 + d * 4);
        qs[g][d] = q_round<TK>(x);
    }
    if constexpr (kv_q8dot<TK>()) {
        __syncthreads();
        for (int b = tid; b < G * D / 32; b += blockDim.x) {
            float * qb = &qs[0][0] + (b / (D / 32)) * D + (b % (D / 32)) * 32;
            float amax = 0.f;
            for (int j = 0; j < 32; ++j) amax = fmaxf(amax, fabsf(qb[j]));
            const float dq = amax / 127.0f, id = dq != 0.0f ? 1.0f / dq : 0.0f;
            const float dh = (float) (_Float16) dq;
            for (int j = 0; j < 32; ++j) qb[j] = dh * roundf(qb[j] * id);
        }
    }
    if (tid < G) { mrun[tid] = -INFINITY; lrun[tid] = 0.f; }
    float slope[FA_MAXG];
#pragma unroll
    for (int g = 0; g < FA_MAXG; ++g) {
        const uint32_t h = (uint32_t) (hk * G + g);
        slope[g] = p.max_bias > 0.0f ? (h < p.n_head_log2 ? powf(p.m0, h + 1) : powf(p.m1f, 2 * (h - p.n_head_log2) + 1)) : 1.0f;
    }
    // output accumulators: thread owns (g, d) pairs o = tid + 256*j
    constexpr int NO = (FA_MAXG * D + 255) / 256;
    float oacc[NO];
#pragma unroll
    for (int j = 0; j < NO; ++j) oacc[j] = 0.f;
    __syncthreads();

    const char * kb = p.k + (hk) * p.k2 + (iq3 % p.ns) * p.k3;
    const char * vb = p.v + (hk) * p.v2 + (iq3 % p.ns) * p.v3;
    const char * mrow = p.mask ? p.mask + iq1 * p.m1 + ((hk * G) % p.mne2) * p.m2 + (iq3 % p.mne3) * p.m3 : nullptr;
    const bool mask_per_head = p.mask && p.mne2 > 1;

    for (int64_t t0 = kbeg; t0 < kend; t0 += FA_TILE) {
        // ---- scores: lane per key
        {
            const int64_t key = t0 + tid;
            float s[FA_MAXG];
#pragma unroll
            for (int g = 0; g < FA_MAXG; ++g) s[g] = -INFINITY;
            if (key < kend) {
                float acc[FA_MAXG];
#pragma unroll
                for (int g = 0; g < FA_MAXG; ++g) acc[g] = 0.f;
                const char * kr = kb + key * p.k1;
                for (int d = 0; d < D; d += 8) {
                    float kv[8];
                    if (std::is_same<TK, uint16_t>::value && p.k_aligned) {
                        const uint4 raw = *(const uint4 *) (kr + 2 * d);
                        const uint16_t * hh = (const uint16_t *) &raw;
#pragma unroll
                        for (int i = 0; i < 8; ++i) kv[i] = h2f(hh[i]);
                    } else {
#pragma unroll
                        for (int i = 0; i < 8; ++i) kv[i] = kv_get<TK>(kr, d + i);
                    }
#pragma unroll
                    for (int g = 0; g < FA_MAXG; ++g) {
                        if (g < G) {
#pragma unroll
                            for (int i = 0; i < 8; ++i) acc[g] += qs[g][d + i] * kv[i];
                        }
                    }
                }
#pragma unroll
                for (int g = 0; g < FA_MAXG; ++g) {
                    if (g >= G) continue;
                    float mv = 0.f;
                    if (mrow) {
                        const char * mr = mask_per_head ? p.mask + iq1 * p.m1 + ((hk * G + g) % p.mne2) * p.m2 + (iq3 % p.mne3) * p.m3 : mrow;
                        mv = slope[g] * h2f(((const uint16_t *) mr)[key]);
                    }
                    if (mv == -INFINITY) continue;
                    float x = acc[g] * p.scale;
                    if (p.softcap != 0.0f) x = p.softcap * tanhf(x);
                    s[g] = x + mv;
                }
            }
#pragma unroll
            for (int g = 0; g < FA_MAXG; ++g) if (g < G) sc[g][tid] = s[g];
        }
        __syncthreads();
        // ---- softmax update per head: wave w handles heads w, w+4
        for (int g = wave; g < G; g += 4) {
            float mx = -INFINITY;
            for (int i = lane; i < FA_TILE; i += 64) mx = fmaxf(mx, sc[g][i]);
            mx = wave_max(mx);
            const float mold = mrun[g];
            const float mnew = fmaxf(mold, mx);
            float sum = 0.f;
            for (int i = lane; i < FA_TILE; i += 64) {
                const float e = mnew == -INFINITY ? 0.f : fa_exp(sc[g][i] - mnew);
                sc[g][i] = e;
                sum += e;
            }
            sum = wave_sum(sum);
            if (lane == 0) {
                const float a = mold == -INFINITY ? 0.f : fa_exp(mold - mnew);
                alpha[g] = a;
                lrun[g] = lrun[g] * a + sum;
                mrun[g] = mnew;
            }
        }
        __syncthreads();
        // ---- P·V: thread owns outputs o = tid + 256*j → (g, d)
        const int64_t nk = min((int64_t) FA_TILE, kend - t0);
#pragma unroll
        for (int j = 0; j < NO; ++j) {
            const int o = tid + 256 * j;
            const int g = o / D, d = o % D;
            if (g < G) {
                float a = oacc[j] * alpha[g];
                const char * vp = vb + t0 * p.v1;
                for (int64_t i = 0; i < nk; ++i) {
                    const float pw = sc[g][i];
                    a += pw * kv_get<TV>(vp + i * p.v1, d);
                }
                oacc[j] = a;
            }
        }
        __syncthreads();
    }
    // ---- write partials
    const int64_t row = (iq3 * p.n_q + iq1) * p.H;   // (seq, query) major, head minor
#pragma unroll
    for (int j = 0; j < NO; ++j) {
        const int o = tid + 256 * j;
        const int g = o / D, d = o % D;
        if (g < G) p.opart[((split * p.ns * p.n_q * p.H) + row + hk * G + g) * D + d] = oacc[j];
    }
    if (tid < G) {
        p.mpart[split * p.ns * p.n_q * p.H + row + hk * G + tid] = mrun[tid];
        p.lpart[split * p.ns * p.n_q * p.H + row + hk * G + tid] = lrun[tid];
    }
}

// ---------------------------------------------------------------------------
// Decode kernel (n_q <= 4, f16 K/V): one block = (query row, KV head, 256-key split),
// the G query heads of the KV head together (G compile-time). Wave w owns keys
// [64w, 64w+64) of the split, one key per lane: the lane's K row and (D <= 128) its
// wave's V rows are all loaded before any arithmetic. Per wave: scores for the G heads
// (q broadcast from LDS), wave softmax, P·V with lanes over head dims; the four waves
// merge in LDS (flash-decoding inside the block). A single split (n_kv <= 256, every
// tg128 step) writes the output directly: no combine launch. Longer caches write
// partials (unnormalised O, m, l) for k_fattn_combine.
// ---------------------------------------------------------------------------
constexpr int FW_CH = 256;

struct FaOut {
    const float * sinks;
    char * dst; size_t nb1, nb2, nb3;
    int direct;
};

typedef _Float16 h2_t __attribute__((ext_vector_type(2)));

__device__ __forceinline__ void h8(const uint4 v, float (&f)[8]) {
    f[0] = h2f((uint16_t) (v.x & 0xFFFF)); f[1] = h2f((uint16_t) (v.x >> 16));
    f[2] = h2f((uint16_t) (v.y & 0xFFFF)); f[3] = h2f((uint16_t) (v.y >> 16));
    f[4] = h2f((uint16_t) (v.z & 0xFFFF)); f[5] = h2f((uint16_t) (v.z >> 16));
    f[6] = h2f((uint16_t) (v.w & 0xFFFF)); f[7] = h2f((uint16_t) (v.w >> 16));
}

template <int D, int G>
__global__ __launch_bounds__(256) void k_fattn_dec(FaArgs p, FaOut fo) {
    static_assert(D % 64 == 0 && D <= 256, "decode FA head size");
    constexpr int NKL = D / 8;                 // 16-byte K loads per lane (its key's row)
    constexpr int D8 = D / 8;                  // 16-byte chunks of a V row
    constexpr int KQ = 64 / D8;                // key subsets of a wave in P·V
    constexpr int KPL = 64 / KQ;               // V rows per lane
    constexpr bool V_EARLY = D <= 128;         // V loads issued with K (register budget)
    __shared__ __align__(16) _Float16 qs[G][D];
    __shared__ __align__(16) float pw[4][G][64];
    __shared__ float wm[4][G], wl[4][G];
    __shared__ __align__(16) float wo[4][G][D];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int Hkv = (int) p.Hkv, n_q = (int) p.n_q, n_kv = (int) p.n_kv;
    // G = query heads per workgroup (a divisor of the GQA group Gt = H/Hkv): splitting a
    // GQA group over workgroups trades K/V re-reads (L2) for shorter per-wave chains
    const int Gt = (int) (p.H / p.Hkv), NGB = Gt / G;
    const int bx = blockIdx.x;
    const int hk = bx % Hkv;
    const int gb = (bx / Hkv) % NGB;
    const int iq1 = (bx / (Hkv * NGB)) % n_q;
    const int iq3 = bx / (Hkv * NGB * n_q);
    const int hb = hk * Gt + gb * G;                    // first query head of this workgroup
    const int split = blockIdx.y;
    const int kw0 = split * FW_CH + wave * 64;          // first key of this wave
    const int key = kw0 + lane;
    const char * kb = p.k + hk * p.k2 + (iq3 % (int) p.ns) * p.k3;
    const char * vb = p.v + hk * p.v2 + (iq3 % (int) p.ns) * p.v3;
    const int vc = lane % D8, vq = lane / D8;           // P·V: 16-byte chunk, key subset

    FA_TRACE(0);
    MX_TRACE_BLK(p.trace_blk, 0);
    // q first: loads retire in issue order, so the LDS fill below waits only for these
    constexpr int QPT = (G * D + 255) / 256;
    float qreg[QPT];
#pragma unroll
    for (int j = 0; j < QPT; ++j) {
        const int i = tid + 256 * j;
        qreg[j] = i < G * D ? *(const float *) (p.q + iq1 * p.q1 + (hb + i / D) * p.q2 + iq3 * p.q3 + (i % D) * 4) : 0.f;
    }
    const bool live = key < n_kv;
    float mv = 0.f;
    if (p.mask && live) mv = h2f(((const uint16_t *) (p.mask + iq1 * p.m1 + (iq3 % (int) p.mne3) * p.m3))[key]);
    uint4 kr[NKL];
    {
        const uint4 * src = (const uint4 *) (kb + (size_t) min(key, n_kv - 1) * p.k1);
#pragma unroll
        for (int j = 0; j < NKL; ++j) kr[j] = src[j];
    }
    uint4 vr[KPL];
    auto load_v = [&] {
#pragma unroll
        for (int j = 0; j < KPL; ++j)
            vr[j] = *(const uint4 *) (vb + (size_t) min(kw0 + vq * KPL + j, n_kv - 1) * p.v1 + vc * 16);
    };
    if constexpr (V_EARLY) load_v();
#pragma unroll
    for (int j = 0; j < QPT; ++j) {
        const int i = tid + 256 * j;
        if (i < G * D) qs[i / D][i % D] = (_Float16) qreg[j];   // the CPU vec-dot rounds q to the K type
    }
    __syncthreads();
    FA_TRACE(1);
    if constexpr (!V_EARLY) load_v();
    // ---- scores (lane = key) and wave softmax, one head at a time (bounded live ranges):
    // q·k as packed f16 pairs with f32 accumulation (v_dot2_f32_f16), q broadcast from LDS
#pragma unroll 1
    for (int g = 0; g < G; ++g) {
        uint4 qv[NKL];
#pragma unroll
        for (int j = 0; j < NKL; ++j) qv[j] = *(const uint4 *) &qs[g][8 * j];
        float a4[4] = {0.f, 0.f, 0.f, 0.f};   // four independent chains
#pragma unroll
        for (int j = 0; j < NKL; ++j) {
            a4[0] = __builtin_amdgcn_fdot2(__builtin_bit_cast(h2_t, kr[j].x), __builtin_bit_cast(h2_t, qv[j].x), a4[0], false);
            a4[1] = __builtin_amdgcn_fdot2(__builtin_bit_cast(h2_t, kr[j].y), __builtin_bit_cast(h2_t, qv[j].y), a4[1], false);
            a4[2] = __builtin_amdgcn_fdot2(__builtin_bit_cast(h2_t, kr[j].z), __builtin_bit_cast(h2_t, qv[j].z), a4[2], false);
            a4[3] = __builtin_amdgcn_fdot2(__builtin_bit_cast(h2_t, kr[j].w), __builtin_bit_cast(h2_t, qv[j].w), a4[3], false);
        }
        const float acc = (a4[0] + a4[1]) + (a4[2] + a4[3]);
        float s = -INFINITY;
        const int h = hb + g;
        float m = mv;
        if (p.mask && p.mne2 > 1)
            m = live ? h2f(((const uint16_t *) (p.mask + iq1 * p.m1 + (h % (int) p.mne2) * p.m2 + (iq3 % (int) p.mne3) * p.m3))[key]) : 0.f;
        if (p.max_bias > 0.0f)
            m *= (uint32_t) h < p.n_head_log2 ? powf(p.m0, h + 1) : powf(p.m1f, 2 * (h - (int) p.n_head_log2) + 1);
        if (live && m != -INFINITY) {
            float x = acc * p.scale;
            if (p.softcap != 0.0f) x = p.softcap * tanhf(x);
            s = x + m;
        }
        const float mx = wave_max(s);
        const float e = mx == -INFINITY ? 0.f : fa_exp(s - mx);
        const float l = wave_sum(e);
        pw[wave][g][lane] = e;
        if (lane == 0) { wm[wave][g] = mx; wl[wave][g] = l; }
    }
    FA_TRACE(2);
    __syncthreads();
    FA_TRACE(3);
    // ---- P·V: lane = (16-byte chunk vc, key subset vq); the G heads share each V row
    float o[G][8];
#pragma unroll
    for (int g = 0; g < G; ++g)
#pragma unroll
        for (int i = 0; i < 8; ++i) o[g][i] = 0.f;
#pragma unroll
    for (int j4 = 0; j4 < KPL; j4 += 4) {
        float4 w4[G];
#pragma unroll
        for (int g = 0; g < G; ++g) w4[g] = *(const float4 *) &pw[wave][g][vq * KPL + j4];
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
            float v[8];
            h8(vr[j4 + jj], v);
#pragma unroll
            for (int g = 0; g < G; ++g) {
                const float w = jj == 0 ? w4[g].x : (jj == 1 ? w4[g].y : (jj == 2 ? w4[g].z : w4[g].w));
#pragma unroll
                for (int i = 0; i < 8; ++i) o[g][i] += w * v[i];
            }
        }
    }
#pragma unroll
    for (int g = 0; g < G; ++g)
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
            for (int off = D8; off < 64; off <<= 1) o[g][i] += __shfl_xor(o[g][i], off, 64);
    if (vq == 0) {
#pragma unroll
        for (int g = 0; g < G; ++g) {
            *(float4 *) &wo[wave][g][vc * 8] = make_float4(o[g][0], o[g][1], o[g][2], o[g][3]);
            *(float4 *) &wo[wave][g][vc * 8 + 4] = make_float4(o[g][4], o[g][5], o[g][6], o[g][7]);
        }
    }
    FA_TRACE(4);
    __syncthreads();
    FA_TRACE(5);
    // ---- merge the four waves
    const int rows = (int) (p.ns * p.n_q * p.H);
    const int row0 = (iq3 * n_q + iq1) * (int) p.H + hb;
    for (int i = tid; i < G * D; i += 256) {
        const int g = i / D, d = i % D;
        float M = fmaxf(fmaxf(wm[0][g], wm[1][g]), fmaxf(wm[2][g], wm[3][g]));
        const int h = hb + g;
        const float sk = (fo.direct && fo.sinks) ? fo.sinks[h] : -INFINITY;
        M = fmaxf(M, sk);
        float L = 0.f, O = 0.f;
#pragma unroll
        for (int w = 0; w < 4; ++w) {
            const float f = wm[w][g] == -INFINITY ? 0.f : fa_exp(wm[w][g] - M);
            L += wl[w][g] * f;
            O += wo[w][g][d] * f;
        }
        if (sk != -INFINITY) L += fa_exp(sk - M);
        if (fo.direct) {
            float * out = (float *) (fo.dst + h * fo.nb1 + iq1 * fo.nb2 + iq3 * fo.nb3);
            out[d] = L == 0.f ? 0.f : O / L;
        } else {
            p.opart[((size_t) split * rows + row0 + g) * D + d] = O;
            if (d == 0) {
                p.mpart[split * rows + row0 + g] = M;
                p.lpart[split * rows + row0 + g] = L;
            }
        }
    }
    FA_TRACE(6);
    MX_TRACE_BLK(p.trace_blk, 1);
}

// Merge the split partials of one output row (block = row, 64 threads). All loads of
// the first 8 splits are issued before any arithmetic: one memory round trip.
template <int D>
__global__ __launch_bounds__(64) void k_fattn_combine(const float * __restrict__ op, const float * __restrict__ mp, const float * __restrict__ lp,
                                const float * __restrict__ sinks, char * __restrict__ dst, size_t nb1, size_t nb2, size_t nb3,
                                int64_t nrows_, int64_t nsplit_, int64_t H, int64_t n_q,
                                int8_t * __restrict__ q8, float * __restrict__ q8d, float * __restrict__ q8s, int64_t q8kp) {
    constexpr int DPT = (D + 63) / 64;
    constexpr int PRE = 8;
    const int nrows = (int) nrows_, nsplit = (int) nsplit_;
    const int r = blockIdx.x;          // (iq3, iq1, h)
    const int lane = threadIdx.x;
    const int h = r % (int) H, iq1 = (r / (int) H) % (int) n_q, iq3 = r / (int) (H * n_q);
    float ov[PRE][DPT];
#pragma unroll
    for (int s = 0; s < PRE; ++s)
#pragma unroll
        for (int i = 0; i < DPT; ++i) {
            const int d = lane + 64 * i;
            ov[s][i] = (s < nsplit && d < D) ? op[((size_t) s * nrows + r) * D + d] : 0.f;
        }
    // per-split maxima and sums: lane s holds split s (splits >= 64 fold into lane s % 64)
    float m_l = -INFINITY;
    for (int s = lane; s < nsplit; s += 64) m_l = fmaxf(m_l, mp[(size_t) s * nrows + r]);
    float M = wave_max(m_l);
    const bool has_sink = sinks != nullptr;
    const float sk = has_sink ? sinks[h] : 0.f;
    if (has_sink) M = fmaxf(M, sk);
    float l_l = 0.f;
    for (int s = lane; s < nsplit; s += 64) {
        const float ms = mp[(size_t) s * nrows + r];
        if (ms != -INFINITY) l_l += lp[(size_t) s * nrows + r] * fa_exp(ms - M);
    }
    float L = wave_sum(l_l);
    if (has_sink) L += fa_exp(sk - M);
    const float inv = L == 0.f ? 0.f : 1.0f / L;
    float o[DPT];
#pragma unroll
    for (int i = 0; i < DPT; ++i) o[i] = 0.f;
    for (int s0 = 0; s0 < nsplit; s0 += PRE) {
        if (s0 > 0) {
#pragma unroll
            for (int s = 0; s < PRE; ++s)
#pragma unroll
                for (int i = 0; i < DPT; ++i) {
                    const int d = lane + 64 * i;
                    ov[s][i] = (s0 + s < nsplit && d < D) ? op[((size_t) (s0 + s) * nrows + r) * D + d] : 0.f;
                }
        }
#pragma unroll
        for (int s = 0; s < PRE; ++s) {
            if (s0 + s >= nsplit) break;
            const float ms = mp[(size_t) (s0 + s) * nrows + r];
            const float w = ms == -INFINITY ? 0.f : fa_exp(ms - M);
#pragma unroll
            for (int i = 0; i < DPT; ++i) o[i] += w * ov[s][i];
        }
    }
    float * out = (float *) (dst + h * nb1 + iq1 * nb2 + iq3 * nb3);
#pragma unroll
    for (int i = 0; i < DPT; ++i) {
        const int d = lane + 64 * i;
        const float v = o[i] * inv;
        if (d < D) out[d] = v;
        if (q8 && (D % 32) == 0) {
            // q8 form of the attention output row (the multi-column GEMV input):
            // column = query row, element = h*D + d, one 32-block per half-wave
            float amax = d < D ? fabsf(v) : 0.f;
#pragma unroll
            for (int off = 16; off > 0; off >>= 1) amax = fmaxf(amax, __shfl_xor(amax, off, 32));
            const Q8Scale qsc = q8_scale(amax);
            const float dd = qsc.d;
            const int qi = q8_round(v, qsc.id);
            int sum = qi;
#pragma unroll
            for (int off = 16; off > 0; off >>= 1) sum += __shfl_xor(sum, off, 32);
            if (d < D) {
                const int64_t col = (int64_t) iq3 * n_q + iq1;
                const int64_t e = (int64_t) h * D + d;
                q8[col * q8kp + e] = (int8_t) qi;
                if ((lane & 31) == 0) {
                    q8d[col * (q8kp / 32) + e / 32] = dd;
                    q8s[col * (q8kp / 32) + e / 32] = dd * (float) sum;
                }
            }
        }
    }
}

// decode kernel eligibility: few query rows, f16 K/V with 16-byte aligned rows
static bool fa_use_dec(const ggml_tensor * dst) {
    const ggml_tensor * q = dst->src[0];
    const ggml_tensor * k = dst->src[1];
    const ggml_tensor * v = dst->src[2];
    const int64_t D = k->ne[0];
    if (q->ne[1] > 4 || k->type != GGML_TYPE_F16 || v->type != GGML_TYPE_F16) return false;
    if (D != 64 && D != 128 && D != 256) return false;
    if (k->ne[1] > INT32_MAX / 2) return false;
    const int64_t G = q->ne[2] / k->ne[2];
    if (G != 1 && G != 2 && G != 4 && G != 8) return false;
    if (k->nb[1] % 16 || k->nb[2] % 16 || k->nb[3] % 16 || v->nb[1] % 16 || v->nb[2] % 16 || v->nb[3] % 16) return false;
    if (k->data && ((uintptr_t) k->data % 16 || (uintptr_t) v->data % 16)) return false;
    return true;
}

static int64_t fa_chunk(const ggml_tensor * dst, int64_t * nsplit_out) {
    const ggml_tensor * q = dst->src[0];
    const ggml_tensor * k = dst->src[1];
    const int64_t n_kv = k->ne[1];
    if (fa_use_dec(dst)) {
        *nsplit_out = mx_ceil_div(n_kv, FW_CH);
        return FW_CH;
    }
    const int64_t blocks = q->ne[1] * k->ne[2] * q->ne[3];
    // enough blocks to cover the chip: split KV when there are few query rows
    int64_t nsplit = std::max<int64_t>(1, std::min<int64_t>(mx_ceil_div(n_kv, FA_TILE), mx_ceil_div(512, blocks)));
    int64_t chunk = mx_ceil_div(mx_ceil_div(n_kv, nsplit), FA_TILE) * FA_TILE;
    nsplit = mx_ceil_div(n_kv, chunk);
    *nsplit_out = nsplit;
    return chunk;
}

bool fa_dec2_ok(const ggml_tensor * dst);
bool fa_mma_ok(const ggml_tensor * dst);
size_t fa_dec2_scratch(const ggml_tensor * dst);
void fa_dec2_run(OpCtx & c, ggml_tensor * dst);
static bool g_fa_dec1 = getenv("GGML_MI355X_FA_DEC1") != nullptr;   // A/B: the v1 decode kernel

size_t flash_attn_scratch(const ggml_tensor * dst) {
    const ggml_tensor * q = dst->src[0];
    const ggml_tensor * v = dst->src[2];
    int64_t nsplit;
    fa_chunk(dst, &nsplit);
    const int64_t rows = q->ne[1] * q->ne[2] * q->ne[3];
    size_t need = nsplit * rows * (v->ne[0] + 2) * sizeof(float) + 4 * 256;
    if (fa_dec2_ok(dst)) need = std::max(need, fa_dec2_scratch(dst));
    const ggml_tensor * k = dst->src[1];
    if ((k->type != GGML_TYPE_F16 || v->type != GGML_TYPE_F16) && fa_mma_ok(dst))   // f16 copies of quantised / bf16 K and / or V
        need = std::max(need, (size_t) ((k->type != GGML_TYPE_F16) + (v->type != GGML_TYPE_F16)) * (mx_nelements(k) / k->ne[3]) * 2 + 512);
    return need;
}

bool flash_attn_supported(const ggml_tensor * dst) {
    const ggml_tensor * q = dst->src[0];
    const ggml_tensor * k = dst->src[1];
    const ggml_tensor * v = dst->src[2];
    const ggml_tensor * m = dst->src[3];
    if (q->type != GGML_TYPE_F32 || dst->type != GGML_TYPE_F32) return false;
    // K and V types: equal, or (round 6) any pair of f16 / q8_0 / q4_0 — the reference's
    // GGML_CUDA_FA_ALL_QUANTS set the fork builds with (fattn.cu:220-260); its own llama-bench
    // line is -ctk q8_0 -ctv f16 (AGENTS.md:166-176)
    auto mixable = [](ggml_type t) { return t == GGML_TYPE_F16 || t == GGML_TYPE_Q8_0 || t == GGML_TYPE_Q4_0; };
    if (k->type != v->type && !(mixable(k->type) && mixable(v->type))) return false;
    if (k->ne[0] != v->ne[0]) return false;
    const int64_t D = k->ne[0];
    auto plain = [](ggml_type t) { return t == GGML_TYPE_F16 || t == GGML_TYPE_F32; };
    auto coded = [](ggml_type t) { return t == GGML_TYPE_BF16 || t == GGML_TYPE_Q8_0 || t == GGML_TYPE_Q4_0; };
    if (plain(k->type) && plain(v->type)) {
        if (D != 32 && D != 40 && D != 48 && D != 64 && D != 80 && D != 96 && D != 112 && D != 128 && D != 256) return false;
    } else if ((plain(k->type) || coded(k->type)) && (plain(v->type) || coded(v->type))) {
        if (D != 64 && D != 128 && D != 256) return false;   // quantised / bf16 caches: the tile kernel's common head sizes
    } else return false;
    if (q->ne[2] % k->ne[2] != 0 || q->ne[2] / k->ne[2] > FA_MAXG) return false;
    if (k->ne[2] != v->ne[2]) return false;
    if (m && m->type != GGML_TYPE_F16) return false;
    if (q->nb[0] != 4 || k->nb[0] != (size_t) mx_type(k->type).size || v->nb[0] != (size_t) mx_type(v->type).size) return false;
    if (q->ne[3] != k->ne[3] && k->ne[3] != 1) return false;
    if (dst->src[4] && dst->src[4]->type != GGML_TYPE_F32) return false;
    return true;
}

template <typename TK, typename TV>
static void fa_launch(OpCtx & c, int D, dim3 grid, const FaArgs & a) {
    constexpr bool plain = (std::is_same<TK, uint16_t>::value || std::is_same<TK, float>::value) &&
                           (std::is_same<TV, uint16_t>::value || std::is_same<TV, float>::value);
    if constexpr (!plain) {
        switch (D) {
            case 64:  k_fattn<TK, TV, 64><<<grid, 256, 0, c.st>>>(a); return;
            case 128: k_fattn<TK, TV, 128><<<grid, 256, 0, c.st>>>(a); return;
            case 256: k_fattn<TK, TV, 256><<<grid, 256, 0, c.st>>>(a); return;
            default: MX_ABORT("fattn D=%d", D);
        }
    }
    switch (D) {
        case 32:  k_fattn<TK, TV, 32><<<grid, 256, 0, c.st>>>(a); break;
        case 40:  k_fattn<TK, TV, 40><<<grid, 256, 0, c.st>>>(a); break;
        case 48:  k_fattn<TK, TV, 48><<<grid, 256, 0, c.st>>>(a); break;
        case 64:  k_fattn<TK, TV, 64><<<grid, 256, 0, c.st>>>(a); break;
        case 80:  k_fattn<TK, TV, 80><<<grid, 256, 0, c.st>>>(a); break;
        case 96:  k_fattn<TK, TV, 96><<<grid, 256, 0, c.st>>>(a); break;
        case 112: k_fattn<TK, TV, 112><<<grid, 256, 0, c.st>>>(a); break;
        case 128: k_fattn<TK, TV, 128><<<grid, 256, 0, c.st>>>(a); break;
        case 256: k_fattn<TK, TV, 256><<<grid, 256, 0, c.st>>>(a); break;
        default: MX_ABORT("fattn D=%d", D);
    }
}

bool fa_mma_ok(const ggml_tensor * dst);
void fa_mma_run(OpCtx & c, ggml_tensor * dst);

// bf16 / q8_0 / q4_0 K or V ([D, n_kv, Hkv] view) -> contiguous f16 [D, n_kv, Hkv] for the
// MFMA prefill kernel (the reference's CUDA backend converts quantised K/V to f16 for its
// tile / mma kernels the same way, fattn-common.cuh launch_fattn)
template <typename T>
__global__ void k_kv_to_f16(const char * __restrict__ src, size_t s1, size_t s2, int D, int n_kv, int Hkv, uint16_t * __restrict__ dst) {
    const int64_t i = (int64_t) blockIdx.x * blockDim.x + threadIdx.x;   // one 8-element group
    const int64_t ng = (int64_t) D / 8 * n_kv * Hkv;
    if (i >= ng) return;
    const int d0 = (int) (i % (D / 8)) * 8;
    const int64_t r = i / (D / 8);
    const int key = (int) (r % n_kv), h = (int) (r / n_kv);
    const char * row = src + (size_t) h * s2 + (size_t) key * s1;
    uint16_t o[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = f2h(kv_get<T>(row, d0 + j));
    uint4 w;
    __builtin_memcpy(&w, o, 16);
    *(uint4 *) (dst + (size_t) r * D + d0) = w;
}

void fa_kv_to_f16(OpCtx & c, const ggml_tensor * t, uint16_t * dst) {
    const int D = (int) t->ne[0], n_kv = (int) t->ne[1], Hkv = (int) t->ne[2];
    const int64_t ng = (int64_t) D / 8 * n_kv * Hkv;
    const unsigned blocks = (unsigned) mx_ceil_div(ng, 256);
    MX_KLOG("fa_kv_to_f16 type=%d D=%d n_kv=%d Hkv=%d", (int) t->type, D, n_kv, Hkv);
    switch (t->type) {
        case GGML_TYPE_BF16: k_kv_to_f16<KvBF16><<<blocks, 256, 0, c.st>>>((const char *) t->data, t->nb[1], t->nb[2], D, n_kv, Hkv, dst); break;
        case GGML_TYPE_Q8_0: k_kv_to_f16<KvQ8><<<blocks, 256, 0, c.st>>>((const char *) t->data, t->nb[1], t->nb[2], D, n_kv, Hkv, dst); break;
        case GGML_TYPE_Q4_0: k_kv_to_f16<KvQ4><<<blocks, 256, 0, c.st>>>((const char *) t->data, t->nb[1], t->nb[2], D, n_kv, Hkv, dst); break;
        default: MX_ABORT("fa_kv_to_f16 type %d", (int) t->type);
    }
}
static bool g_fa_mma_off = getenv("GGML_MI355X_FA_TILE") != nullptr;

bool fa_dec2_will_run(const ggml_tensor * dst) { return !g_fa_dec1 && g_tune[10] != 1 && fa_dec2_ok(dst); }

void op_flash_attn_ext(OpCtx & c, ggml_tensor * dst) {
    if (fa_dec2_will_run(dst)) { fa_dec2_run(c, dst); return; }
    kv_new_row_flush(c);   // (the executor flushes before any other consumer; the other kernels read the cache)
    if (!g_fa_mma_off && !fa_use_dec(dst) && fa_mma_ok(dst)) { fa_mma_run(c, dst); return; }
    const ggml_tensor * q = dst->src[0];
    const ggml_tensor * k = dst->src[1];
    const ggml_tensor * v = dst->src[2];
    const ggml_tensor * m = dst->src[3];
    const ggml_tensor * sk = dst->src[4];
    FaArgs a{};
    a.q = (const char *) q->data; a.q1 = q->nb[1]; a.q2 = q->nb[2]; a.q3 = q->nb[3];
    a.k = (const char *) k->data; a.k1 = k->nb[1]; a.k2 = k->nb[2]; a.k3 = k->nb[3];
    a.v = (const char *) v->data; a.v1 = v->nb[1]; a.v2 = v->nb[2]; a.v3 = v->nb[3];
    if (m) { a.mask = (const char *) m->data; a.m1 = m->nb[1]; a.m2 = m->nb[2]; a.m3 = m->nb[3]; a.mne2 = m->ne[2]; a.mne3 = m->ne[3]; }
    a.n_q = q->ne[1]; a.n_kv = k->ne[1]; a.H = q->ne[2]; a.Hkv = k->ne[2]; a.ns = k->ne[3];
    a.scale = mx_op_param<float>(dst, 0);
    a.max_bias = mx_op_param<float>(dst, 1);
    a.softcap = mx_op_param<float>(dst, 2);
    if (a.softcap != 0.0f) a.scale /= a.softcap;
    const uint32_t n_head = (uint32_t) q->ne[2];
    a.n_head_log2 = 1u << (uint32_t) floor(log2((double) n_head));
    a.m0 = powf(2.0f, -(a.max_bias) / a.n_head_log2);
    a.m1f = powf(2.0f, -(a.max_bias / 2.0f) / a.n_head_log2);
    int64_t nsplit;
    a.chunk = fa_chunk(dst, &nsplit);
    a.nsplit = nsplit;
    const int64_t rows = q->ne[1] * q->ne[2] * q->ne[3];
    const int D = (int) v->ne[0];
    a.opart = (float *) c.scratch->take(nsplit * rows * D * sizeof(float));
    a.mpart = (float *) c.scratch->take(nsplit * rows * sizeof(float));
    a.lpart = (float *) c.scratch->take(nsplit * rows * sizeof(float));
    // fold the sequence dim of q into the grid; K/V streams broadcast when ns == 1
    a.ns = k->ne[3];
    dim3 grid((unsigned) (q->ne[1] * k->ne[2] * q->ne[3]), (unsigned) nsplit);
    // FaArgs::ns is used both as kv-stream count (k3 index = iq3 % ns) and in partial indexing below
    FaArgs b = a;
    b.ns = q->ne[3];
    // kernel indexes K/V by (iq3 % ns): pass kv stream count through k3 stride when ns==1
    if (k->ne[3] == 1) { b.k3 = 0; b.v3 = 0; }
    b.trace = mx_trace_slot(0);
    b.trace_blk = mx_trace_blocks();
    b.k_aligned = ((uintptr_t) k->data % 16 == 0) && k->nb[1] % 16 == 0 && k->nb[2] % 16 == 0 && k->nb[3] % 16 == 0;
    const float * psk = sk ? (const float *) sk->data : nullptr;
    if (fa_use_dec(dst)) {
        const int Gt = (int) (q->ne[2] / k->ne[2]);
        const FaOut fo{psk, (char *) dst->data, dst->nb[1], dst->nb[2], dst->nb[3], nsplit == 1};
        // heads per workgroup: one while the grid is small (short caches), the whole
        // GQA group once there are enough splits to fill the chip
        const int64_t blocks_full = k->ne[2] * q->ne[1] * q->ne[3] * nsplit;
        int G = blocks_full >= 128 ? Gt : 1;
        if (g_tune[7]) G = std::min(g_tune[7], Gt);
        const dim3 gridd((unsigned) (q->ne[1] * k->ne[2] * (Gt / G) * q->ne[3]), (unsigned) nsplit);
        MX_KLOG("fattn_dec D=%d G=%d nsplit=%d n_kv=%d", D, G, (int) nsplit, (int) k->ne[1]);
#define DEC(DD, GG) if (D == DD && G == GG) k_fattn_dec<DD, GG><<<gridd, 256, 0, c.st>>>(b, fo); else
#define DECG(DD) DEC(DD, 1) DEC(DD, 2) DEC(DD, 4) DEC(DD, 8)
        DECG(64) DECG(128) DECG(256) MX_ABORT("fattn dec D=%d G=%d", D, G);
#undef DECG
#undef DEC
        if (nsplit == 1) return;
    } else {
        MX_KLOG("fattn_tile D=%d type=%d vtype=%d", D, (int) k->type, (int) v->type);
        if (k->type != v->type) {   // mixed f16 / q8_0 / q4_0 pairs (flash_attn_supported)
            auto vl = [&](auto ktag) {
                using TK = decltype(ktag);
                switch (v->type) {
                    case GGML_TYPE_F16:  fa_launch<TK, uint16_t>(c, D, grid, b); break;
                    case GGML_TYPE_Q8_0: fa_launch<TK, KvQ8>(c, D, grid, b); break;
                    case GGML_TYPE_Q4_0: fa_launch<TK, KvQ4>(c, D, grid, b); break;
                    default: MX_ABORT("fattn v type %d", (int) v->type);
                }
            };
            switch (k->type) {
                case GGML_TYPE_F16:  vl(uint16_t{}); break;
                case GGML_TYPE_Q8_0: vl(KvQ8{}); break;
                case GGML_TYPE_Q4_0: vl(KvQ4{}); break;
                default: MX_ABORT("fattn k type %d", (int) k->type);
            }
        } else switch (k->type) {
            case GGML_TYPE_F16:  fa_launch<uint16_t, uint16_t>(c, D, grid, b); break;
            case GGML_TYPE_BF16: fa_launch<KvBF16, KvBF16>(c, D, grid, b); break;
            case GGML_TYPE_Q8_0: fa_launch<KvQ8, KvQ8>(c, D, grid, b); break;
            case GGML_TYPE_Q4_0: fa_launch<KvQ4, KvQ4>(c, D, grid, b); break;
            default:             fa_launch<float, float>(c, D, grid, b); break;
        }
    }
    // decode: also emit the q8 activation of the output for the O-projection GEMV
    ActQ * q8 = nullptr;
    if (D % 32 == 0 && q->ne[1] * q->ne[3] > 1 && q->ne[1] * q->ne[3] <= 8 && mx_is_contiguous(dst))
        q8 = act_cache_alloc_raw(c.s, dst->data, D * q->ne[2], q->ne[1] * q->ne[3], mx_nbytes(dst));
    switch (D) {
#define CMB(DD) case DD: k_fattn_combine<DD><<<(unsigned) rows, 64, 0, c.st>>>(a.opart, a.mpart, a.lpart, psk, (char *) dst->data, \
                                                       dst->nb[1], dst->nb[2], dst->nb[3], rows, nsplit, q->ne[2], q->ne[1], \
                                                       q8 ? (int8_t *) q8->q : nullptr, q8 ? (float *) q8->d : nullptr, \
                                                       q8 ? (float *) q8->s : nullptr, q8 ? q8->kp : 0); break;
        CMB(32) CMB(40) CMB(48) CMB(64) CMB(80) CMB(96) CMB(112) CMB(128) CMB(256)
#undef CMB
    }
}

}  // namespace mx
