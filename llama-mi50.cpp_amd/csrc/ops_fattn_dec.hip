// ops_fattn_dec.hip — single-token FLASH_ATTN_EXT (decode) on gfx950, v2.
//
// Semantics: ggml_compute_forward_flash_attn_ext_f16_one_chunk (ggml-cpu/ops.cpp:
// 8045-8260): q rounded to f16 (the K vec-dot type), s = (q·k)·scale + mask, keys whose
// mask is −inf skipped, softmax over keys, O = Σ p·V. Reference GPU: fattn-vec.cuh:21 +
// the split-KV combine fattn-common.cuh:730-782.
//
// Why v2: the first decode kernel gave each lane one key and had it read that key's
// whole 256-B K row (16 loads, 2 KB apart between lanes): every wave instruction
// touched 64 cache lines, and at llama-bench tg128's 256-key cache the kernel spent
// ~5 of its 8.5 µs in the vector-memory pipe of the 32 CUs it ran on.
// v2 (MI355X-first):
//  * D/8 lanes share one key row (16 B each, 8 f16 dims): a wave instruction reads
//    64/(D/8) whole rows — coalesced; q·k partials reduce over the row's lanes by DPP;
//  * one workgroup = one KV head x all G query heads of its GQA group (K/V read once)
//    x a split of 64/128-key chunks (online softmax over its chunks), at most 16 splits,
//    so a short cache still spreads over Hkv x nsplit CUs;
//  * every load (q, K, V, mask) is issued before any arithmetic: one memory round trip;
//  * splits merge in the same launch: each workgroup publishes (O, max, sum) and the
//    last one to arrive (device-scope counter, reset by it for the next launch / graph
//    replay) combines them — no second kernel, no second launch gap.
#include "backend.h"
#include "quants.cuh"
#include "gemv.h"
#include <type_traits>

namespace mx { extern int g_tune[48]; }

namespace mx {

struct FaDecArgs {
    const char * q; size_t q1, q2, q3;
    const char * k; size_t k1, k2, k3;
    const char * v; size_t v1, v2, v3;
    const char * mask; size_t m1, m3; int mne3;
    char * dst; size_t d1, d2, d3;
    float * part;                  // [rows][nsplit][G*(D+2)] partials (scratch)
    int to_part;                   // LONG: partials even for one split (fa_dec2_partials)
    unsigned int * cnt;            // per (q row, seq, KV head) arrival counters, zero between launches
    int n_q, n_kv, H, Hkv, ns_kv, nsplit;
    float scale;
    unsigned long long * trace;    // debug (MX_TRACE), workgroup 0
    unsigned long long * trace_blk;
    // weight prefetch (grid rows y >= nsplit, see fa_prefetch_plan in exec.cpp): one dword
    // per 128-B line of each range, so the next GEMV launches hit the Infinity Cache
    const char * pf[4]; size_t pf_eighth[4]; unsigned pf_lines[4]; int pf_n;   // lines per eighth
    // round 6: this token's q8_0 K / V row, staged in f32 by the fused decode QKV launch
    // (KvNewRow, ops_qkv.hip) instead of a k_kv_store_q8 launch: every workgroup quantises
    // its head's part itself and uses it in place of the cache row (read stale), one per KV
    // head writes it to the cache. null: the row is in the cache already
    const float * nr_k; const float * nr_v; const int64_t * nr_ik; const int64_t * nr_iv;
};

constexpr int FD_NI = 4;          // key-row load instructions per wave per chunk
constexpr int FD_MAXSPLIT = 16;   // workgroups per (q row, KV head); longer caches loop over chunks

// q8_0 K/V (KQ, `-ctk q8_0 -ctv q8_0`): a lane's 8 dimensions are 8 int8 of one 32-block
// (its f16 scale first: block_q8_0), q is quantised to q8_0 per 32-block as the CPU's
// vec_dot_type conversion does (amax over the block's 4 lanes by DPP, d = amax/127 kept
// as f16), q·k = Σ_blocks d_q·d_k·Σ q_i k_i, V dequantised d·q_i into the f32 sums.
// Round 6: K and V types are independent (template KV: fd_kv_code) — the fork's own line is
// `-ctk q8_0 -ctv f16` (K q8_0, V f16; reference fattn.cu:220-226 under FA_ALL_QUANTS).
// KV 0: f16 / f16, 1: q8_0 / q8_0, 2: q8_0 K / f16 V, 3: f16 K / q8_0 V.
constexpr bool fd_kq(int kv) { return kv == 1 || kv == 2; }
constexpr bool fd_vq(int kv) { return kv == 1 || kv == 3; }
static int fd_kv_code(const ggml_tensor * k, const ggml_tensor * v) {
    const bool kq = k->type == GGML_TYPE_Q8_0, vq = v->type == GGML_TYPE_Q8_0;
    return kq ? (vq ? 1 : 2) : (vq ? 3 : 0);
}
// f(std::integral_constant<int, KV>{}) for the runtime code kv (one instantiation per pair)
template <typename F>
static void fd_kv_dispatch(int kv, F && f) {
    switch (kv) {
        case 1: f(std::integral_constant<int, 1>{}); break;
        case 2: f(std::integral_constant<int, 2>{}); break;
        case 3: f(std::integral_constant<int, 3>{}); break;
        default: f(std::integral_constant<int, 0>{}); break;
    }
}
__device__ __forceinline__ uint2 ldu8(const char * p) {   // 8 bytes, any 2-byte alignment
    uint2 v;
    __builtin_memcpy(&v, __builtin_assume_aligned(p, 2), 8);
    return v;
}

// Reductions over the key rows of a wave: lanes l ^ LPK, l ^ 2 LPK, ... For LPK = 16 (D 128)
// by the gfx950 row-swap instructions (VALU; with both operands = v the two results add up
// to v[l] + v[l ^ 16] / v[l ^ 32]) instead of ds_bpermute shuffles (the same change took
// ~1 us of latency out of ops_attn_o.hip's attention); other LPK by shuffles.
template <int LPK>
__device__ __forceinline__ float kr_sum(float v) {
    if constexpr (LPK == 16) {
        auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
        v = __uint_as_float(a[0]) + __uint_as_float(a[1]);
        auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
        return __uint_as_float(b[0]) + __uint_as_float(b[1]);
    } else {
#pragma unroll
        for (int off = LPK; off < 64; off <<= 1) v += __shfl_xor(v, off, 64);
        return v;
    }
}
template <int LPK>
__device__ __forceinline__ float kr_max(float v) {
    if constexpr (LPK == 16) {
        auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
        v = fmaxf(__uint_as_float(a[0]), __uint_as_float(a[1]));
        auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
        return fmaxf(__uint_as_float(b[0]), __uint_as_float(b[1]));
    } else {
#pragma unroll
        for (int off = LPK; off < 64; off <<= 1) v = fmaxf(v, __shfl_xor(v, off, 64));
        return v;
    }
}

// G = query heads per workgroup (a divisor of the GQA ratio Gt; K/V are read once per
// workgroup), NW = waves per workgroup (the chunk is NW x NI x 64/(D/8) keys), NI = key-row
// load instructions per wave and chunk. LONG (round 3, caches beyond one chunk): every
// workgroup takes exactly ONE chunk, so all of a split's K/V bytes are in flight at once
// (the looping split form paid one memory round trip per 64-key chunk: 34.5 us at 16k
// keys), any number of splits; the (O, max, sum) partials are merged by
// k_fattn_dec2_combine, a parallel second launch (one workgroup per query head).
template <int D, int G, int NW, int KV = 0, int NI = FD_NI, bool LONG = false, int CPW = 1>
__global__ __launch_bounds__(64 * NW) void k_fattn_dec2(FaDecArgs p) {
    constexpr bool KQ = fd_kq(KV), VQ = fd_vq(KV);
    constexpr int NT = 64 * NW;
    constexpr int LPK = D / 8;            // lanes per key row
    constexpr int KPI = 64 / LPK;         // keys per wave instruction
    constexpr int KPW = NI * KPI;         // keys per wave per chunk
    constexpr int CS = NW * KPW;          // keys per chunk (workgroup)
    typedef _Float16 h2v __attribute__((ext_vector_type(2)));
    __shared__ float wm[NW][G], wl[NW][G];
    __shared__ __align__(16) float wo[NW][G][D];
    __shared__ float sM[G][LONG ? 1 : FD_MAXSPLIT], sF[G][LONG ? 1 : FD_MAXSPLIT], sL[G];
    __shared__ int s_last;

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if ((int) blockIdx.y >= p.nsplit) {       // prefetch rows (workgroup-uniform: no barrier below)
        // linear workgroup id L runs on XCD L % 8 (fa_dec2_run keeps the first prefetch id
        // and their count multiples of 8); XCD x touches the head of the x-th eighth of
        // every range, the rows its GEMV blocks will read first
        const unsigned L = blockIdx.x + gridDim.x * blockIdx.y, P0 = gridDim.x * p.nsplit;
        const unsigned xcd = L & 7, T = (gridDim.x * (gridDim.y - p.nsplit) >> 3) * NT;
        const unsigned t0 = ((L - P0) >> 3) * NT + tid;
        unsigned acc = 0;
        for (int r = 0; r < p.pf_n; ++r) {
            const unsigned * w = (const unsigned *) (p.pf[r] + (size_t) xcd * p.pf_eighth[r]);
#pragma unroll 4
            for (unsigned l = t0; l < p.pf_lines[r]; l += T) acc ^= w[(size_t) l * 32];
        }
        if (acc == 0x9E3779B9u && p.n_kv < 0) p.part[0] = 0.f;   // never (n_kv > 0): keeps the loads
        return;
    }
    const int c = lane % LPK, kq = lane / LPK;
    const int Gt = p.H / p.Hkv, NGB = Gt / G;
    const int hk = blockIdx.x % p.Hkv;
    const int gb = (blockIdx.x / p.Hkv) % NGB;
    const int iq1 = (blockIdx.x / (p.Hkv * NGB)) % p.n_q;
    const int iq3 = blockIdx.x / (p.Hkv * NGB * p.n_q);
    const int split = blockIdx.y;
    const int hb = hk * Gt + gb * G;                         // first query head
    const int hslot = hk * NGB + gb;                         // partial / counter slot
    // this lane's 8 dimensions of a row: f16 at 16 c; q8_0 at block c/4 (34 B), byte 8 (c%4)
    const int lofs8 = (c >> 2) * 34 + 2 + 8 * (c & 3), lofs16 = c * 16;
    const int lofsk = KQ ? lofs8 : lofs16, lofsv = VQ ? lofs8 : lofs16;
    const int dofs = (c >> 2) * 34;
    const char * kb = p.k + (size_t) hk * p.k2 + (size_t) (iq3 % p.ns_kv) * p.k3 + lofsk;
    const char * vb = p.v + (size_t) hk * p.v2 + (size_t) (iq3 % p.ns_kv) * p.v3 + lofsv;
    const uint16_t * mrow = (const uint16_t *) (p.mask ? p.mask + (size_t) iq1 * p.m1 + (size_t) (iq3 % p.mne3) * p.m3 : p.k);
    const int nch = (p.n_kv + CS - 1) / CS, cpb = LONG ? 1 : (nch + p.nsplit - 1) / p.nsplit;
    unsigned long long * tr = (blockIdx.x == 0 && blockIdx.y == 0) ? p.trace : nullptr;
    MX_TRACE(tr, 0);
    MX_TRACE_BLK(p.trace_blk, 0);

    // q and (round 6) this token's new K / V row are LOADED first, but converted only after
    // the first chunk's K / V loads are issued (prep below): their conversion no longer holds
    // the chunk loads back by a memory round trip. The CPU vec-dot rounds q to the K type:
    // f16, or q8_0 blocks for a q8_0 K (amax over the block's 4 lanes by DPP, d = amax/127)
    float4 qa[G], qb[G];
#pragma unroll
    for (int h = 0; h < G; ++h) {
        const float * qp = (const float *) (p.q + (size_t) iq1 * p.q1 + (size_t) (hb + h) * p.q2 + (size_t) iq3 * p.q3) + 8 * c;
        qa[h] = *(const float4 *) qp;
        qb[h] = *(const float4 *) (qp + 4);
    }
    // the new row (q8_0 caches, FaDecArgs::nr_*): unconditional loads (a dummy source when
    // absent: a load under a branch waits at the join)
    const float * nks = KQ && p.nr_k ? p.nr_k + hk * D + 8 * c : (const float *) p.q;
    const float * nvs = VQ && p.nr_v ? p.nr_v + hk * D + 8 * c : (const float *) p.q;
    const float4 nk0 = *(const float4 *) nks, nk1 = *(const float4 *) (nks + 4);
    const float4 nv0 = *(const float4 *) nvs, nv1 = *(const float4 *) (nvs + 4);
    const int64_t nik = *(KQ && p.nr_k ? p.nr_ik : (const int64_t *) p.q), niv = *(VQ && p.nr_v ? p.nr_iv : (const int64_t *) p.q);
    h2v qh[G][4];
    int qq8[G][2];                                           // KQ: q as q8_0, 8 int8
    float qd[G];                                             // KQ: its block scale (f16-rounded)
    int64_t nrk = -1, nrv = -1;
    uint2 nkq = {0, 0}, nvq = {0, 0};
    uint16_t nkd = 0, nvd = 0;
    // quantize_row_q8_0 of a lane's 8 values (the 32-block over 4 lanes): the bytes
    // k_kv_store_q8 would have written for the new row
    auto nr_quant = [&](float4 a0, float4 a1, uint2 & q8, uint16_t & dh) {
        const float x[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
        float amax = 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j) amax = fmaxf(amax, fabsf(x[j]));
        amax = dpp_max_group<4>(amax);
        const float d = amax / 127.0f, id = d != 0.0f ? 1.0f / d : 0.0f;
        dh = f2h(d);
        uint32_t w0 = 0, w1 = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            w0 |= ((uint32_t) (int8_t) roundf(__fmul_rn(x[j], id)) & 0xFFu) << (8 * j);
            w1 |= ((uint32_t) (int8_t) roundf(__fmul_rn(x[4 + j], id)) & 0xFFu) << (8 * j);
        }
        q8 = make_uint2(w0, w1);
    };
    // the new row concerns only the workgroup whose keys hold it and the one that stores it
    // (below): the others skip its quantisation (workgroup-uniform)
    auto nr_mine = [&](int64_t r) {
        const int cw = LONG ? CPW : cpb;                       // chunks of this workgroup
        const int64_t lo = (int64_t) split * cw * CS, hi = lo + (int64_t) cw * CS;
        return (gb == 0 && split == 0 && iq1 == 0 && iq3 == 0) || (r >= lo && r < hi);
    };
    auto prep = [&]() {
        if constexpr (KQ) {
#pragma unroll
            for (int h = 0; h < G; ++h) {
                const float x[8] = {qa[h].x, qa[h].y, qa[h].z, qa[h].w, qb[h].x, qb[h].y, qb[h].z, qb[h].w};
                float amax = 0.f;
#pragma unroll
                for (int j = 0; j < 8; ++j) amax = fmaxf(amax, fabsf(x[j]));
                amax = dpp_max_group<4>(amax);
                const float dq = amax / 127.0f, id = dq != 0.0f ? 1.0f / dq : 0.0f;
                qd[h] = (float) (_Float16) dq;
                int w0 = 0, w1 = 0;
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    w0 |= ((int) roundf(x[j] * id) & 0xFF) << (8 * j);
                    w1 |= ((int) roundf(x[4 + j] * id) & 0xFF) << (8 * j);
                }
                qq8[h][0] = w0; qq8[h][1] = w1;
            }
            if (p.nr_k && nr_mine(nik)) { nrk = nik; nr_quant(nk0, nk1, nkq, nkd); }
        } else {
#pragma unroll
            for (int h = 0; h < G; ++h) {
                qh[h][0] = h2v{(_Float16) qa[h].x, (_Float16) qa[h].y}; qh[h][1] = h2v{(_Float16) qa[h].z, (_Float16) qa[h].w};
                qh[h][2] = h2v{(_Float16) qb[h].x, (_Float16) qb[h].y}; qh[h][3] = h2v{(_Float16) qb[h].z, (_Float16) qb[h].w};
            }
        }
        if constexpr (VQ) if (p.nr_v && nr_mine(niv)) { nrv = niv; nr_quant(nv0, nv1, nvq, nvd); }
    };
    // running (max, sum, O) of this wave; O not yet reduced over the wave's key rows
    float M[G], L[G], o[G][8];
#pragma unroll
    for (int h = 0; h < G; ++h) {
        M[h] = -INFINITY; L[h] = 0.f;
#pragma unroll
        for (int i = 0; i < 8; ++i) o[h][i] = 0.f;
    }
    // one chunk's loads, unconditional (clamped: a load under a branch costs a wait at
    // the join): mask, K rows, V rows — coalesced, LPK lanes per row
    struct Chunk { uint16_t mraw[NI]; uint4 kr[NI], vr[NI]; uint16_t kd[NI], vd[NI]; };
    auto load = [&](int ch, Chunk & b) {
        const int key0 = ch * CS + wave * KPW + kq;
#pragma unroll
        for (int t = 0; t < NI; ++t) b.mraw[t] = mrow[min(key0 + t * KPI, p.n_kv - 1)];
        if constexpr (KQ) {
#pragma unroll
            for (int t = 0; t < NI; ++t) {
                const size_t ko = (size_t) min(key0 + t * KPI, p.n_kv - 1) * p.k1;
                const uint2 w = ldu8(kb + ko);
                b.kr[t] = make_uint4(w.x, w.y, 0, 0);
                b.kd[t] = ld_u16(kb - lofsk + dofs + ko);
            }
        } else {
#pragma unroll
            for (int t = 0; t < NI; ++t) b.kr[t] = *(const uint4 *) (kb + (size_t) min(key0 + t * KPI, p.n_kv - 1) * p.k1);
        }
        if constexpr (VQ) {
#pragma unroll
            for (int t = 0; t < NI; ++t) {
                const size_t vo = (size_t) min(key0 + t * KPI, p.n_kv - 1) * p.v1;
                const uint2 w = ldu8(vb + vo);
                b.vr[t] = make_uint4(w.x, w.y, 0, 0);
                b.vd[t] = ld_u16(vb - lofsv + dofs + vo);
            }
        } else {
#pragma unroll
            for (int t = 0; t < NI; ++t) b.vr[t] = *(const uint4 *) (vb + (size_t) min(key0 + t * KPI, p.n_kv - 1) * p.v1);
        }
    };
    // scores and the online softmax of one loaded chunk (keys past n_kv count as masked:
    // a chunk wholly past the cache contributes nothing)
    auto process = [&](int ch, const Chunk & b, bool first) {
        const int key0 = ch * CS + wave * KPW + kq;
        float mk[NI];
#pragma unroll
        for (int t = 0; t < NI; ++t) mk[t] = key0 + t * KPI < p.n_kv ? (p.mask ? h2f(b.mraw[t]) : 0.f) : -INFINITY;
        // scores: q·k over the row's LPK lanes (DPP), one per (head, key) in every lane of the row
        float s[G][NI];
        if (first) { asm volatile("" :: "v"(b.kr[0].x), "v"(b.vr[0].x), "v"(b.vr[NI - 1].w)); MX_TRACE(tr, 2); }
#pragma unroll
        for (int t = 0; t < NI; ++t) {
            // the new row replaces its stale cache copy (selects, no branch)
            const bool isnk = key0 + t * KPI == nrk;
            const uint32_t kx = isnk ? nkq.x : b.kr[t].x, ky = isnk ? nkq.y : b.kr[t].y;
            const uint16_t kdd = isnk ? nkd : b.kd[t];
#pragma unroll
            for (int h = 0; h < G; ++h) {
                float acc;
                if constexpr (KQ) {
                    const int si = dot4_i8((int) ky, qq8[h][1], dot4_i8((int) kx, qq8[h][0], 0));
                    acc = (float) si * (qd[h] * h2f(kdd));
                } else {
                    acc = __builtin_amdgcn_fdot2(__builtin_bit_cast(h2v, b.kr[t].x), qh[h][0], 0.f, false);
                    acc = __builtin_amdgcn_fdot2(__builtin_bit_cast(h2v, b.kr[t].y), qh[h][1], acc, false);
                    acc = __builtin_amdgcn_fdot2(__builtin_bit_cast(h2v, b.kr[t].z), qh[h][2], acc, false);
                    acc = __builtin_amdgcn_fdot2(__builtin_bit_cast(h2v, b.kr[t].w), qh[h][3], acc, false);
                }
                acc = dpp_sum_group<LPK>(acc);
                // log2 domain (v_exp_f32 below): s = (q·k·scale + mask) · log2(e)
                s[h][t] = mk[t] == -INFINITY ? -INFINITY : (acc * p.scale + mk[t]) * 1.4426950408889634f;
            }
        }
        // online softmax (the wave's keys of this chunk: xor over the key rows kq)
#pragma unroll
        for (int h = 0; h < G; ++h) {
            float mc = s[h][0];
#pragma unroll
            for (int t = 1; t < NI; ++t) mc = fmaxf(mc, s[h][t]);
            mc = kr_max<LPK>(mc);
            const float Mn = fmaxf(M[h], mc);
            const float a = M[h] == -INFINITY ? 0.f : __builtin_amdgcn_exp2f(M[h] - Mn);
            float pr[NI], lc = 0.f;
#pragma unroll
            for (int t = 0; t < NI; ++t) { pr[t] = Mn == -INFINITY ? 0.f : __builtin_amdgcn_exp2f(s[h][t] - Mn); lc += pr[t]; }
            lc = kr_sum<LPK>(lc);
            L[h] = L[h] * a + lc;
            M[h] = Mn;
#pragma unroll
            for (int i = 0; i < 8; ++i) o[h][i] *= a;
#pragma unroll
            for (int t = 0; t < NI; ++t) {
                if constexpr (VQ) {
                    const bool isnv = key0 + t * KPI == nrv;
                    const float dv = h2f(isnv ? nvd : b.vd[t]);
                    const uint32_t vw[2] = {isnv ? nvq.x : b.vr[t].x, isnv ? nvq.y : b.vr[t].y};
                    const float pdv = pr[t] * dv;     // (the block scale folded into the weight)
#pragma unroll
                    for (int i = 0; i < 8; ++i)
                        o[h][i] += pdv * (float) (int8_t) ((vw[i >> 2] >> (8 * (i & 3))) & 0xFF);
                } else {
                    const uint32_t vw[4] = {b.vr[t].x, b.vr[t].y, b.vr[t].z, b.vr[t].w};
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        o[h][2 * i] += pr[t] * h2f((uint16_t) (vw[i] & 0xFFFF));
                        o[h][2 * i + 1] += pr[t] * h2f((uint16_t) (vw[i] >> 16));
                    }
                }
            }
        }
    };
    if constexpr (LONG && CPW > 1) {
        // round 4: CPW chunks per workgroup, double-buffered — chunk c+1's loads are in
        // flight while chunk c computes (the one-chunk form left every workgroup's compute
        // exposed after its single round trip, and 4x the splits for the combine)
        Chunk bf[2];
        load(min(split * CPW, nch - 1), bf[0]);
        __builtin_amdgcn_sched_barrier(0);
        prep();
#pragma unroll
        for (int ci = 0; ci < CPW; ++ci) {
            // (compiler memory barrier: the next chunk's loads are issued here, not hoisted
            // above the previous chunk's processing — two register buffers, not CPW)
            asm volatile("" ::: "memory");
            if (ci + 1 < CPW) load(min(split * CPW + ci + 1, nch - 1), bf[(ci + 1) & 1]);
            __builtin_amdgcn_sched_barrier(0);
            process(split * CPW + ci, bf[ci & 1], ci == 0);
        }
    } else {
        for (int ci = 0; ci < cpb; ++ci) {
            const int ch = split * cpb + ci;
            if (ch >= nch) break;                                 // workgroup-uniform
            Chunk b;
            load(ch, b);
            __builtin_amdgcn_sched_barrier(0);
            if (ci == 0) { MX_TRACE(tr, 1); prep(); }
            process(ch, b, ci == 0);
        }
    }
    // one workgroup per KV head stores the new q8_0 rows (the others read the stale copy and
    // replaced it): lanes of key row 0 of wave 0, 8 quants each, the block scale by its first lane
    if ((KQ || VQ) && gb == 0 && split == 0 && iq1 == 0 && iq3 == 0 && wave == 0 && kq == 0) {
        auto put = [&](const char * base, size_t stride, int64_t row, uint2 q8, uint16_t dh) {
            char * rp = const_cast<char *>(base) + (size_t) row * stride;
            uint16_t * qp = (uint16_t *) (rp + lofs8);           // 2-byte aligned (34-B blocks)
            qp[0] = (uint16_t) q8.x; qp[1] = (uint16_t) (q8.x >> 16); qp[2] = (uint16_t) q8.y; qp[3] = (uint16_t) (q8.y >> 16);
            if ((c & 3) == 0) *(uint16_t *) (rp + dofs) = dh;
        };
        if (KQ && nrk >= 0) put(kb - lofsk, p.k1, nrk, nkq, nkd);
        if (VQ && nrv >= 0) put(vb - lofsv, p.v1, nrv, nvq, nvd);
    }
#pragma unroll
    for (int h = 0; h < G; ++h) {
#pragma unroll
        for (int i = 0; i < 8; ++i) o[h][i] = kr_sum<LPK>(o[h][i]);
        if (lane == 0) { wm[wave][h] = M[h]; wl[wave][h] = L[h]; }
        if (kq == 0) {
            *(float4 *) &wo[wave][h][8 * c] = make_float4(o[h][0], o[h][1], o[h][2], o[h][3]);
            *(float4 *) &wo[wave][h][8 * c + 4] = make_float4(o[h][4], o[h][5], o[h][6], o[h][7]);
        }
    }
    MX_TRACE(tr, 3);
    __syncthreads();
    MX_TRACE(tr, 4);

    // ---- merge the four waves: (O, M, L) of this split for the G heads
    constexpr int PW = G * (D + 2);                          // partial floats per workgroup
    const int slots = p.Hkv * NGB;
    float * part = p.part + ((size_t) ((iq3 * p.n_q + iq1) * slots + hslot) * p.nsplit + split) * PW;
    for (int i = tid; i < G * D; i += NT) {
        const int h = i / D, d = i % D;
        float Mw = wm[0][h];
#pragma unroll
        for (int w = 1; w < NW; ++w) Mw = fmaxf(Mw, wm[w][h]);
        float Lw = 0.f, O = 0.f;
#pragma unroll
        for (int w = 0; w < NW; ++w) {
            const float f = wm[w][h] == -INFINITY ? 0.f : __builtin_amdgcn_exp2f(wm[w][h] - Mw);
            Lw += wl[w][h] * f;
            O += wo[w][h][d] * f;
        }
        if (p.nsplit == 1 && !(LONG && p.to_part)) {
            float * out = (float *) (p.dst + (size_t) (hb + h) * p.d1 + (size_t) iq1 * p.d2 + (size_t) iq3 * p.d3);
            out[d] = Lw == 0.f ? 0.f : O / Lw;
        } else if constexpr (LONG) {      // plain stores: the combine is a later launch
            part[h * (D + 2) + d] = O;
            if (d == 0) { part[h * (D + 2) + D] = Mw; part[h * (D + 2) + D + 1] = Lw; }
        } else {
            // agent-scope (write-through) stores: visible to every XCD once completed,
            // without the L2 writeback a __threadfence() release does
            __hip_atomic_store(part + h * (D + 2) + d, O, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (d == 0) {
                __hip_atomic_store(part + h * (D + 2) + D, Mw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(part + h * (D + 2) + D + 1, Lw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
    }
    MX_TRACE(tr, 5);
    MX_TRACE_BLK(p.trace_blk, 1);
    if (p.nsplit == 1 || LONG) return;

    // ---- split merge by the last workgroup of this (q row, KV head) to arrive
    __builtin_amdgcn_s_waitcnt(0);           // this thread's partial stores have completed
    __syncthreads();                         // ... and every thread's
    unsigned int * cnt = p.cnt + (iq3 * p.n_q + iq1) * slots + hslot;
    // acq_rel at agent scope: the release orders this workgroup's partial stores before the
    // count, the acquire makes every other split's partials visible to the last arrival
    // (the memory model's guarantee, not only the write-through stores' hardware behaviour)
    if (tid == 0) s_last = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == (unsigned) (p.nsplit - 1);
    __syncthreads();
    if (!s_last) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");   // every thread of the merging workgroup
    const float * pb = p.part + (size_t) ((iq3 * p.n_q + iq1) * slots + hslot) * p.nsplit * PW;
    auto ld = [](const float * a) { return __hip_atomic_load(a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); };
    // (max, sum) of every split in one parallel round trip, then per-split weights
    for (int i = tid; i < G * p.nsplit; i += NT) {
        const int h = i / p.nsplit, sp = i % p.nsplit;
        sM[h][sp] = ld(pb + (size_t) sp * PW + h * (D + 2) + D);
        sF[h][sp] = ld(pb + (size_t) sp * PW + h * (D + 2) + D + 1);
    }
    __syncthreads();
    if (tid < G) {
        float Mx = -INFINITY, Ls = 0.f;
        for (int sp = 0; sp < p.nsplit; ++sp) Mx = fmaxf(Mx, sM[tid][sp]);
        for (int sp = 0; sp < p.nsplit; ++sp) {
            const float f = sM[tid][sp] == -INFINITY ? 0.f : __builtin_amdgcn_exp2f(sM[tid][sp] - Mx);
            Ls += sF[tid][sp] * f;
            sM[tid][sp] = f;                 // now the weight of split sp
        }
        sL[tid] = Ls;
    }
    __syncthreads();
    for (int i = tid; i < G * D; i += NT) {
        const int h = i / D, d = i % D;
        float ov[FD_MAXSPLIT];
#pragma unroll
        for (int sp = 0; sp < FD_MAXSPLIT; ++sp)            // all loads in flight at once
            ov[sp] = sp < p.nsplit ? ld(pb + (size_t) sp * PW + h * (D + 2) + d) : 0.f;
        float O = 0.f;
#pragma unroll
        for (int sp = 0; sp < FD_MAXSPLIT; ++sp) if (sp < p.nsplit) O += sM[h][sp] * ov[sp];
        float * out = (float *) (p.dst + (size_t) (hb + h) * p.d1 + (size_t) iq1 * p.d2 + (size_t) iq3 * p.d3);
        out[d] = sL[h] == 0.f ? 0.f : O / sL[h];
    }
    if (tid == 0) __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // next launch / replay
}

// Merge of the LONG geometry's split partials: one workgroup per query head; the (max,
// sum) of every split first (threads over splits), then O = Σ_s w_s O_s with the four waves
// taking every fourth split and each lane D/64 dimensions (all of a wave's loads of a
// split in one instruction), the waves' sums added through LDS. Max in the log2 domain
// as the partials are. Replaces the looping in-launch merge for caches of > 16 chunks.
template <int D, int G>
__global__ __launch_bounds__(256) void k_fattn_dec2_combine(FaDecArgs p) {
    constexpr int PW = G * (D + 2), DPL = D / 64;
    extern __shared__ float wsp[];                            // [nsplit] split weights
    __shared__ float red[4][D], rm[4], rl[4];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int h = blockIdx.x % G, rs = blockIdx.x / G;        // rs = (iq3 n_q + iq1) slots + hslot
    const int Gt = p.H / p.Hkv, NGB = Gt / G, slots = p.Hkv * NGB;
    const int hslot = rs % slots, iq1 = (rs / slots) % p.n_q, iq3 = rs / (slots * p.n_q);
    const int hb = (hslot / NGB) * Gt + (hslot % NGB) * G;
    const float * pb = p.part + (size_t) rs * p.nsplit * PW + h * (D + 2);
    float m = -INFINITY;
    for (int sp = tid; sp < p.nsplit; sp += 256) m = fmaxf(m, pb[(size_t) sp * PW + D]);
    m = wave_max(m);
    if (lane == 0) rm[wave] = m;
    __syncthreads();
    const float Mx = fmaxf(fmaxf(rm[0], rm[1]), fmaxf(rm[2], rm[3]));
    float l = 0.f;
    for (int sp = tid; sp < p.nsplit; sp += 256) {
        const float ms = pb[(size_t) sp * PW + D];
        const float f = ms == -INFINITY ? 0.f : __builtin_amdgcn_exp2f(ms - Mx);
        wsp[sp] = f;
        l += f * pb[(size_t) sp * PW + D + 1];
    }
    l = wave_sum(l);
    if (lane == 0) rl[wave] = l;
    __syncthreads();
    const float L = (rl[0] + rl[1]) + (rl[2] + rl[3]);
    float o[DPL] = {};
#pragma unroll 8
    for (int sp = wave; sp < p.nsplit; sp += 4) {
        const float f = wsp[sp];
        const float * op = pb + (size_t) sp * PW + DPL * lane;
        if constexpr (DPL == 2) { const float2 v = *(const float2 *) op; o[0] += f * v.x; o[1] += f * v.y; }
        else o[0] += f * op[0];
    }
#pragma unroll
    for (int j = 0; j < DPL; ++j) red[wave][DPL * lane + j] = o[j];
    __syncthreads();
    if (tid < D) {
        const float O = (red[0][tid] + red[1][tid]) + (red[2][tid] + red[3][tid]);
        float * out = (float *) (p.dst + (size_t) (hb + h) * p.d1 + (size_t) iq1 * p.d2 + (size_t) iq3 * p.d3);
        out[tid] = L == 0.f ? 0.f : O / L;
    }
}

// eligibility: f16 K/V, D 64/128, GQA ratio 1-8, a plain f16 mask broadcast over heads,
// no softcap / ALiBi / sinks, few query rows (decode)
bool fa_dec2_will_run(const ggml_tensor * dst);   // ops_fattn.hip: op_flash_attn_ext's choice
bool fa_dec2_ok(const ggml_tensor * dst) {
    const ggml_tensor * q = dst->src[0], * k = dst->src[1], * v = dst->src[2], * m = dst->src[3];
    const bool kq = k->type == GGML_TYPE_Q8_0, vq = v->type == GGML_TYPE_Q8_0;
    if (q->ne[1] > 4 || !(k->type == GGML_TYPE_F16 || kq) || !(v->type == GGML_TYPE_F16 || vq)) return false;
    const int64_t D = k->ne[0];
    if ((D != 64 && D != 128) || v->ne[0] != D) return false;
    const int64_t G = q->ne[2] / k->ne[2];
    if (q->ne[2] % k->ne[2] || (G != 1 && G != 2 && G != 4 && G != 8)) return false;
    if (dst->src[4]) return false;                                        // sinks
    if (mx_op_param<float>(dst, 1) != 0.0f || mx_op_param<float>(dst, 2) != 0.0f) return false;   // ALiBi, softcap
    if (m && (m->type != GGML_TYPE_F16 || m->ne[2] > 1)) return false;
    // q8_0 rows: 2-byte aligned blocks, 8-byte loads at any 2-byte alignment; f16 rows: 16-B loads
    auto aligned = [](const ggml_tensor * t, bool q8) {
        const size_t a = q8 ? 2 : 16;
        return t->nb[1] % a == 0 && t->nb[2] % a == 0 && (uintptr_t) t->data % a == 0;
    };
    if (!aligned(k, kq) || !aligned(v, vq)) return false;
    if (q->nb[1] % 16 || q->nb[2] % 16 || (uintptr_t) q->data % 16) return false;
    if (q->ne[3] != k->ne[3] && k->ne[3] != 1) return false;
    // counters [0, MX_FA_CNT / 2): the upper half holds k_attn_o's row-chunk epochs (ops_attn_o.hip)
    if (k->ne[1] > INT32_MAX / 2 || q->ne[1] * q->ne[3] * q->ne[2] > MX_FA_CNT / 2) return false;
    // caches beyond one 16-wave chunk take the LONG geometry (fd_cfg); g_tune[10] = 4 keeps
    // them on the v1 kernel + combine (round-2 behaviour: 18.4 + 12.0 us at 16k keys)
    if (g_tune[10] == 4 && !kq && !vq && k->ne[1] > 16 * FD_NI * (64 / (D / 8))) return false;
    if (k->ne[1] > (int64_t) 32768 * 4 * 8 * (64 / (D / 8))) return false;   // FD_LONG_MAXSPLIT chunks
    return true;
}

// launch geometry: a cache that one 16-wave chunk covers (<= 256 keys at D 128, llama-
// bench tg128) runs as one split with ONE query head per workgroup (Hkv x Gt workgroups,
// K/V re-read from L2 by the GQA group): no split merge, whose publish / count / gather
// round trips cost ~4 us; longer caches use 4-wave workgroups over the whole GQA group
// and up to 16 splits merged in the same launch.
// LONG: 4-wave workgroups over min(Gt, 2) query heads (K/V read once per workgroup for
// those heads, from L2 by the group's other workgroup), 8 key rows per lane per chunk —
// 128 keys (64 KB of f16 K/V at D 128) in flight per workgroup, one chunk each.
struct FdCfg { int G, NW, nsplit; bool lng; int cpw = 1; };
constexpr int FD_LONG_NI = 8;
constexpr int FD_LONG_MAXSPLIT = 32768;   // the combine's split weights in LDS (128 KB): 4M keys at D 128
static FdCfg fd_cfg(int D, int Gt, int64_t n_kv, int64_t rows, int kv) {   // rows = Hkv x n_q x sequences; kv: fd_kv_code
    const int cs16 = 16 * FD_NI * (64 / (D / 8)), cs4 = 4 * FD_NI * (64 / (D / 8));
    // g_tune[1] = NI (2 / 4, experiment): short caches too take the LONG geometry — chunks of
    // 4 NI 64/(D/8) keys, one per workgroup, G = g_tune[29] (default 1) heads, plus the combine
    if (g_tune[1] && D == 128 && n_kv <= cs16 && n_kv > 4 * g_tune[1] * (64 / (D / 8))) {   // >= 2 splits
        const int g = g_tune[29] ? std::min(g_tune[29], Gt) : 1;
        return {g, 4, (int) mx_ceil_div(n_kv, 4 * g_tune[1] * (64 / (D / 8))), true};
    }
    if (g_tune[10] == 2 || (g_tune[10] != 3 && n_kv <= cs16)) return {1, 16, (int) mx_ceil_div(n_kv, cs16), false};
    if (g_tune[10] == 3) return {Gt, 4, (int) std::min<int64_t>(FD_MAXSPLIT, mx_ceil_div(n_kv, cs4)), false};
    // sweeps: g_tune[28] keys rows per lane (4 / 8 / 16), g_tune[29] heads per workgroup (D 128, f16)
    const int ni = D == 128 && g_tune[28] ? g_tune[28] : FD_LONG_NI;
    // two heads per workgroup measured best (fa_4096 7.7 vs 8.5 us for four, fa_16384 17.7
    // vs 18.5; profiles/r03/opbench_fa_long_sweep.txt)
    const int g = D == 128 && g_tune[29] ? std::min(g_tune[29], Gt) : std::min(Gt, 2);
    const int csl = 4 * ni * (64 / (D / 8));
    const int64_t nch = mx_ceil_div(n_kv, csl);
    // round 4 experiment, g_tune[2] = CPW (2 / 4 / 8): CPW chunks per workgroup, double-
    // buffered (chunk c+1's loads in flight while chunk c computes). Measured slower than one
    // chunk per workgroup at every length (opbench, profiles/r04/fa_long_cpw_ab.txt: 16k keys
    // 17.4 / 19.3 / 21.5 / 47 us for CPW 1 / 2 / 4 / 8; drop-in tg128 at depth 16384 354 -> 319
    // tok/s with CPW 4): with all chunks of all workgroups resident at once the loads are
    // already in flight together, and a second register buffer halves the waves per SIMD.
    int cpw = 1;
    (void) rows;
    if (g_tune[2] == 2 || g_tune[2] == 4 || g_tune[2] == 8) cpw = g_tune[2];
    if (ni != FD_LONG_NI || g > 2 || kv > 1) cpw = 1;         // (instantiated for the default NI, G <= 2, same K/V types)
    return {g, 4, (int) mx_ceil_div(nch, cpw), true, cpw};
}

static size_t fd3_scratch(const ggml_tensor * dst);
static bool fd3_run(OpCtx & c, ggml_tensor * dst);

// Round 6: the fused QKV launch's pending q8_0 row(s) (Stream::kvnew) belong to this
// attention when it reads exactly those caches, one token of one sequence
static bool fd_new_row_match(const KvNewRow & r, const ggml_tensor * fa) {
    const ggml_tensor * q = fa->src[0], * k = fa->src[1], * v = fa->src[2];
    if (!r.on || q->ne[1] != 1 || q->ne[3] != 1 || k->ne[3] != 1 || v->ne[3] != 1) return false;
    const int64_t D = k->ne[0];
    auto same = [&](const ggml_tensor * t, const char * base, size_t nb1, int n) {
        return t->type == GGML_TYPE_Q8_0 && (const char *) t->data == base && t->nb[1] == nb1 && t->nb[2] == (size_t) (D / 32) * 34 &&
               t->ne[0] * t->ne[2] == n;
    };
    if (r.k && !same(k, r.kc, r.kc_nb1, r.nk)) return false;
    if (r.v && !same(v, r.vc, r.vc_nb1, r.nv)) return false;
    // (a cache that took its row in the QKV launch must still be this attention's)
    if (!r.k && (const char *) k->data != r.kc) return false;
    if (!r.v && (const char *) v->data != r.vc) return false;
    return true;
}
bool fa_takes_new_row(const Stream * s, const ggml_tensor * fa) {
    return fa->op == GGML_OP_FLASH_ATTN_EXT && fd_new_row_match(s->kvnew, fa) && fa_dec2_will_run(fa);
}
static void fd_take_new_row(OpCtx & c, const ggml_tensor * dst, FaDecArgs & a) {
    KvNewRow & r = c.s->kvnew;
    if (!r.on) return;
    if (!fd_new_row_match(r, dst)) { kv_new_row_flush(c); return; }   // (the executor normally did)
    a.nr_k = r.k; a.nr_ik = r.kidx;
    a.nr_v = r.v; a.nr_iv = r.vidx;
    r.on = false;
}

size_t fa_dec2_scratch(const ggml_tensor * dst) {
    if (const size_t s3 = fd3_scratch(dst)) return s3;
    const ggml_tensor * q = dst->src[0], * k = dst->src[1];
    const int64_t D = k->ne[0];
    const FdCfg f = fd_cfg((int) D, (int) (q->ne[2] / k->ne[2]), k->ne[1], k->ne[2] * q->ne[1] * q->ne[3], fd_kv_code(k, dst->src[2]));
    return (size_t) (q->ne[1] * q->ne[3] * q->ne[2]) * (f.lng ? f.nsplit : std::min(f.nsplit, FD_MAXSPLIT)) * (D + 2) * sizeof(float) + 256;
}

// the LONG geometry's launch: every K/V type pair at one chunk per workgroup; the CPW > 1
// experiment (g_tune[2]) only for caches of one type (fd_cfg)
template <int DD, int GG, int CP>
static void fd_long_launch(int kv, dim3 grid, const FaDecArgs & a, hipStream_t st) {
    if constexpr (CP == 1) fd_kv_dispatch(kv, [&](auto KVC) { k_fattn_dec2<DD, GG, 4, decltype(KVC)::value, FD_LONG_NI, true, 1><<<grid, 256, 0, st>>>(a); });
    else if (kv == 1) k_fattn_dec2<DD, GG, 4, 1, FD_LONG_NI, true, CP><<<grid, 256, 0, st>>>(a);
    else k_fattn_dec2<DD, GG, 4, 0, FD_LONG_NI, true, CP><<<grid, 256, 0, st>>>(a);
}

void fa_dec2_run(OpCtx & c, ggml_tensor * dst) {
    if (fd3_run(c, dst)) return;                 // long caches: the streaming form (k_fattn_dec3)
    const ggml_tensor * q = dst->src[0], * k = dst->src[1], * v = dst->src[2], * m = dst->src[3];
    FaDecArgs a{};
    a.q = (const char *) q->data; a.q1 = q->nb[1]; a.q2 = q->nb[2]; a.q3 = q->nb[3];
    a.k = (const char *) k->data; a.k1 = k->nb[1]; a.k2 = k->nb[2]; a.k3 = k->nb[3];
    a.v = (const char *) v->data; a.v1 = v->nb[1]; a.v2 = v->nb[2]; a.v3 = v->nb[3];
    if (m) { a.mask = (const char *) m->data; a.m1 = m->nb[1]; a.m3 = m->nb[3]; a.mne3 = (int) m->ne[3]; }
    else a.mne3 = 1;
    a.dst = (char *) dst->data; a.d1 = dst->nb[1]; a.d2 = dst->nb[2]; a.d3 = dst->nb[3];
    a.n_q = (int) q->ne[1]; a.n_kv = (int) k->ne[1]; a.H = (int) q->ne[2]; a.Hkv = (int) k->ne[2];
    a.ns_kv = (int) k->ne[3];
    a.scale = mx_op_param<float>(dst, 0);
    const int D = (int) k->ne[0], Gt = a.H / a.Hkv;
    const FdCfg f = fd_cfg(D, Gt, a.n_kv, (int64_t) a.Hkv * a.n_q * q->ne[3], fd_kv_code(k, v));
    MX_ASSERT(f.lng ? f.nsplit <= 65535 : f.nsplit <= FD_MAXSPLIT);
    a.nsplit = f.nsplit;
    a.part = (float *) c.scratch->take(fa_dec2_scratch(dst));
    a.cnt = c.s->fa_cnt;
    fd_take_new_row(c, dst, a);
    a.trace = mx_trace_slot(0);
    a.trace_blk = mx_trace_blocks();
    const unsigned gx = (unsigned) (a.Hkv * (Gt / f.G) * a.n_q * q->ne[3]);
    unsigned pf_rows = 0;
    a.pf_n = c.s->pf_n;
    for (int r = 0; r < a.pf_n; ++r) {
        a.pf[r] = c.s->pf_ptr[r]; a.pf_eighth[r] = c.s->pf_len[r] / 8; a.pf_lines[r] = (unsigned) (c.s->pf_take[r] / 128);
    }
    // ~160 otherwise idle workgroups, first id and count multiples of 8 (XCD = id % 8)
    if (a.pf_n && (gx * a.nsplit) % 8 == 0) {
        pf_rows = (unsigned) mx_ceil_div(160, gx);
        while ((gx * pf_rows) % 8) ++pf_rows;
    } else a.pf_n = 0;
    const dim3 grid(gx, (unsigned) a.nsplit + pf_rows);
    const int kv = fd_kv_code(k, v);
    MX_KLOG("fattn_dec2 D=%d G=%d NW=%d nsplit=%d n_kv=%d H=%d Hkv=%d kq8=%d vq8=%d pf_rows=%u long=%d cpw=%d newrow=%d", D, f.G, f.NW,
            f.nsplit, a.n_kv, a.H, a.Hkv, (int) fd_kq(kv), (int) fd_vq(kv), pf_rows, (int) f.lng, f.cpw, (int) (a.nr_k || a.nr_v));
    if (f.lng) {
        const unsigned gc = gx * (unsigned) f.G;                     // one combine workgroup per query head
        const size_t lds = (size_t) f.nsplit * sizeof(float);
#define FLC(DD, GG, CP) if (f.cpw == CP) fd_long_launch<DD, GG, CP>(kv, grid, a, c.st);
#define FLW(DD, GG, CPWS) if (D == DD && f.G == GG) { \
            CPWS \
            MX_LDS_OPTIN((k_fattn_dec2_combine<DD, GG>), FD_LONG_MAXSPLIT * (int) sizeof(float)); \
            k_fattn_dec2_combine<DD, GG><<<gc, 256, lds, c.st>>>(a); \
            return; }
        const int ni = D == 128 && g_tune[1] && a.n_kv <= 16 * FD_NI * (64 / (D / 8)) && a.n_kv > 4 * g_tune[1] * (64 / (D / 8)) ? g_tune[1] :
                       D == 128 && g_tune[28] ? g_tune[28] : FD_LONG_NI;
        if (ni != FD_LONG_NI && kv == 0) {   // sweep geometries (f16, D 128)
#define FS(NI_, GG) if (ni == NI_ && f.G == GG) { \
                k_fattn_dec2<128, GG, 4, false, NI_, true><<<grid, 256, 0, c.st>>>(a); \
                k_fattn_dec2_combine<128, GG><<<gc, 256, lds, c.st>>>(a); return; }
            FS(2, 1) FS(2, 2) FS(4, 1) FS(4, 2) FS(4, 4) FS(16, 1) FS(16, 2) FS(16, 4)
#undef FS
        }
        if (ni == 16 && kv != 0 && D == 128 && f.G == 2) {   // sweep: 16 key rows per lane, quantised caches
            fd_kv_dispatch(kv, [&](auto KVC) { k_fattn_dec2<128, 2, 4, decltype(KVC)::value, 16, true><<<grid, 256, 0, c.st>>>(a); });
            k_fattn_dec2_combine<128, 2><<<gc, 256, lds, c.st>>>(a);
            return;
        }
        // fd_cfg sized the splits for `ni` keys rows per lane: a kernel of another NI would
        // cover only part of the cache (a sweep knob outside the instantiated set)
        MX_ASSERT(ni == FD_LONG_NI);
#define CPW4(DD, GG) FLC(DD, GG, 2) else FLC(DD, GG, 4) else FLC(DD, GG, 8) else FLC(DD, GG, 1)
        FLW(128, 1, CPW4(128, 1)) FLW(128, 2, CPW4(128, 2)) FLW(128, 4, FLC(128, 4, 1))
        FLW(64, 1, CPW4(64, 1)) FLW(64, 2, CPW4(64, 2)) FLW(64, 4, FLC(64, 4, 1))
#undef CPW4
#undef FLW
#undef FLC
        MX_ABORT("fattn dec2 long D=%d G=%d", D, f.G);
    }
#define FD(DD, GG, NWW) if (D == DD && f.G == GG && f.NW == NWW) { \
        fd_kv_dispatch(kv, [&](auto KVC) { k_fattn_dec2<DD, GG, NWW, decltype(KVC)::value><<<grid, 64 * NWW, 0, c.st>>>(a); }); \
        return; }
    FD(128, 1, 16) FD(64, 1, 16)
    FD(128, 4, 4) FD(128, 1, 4) FD(128, 2, 4) FD(128, 8, 4) FD(64, 1, 4) FD(64, 2, 4) FD(64, 4, 4) FD(64, 8, 4)
#undef FD
    MX_ABORT("fattn dec2 D=%d G=%d NW=%d", D, f.G, f.NW);
}

// Round 5: decode attention whose split partials the output projection merges in its
// prologue (exec.cpp fuse_attn_split_o, XStage::fap). At llama-bench tg128 (256 keys) the
// one-split form ran 32 workgroups of 16 waves, each pulling 128 KB of K/V through one
// CU (~6.5 us per layer, 82 % of wave time parked on waits); the LONG geometry with 64-key
// chunks runs Hkv x Gt x 4 four-wave workgroups with 32 KB each, and its (O, max, sum)
// partials need no combine launch (~4 us, profiles/r04/fa256_split_ab.txt) because the
// output projection's 256 workgroups merge them while their weight loads are in flight.
// Partial layout (G = 1): head hh, split s at part + (hh * nsplit + s) * (D + 2).
static int fa_split_ni() {   // key rows per lane per chunk: 4 (64-key chunks), 2 (32) or 8 (128); g_tune[33]
    static const int ni = [] { const char * v = getenv("GGML_MI355X_FA_SPLIT_NI"); const int n = v ? atoi(v) : 4; return n == 2 || n == 8 ? n : 4; }();
    return g_tune[33] == 2 || g_tune[33] == 4 || g_tune[33] == 8 ? g_tune[33] : ni;
}
int fa_dec2_partials_nsplit(const ggml_tensor * fa) {
    const ggml_tensor * q = fa->src[0], * k = fa->src[1];
    if (!fa_dec2_ok(fa) || k->ne[0] != 128 || q->ne[1] != 1 || q->ne[3] != 1 || k->ne[3] != 1) return 0;
    if (fa->src[3] && fa->src[3]->ne[3] != 1) return 0;
    const int64_t cs = 4 * fa_split_ni() * 4;                   // 4 waves x NI rows x 4 keys per instruction
    const int64_t ns = mx_ceil_div(k->ne[1], cs);
    return ns >= 1 && ns <= 8 ? (int) ns : 0;
}
void fa_dec2_partials(OpCtx & c, ggml_tensor * dst, float * part, int nsplit) {
    const ggml_tensor * q = dst->src[0], * k = dst->src[1], * v = dst->src[2], * m = dst->src[3];
    FaDecArgs a{};
    a.q = (const char *) q->data; a.q1 = q->nb[1]; a.q2 = q->nb[2]; a.q3 = q->nb[3];
    a.k = (const char *) k->data; a.k1 = k->nb[1]; a.k2 = k->nb[2]; a.k3 = k->nb[3];
    a.v = (const char *) v->data; a.v1 = v->nb[1]; a.v2 = v->nb[2]; a.v3 = v->nb[3];
    if (m) { a.mask = (const char *) m->data; a.m1 = m->nb[1]; a.m3 = m->nb[3]; a.mne3 = (int) m->ne[3]; }
    else a.mne3 = 1;
    a.dst = (char *) dst->data; a.d1 = dst->nb[1]; a.d2 = dst->nb[2]; a.d3 = dst->nb[3];
    a.n_q = 1; a.n_kv = (int) k->ne[1]; a.H = (int) q->ne[2]; a.Hkv = (int) k->ne[2];
    a.ns_kv = 1;
    a.scale = mx_op_param<float>(dst, 0);
    a.nsplit = nsplit;
    a.part = part;
    a.to_part = 1;
    a.cnt = c.s->fa_cnt;
    fd_take_new_row(c, dst, a);
    a.trace = mx_trace_slot(0);
    a.trace_blk = mx_trace_blocks();
    const unsigned gx = (unsigned) a.H;                          // G = 1: one query head per workgroup
    unsigned pf_rows = 0;
    // the gate/up weight prefetch rows (exec.cpp fa_prefetch_plan) only on request
    // (GGML_MI355X_FA_PREFETCH_MB or g_tune[23] > 0): this launch is short enough that the
    // default 16 MB outlasts it — same box, drop-in tg128 630 (16 MB) / 640 (8) / 644 tok/s
    // without (profiles/r05/fa_split_prefetch_ab.txt)
    static const bool pf_env = getenv("GGML_MI355X_FA_PREFETCH_MB") != nullptr;
    a.pf_n = pf_env || g_tune[23] > 0 ? c.s->pf_n : 0;
    for (int r = 0; r < a.pf_n; ++r) {
        a.pf[r] = c.s->pf_ptr[r]; a.pf_eighth[r] = c.s->pf_len[r] / 8; a.pf_lines[r] = (unsigned) (c.s->pf_take[r] / 128);
    }
    if (a.pf_n && (gx * a.nsplit) % 8 == 0) {   // ~160 prefetch workgroups (see fa_dec2_run)
        pf_rows = (unsigned) mx_ceil_div(160, gx);
        while ((gx * pf_rows) % 8) ++pf_rows;
    } else a.pf_n = 0;
    const dim3 grid(gx, (unsigned) a.nsplit + pf_rows);
    const int kv = fd_kv_code(k, v);
    const int ni = fa_split_ni();
    MX_KLOG("fattn_dec2_part D=128 G=1 NI=%d nsplit=%d n_kv=%d H=%d Hkv=%d kq8=%d vq8=%d pf_rows=%u newrow=%d", ni, nsplit, a.n_kv, a.H,
            a.Hkv, (int) fd_kq(kv), (int) fd_vq(kv), pf_rows, (int) (a.nr_k || a.nr_v));
    if (ni == 2) fd_kv_dispatch(kv, [&](auto KVC) { k_fattn_dec2<128, 1, 4, decltype(KVC)::value, 2, true><<<grid, 256, 0, c.st>>>(a); });
    else if (ni == 8) fd_kv_dispatch(kv, [&](auto KVC) { k_fattn_dec2<128, 1, 4, decltype(KVC)::value, 8, true><<<grid, 256, 0, c.st>>>(a); });
    else fd_kv_dispatch(kv, [&](auto KVC) { k_fattn_dec2<128, 1, 4, decltype(KVC)::value, 4, true><<<grid, 256, 0, c.st>>>(a); });
}

// ---------------------------------------------------------------------------
// Round 5: long-context decode attention as a stream (k_fattn_dec3). The LONG geometry
// above gives every workgroup one 128-key chunk held in registers (124 VGPRs: 4 waves per
// SIMD), so 16k keys x 8 KV heads x 2 head pairs ran as two rounds of 1,024 workgroups
// that all issue, wait, compute and leave together, and its 128 partials per head needed
// a combine launch: 20.7 + 5.0 us per layer at depth 16384 (0.40 of HBM).
// Here one workgroup per CU (Hkv x NS of them, ~256) streams a contiguous key range of
// one KV head for ALL Gt query heads of its GQA group (K/V read once), through an LDS ring
// filled by LDS-DMA (global_load_lds, no registers held): each wave owns its own slots of
// the ring — it DMAs and later reads back only its own 16-key wave-stages — so the loop has
// no barrier, only per-wave vmcnt waits, with S - 1 wave-stages (3 x 8 KB) ahead per wave.
// Splits merge in the same launch (agent-scope partial stores, the last of a KV head's NS
// workgroups to arrive combines, as k_fattn_dec2's short-cache form): no combine launch.
// Semantics as k_fattn_dec2 (f16 K/V, D 128, log2-domain online softmax).
// ---------------------------------------------------------------------------
constexpr int FD3_SK = 16;                 // keys per wave-stage: 4 DMA rows x 4 keys
constexpr int FD3_MAXNS = 64;              // splits per KV head (merge weights in LDS)
constexpr int FD3_WST = 2 * 4 * 64 + 16;   // uint4 per wave-stage: K 4 KB, V 4 KB, mask 256 B

template <int N>
__device__ __forceinline__ void fd3_wait_vm() {   // s_waitcnt vmcnt(N) alone
    static_assert(N >= 0 && N < 64, "vmcnt range");
    __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}
typedef __attribute__((address_space(3))) void * fd3_lds_t;
typedef uint32_t v4u_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint32_t fd3_lds_off(const void * p) {
    return (uint32_t) (uintptr_t) (const __attribute__((address_space(3))) char *) p;
}

template <int G, int NW, int S>
__global__ __launch_bounds__(64 * NW) void k_fattn_dec3(FaDecArgs p, int kps) {
    constexpr int D = 128, LPK = 16, KPI = 4, NI = 4, NT = 64 * NW;
    static_assert(S >= 2 && S <= 4, "ring depth");
    typedef _Float16 h2v __attribute__((ext_vector_type(2)));
    extern __shared__ __align__(16) uint4 ring[];            // [NW][S][FD3_WST]
    __shared__ float wm[NW][G], wl[NW][G];
    __shared__ int s_last;
    float (*wo)[G][D] = (float (*)[G][D]) ring;               // after the loop: the waves' O (ring reused)

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int c = lane % LPK, kq = lane / LPK;
    const int hk = blockIdx.x % p.Hkv, split = blockIdx.x / p.Hkv;
    const int Gt = p.H / p.Hkv, hb = hk * Gt;
    const char * kb = p.k + (size_t) hk * p.k2 + c * 16;
    const char * vb = p.v + (size_t) hk * p.v2 + c * 16;
    const char * mrow = p.mask ? p.mask : p.k;               // (no mask: loads land unused)
    const int ks0 = split * kps, nj = kps / (FD3_SK * NW);   // this wave's wave-stages
    uint4 * my = ring + wave * S * FD3_WST;
    unsigned long long * tr = blockIdx.x == 0 ? p.trace : nullptr;
    MX_TRACE(tr, 0);
    MX_TRACE_BLK(p.trace_blk, 0);

    auto key0_of = [&](int j) { return ks0 + (j * NW + wave) * FD3_SK; };
    // wave-stage j into slot j % S: 4 K rows-of-4, 4 V rows-of-4, the 16 mask values
    // (lanes 0-7 one dword each; the others repeat lane 7's) — 9 DMA instructions
    auto issue = [&](int j) {
        uint4 * st = my + (j % S) * FD3_WST;
        const int key0 = key0_of(j);
#pragma unroll
        for (int t = 0; t < NI; ++t) {
            const size_t r = (size_t) min(key0 + t * KPI + kq, p.n_kv - 1);
            __builtin_amdgcn_global_load_lds(kb + r * p.k1, (fd3_lds_t) (st + t * 64), 16, 0, 0);
        }
#pragma unroll
        for (int t = 0; t < NI; ++t) {
            const size_t r = (size_t) min(key0 + t * KPI + kq, p.n_kv - 1);
            __builtin_amdgcn_global_load_lds(vb + r * p.v1, (fd3_lds_t) (st + 256 + t * 64), 16, 0, 0);
        }
        const int mk = min(key0 + 2 * min(lane, 7), p.n_kv - 2);   // (n_kv even: fd3_cfg)
        __builtin_amdgcn_global_load_lds(mrow + (size_t) mk * 2, (fd3_lds_t) (st + 512), 4, 0, 0);
    };

    float M[G], L[G], o[G][8];
#pragma unroll
    for (int h = 0; h < G; ++h) {
        M[h] = -INFINITY; L[h] = 0.f;
#pragma unroll
        for (int i = 0; i < 8; ++i) o[h][i] = 0.f;
    }
#pragma unroll
    for (int j = 0; j < S - 1; ++j) if (j < nj) issue(j);
    // q of the G heads, rounded to f16 (the K vec-dot type), loaded behind the ring's first
    // stages (loaded first, its conversion held the DMA issue back one memory latency)
    asm volatile("" ::: "memory");
    h2v qh[G][4];
#pragma unroll
    for (int h = 0; h < G; ++h) {
        const float * qp = (const float *) (p.q + (size_t) (hb + h) * p.q2) + 8 * c;
        const float4 a = *(const float4 *) qp, b = *(const float4 *) (qp + 4);
        qh[h][0] = h2v{(_Float16) a.x, (_Float16) a.y}; qh[h][1] = h2v{(_Float16) a.z, (_Float16) a.w};
        qh[h][2] = h2v{(_Float16) b.x, (_Float16) b.y}; qh[h][3] = h2v{(_Float16) b.z, (_Float16) b.w};
    }
    MX_TRACE(tr, 1);
    for (int j = 0; j < nj; ++j) {
        if (j + S - 1 < nj) issue(j + S - 1);
        const int rem = min(nj - 1 - j, S - 1);             // wave-stages issued after j
        if (rem >= 3) fd3_wait_vm<27>();
        else if (rem == 2) fd3_wait_vm<18>();
        else if (rem == 1) fd3_wait_vm<9>();
        else fd3_wait_vm<0>();
        asm volatile("" ::: "memory");
        if (j == 0) MX_TRACE(tr, 2);
        const uint4 * st = my + (j % S) * FD3_WST;
        const int key0 = key0_of(j);
        // the wave-stage back from LDS in one batch (inline asm: through plain loads the
        // compiler puts a vmcnt(0) for the LDS-DMA in front of them, draining the ring)
        uint4 kr[NI], vr[NI];
        float mk[NI];
        {
            v4u_t a0, a1, a2, a3, b0, b1, b2, b3;
            uint32_t m0, m1, m2, m3;
            const uint32_t ad = fd3_lds_off(st + lane), am = fd3_lds_off(st + 512) + 2 * kq;
            asm volatile("ds_read_b128 %0, %12\n\tds_read_b128 %1, %12 offset:1024\n\tds_read_b128 %2, %12 offset:2048\n\t"
                         "ds_read_b128 %3, %12 offset:3072\n\tds_read_b128 %4, %12 offset:4096\n\tds_read_b128 %5, %12 offset:5120\n\t"
                         "ds_read_b128 %6, %12 offset:6144\n\tds_read_b128 %7, %12 offset:7168\n\tds_read_u16 %8, %13\n\t"
                         "ds_read_u16 %9, %13 offset:8\n\tds_read_u16 %10, %13 offset:16\n\tds_read_u16 %11, %13 offset:24\n\t"
                         "s_waitcnt lgkmcnt(0)"
                         : "=&v"(a0), "=&v"(a1), "=&v"(a2), "=&v"(a3), "=&v"(b0), "=&v"(b1), "=&v"(b2), "=&v"(b3),
                           "=&v"(m0), "=&v"(m1), "=&v"(m2), "=&v"(m3)
                         : "v"(ad), "v"(am) : "memory");
            const v4u_t av[NI] = {a0, a1, a2, a3}, bv[NI] = {b0, b1, b2, b3};
            const uint32_t mr[NI] = {m0, m1, m2, m3};
#pragma unroll
            for (int t = 0; t < NI; ++t) {
                kr[t] = make_uint4(av[t][0], av[t][1], av[t][2], av[t][3]);
                vr[t] = make_uint4(bv[t][0], bv[t][1], bv[t][2], bv[t][3]);
                const int key = key0 + t * KPI + kq;
                mk[t] = key < p.n_kv ? (p.mask ? h2f((uint16_t) mr[t]) : 0.f) : -INFINITY;
            }
        }
        float s[G][NI];
#pragma unroll
        for (int t = 0; t < NI; ++t)
#pragma unroll
            for (int h = 0; h < G; ++h) {
                float acc = __builtin_amdgcn_fdot2(__builtin_bit_cast(h2v, kr[t].x), qh[h][0], 0.f, false);
                acc = __builtin_amdgcn_fdot2(__builtin_bit_cast(h2v, kr[t].y), qh[h][1], acc, false);
                acc = __builtin_amdgcn_fdot2(__builtin_bit_cast(h2v, kr[t].z), qh[h][2], acc, false);
                acc = __builtin_amdgcn_fdot2(__builtin_bit_cast(h2v, kr[t].w), qh[h][3], acc, false);
                acc = dpp_sum_group<LPK>(acc);
                s[h][t] = mk[t] == -INFINITY ? -INFINITY : (acc * p.scale + mk[t]) * 1.4426950408889634f;
            }
        float vf[NI][8];
#pragma unroll
        for (int t = 0; t < NI; ++t) {
            const uint32_t vw[4] = {vr[t].x, vr[t].y, vr[t].z, vr[t].w};
#pragma unroll
            for (int i = 0; i < 4; ++i) { vf[t][2 * i] = h2f((uint16_t) (vw[i] & 0xFFFF)); vf[t][2 * i + 1] = h2f((uint16_t) (vw[i] >> 16)); }
        }
#pragma unroll
        for (int h = 0; h < G; ++h) {
            float mc = s[h][0];
#pragma unroll
            for (int t = 1; t < NI; ++t) mc = fmaxf(mc, s[h][t]);
            mc = kr_max<LPK>(mc);
            const float Mn = fmaxf(M[h], mc);
            const float a = M[h] == -INFINITY ? 0.f : __builtin_amdgcn_exp2f(M[h] - Mn);
            float pr[NI], lc = 0.f;
#pragma unroll
            for (int t = 0; t < NI; ++t) { pr[t] = Mn == -INFINITY ? 0.f : __builtin_amdgcn_exp2f(s[h][t] - Mn); lc += pr[t]; }
            lc = kr_sum<LPK>(lc);
            L[h] = L[h] * a + lc;
            M[h] = Mn;
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                float v = o[h][i] * a;
#pragma unroll
                for (int t = 0; t < NI; ++t) v += pr[t] * vf[t][i];
                o[h][i] = v;
            }
        }
    }
    MX_TRACE(tr, 3);
    __syncthreads();                                          // every wave is done with its ring slots
    // the NW waves' (O, M, L) -> this split's partial
#pragma unroll
    for (int h = 0; h < G; ++h) {
#pragma unroll
        for (int i = 0; i < 8; ++i) o[h][i] = kr_sum<LPK>(o[h][i]);
        if (lane == 0) { wm[wave][h] = M[h]; wl[wave][h] = L[h]; }
        if (kq == 0) {
            *(float4 *) &wo[wave][h][8 * c] = make_float4(o[h][0], o[h][1], o[h][2], o[h][3]);
            *(float4 *) &wo[wave][h][8 * c + 4] = make_float4(o[h][4], o[h][5], o[h][6], o[h][7]);
        }
    }
    __syncthreads();
    constexpr int PW = G * (D + 2);
    const int ns = p.nsplit;
    float * part = p.part + ((size_t) hk * ns + split) * PW;
    for (int i = tid; i < G * D; i += NT) {
        const int h = i / D, d = i % D;
        float Mw = wm[0][h];
#pragma unroll
        for (int w = 1; w < NW; ++w) Mw = fmaxf(Mw, wm[w][h]);
        float Lw = 0.f, O = 0.f;
#pragma unroll
        for (int w = 0; w < NW; ++w) {
            const float f = wm[w][h] == -INFINITY ? 0.f : __builtin_amdgcn_exp2f(wm[w][h] - Mw);
            Lw += wl[w][h] * f;
            O += wo[w][h][d] * f;
        }
        if (ns == 1) {
            ((float *) (p.dst + (size_t) (hb + h) * p.d1))[d] = Lw == 0.f ? 0.f : O / Lw;
            continue;
        }
        // agent-scope (write-through) stores: visible to every XCD once completed
        __hip_atomic_store(part + h * (D + 2) + d, O, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (d == 0) {   // (max, sum) as one 8-byte store: the merge reads them as one
            const uint64_t ml = (uint64_t) __float_as_uint(Mw) | ((uint64_t) __float_as_uint(Lw) << 32);
            __hip_atomic_store((uint64_t *) (part + h * (D + 2) + D), ml, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    MX_TRACE_BLK(p.trace_blk, 1);
    if (ns == 1) return;
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    MX_TRACE(tr, 4);
    unsigned int * cnt = p.cnt + hk;
    // relaxed count: the partials went out as agent-scope (write-through) atomic stores and
    // have completed (waitcnt above); the merge reads them back with agent-scope loads. An
    // acq_rel count adds an L2 writeback (buffer_wbl2) to every workgroup and an L2
    // invalidate to the merging one, ~2 us of this launch's tail.
    // Hardware assumption (gfx950, coarse-grained device memory): an agent-scope atomic
    // store is written through the XCD's L2 to the device coherence point and s_waitcnt
    // vmcnt(0) returns only once it is there; an agent-scope atomic load reads that point.
    // Every byte the merge reads is such a store, so no fence is needed for them — only for
    // ordinary stores, which this protocol never relies on. Pinned by
    // tests/test_ops_gpu.py::test_flash_attn_stream_merge_visibility (64K keys, 24 runs).
    if (tid == 0) s_last = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (unsigned) (ns - 1);
    __syncthreads();
    if (!s_last) return;
    // the merge in ONE memory round trip per 8 splits of a wave: wave w takes splits w,
    // w + NW, ...; each lane loads (O of its 2 dimensions, max, sum) of every head for all of
    // them at once, merges them under the wave's own max, and the NW wave results merge
    // through LDS (a first version loaded the maxima, then the sums one split at a time,
    // then O: ~30 dependent round trips, 33 us per launch at 16k keys)
    const float * pb = p.part + (size_t) hk * ns * PW;
    auto ld2 = [](const float * a) {      // two adjacent floats (8-byte aligned) in one agent-scope load
        const uint64_t v = __hip_atomic_load((const uint64_t *) a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return make_float2(__uint_as_float((uint32_t) v), __uint_as_float((uint32_t) (v >> 32)));
    };
    float wmx[G], wls[G], acc[G][2];
#pragma unroll
    for (int h = 0; h < G; ++h) { wmx[h] = -INFINITY; wls[h] = 0.f; acc[h][0] = acc[h][1] = 0.f; }
    for (int s0 = wave; s0 < ns; s0 += 8 * NW) {           // wave-uniform
        float vo[8][G][2], vm[8][G], vl[8][G];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const float * ps = pb + (size_t) min(s0 + u * NW, ns - 1) * PW;
#pragma unroll
            for (int h = 0; h < G; ++h) {
                const float2 o2 = ld2(ps + h * (D + 2) + 2 * lane), ml = ld2(ps + h * (D + 2) + D);
                vo[u][h][0] = o2.x; vo[u][h][1] = o2.y;
                vm[u][h] = ml.x; vl[u][h] = ml.y;
            }
        }
#pragma unroll
        for (int h = 0; h < G; ++h) {
            float mn = wmx[h];
#pragma unroll
            for (int u = 0; u < 8; ++u) if (s0 + u * NW < ns) mn = fmaxf(mn, vm[u][h]);
            const float a = wmx[h] == -INFINITY ? 0.f : __builtin_amdgcn_exp2f(wmx[h] - mn);
            float l = wls[h] * a, o0 = acc[h][0] * a, o1 = acc[h][1] * a;
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const float f = s0 + u * NW < ns && vm[u][h] != -INFINITY ? __builtin_amdgcn_exp2f(vm[u][h] - mn) : 0.f;
                l += f * vl[u][h];
                o0 += f * vo[u][h][0];
                o1 += f * vo[u][h][1];
            }
            wmx[h] = mn; wls[h] = l; acc[h][0] = o0; acc[h][1] = o1;
        }
    }
    // (every wave has >= 1 split: ns >= NW is not guaranteed — empty waves carry -inf / 0)
#pragma unroll
    for (int h = 0; h < G; ++h) {
        if (lane == 0) { wm[wave][h] = wmx[h]; wl[wave][h] = wls[h]; }
        *(float2 *) &wo[wave][h][2 * lane] = make_float2(acc[h][0], acc[h][1]);
    }
    __syncthreads();
    for (int i = tid; i < G * D; i += NT) {
        const int h = i / D, d = i % D;
        float Mx = wm[0][h];
#pragma unroll
        for (int w = 1; w < NW; ++w) Mx = fmaxf(Mx, wm[w][h]);
        float Ls = 0.f, O = 0.f;
#pragma unroll
        for (int w = 0; w < NW; ++w) {
            const float f = wm[w][h] == -INFINITY ? 0.f : __builtin_amdgcn_exp2f(wm[w][h] - Mx);
            Ls += wl[w][h] * f;
            O += wo[w][h][d] * f;
        }
        ((float *) (p.dst + (size_t) (hb + h) * p.d1))[d] = Ls == 0.f ? 0.f : O / Ls;
    }
    if (tid == 0) __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // next launch / replay
    MX_TRACE(tr, 5);
    MX_TRACE_BLK(p.trace_blk, 1);                             // (the merging workgroup: its end after the merge)
}

// geometry: ~256 workgroups (one per CU), NS splits per KV head of kps keys each (a whole
// number of 16 x NW-key workgroup stages). GGML_MI355X_FA_STREAM=0 / g_tune[39] = 1 off;
// g_tune[35] = minimum cache length in units of 256 keys (default 16384 keys).
struct Fd3Cfg { int ns = 0, kps = 0, nw = 4, st = 4; };
// geometry: 4 waves x 4 ring stages (one wave per SIMD), or g_tune[37] = 1: 8 waves x 2
// stages (two waves per SIMD: a lone wave issues VALU at half the SIMD's rate, and the
// loop is VALU-bound — 0.56 of wave time issuing, pmc_decode_d16384_sq.json)
static int fd3_geom() {
    static const int env = [] { const char * v = getenv("GGML_MI355X_FA_STREAM_GEOM"); return v ? atoi(v) : 0; }();
    return g_tune[37] ? g_tune[37] : env;
}
static Fd3Cfg fd3_cfg(const ggml_tensor * dst) {
    static const bool off = [] { const char * v = getenv("GGML_MI355X_FA_STREAM"); return v && !strcmp(v, "0"); }();
    const ggml_tensor * q = dst->src[0], * k = dst->src[1], * v = dst->src[2], * m = dst->src[3];
    if (off || g_tune[39] == 1 || !fa_dec2_ok(dst)) return {};
    if (k->type != GGML_TYPE_F16 || v->type != GGML_TYPE_F16 || k->ne[0] != 128 || q->ne[1] != 1 || q->ne[3] != 1 || k->ne[3] != 1) return {};
    if (m && (m->ne[3] != 1 || (uintptr_t) m->data % 4 || m->nb[1] % 4)) return {};
    const int64_t n_kv = k->ne[1], Hkv = k->ne[2];
    // (from 16384 keys: the LONG kernel + combine measured better at -d 4096 (547 vs 529
    // tok/s) and -d 8192 (511.6 vs 498.2), this form at -d 16384 (453 vs 449.5) — same-box
    // passes on two boxes, profiles/r05/fa_stream_ab.txt)
    const int64_t min_kv = g_tune[35] > 0 ? (int64_t) g_tune[35] * 256 : 16384;
    if (n_kv < min_kv || n_kv % 2 || Hkv > MX_FA_CNT / 2) return {};
    const int nw = fd3_geom() == 1 ? 8 : 4, st = fd3_geom() == 1 ? 2 : 4;
    const int64_t wst = FD3_SK * nw;
    int64_t ns = std::max<int64_t>(1, 256 / Hkv);
    ns = std::min<int64_t>({ns, FD3_MAXNS, mx_ceil_div(n_kv, wst)});
    const int64_t kps = mx_ceil_div(mx_ceil_div(n_kv, ns), wst) * wst;
    return {(int) mx_ceil_div(n_kv, kps), (int) kps, nw, st};
}

static size_t fd3_scratch(const ggml_tensor * dst) {
    const Fd3Cfg f = fd3_cfg(dst);
    return f.ns ? (size_t) dst->src[0]->ne[2] * f.ns * (128 + 2) * sizeof(float) + 256 : 0;
}

static bool fd3_run(OpCtx & c, ggml_tensor * dst) {
    const Fd3Cfg f = fd3_cfg(dst);
    if (!f.ns) return false;
    const ggml_tensor * q = dst->src[0], * k = dst->src[1], * v = dst->src[2], * m = dst->src[3];
    FaDecArgs a{};
    a.q = (const char *) q->data; a.q2 = q->nb[2];
    a.k = (const char *) k->data; a.k1 = k->nb[1]; a.k2 = k->nb[2];
    a.v = (const char *) v->data; a.v1 = v->nb[1]; a.v2 = v->nb[2];
    if (m) a.mask = (const char *) m->data;
    a.dst = (char *) dst->data; a.d1 = dst->nb[1];
    a.n_q = 1; a.n_kv = (int) k->ne[1]; a.H = (int) q->ne[2]; a.Hkv = (int) k->ne[2]; a.ns_kv = 1;
    a.scale = mx_op_param<float>(dst, 0);
    a.nsplit = f.ns;
    a.part = (float *) c.scratch->take(fd3_scratch(dst));
    a.cnt = c.s->fa_cnt;
    a.trace = mx_trace_slot(0);
    a.trace_blk = mx_trace_blocks();
    const int Gt = a.H / a.Hkv;
    const dim3 grid((unsigned) (a.Hkv * f.ns));
    const size_t lds = (size_t) f.nw * f.st * FD3_WST * 16;
    MX_KLOG("fattn_dec3 D=128 G=%d ns=%d kps=%d n_kv=%d H=%d Hkv=%d nw=%d", Gt, f.ns, f.kps, a.n_kv, a.H, a.Hkv, f.nw);
#define F3(GG, NWW, SS) if (Gt == GG && f.nw == NWW) { \
        MX_LDS_OPTIN((k_fattn_dec3<GG, NWW, SS>), lds); \
        k_fattn_dec3<GG, NWW, SS><<<grid, 64 * NWW, lds, c.st>>>(a, f.kps); return true; }
    F3(1, 4, 4) F3(2, 4, 4) F3(4, 4, 4) F3(8, 4, 4)
    F3(1, 8, 2) F3(2, 8, 2) F3(4, 8, 2) F3(8, 8, 2)
#undef F3
    return false;
}

// ---------------------------------------------------------------------------
// Non-flash-attention decode (llama-bench's default -fa 0): build_attn_mha's chain
// MUL_MAT(k, q) -> SOFT_MAX(mask, scale) -> MUL_MAT(v, kq) -> PERMUTE -> CONT
// (src/llama-graph.cpp:1740-1796) for one query token in ONE launch instead of four
// (2 dense GEMVs of 7.5 us, the softmax and the copy: 24.8 us per layer in the -fa 0
// drop-in profile). One workgroup per query head. Semantics per node: kq = f16(q)·k (the
// first mul_mat converts q to K's vec_dot_type f16), softmax over the row in f32
// (x·scale + mask, exp(x - max), times 1/sum), kqv = f16(p)·v (the second mul_mat
// converts p to f16), f32 accumulation. V is the transposed cache view: one contiguous
// row of n_kv values per dimension.
struct NfArgs {
    const char * q; size_t q2;          // q [D, 1, H] f32: head stride (bytes)
    const char * k; size_t k1, k2;      // k [D, n_kv, Hkv] f16: key stride, head stride
    const char * v; size_t v1, v2;      // v [n_kv, D, Hkv] f16: dimension stride, head stride
    const char * mask; int mask_f16;    // the token's mask row [n_kv] (f16 or f32), nullable
    float * dst;                        // [H * D]
    int n_kv, H, Hkv;
    float scale;
    const char * pf[4]; size_t pf_eighth[4]; unsigned pf_lines[4]; int pf_n;   // as FaDecArgs
};

constexpr int NF_NI = 8;                // key rows per lane in flight
constexpr int NF_MAX_KV = 16384;        // scores in LDS: 64 KB dynamic + ~1 KB static (> the 64 KB default)

// NI key rows per lane per pass, NT threads; VPRE > 0 (round 4, caches of one pass): the
// lane's V row segment (VPRE x 16 B) and the mask values are loaded together with the K
// rows, before any arithmetic — one memory round trip instead of K (two passes at NI 8 for
// 256 keys), then the mask, then V after the softmax. At 256 keys, 1,024 threads (NI 4,
// VPRE 4: 32 B of K and 64 B of V per lane): 10.1 -> 8.05 us per layer in the drop-in -fa 0
// decode, tg128 557.6 -> 577.0 tok/s (256 threads, NI 16 / VPRE 16: 9.1 us, 568;
// profiles/r04/nofa_decode_ab.txt; g_tune[2] = 10 / 9 select those)
template <int D, int NI = NF_NI, int VPRE = 0, int NT = 256>
__global__ __launch_bounds__(NT) void k_attn_nofa_dec(NfArgs p) {
    constexpr int NW = NT / 64;
    extern __shared__ __align__(16) float sc[];   // [n_kv]: scores, then f16-rounded probabilities
    __shared__ float red[NW];
    __shared__ float opart[NT / D][D];
    typedef _Float16 h2v __attribute__((ext_vector_type(2)));
    constexpr int LPK = D / 8, KPI = 64 / LPK, PER = NW * NI * KPI;   // keys per workgroup pass
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if (blockIdx.y > 0) {                      // weight prefetch rows, as in k_fattn_dec2
        const unsigned L = blockIdx.x + gridDim.x * blockIdx.y, xcd = L & 7;
        const unsigned T = (gridDim.x * (gridDim.y - 1) >> 3) * NT, t0 = ((L - gridDim.x) >> 3) * NT + tid;
        unsigned acc = 0;
        for (int r = 0; r < p.pf_n; ++r) {
            const unsigned * w = (const unsigned *) (p.pf[r] + (size_t) xcd * p.pf_eighth[r]);
#pragma unroll 4
            for (unsigned l = t0; l < p.pf_lines[r]; l += T) acc ^= w[(size_t) l * 32];
        }
        if (acc == 0x9E3779B9u && p.n_kv < 0) p.dst[0] = 0.f;   // never (n_kv > 0): keeps the loads
        return;
    }
    const int h = blockIdx.x, hk = h / (p.H / p.Hkv);
    const int c = lane % LPK, kq = lane / LPK;
    h2v qh[4];
    {
        const float * qp = (const float *) (p.q + (size_t) h * p.q2) + 8 * c;
        const float4 a = *(const float4 *) qp, b = *(const float4 *) (qp + 4);
        qh[0] = h2v{(_Float16) a.x, (_Float16) a.y}; qh[1] = h2v{(_Float16) a.z, (_Float16) a.w};
        qh[2] = h2v{(_Float16) b.x, (_Float16) b.y}; qh[3] = h2v{(_Float16) b.z, (_Float16) b.w};
    }
    const char * kb = p.k + (size_t) hk * p.k2 + c * 16;
    // P·V geometry (below): NT/D threads per dimension, each a contiguous key range
    constexpr int SPLIT = NT / D;
    const int d = tid % D, part = tid / D;
    const int nk = p.n_kv / SPLIT;                           // host: n_kv % (8 SPLIT) == 0
    const char * vr = p.v + (size_t) hk * p.v2 + (size_t) d * p.v1 + (size_t) part * nk * 2;
    uint4 vpre[VPRE > 0 ? VPRE : 1];
    if constexpr (VPRE > 0) {
#pragma unroll
        for (int j = 0; j < VPRE; ++j) vpre[j] = *(const uint4 *) (vr + 16 * min(j, nk / 8 - 1));
    }
    for (int base = 0; base < p.n_kv; base += PER) {
        uint4 kr[NI];
        int key[NI];
        float mval[NI];
#pragma unroll
        for (int t = 0; t < NI; ++t) {
            key[t] = base + (wave * NI + t) * KPI + kq;
            kr[t] = *(const uint4 *) (kb + (size_t) min(key[t], p.n_kv - 1) * p.k1);
        }
        if constexpr (VPRE > 0) {     // the mask values with the rows (unconditional, clamped)
#pragma unroll
            for (int t = 0; t < NI; ++t) {
                const int kk = min(key[t], p.n_kv - 1);
                mval[t] = !p.mask ? 0.f : p.mask_f16 ? h2f(((const uint16_t *) p.mask)[kk]) : ((const float *) p.mask)[kk];
            }
        }
#pragma unroll
        for (int t = 0; t < NI; ++t) {
            float acc = __builtin_amdgcn_fdot2(__builtin_bit_cast(h2v, kr[t].x), qh[0], 0.f, false);
            acc = __builtin_amdgcn_fdot2(__builtin_bit_cast(h2v, kr[t].y), qh[1], acc, false);
            acc = __builtin_amdgcn_fdot2(__builtin_bit_cast(h2v, kr[t].z), qh[2], acc, false);
            acc = __builtin_amdgcn_fdot2(__builtin_bit_cast(h2v, kr[t].w), qh[3], acc, false);
            acc = dpp_sum_group<LPK>(acc);
            if (c == LPK - 1 && key[t] < p.n_kv) {
                float m = 0.f;
                if constexpr (VPRE > 0) m = mval[t];
                else if (p.mask) m = p.mask_f16 ? h2f(((const uint16_t *) p.mask)[key[t]]) : ((const float *) p.mask)[key[t]];
                sc[key[t]] = acc * p.scale + m;
            }
        }
    }
    __syncthreads();
    // softmax (ggml_vec_soft_max_f32: exp(x - max), Σ, times 1/Σ)
    float mx = -INFINITY;
    for (int k = tid; k < p.n_kv; k += NT) mx = fmaxf(mx, sc[k]);
    mx = wave_max(mx);
    if (lane == 0) red[wave] = mx;
    __syncthreads();
#pragma unroll
    for (int w = 0; w < NW; ++w) mx = fmaxf(mx, red[w]);
    __syncthreads();
    float sum = 0.f;
    for (int k = tid; k < p.n_kv; k += NT) {
        const float e = sc[k] == -INFINITY ? 0.f : expf(sc[k] - mx);
        sc[k] = e;
        sum += e;
    }
    sum = wave_sum(sum);
    if (lane == 0) red[wave] = sum;
    __syncthreads();
    float tot = 0.f;
#pragma unroll
    for (int w = 0; w < NW; ++w) tot += red[w];
    const float inv = 1.0f / tot;
    for (int k = tid; k < p.n_kv; k += NT) sc[k] = (float) (_Float16) (sc[k] * inv);
    __syncthreads();
    // P·V over the transposed rows
    const float * pp = sc + part * nk;
    float o = 0.f;
    if constexpr (VPRE > 0) {
#pragma unroll
        for (int j = 0; j < VPRE; ++j) {
            if (8 * j >= nk) break;
            const uint32_t ww[4] = {vpre[j].x, vpre[j].y, vpre[j].z, vpre[j].w};
#pragma unroll
            for (int i2 = 0; i2 < 4; ++i2) {
                o += pp[8 * j + 2 * i2] * h2f((uint16_t) (ww[i2] & 0xFFFF));
                o += pp[8 * j + 2 * i2 + 1] * h2f((uint16_t) (ww[i2] >> 16));
            }
        }
    }
    for (int k = 8 * VPRE; k < nk; k += 8) {
        const uint4 w = *(const uint4 *) (vr + 2 * k);
        const uint32_t ww[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            o += pp[k + 2 * j] * h2f((uint16_t) (ww[j] & 0xFFFF));
            o += pp[k + 2 * j + 1] * h2f((uint16_t) (ww[j] >> 16));
        }
    }
    opart[part][d] = o;
    __syncthreads();
    if (tid < D) {
        float r = 0.f;
#pragma unroll
        for (int s2 = 0; s2 < SPLIT; ++s2) r += opart[s2][tid];
        p.dst[(size_t) h * D + tid] = r;
    }
}

// ---------------------------------------------------------------------------
// Round 5: the -fa 0 decode chain for long caches. k_attn_nofa_dec keeps a head's scores in
// LDS (<= 16384 keys) and runs one workgroup per query head; beyond that the chain fell to
// the generic f16 GEMVs (llama-bench's default -fa 0 at -d 16384: 54 tok/s). Three launches
// over the whole chip instead:
//  k_nofa_scores: (KV head, 128-key chunk) workgroups for all Gt query heads of the group
//    (K read once): s = f16(q)·k · scale + mask into scratch, and per chunk the (max,
//    Σ exp(s - max)) of each head;
//  k_nofa_pv: (KV head, 512-key block) workgroups: each head's global max and sum from the
//    chunk partials, p = f16(exp(s - max) / sum) for the block — the softmax, then the
//    second mul_mat's f16 conversion, as the node chain computes them — and Σ p·v over the
//    block's keys of the transposed V rows (two threads per dimension) -> a partial O;
//  k_nofa_sum: O = Σ of the block partials in block order (p is normalised: a plain,
//    deterministic sum).
// ---------------------------------------------------------------------------
struct NlArgs {
    const char * q; size_t q2;
    const char * k; size_t k1, k2;
    const char * v; size_t v1, v2;
    const char * mask; int mask_f16;
    float * s;            // [H][n_kv] scores
    float2 * cp;          // [H][nc] chunk (max, sum)
    float * op;           // [nb][H][D] block partials of O
    float * dst;          // [H][D]
    int n_kv, H, Hkv, nc, nb;
    float scale;
};
constexpr int NL_CK = 128, NL_KB = 512;

template <int G>
__global__ __launch_bounds__(256) void k_nofa_scores(NlArgs p) {
    constexpr int LPK = 16, KPI = 4, NI = 8;
    typedef _Float16 h2v __attribute__((ext_vector_type(2)));
    __shared__ float rm[4][G], rl[4][G];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, c = lane % LPK, kq = lane / LPK;
    const int hk = blockIdx.x % p.Hkv, ch = blockIdx.x / p.Hkv, hb = hk * G;
    const char * kb = p.k + (size_t) hk * p.k2 + c * 16;
    uint4 kr[NI];
    int key[NI];
    float mv[NI];
#pragma unroll
    for (int t = 0; t < NI; ++t) {
        key[t] = ch * NL_CK + (wave * NI + t) * KPI + kq;
        kr[t] = *(const uint4 *) (kb + (size_t) min(key[t], p.n_kv - 1) * p.k1);
    }
#pragma unroll
    for (int t = 0; t < NI; ++t) {
        const int kk = min(key[t], p.n_kv - 1);
        mv[t] = !p.mask ? 0.f : p.mask_f16 ? h2f(((const uint16_t *) p.mask)[kk]) : ((const float *) p.mask)[kk];
    }
    h2v qh[G][4];
#pragma unroll
    for (int h = 0; h < G; ++h) {
        const float * qp = (const float *) (p.q + (size_t) (hb + h) * p.q2) + 8 * c;
        const float4 a = *(const float4 *) qp, b = *(const float4 *) (qp + 4);
        qh[h][0] = h2v{(_Float16) a.x, (_Float16) a.y}; qh[h][1] = h2v{(_Float16) a.z, (_Float16) a.w};
        qh[h][2] = h2v{(_Float16) b.x, (_Float16) b.y}; qh[h][3] = h2v{(_Float16) b.z, (_Float16) b.w};
    }
    float sc[G][NI];
#pragma unroll
    for (int t = 0; t < NI; ++t)
#pragma unroll
        for (int h = 0; h < G; ++h) {
            float acc = __builtin_amdgcn_fdot2(__builtin_bit_cast(h2v, kr[t].x), qh[h][0], 0.f, false);
            acc = __builtin_amdgcn_fdot2(__builtin_bit_cast(h2v, kr[t].y), qh[h][1], acc, false);
            acc = __builtin_amdgcn_fdot2(__builtin_bit_cast(h2v, kr[t].z), qh[h][2], acc, false);
            acc = __builtin_amdgcn_fdot2(__builtin_bit_cast(h2v, kr[t].w), qh[h][3], acc, false);
            acc = dpp_sum_group<LPK>(acc);                    // (in every lane of the row)
            sc[h][t] = key[t] < p.n_kv ? acc * p.scale + mv[t] : -INFINITY;
            if (c == 0 && key[t] < p.n_kv) p.s[(size_t) (hb + h) * p.n_kv + key[t]] = sc[h][t];
        }
    // the chunk's (max, sum) per head: over t in the lane, the row groups kq, then the waves
#pragma unroll
    for (int h = 0; h < G; ++h) {
        float m = sc[h][0];
#pragma unroll
        for (int t = 1; t < NI; ++t) m = fmaxf(m, sc[h][t]);
        m = kr_max<LPK>(m);
        if (lane == 0) rm[wave][h] = m;
    }
    __syncthreads();
#pragma unroll
    for (int h = 0; h < G; ++h) {
        const float M = fmaxf(fmaxf(rm[0][h], rm[1][h]), fmaxf(rm[2][h], rm[3][h]));
        float l = 0.f;
#pragma unroll
        for (int t = 0; t < NI; ++t) l += sc[h][t] == -INFINITY ? 0.f : expf(sc[h][t] - M);
        l = kr_sum<LPK>(l);
        if (lane == 0) rl[wave][h] = l;
    }
    __syncthreads();
    if (tid < G) {
        const float M = fmaxf(fmaxf(rm[0][tid], rm[1][tid]), fmaxf(rm[2][tid], rm[3][tid]));
        p.cp[(size_t) (hb + tid) * p.nc + ch] = make_float2(M, (rl[0][tid] + rl[1][tid]) + (rl[2][tid] + rl[3][tid]));
    }
}

// KB keys per workgroup (512, or 128 for shorter caches: >= ~256 workgroups); the V rows of
// the block are loaded first, so their round trip overlaps the (max, sum) reductions
template <int G, int KB>
__global__ __launch_bounds__(256) void k_nofa_pv(NlArgs p) {
    constexpr int D = 128, NV = KB / 16;                   // 16-byte V loads per thread
    __shared__ float pl[G][KB];
    __shared__ float red[4][G], sM[G], sInv[G];
    __shared__ float oh[G][D];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int hk = blockIdx.x % p.Hkv, blk = blockIdx.x / p.Hkv, hb = hk * G, k0 = blk * KB;
    // P·V geometry: thread -> dimension d, key half (KB / 2 keys)
    const int d = tid & (D - 1), half = tid >> 7;
    const int kb0 = k0 + half * (KB / 2);
    const char * vr = p.v + (size_t) hk * p.v2 + (size_t) d * p.v1 + (size_t) kb0 * 2;
    uint4 vv[NV];
    auto load_v = [&] {
#pragma unroll
        for (int j = 0; j < NV; ++j) vv[j] = kb0 + 8 * j + 8 <= p.n_kv ? *(const uint4 *) (vr + 16 * j) : make_uint4(0, 0, 0, 0);
    };
    // (512-key blocks: after the probabilities — 128 VGPRs of V held across the reductions
    // measured 23 vs 20 us per launch at 16k keys)
    if constexpr (KB <= 128) load_v();
    // global max and sum of each head (every workgroup of the head recomputes them: nc pairs)
    float m[G], l[G];
#pragma unroll
    for (int h = 0; h < G; ++h) {
        m[h] = -INFINITY;
        for (int cc = tid; cc < p.nc; cc += 256) m[h] = fmaxf(m[h], p.cp[(size_t) (hb + h) * p.nc + cc].x);
        m[h] = wave_max(m[h]);
        if (lane == 0) red[wave][h] = m[h];
    }
    __syncthreads();
#pragma unroll
    for (int h = 0; h < G; ++h) {
        m[h] = fmaxf(fmaxf(red[0][h], red[1][h]), fmaxf(red[2][h], red[3][h]));
        l[h] = 0.f;
        for (int cc = tid; cc < p.nc; cc += 256) {
            const float2 v = p.cp[(size_t) (hb + h) * p.nc + cc];
            l[h] += v.x == -INFINITY ? 0.f : v.y * expf(v.x - m[h]);
        }
        l[h] = wave_sum(l[h]);
    }
    __syncthreads();
    if (lane == 0) {
#pragma unroll
        for (int h = 0; h < G; ++h) red[wave][h] = l[h];
    }
    __syncthreads();
    if (tid < G) { sM[tid] = m[tid]; sInv[tid] = 1.0f / ((red[0][tid] + red[1][tid]) + (red[2][tid] + red[3][tid])); }
    __syncthreads();
    // this block's probabilities, f16-rounded
    for (int k = tid; k < KB; k += 256) {
        const int key = k0 + k;
#pragma unroll
        for (int h = 0; h < G; ++h) {
            const float sv = key < p.n_kv ? p.s[(size_t) (hb + h) * p.n_kv + key] : -INFINITY;
            pl[h][k] = sv == -INFINITY ? 0.f : (float) (_Float16) (expf(sv - sM[h]) * sInv[h]);
        }
    }
    __syncthreads();
    if constexpr (KB > 128) load_v();
    float o[G];
#pragma unroll
    for (int h = 0; h < G; ++h) o[h] = 0.f;
#pragma unroll
    for (int j = 0; j < NV; ++j) {
        const uint32_t ww[4] = {vv[j].x, vv[j].y, vv[j].z, vv[j].w};
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            const float x = h2f((uint16_t) (ww[e >> 1] >> (16 * (e & 1))));
#pragma unroll
            for (int h = 0; h < G; ++h) o[h] += pl[h][half * (KB / 2) + 8 * j + e] * x;
        }
    }
    if (half == 1) {
#pragma unroll
        for (int h = 0; h < G; ++h) oh[h][d] = o[h];
    }
    __syncthreads();
    if (half == 0) {
#pragma unroll
        for (int h = 0; h < G; ++h) p.op[((size_t) blk * p.H + hb + h) * D + d] = o[h] + oh[h][d];
    }
}

__global__ __launch_bounds__(128) void k_nofa_sum(NlArgs p) {
    const int h = blockIdx.x, d = threadIdx.x;
    float acc = 0.f;
#pragma unroll 8
    for (int b = 0; b < p.nb; ++b) acc += p.op[((size_t) b * p.H + h) * 128 + d];
    p.dst[(size_t) h * 128 + d] = acc;
}

// the long-cache form: D 128, one query token, GQA 1/2/4/8, n_kv % 8 == 0, from
// GGML_MI355X_NOFA_LONG_MIN keys (default 512: drop-in -fa 0 tg128 at -d 512 / 1024 / 4096 /
// 16384 453 -> 499, 376 -> 507, 184 -> 461, 54 -> 362 tok/s; g_tune[36] in units of 1024) and for every
// cache the one-workgroup kernel cannot hold (> 16384 keys)
static int nl_min_kv() {
    static const int env = [] { const char * v = getenv("GGML_MI355X_NOFA_LONG_MIN"); return v ? atoi(v) : 512; }();
    return g_tune[36] > 0 ? g_tune[36] * 1024 : env;
}
static bool nl_ok(int D, int n_kv, int H, int Hkv) {
    const int G = H / Hkv;
    return D == 128 && n_kv % 8 == 0 && (n_kv > NF_MAX_KV || n_kv >= nl_min_kv()) && (G == 1 || G == 2 || G == 4 || G == 8);
}
static size_t nl_scratch(int n_kv, int H) {
    const size_t nc = mx_ceil_div(n_kv, NL_CK), nb = mx_ceil_div(n_kv, NL_KB);
    return (size_t) H * n_kv * 4 + 256 + (size_t) H * nc * 8 + 256 + 4 * nb * H * 128 * 4 + 256;   // (blocks of 128 keys: 4 nb)
}
// scratch of the chain, sized at its SOFT_MAX node (one query row of n_kv keys, H heads)
size_t nofa_long_scratch(const ggml_tensor * sm) {
    if (sm->op != GGML_OP_SOFT_MAX || sm->ne[1] != 1 || sm->ne[3] != 1 || sm->ne[0] % 8) return 0;
    if (sm->ne[0] <= NF_MAX_KV && sm->ne[0] < nl_min_kv()) return 0;
    return nl_scratch((int) sm->ne[0], (int) sm->ne[2]);
}
static void nl_run(OpCtx & c, const NfArgs & a, float * dst) {
    NlArgs p{};
    p.q = a.q; p.q2 = a.q2; p.k = a.k; p.k1 = a.k1; p.k2 = a.k2; p.v = a.v; p.v1 = a.v1; p.v2 = a.v2;
    p.mask = a.mask; p.mask_f16 = a.mask_f16; p.dst = dst;
    p.n_kv = a.n_kv; p.H = a.H; p.Hkv = a.Hkv; p.scale = a.scale;
    p.nc = (int) mx_ceil_div(a.n_kv, NL_CK);
    const int kb = a.Hkv * mx_ceil_div(a.n_kv, NL_KB) >= 256 ? NL_KB : 128;
    p.nb = (int) mx_ceil_div(a.n_kv, kb);
    p.s = (float *) c.scratch->take((size_t) a.H * a.n_kv * 4);
    p.cp = (float2 *) c.scratch->take((size_t) a.H * p.nc * 8);
    p.op = (float *) c.scratch->take((size_t) p.nb * a.H * 128 * 4);
    const int G = a.H / a.Hkv;
    MX_KLOG("attn_nofa_long D=128 n_kv=%d H=%d Hkv=%d chunks=%d blocks=%d kb=%d", a.n_kv, a.H, a.Hkv, p.nc, p.nb, kb);
    const dim3 g1((unsigned) (a.Hkv * p.nc)), g2((unsigned) (a.Hkv * p.nb));
#define NL(GG) if (G == GG) { k_nofa_scores<GG><<<g1, 256, 0, c.st>>>(p); \
        if (kb == NL_KB) k_nofa_pv<GG, NL_KB><<<g2, 256, 0, c.st>>>(p); else k_nofa_pv<GG, 128><<<g2, 256, 0, c.st>>>(p); }
    NL(1) NL(2) NL(4) NL(8)
#undef NL
    k_nofa_sum<<<(unsigned) a.H, 128, 0, c.st>>>(p);
}

// ---------------------------------------------------------------------------
// Round 5: the -fa 0 decode chain of a short cache (<= 512 keys, D 128) as split partials
// for the output projection's prologue (XS_FAP, as fa_dec2_partials does for -fa 1): one
// 4-wave workgroup per (query head, 64-key split) computes the split's scores, its max
// (log2 domain), Σ exp2(s - max) and the unnormalised Σ p·v over the transposed V rows,
// all loads (K rows, mask, V row segments) issued before any arithmetic. The output
// projection merges the splits while its weight loads are in flight: no one-workgroup-
// per-head pass over the whole cache, no separate f32 x. Numerics: the probabilities stay
// f32 here (the node chain rounds the normalised p to f16 for the second mul_mat).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_nofa_part(NfArgs p, float * part, int nsplit) {
    constexpr int D = 128, LPK = 16, KPI = 4, NI = 4;
    typedef _Float16 h2v __attribute__((ext_vector_type(2)));
    __shared__ float sc[64], red[4], oh[D];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, c = lane % LPK, kq = lane / LPK;
    const int h = blockIdx.x, sp = blockIdx.y, hk = h / (p.H / p.Hkv), k0 = sp * 64;
    const char * kb = p.k + (size_t) hk * p.k2 + c * 16;
    // K rows: wave w has keys k0 + 16 w + 4 t + kq
    uint4 kr[NI];
    int key[NI];
#pragma unroll
    for (int t = 0; t < NI; ++t) {
        key[t] = k0 + wave * 16 + t * KPI + kq;
        kr[t] = *(const uint4 *) (kb + (size_t) min(key[t], p.n_kv - 1) * p.k1);
    }
    // V: thread -> dimension d, half of the split's keys (32 keys = 4 x 16 B)
    const int d = tid & (D - 1), half = tid >> 7;
    const int kv0 = k0 + half * 32;
    const char * vr = p.v + (size_t) hk * p.v2 + (size_t) d * p.v1 + (size_t) kv0 * 2;
    uint4 vv[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) vv[j] = kv0 + 8 * j + 8 <= p.n_kv ? *(const uint4 *) (vr + 16 * j) : make_uint4(0, 0, 0, 0);
    float mv[NI];
#pragma unroll
    for (int t = 0; t < NI; ++t) {
        const int kk = min(key[t], p.n_kv - 1);
        mv[t] = !p.mask ? 0.f : p.mask_f16 ? h2f(((const uint16_t *) p.mask)[kk]) : ((const float *) p.mask)[kk];
    }
    h2v qh[4];
    {
        const float * qp = (const float *) (p.q + (size_t) h * p.q2) + 8 * c;
        const float4 a = *(const float4 *) qp, b = *(const float4 *) (qp + 4);
        qh[0] = h2v{(_Float16) a.x, (_Float16) a.y}; qh[1] = h2v{(_Float16) a.z, (_Float16) a.w};
        qh[2] = h2v{(_Float16) b.x, (_Float16) b.y}; qh[3] = h2v{(_Float16) b.z, (_Float16) b.w};
    }
#pragma unroll
    for (int t = 0; t < NI; ++t) {
        float acc = __builtin_amdgcn_fdot2(__builtin_bit_cast(h2v, kr[t].x), qh[0], 0.f, false);
        acc = __builtin_amdgcn_fdot2(__builtin_bit_cast(h2v, kr[t].y), qh[1], acc, false);
        acc = __builtin_amdgcn_fdot2(__builtin_bit_cast(h2v, kr[t].z), qh[2], acc, false);
        acc = __builtin_amdgcn_fdot2(__builtin_bit_cast(h2v, kr[t].w), qh[3], acc, false);
        acc = dpp_sum_group<LPK>(acc);
        if (c == 0) {
            const float sv = key[t] < p.n_kv ? acc * p.scale + mv[t] : -INFINITY;
            sc[wave * 16 + t * KPI + kq] = sv == -INFINITY ? -INFINITY : sv * 1.4426950408889634f;   // log2 domain
        }
    }
    __syncthreads();
    // the split's max and Σ exp2 (wave 0), p into LDS
    if (wave == 0) {
        const float v = sc[lane];
        const float m = wave_max(v);
        const float e = m == -INFINITY || v == -INFINITY ? 0.f : __builtin_amdgcn_exp2f(v - m);
        sc[lane] = e;
        const float l = wave_sum(e);
        if (lane == 0) { red[0] = m; red[1] = l; }
    }
    __syncthreads();
    float o = 0.f;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const uint32_t ww[4] = {vv[j].x, vv[j].y, vv[j].z, vv[j].w};
#pragma unroll
        for (int e = 0; e < 8; ++e) o += sc[half * 32 + 8 * j + e] * h2f((uint16_t) (ww[e >> 1] >> (16 * (e & 1))));
    }
    if (half == 1) oh[d] = o;
    __syncthreads();
    float * pw = part + ((size_t) h * nsplit + sp) * (D + 2);
    if (half == 0) pw[d] = o + oh[d];
    if (tid == 0) { pw[D] = red[0]; pw[D + 1] = red[1]; }
}

static bool nf_view(const ggml_tensor * t) {
    return t->op == GGML_OP_RESHAPE || t->op == GGML_OP_VIEW || t->op == GGML_OP_PERMUTE || t->op == GGML_OP_TRANSPOSE;
}
static const ggml_tensor * nf_base(const ggml_tensor * t) {
    while (t && nf_view(t)) t = t->src[0];
    return t;
}

static const bool g_no_attn_nofa_pp = getenv("GGML_MI355X_NO_ATTN_FUSION_PP") != nullptr;   // A/B: prefill chain node by node

// the chain's CONT output feeding the output projection + residual ADD (decode, <= 512 keys,
// D 128): split partials + the projection's FAP prologue; returns the nodes consumed from
// i (0: not this shape — the caller runs the one-launch chain kernel)
static const bool g_no_nofa_split_o = getenv("GGML_MI355X_NO_NOFA_SPLIT_O") != nullptr;   // A/B
static int nofa_split_o(OpCtx & c, ggml_cgraph * g, int i, int last, const NfArgs & a, ggml_tensor * out, const UseCount & uses) {
    if (g_no_nofa_split_o || g_tune[38] == 1 || !g_gemv2 || a.n_kv > 512 || a.n_kv % 64 || a.n_kv < 64) return 0;
    auto use = [&](const ggml_tensor * t) { auto it = uses.find(t); return it == uses.end() ? 0 : it->second; };
    const ggml_tensor * q = g->nodes[i]->src[1];
    const int D = (int) q->ne[0], H = (int) q->ne[2], ns = a.n_kv / 64;
    if (D != 128 || use(out) != 1 || (out->flags & GGML_TENSOR_FLAG_OUTPUT)) return 0;
    ggml_tensor * mm = nullptr;
    int jm = -1;
    for (int j = last + 1; j < g->n_nodes && j < last + 4; ++j) {
        ggml_tensor * n = g->nodes[j];
        if (nf_view(n)) { if (nf_base(n) != out) return 0; continue; }
        if (n->op == GGML_OP_MUL_MAT && nf_base(n->src[1]) == out) { mm = n; jm = j; }
        break;
    }
    if (!mm || jm + 1 >= g->n_nodes) return 0;
    const ggml_tensor * x = mm->src[1];
    if (x != out && (x->op != GGML_OP_RESHAPE || use(x) != 1 || (x->flags & GGML_TENSOR_FLAG_OUTPUT))) return 0;
    if (mx_nelements(x) != (int64_t) D * H || mx_nrows(x) != 1) return 0;
    const ggml_tensor * wo = mm->src[0];
    if (!gemv2_fap_o_ok(c.s, wo, x, mm)) return 0;
    if (use(mm) != 1 || (mm->flags & GGML_TENSOR_FLAG_OUTPUT)) return 0;
    // the tail: ADD(mm, res) right after, or (the last layer) libllama's one-row inp_out_ids
    // pair GET_ROWS(mm), GET_ROWS(res) -> ADD: one token, both GET_ROWS are the identity
    ggml_tensor * add = nullptr, * g1 = nullptr, * g2 = nullptr;
    const ggml_tensor * res = nullptr;
    int lastn = -1;
    if (g->nodes[jm + 1]->op == GGML_OP_ADD) {
        add = g->nodes[jm + 1];
        res = add->src[0] == mm ? add->src[1] : (add->src[1] == mm ? add->src[0] : nullptr);
        lastn = jm + 1;
    } else {
        for (int j = jm + 1; j < g->n_nodes && j <= jm + 4; ++j) {
            ggml_tensor * n = g->nodes[j];
            if (nf_view(n)) continue;
            if (n->op == GGML_OP_GET_ROWS && !g1 && n->src[0] == mm) { g1 = n; continue; }
            if (n->op == GGML_OP_GET_ROWS && !g2 && n->src[0] != mm) { g2 = n; continue; }
            if (n->op == GGML_OP_ADD && g1 && g2 && ((n->src[0] == g1 && n->src[1] == g2) || (n->src[0] == g2 && n->src[1] == g1))) {
                add = n; lastn = j;
            }
            break;
        }
        if (!add) return 0;
        for (const ggml_tensor * gr : {g1, g2}) {
            if (gr->type != GGML_TYPE_F32 || gr->src[0]->type != GGML_TYPE_F32 || mx_nrows(gr->src[0]) != 1 || mx_nrows(gr) != 1 ||
                mx_nelements(gr->src[1]) != 1 || use(gr) != 1 || (gr->flags & GGML_TENSOR_FLAG_OUTPUT)) return 0;
        }
        res = g2->src[0];
    }
    if (!res || res == mm || add->type != GGML_TYPE_F32 || res->type != GGML_TYPE_F32) return 0;
    if (!mx_are_same_shape(res, mm) || !mx_are_same_shape(add, mm) || !mx_is_contiguous(res) || !mx_is_contiguous(add)) return 0;
    const bool same = res->nb[1] == add->nb[1];
    if (!fused_io_ok({add}, {res}, {{add, same ? res : nullptr}})) return 0;
    const size_t part_bytes = (size_t) H * ns * (D + 2) * sizeof(float) + 256;
    if (c.scratch->avail() < part_bytes) return 0;
    for (int j = last + 1; j <= lastn; ++j) {
        deferred_guard_node_ext(c, g->nodes[j]);
        act_cache_invalidate(c.s, g->nodes[j]);
    }
    float * part = (float *) c.scratch->take(part_bytes);
    MX_KLOG("attn_nofa_part D=128 n_kv=%d H=%d Hkv=%d nsplit=%d", a.n_kv, a.H, a.Hkv, ns);
    k_nofa_part<<<dim3((unsigned) H, (unsigned) ns), 256, 0, c.st>>>(a, part, ns);
    XStage xs{nullptr, nullptr, 0.0f, 0};
    xs.xcd = g_tune[15] != 1;
    xs.fap = part; xs.fap_ns = ns; xs.fap_d = D;
    gemv2_fap_o_launch(c, wo, xs, (float *) add->data, (const float *) res->data);
    return lastn - i + 1;
}
void fa_mma_nofa_launch(OpCtx & c, const ggml_tensor * q, const ggml_tensor * k, const ggml_tensor * v, const ggml_tensor * m,
                        float scale, ggml_tensor * out);   // ops_fattn_mma.hip

// returns the number of graph nodes consumed from i (0: no match). One query token: the
// decode kernel above; n_q >= 16 (prefill ubatches): the transposed-V MFMA flash kernel
// (fa_mma_nofa_launch), D = 128, n_kv % 64 == 0 (libllama pads the cache view to 256).
int fuse_attn_nofa(OpCtx & c, ggml_cgraph * g, int i, const UseCount & uses) {
    auto use = [&](const ggml_tensor * t) { auto it = uses.find(t); return it == uses.end() ? 0 : it->second; };
    ggml_tensor * kq = g->nodes[i];
    if (kq->op != GGML_OP_MUL_MAT) return 0;
    const ggml_tensor * k = kq->src[0], * q = kq->src[1];
    if (k->type != GGML_TYPE_F16 || q->type != GGML_TYPE_F32 || kq->type != GGML_TYPE_F32) return 0;
    const int D = (int) k->ne[0];
    const int n_q = (int) q->ne[1];
    const bool pre = n_q >= 16 && !g_no_attn_nofa_pp;
    if (!pre && n_q != 1) return 0;
    if ((D != 64 && D != 128) || (pre && D != 128) || q->ne[0] != D || q->ne[3] != 1 || k->ne[3] != 1) return 0;
    const int n_kv = (int) k->ne[1], H = (int) q->ne[2], Hkv = (int) k->ne[2];
    // decode P·V: 256/D threads per dimension, each a contiguous key range stepped by 8 keys
    // (16-byte V loads), so n_kv must split into 256/D parts of a multiple of 8 keys
    if (H % Hkv || k->nb[0] != 2 || k->nb[1] % 16 || k->nb[2] % 16 || (uintptr_t) k->data % 16) return 0;
    const bool lng = !pre && nl_ok(D, n_kv, H, Hkv);
    if (pre ? (n_kv % 64 || n_kv < 64) : lng ? false : (n_kv % (8 * (256 / D)) || n_kv > NF_MAX_KV)) return 0;
    if (lng && c.scratch->avail() < nl_scratch(n_kv, H)) return 0;
    if (q->nb[0] != 4 || q->nb[2] % 16 || (uintptr_t) q->data % 16 || (pre && q->nb[1] % 16)) return 0;
    ggml_tensor * sm = nullptr, * kqv = nullptr, * out = nullptr;
    int last = i;
    for (int j = i + 1; j < g->n_nodes && j < i + 12; ++j) {
        ggml_tensor * n = g->nodes[j];
        if (nf_view(n)) continue;
        if (!sm && n->op == GGML_OP_SOFT_MAX && n->src[0] == kq) { sm = n; last = j; continue; }
        if (sm && !kqv && n->op == GGML_OP_MUL_MAT && n->src[1] == sm) { kqv = n; last = j; continue; }
        if (kqv && !out && (n->op == GGML_OP_CONT || n->op == GGML_OP_CPY || n->op == GGML_OP_DUP) && nf_base(n->src[0]) == kqv &&
            n->src[0]->op == GGML_OP_PERMUTE) { out = n; last = j; break; }
        break;
    }
    if (!sm || !kqv || !out) return 0;
    // the softmax: plain scale + mask, no ALiBi / sinks
    if (sm->src[2] || mx_op_param<float>(sm, 1) != 0.0f || sm->type != GGML_TYPE_F32 || !mx_is_contiguous(sm)) return 0;
    if (kq->ne[0] != n_kv || kq->ne[1] != n_q || kq->ne[2] != H) return 0;
    const ggml_tensor * m = sm->src[1];
    if (m && ((m->type != GGML_TYPE_F16 && m->type != GGML_TYPE_F32) || m->ne[0] < n_kv || !mx_is_contiguous(m))) return 0;
    if (m && pre && (m->ne[1] < n_q || m->ne[2] != 1 || m->ne[3] != 1 || m->nb[1] % 16 || (uintptr_t) m->data % 16)) return 0;
    if (m && pre && m->type == GGML_TYPE_F32 && c.scratch->avail() < (size_t) n_kv * n_q * 2 + 256) return 0;
    // v: the transposed cache view [n_kv, D, Hkv], contiguous keys per dimension
    const ggml_tensor * v = kqv->src[0];
    if (v->type != GGML_TYPE_F16 || v->ne[0] != n_kv || v->ne[1] != D || v->ne[2] != Hkv || v->ne[3] != 1 || v->nb[0] != 2) return 0;
    if (v->nb[1] % 16 || v->nb[2] % 16 || (uintptr_t) v->data % 16) return 0;
    if (kqv->ne[0] != D || kqv->ne[1] != n_q || kqv->ne[2] != H || kqv->type != GGML_TYPE_F32) return 0;
    if (out->type != GGML_TYPE_F32 || !mx_is_contiguous(out) || mx_nelements(out) != (int64_t) D * H * n_q) return 0;
    const ggml_tensor * pm = out->src[0];   // permute(kqv, 0, 2, 1, 3): element (d, h, t) -> out[(t H + h) D + d]
    if (pm->ne[0] != D || pm->ne[1] != H || pm->ne[2] != n_q || pm->nb[1] != kqv->nb[2] || pm->nb[2] != kqv->nb[1]) return 0;
    // intermediates read only inside the chain, nothing else in between
    if (use(kq) != 1 || use(sm) != 1 || ((kq->flags | sm->flags | kqv->flags) & GGML_TENSOR_FLAG_OUTPUT)) return 0;
    for (int j = i + 1; j <= last; ++j) {
        const ggml_tensor * n = g->nodes[j];
        if (n != sm && n != kqv && n != out && !nf_view(n)) return 0;
        if (nf_view(n) && nf_base(n) == kqv && n != pm) return 0;   // another reader of kqv
    }
    // the output may sit exactly over q (the allocator reuses the dead q's memory): element
    // (d, h, t) of both is at (t H + h) D + d when q's strides are the permuted contiguous
    // ones, and each workgroup reads its q rows before it writes the same rows
    const bool q_same = q->nb[1] == (size_t) H * D * 4 && q->nb[2] == (size_t) D * 4;
    if (!fused_io_ok({out}, {q, k, v, m}, {{out, q_same ? q : nullptr}})) return 0;
    for (const ggml_tensor * t : {(const ggml_tensor *) kq, (const ggml_tensor *) sm, (const ggml_tensor *) kqv})
        for (int j = last + 1; j < g->n_nodes; ++j)
            for (int s2 = 0; s2 < GGML_MAX_SRC; ++s2)
                if (g->nodes[j]->src[s2] && nf_base(g->nodes[j]->src[s2]) == t) return 0;
    if (pre) {
        for (int j = i; j <= last; ++j) {
            deferred_guard_node_ext(c, g->nodes[j]);
            act_cache_invalidate(c.s, g->nodes[j]);
        }
        fa_mma_nofa_launch(c, q, k, v, m, mx_op_param<float>(sm, 0), out);
        return last - i + 1;
    }
    NfArgs a{};
    a.q = (const char *) q->data; a.q2 = q->nb[2];
    a.k = (const char *) k->data; a.k1 = k->nb[1]; a.k2 = k->nb[2];
    a.v = (const char *) v->data; a.v1 = v->nb[1]; a.v2 = v->nb[2];
    a.mask = m ? (const char *) m->data : nullptr; a.mask_f16 = m && m->type == GGML_TYPE_F16;
    a.dst = (float *) out->data;
    a.n_kv = n_kv; a.H = H; a.Hkv = Hkv;
    a.scale = mx_op_param<float>(sm, 0);
    for (int j = i; j <= last; ++j) {
        deferred_guard_node_ext(c, g->nodes[j]);
        act_cache_invalidate(c.s, g->nodes[j]);
    }
    // (split partials into the O projection first: at <= 512 keys they beat the long form)
    if (const int k = nofa_split_o(c, g, i, last, a, out, uses)) return k;
    if (lng) { nl_run(c, a, (float *) out->data); return last - i + 1; }
    MX_KLOG("attn_nofa D=%d n_kv=%d H=%d Hkv=%d mask=%d pf=%d", D, n_kv, H, Hkv, m ? (int) m->type : -1, H % 8 == 0 ? c.s->pf_n : 0);
    const size_t lds = (size_t) n_kv * 4;
    dim3 grid((unsigned) H, 1);
    a.pf_n = H % 8 == 0 ? c.s->pf_n : 0;       // prefetch ids must start on XCD 0
    for (int r = 0; r < a.pf_n; ++r) {
        a.pf[r] = c.s->pf_ptr[r]; a.pf_eighth[r] = c.s->pf_len[r] / 8; a.pf_lines[r] = (unsigned) (c.s->pf_take[r] / 128);
    }
    if (a.pf_n) grid.y = 1 + (unsigned) mx_ceil_div(640, H);   // ~640 prefetch workgroups of 4 waves
    MX_LDS_OPTIN(k_attn_nofa_dec<128>, NF_MAX_KV * 4);
    MX_LDS_OPTIN(k_attn_nofa_dec<64>, NF_MAX_KV * 4);
    MX_LDS_OPTIN((k_attn_nofa_dec<128, 16, 16>), NF_MAX_KV * 4);
    MX_LDS_OPTIN((k_attn_nofa_dec<128, 4, 4, 1024>), NF_MAX_KV * 4);
    // one pass over a cache of <= 256 keys with V and the mask loaded up front (D 128);
    // g_tune[2] = 10: the 256-thread one-pass form, 9: the round-3 two-pass form (A/B)
    if (D == 128 && n_kv <= 256 && n_kv % 64 == 0 && g_tune[2] != 9 && g_tune[2] != 10) k_attn_nofa_dec<128, 4, 4, 1024><<<grid, 1024, lds, c.st>>>(a);
    else if (D == 128 && n_kv <= 4 * 16 * 4 && g_tune[2] != 9) k_attn_nofa_dec<128, 16, 16><<<grid, 256, lds, c.st>>>(a);
    else if (D == 128) k_attn_nofa_dec<128><<<grid, 256, lds, c.st>>>(a);
    else k_attn_nofa_dec<64><<<grid, 256, lds, c.st>>>(a);
    return last - i + 1;
}

}  // namespace mx
