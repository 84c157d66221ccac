// ops_attn_o.hip — decode attention and the attention output projection in ONE launch.
//
// Node chain (src/llama-graph.cpp build_attn_mha + build_attn, src/models/llama.cpp):
//   FLASH_ATTN_EXT(q, k, v, mask) -> RESHAPE [D*H, 1] -> MUL_MAT(wo, .) -> ADD(., inpSA)
// for one query token. Unfused this is the decode attention (k_fattn_dec2: 32 workgroups,
// ~7.4 us per layer at 256 keys, HBM idle) + a launch boundary + the output-projection
// GEMV (9.4 MB of Q4_K at ~2 TB/s, ~4.7 us): the two latency-bound launches of a layer.
//
// MI355X design: the output projection is a sum over heads, y = x + sum_h Wo[:, h] o_h, and
// one Q4_K super-block of a Wo row spans exactly two heads at D = 128. Workgroup (pair p,
// row chunk r) therefore
//   1. issues its K/V/q/mask loads (one 256-key chunk, every load in flight, the decode
//      v2 geometry: 16 lanes per 256-B key row) and then the loads of super-block p of
//      its RPW rows of Wo (registers; the HBM stream overlaps the attention),
//   2. computes the attention of heads 2p, 2p+1 (both of one KV head: G even) exactly as
//      k_fattn_dec2 does (q rounded to f16, log2-domain online softmax), merges its waves
//      in LDS, normalises, and quantises the 256 outputs to q8_1 in LDS — the same
//      quantisation the output-projection GEMV's prologue applies to the FA output,
//   3. dots its rows' super-block with them (v_dot4, the decode GEMV's unit dot),
//   4. publishes the per-row partial as one {value, tag} granule (an 8-byte agent-scope,
//      write-through store) and exits; the row chunk's merger (the workgroup of its last
//      pair) polls the NP granules of its rows until all carry this launch's tag, sums them
//      in pair order (deterministic), adds the residual and stores y.
// Every workgroup of a pair recomputes the pair's attention (K/V of one KV head, 128 KB,
// from L2 after the first touch: the workgroups of one KV head are placed on one XCD);
// that costs less than the launch boundary and the separate GEMV it replaces.
// Spare workgroups beyond the grid carry the weight prefetch of the next streaming GEMV
// (exec.cpp fa_prefetch_plan), as the unfused attention launch does.
#include "backend.h"
#include "gemv.cuh"

#if !MX_AB_VARIANTS
// product build: the fused form is an A/B experiment (measured slower), the
// chain runs as the decode attention + the output-projection GEMV
namespace mx {
int fuse_attn_oproj(OpCtx &, ggml_cgraph *, int, const UseCount &) { return 0; }
}  // namespace mx
#else

namespace mx {

struct AoArgs {
    const char * q; size_t q2;          // q [D, 1, H] f32: head stride (bytes)
    const char * k; size_t k1, k2;      // K cache view [D, n_kv, Hkv] f16
    const char * v; size_t v1, v2;
    const uint16_t * mask;              // the token's f16 mask row (nullable)
    const char * wo; size_t wo_row;     // Q4_K [D*H, M]
    const float * res;                  // residual [M]
    float * dst;                        // y [M]
    uint2 * part;                       // [NP][M] per-pair partial rows as {value, tag} granules (scratch)
    unsigned int * cnt;                 // [NR] row-chunk epochs (fa_cnt's upper half)
    int n_kv, H, Hkv, M, NP, NR;
    float scale;
    unsigned long long * trace_blk;     // debug (opbench --trace-blocks): {start, end} of every workgroup
    unsigned long long * trace;         // debug (opbench --trace, slot 0): phase stamps of workgroup 0
    int dbg;                            // timing experiments (g_tune[27] >> 1): 1 no K/V/mask loads,
                                        // 2 no row-chunk merge, 4 no Wo loads (results wrong)
    const char * pf[4]; size_t pf_eighth[4]; unsigned pf_lines[4]; int pf_n;   // as FaDecArgs
};

constexpr int AO_D = 128, AO_NW = 8, AO_NT = 64 * AO_NW;
constexpr int AO_LPK = AO_D / 8;                 // lanes per key row
constexpr int AO_KPI = 64 / AO_LPK;              // keys per wave instruction
constexpr int AO_NI = 8;                         // key-row loads per lane
constexpr int AO_CS = AO_NW * AO_NI * AO_KPI;    // keys per launch: 256

// reductions over the four key rows of a wave (lanes l, l^16, l^32, l^48) by the gfx950
// row-swap instructions (VALU) instead of ds_bpermute shuffles: with both operands = v,
// the two results of a swap add up to v[l] + v[l ^ 16] (v[l ^ 32])
__device__ __forceinline__ float ao_sum4(float v) {
    auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    v = __uint_as_float(a[0]) + __uint_as_float(a[1]);
    auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return __uint_as_float(b[0]) + __uint_as_float(b[1]);
}
__device__ __forceinline__ float ao_max4(float v) {
    auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    v = fmaxf(__uint_as_float(a[0]), __uint_as_float(a[1]));
    auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return fmaxf(__uint_as_float(b[0]), __uint_as_float(b[1]));
}

// TPR threads per Wo row (each 4/TPR of the super-block's four 64-weight units); RPW rows
// per workgroup
template <int TPR>
__global__ __launch_bounds__(AO_NT) void k_attn_o(AoArgs p) {
    constexpr int RPW = AO_NT / TPR, UPT = 4 / TPR;
    typedef _Float16 h2v __attribute__((ext_vector_type(2)));
    __shared__ float wm[AO_NW][2], wl[AO_NW][2];
    __shared__ __align__(16) float wo[AO_NW][2][AO_D];
    __shared__ __align__(16) float xa[2 * AO_D];
    __shared__ __align__(16) char q8s[2 * AO_D + 16 * 4];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int T = p.NP * p.NR;
    const int L = (int) blockIdx.x;
    if (L >= T) {                             // prefetch workgroups (block-uniform, no barrier)
        const unsigned xcd = (unsigned) L & 7, P0 = (unsigned) T;
        const unsigned NPF = gridDim.x - P0, TT = (NPF >> 3) * AO_NT;
        const unsigned t0 = (((unsigned) L - P0) >> 3) * AO_NT + tid;
        unsigned acc = 0;
        for (int r = 0; r < p.pf_n; ++r) {
            const unsigned * w = (const unsigned *) (p.pf[r] + (size_t) xcd * p.pf_eighth[r]);
#pragma unroll 4
            for (unsigned l = t0; l < p.pf_lines[r]; l += TT) acc ^= w[(size_t) l * 32];
        }
        if (acc == 0x9E3779B9u && p.n_kv < 0) p.part[0] = make_uint2(0, 0);   // never (n_kv > 0): keeps the loads
        return;
    }
    // XCD x (= L % 8) takes one contiguous run of logical workgroups: all row chunks of
    // consecutive pairs, i.e. (GQA 4) the two pairs of one KV head, whose K/V its L2 keeps
    const int l = (T & 7) == 0 ? (L & 7) * (T >> 3) + (L >> 3) : L;
    const int pr = l / p.NR, rc = l % p.NR;
    const int h0 = 2 * pr, hk = h0 / (p.H / p.Hkv);
    // this launch's granule tag: the row chunk's epoch (advanced by its merger at the end;
    // every producer of the chunk reads it before the merger can finish) as a quiet-NaN
    // payload that neither integer tables nor computed floats in the scratch arena carry
    const unsigned epoch = __hip_atomic_load(p.cnt + rc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned tag = 0x7FE00000u | (epoch % 0x1FFFFFu + 1u);   // v1 tag space (bit 21 set; v2: clear)
    unsigned long long * tr = L == 0 ? p.trace : nullptr;
    MX_TRACE(tr, 0);
    MX_TRACE_BLK(p.trace_blk, 0);

    // ---- loads: q, mask, K, V (one chunk), then this thread's Wo units
    const int c = lane % AO_LPK, kq = lane / AO_LPK;
    const char * kb = p.k + (size_t) hk * p.k2 + c * 16;
    const char * vb = p.v + (size_t) hk * p.v2 + c * 16;
    float4 qa[2], qb[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const float * qp = (const float *) (p.q + (size_t) (h0 + h) * p.q2) + 8 * c;
        qa[h] = *(const float4 *) qp;
        qb[h] = *(const float4 *) (qp + 4);
    }
    const int key0 = wave * (AO_NI * AO_KPI) + kq;
    // unconditional loads (a load under a branch made every one of them its own round trip:
    // the compiler waited at each join); without a mask the K cache stands in, unused
    const uint16_t * mrow = p.mask ? p.mask : (const uint16_t *) p.k;
    uint16_t mraw[AO_NI];
    uint4 kr[AO_NI], vr[AO_NI];
    if (p.dbg & 1) {
#pragma unroll
        for (int t = 0; t < AO_NI; ++t) { mraw[t] = 0; kr[t] = make_uint4(tid, t, 0, 0); vr[t] = make_uint4(t, tid, 0, 0); }
    } else {
#pragma unroll
        for (int t = 0; t < AO_NI; ++t) mraw[t] = mrow[min(key0 + t * AO_KPI, p.n_kv - 1)];
#pragma unroll
        for (int t = 0; t < AO_NI; ++t) kr[t] = *(const uint4 *) (kb + (size_t) min(key0 + t * AO_KPI, p.n_kv - 1) * p.k1);
#pragma unroll
        for (int t = 0; t < AO_NI; ++t) vr[t] = *(const uint4 *) (vb + (size_t) min(key0 + t * AO_KPI, p.n_kv - 1) * p.v1);
    }
    __builtin_amdgcn_sched_barrier(0);
    const int rl = tid / TPR, sub = tid % TPR;
    const int row = rc * RPW + rl;
    const char * wrow = p.wo + (size_t) min(row, p.M - 1) * p.wo_row + (size_t) pr * 144;
    // the super-block header once, then the 32-B qs runs of this thread's units
    W2<GGML_TYPE_Q4_K> wr[UPT];
    if (p.dbg & 4) {
#pragma unroll
        for (int j = 0; j < UPT; ++j) { wr[j].hd = make_int4(tid, 0, 0, 0); wr[j].w0 = make_int4(j, 0, 0, 0); wr[j].w1 = make_int4(0, j, 0, 0); }
    } else {
        const int4 hd = *(const int4 *) wrow;
#pragma unroll
        for (int j = 0; j < UPT; ++j) {
            const int u = sub * UPT + j;
            wr[j].hd = hd;
            wr[j].w0 = *(const int4 *) (wrow + 16 + 32 * u);
            wr[j].w1 = *(const int4 *) (wrow + 32 + 32 * u);
        }
    }
    __builtin_amdgcn_sched_barrier(0);

    MX_TRACE(tr, 1);
    // ---- attention of heads h0, h0 + 1 over the chunk (k_fattn_dec2 semantics)
    h2v qh[2][4];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        qh[h][0] = h2v{(_Float16) qa[h].x, (_Float16) qa[h].y}; qh[h][1] = h2v{(_Float16) qa[h].z, (_Float16) qa[h].w};
        qh[h][2] = h2v{(_Float16) qb[h].x, (_Float16) qb[h].y}; qh[h][3] = h2v{(_Float16) qb[h].z, (_Float16) qb[h].w};
    }
    float mk[AO_NI];
#pragma unroll
    for (int t = 0; t < AO_NI; ++t) mk[t] = key0 + t * AO_KPI < p.n_kv ? (p.mask ? h2f(mraw[t]) : 0.f) : -INFINITY;
    float s[2][AO_NI];
#pragma unroll
    for (int t = 0; t < AO_NI; ++t)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            float acc = __builtin_amdgcn_fdot2(__builtin_bit_cast(h2v, kr[t].x), qh[h][0], 0.f, false);
            acc = __builtin_amdgcn_fdot2(__builtin_bit_cast(h2v, kr[t].y), qh[h][1], acc, false);
            acc = __builtin_amdgcn_fdot2(__builtin_bit_cast(h2v, kr[t].z), qh[h][2], acc, false);
            acc = __builtin_amdgcn_fdot2(__builtin_bit_cast(h2v, kr[t].w), qh[h][3], acc, false);
            acc = dpp_sum_group<AO_LPK>(acc);
            s[h][t] = mk[t] == -INFINITY ? -INFINITY : (acc * p.scale + mk[t]) * 1.4426950408889634f;
        }
    float M[2], Ls[2], o[2][8];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        float mc = s[h][0];
#pragma unroll
        for (int t = 1; t < AO_NI; ++t) mc = fmaxf(mc, s[h][t]);
        mc = ao_max4(mc);
        float pr_[AO_NI], lc = 0.f;
#pragma unroll
        for (int t = 0; t < AO_NI; ++t) { pr_[t] = mc == -INFINITY ? 0.f : __builtin_amdgcn_exp2f(s[h][t] - mc); lc += pr_[t]; }
        lc = ao_sum4(lc);
        M[h] = mc; Ls[h] = lc;
#pragma unroll
        for (int i = 0; i < 8; ++i) o[h][i] = 0.f;
#pragma unroll
        for (int t = 0; t < AO_NI; ++t) {
            const uint32_t vw[4] = {vr[t].x, vr[t].y, vr[t].z, vr[t].w};
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                o[h][2 * i] += pr_[t] * h2f((uint16_t) (vw[i] & 0xFFFF));
                o[h][2 * i + 1] += pr_[t] * h2f((uint16_t) (vw[i] >> 16));
            }
        }
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
#pragma unroll
        for (int i = 0; i < 8; ++i) o[h][i] = ao_sum4(o[h][i]);
        if (lane == 0) { wm[wave][h] = M[h]; wl[wave][h] = Ls[h]; }
        if (kq == 0) {
            *(float4 *) &wo[wave][h][8 * c] = make_float4(o[h][0], o[h][1], o[h][2], o[h][3]);
            *(float4 *) &wo[wave][h][8 * c + 4] = make_float4(o[h][4], o[h][5], o[h][6], o[h][7]);
        }
    }
    MX_TRACE(tr, 2);
    __syncthreads();
    if (tid < 2 * AO_D) {                      // merge the waves: the FA output of the pair
        const int h = tid / AO_D, d = tid % AO_D;
        float Mw = wm[0][h];
#pragma unroll
        for (int w = 1; w < AO_NW; ++w) Mw = fmaxf(Mw, wm[w][h]);
        float Lw = 0.f, O = 0.f;
#pragma unroll
        for (int w = 0; w < AO_NW; ++w) {
            const float f = wm[w][h] == -INFINITY ? 0.f : __builtin_amdgcn_exp2f(wm[w][h] - Mw);
            Lw += wl[w][h] * f;
            O += wo[w][h][d] * f;
        }
        xa[tid] = Lw == 0.f ? 0.f : O / Lw;
    }
    __syncthreads();
    // ---- q8_1 of the 256 outputs (the GEMV prologue's quantisation, gemv.cuh q8_half)
    const LdsAct a = lds_act(q8s, 2 * AO_D);
    if (tid < 2 * AO_D / 16) {
        float v16[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) v16[j] = xa[16 * tid + j];
        q8_half(v16, tid, a);
    }
    __syncthreads();
    MX_TRACE(tr, 3);
    // ---- this row's super-block p against the pair's q8 outputs
    float acc = 0.f;
#pragma unroll
    for (int j = 0; j < UPT; ++j) acc += w2_dot<GGML_TYPE_Q4_K>(wr[j], sub * UPT + j, a);
    acc = dpp_sum_group<TPR>(acc);
    if (sub == 0 && row < p.M) {
        const uint64_t g = (uint64_t) __float_as_uint(acc) | ((uint64_t) tag << 32);
        __hip_atomic_store((unsigned long long *) (p.part + (size_t) pr * p.M + row), (unsigned long long) g, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);   // one write-through 8-byte store: value and tag land together
    }
    MX_TRACE(tr, 4);
    // ---- row chunk rc is merged by its last pair's workgroup: every row's thread polls the
    // NP granules (agent-scope loads, all in flight) until each carries this launch's tag,
    // then sums them in pair order (deterministic) and adds the residual. No arrival
    // counter: a producer stores and exits (an acq_rel count also cost a buffer_wbl2 per
    // workgroup); the merger waits about one hand-off after the last granule lands.
    if ((p.dbg & 2) || pr != p.NP - 1) { MX_TRACE_BLK(p.trace_blk, 1); return; }
    if (tid < RPW) {
        const int r2 = min(rc * RPW + tid, p.M - 1);
        const unsigned long long * gp = (const unsigned long long *) (p.part + r2);
        float y = 0.f;
        for (int p0 = 0; p0 < p.NP; p0 += 16) {
            unsigned long long v[16];
            for (int it = 0; it < (1 << 22); ++it) {   // bounded: a lost granule ends in NaN, not a hang
#pragma unroll
                for (int j = 0; j < 16; ++j)
                    v[j] = __hip_atomic_load(gp + (size_t) min(p0 + j, p.NP - 1) * p.M, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                bool ok = true;
#pragma unroll
                for (int j = 0; j < 16; ++j) ok &= (unsigned) (v[j] >> 32) == tag;
                if (ok) break;
                if (it == (1 << 22) - 1) { y = __int_as_float(0x7FC00000); break; }
                __builtin_amdgcn_s_sleep(1);
            }
#pragma unroll
            for (int j = 0; j < 16; ++j) if (p0 + j < p.NP) y += __uint_as_float((unsigned) v[j]);
        }
        if (rc * RPW + tid < p.M) p.dst[r2] = y + p.res[r2];
    }
    __syncthreads();
    if (tid == 0) __hip_atomic_store(p.cnt + rc, epoch + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // next launch / replay
    MX_TRACE(tr, 6);
    MX_TRACE_BLK(p.trace_blk, 1);
}

// ---------------------------------------------------------------------------
// v2 ("stream beside the chain", MI355X_MICROARCH.md price table): the attention runs on
// NP workgroups (one head pair each, the v1 attention code) and publishes the FA output as
// {value, tag} granules; NG = M / 32 GEMV workgroups stream their Wo rows into registers at
// launch (the whole row, like the unfused output-projection GEMV, overlapping the attention),
// poll the granules, quantise them to q8_1 in LDS (bit-identical to the GEMV prologue's
// q8_half) and finish the rows: no redundant attention, no per-row merge; the remaining
// CUs carry the weight prefetch of the next streaming GEMV. The granule tag comes from a
// launch counter to which every launch adds exactly 2^16 (the GEMV workgroups add 1 each
// when done, workgroup 0 the rest), so every workgroup of a launch reads the same
// floor(count / 2^16) whatever shapes ran before: no reset pass.
// Deadlock-free: attention workgroups have the lowest ids (dispatched first) and wait for
// nothing; only GEMV workgroups wait, and only for them.
// S key splits per head pair (each attention workgroup 256 / S keys: S = 2 halves the
// K/V bytes a CU issues, the attention's critical path); the GEMV workgroups merge the S
// partial (O, max, sum) in their prologue, as k_fattn_dec2's split merge does.
template <int U, int S>   // Q4_K units per lane: K = 1024 U
__global__ __launch_bounds__(AO_NT) void k_attn_o2(AoArgs p) {
    constexpr int K = 1024 * U, KPT = K / AO_NT;   // granules per thread in the GEMV prologue
    constexpr int NI = AO_NI / S;                  // key rows per lane
    typedef _Float16 h2v __attribute__((ext_vector_type(2)));
    __shared__ float wm[AO_NW][2], wl[AO_NW][2];
    __shared__ __align__(16) char smem[K + K / 32 * 8 > AO_NW * 2 * AO_D * 4 ? K + K / 32 * 8 : AO_NW * 2 * AO_D * 4];
    __shared__ __align__(16) float xa[2 * AO_D];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int L = (int) blockIdx.x, NA = p.NP * S, NG = p.NR;
    if (L >= NA + NG) {                       // prefetch workgroups (block-uniform, no barrier)
        const unsigned xcd = (unsigned) L & 7, P0 = (unsigned) (NA + NG);
        const unsigned NPF = gridDim.x - P0, TT = (NPF >> 3) * AO_NT;
        const unsigned t0 = (((unsigned) L - P0) >> 3) * AO_NT + tid;
        unsigned acc = 0;
        for (int r = 0; r < p.pf_n; ++r) {
            const unsigned * w = (const unsigned *) (p.pf[r] + (size_t) xcd * p.pf_eighth[r]);
#pragma unroll 4
            for (unsigned l = t0; l < p.pf_lines[r]; l += TT) acc ^= w[(size_t) l * 32];
        }
        if (acc == 0x9E3779B9u && p.n_kv < 0) p.part[0] = make_uint2(0, 0);   // never (n_kv > 0): keeps the loads
        return;
    }
    const unsigned n = __hip_atomic_load(p.cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >> 16;
    const unsigned tag = 0x7FC00000u | (n % 0x1FFFFFu + 1u);
    unsigned long long * tr = L == 0 ? p.trace : nullptr;
    MX_TRACE(tr, 0);
    MX_TRACE_BLK(p.trace_blk, 0);
    if (L < NA) {
        // ---- attention of heads 2 pr, 2 pr + 1 over key split sp (as k_attn_o), published
        // as granules: per element the split's unnormalised O, per head its (max, sum)
        const int pr = L / S, sp = L % S;
        const int h0 = 2 * pr, hk = h0 / (p.H / p.Hkv);
        const int c = lane % AO_LPK, kq = lane / AO_LPK;
        const char * kb = p.k + (size_t) hk * p.k2 + c * 16;
        const char * vb = p.v + (size_t) hk * p.v2 + c * 16;
        float4 qa[2], qb[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const float * qp = (const float *) (p.q + (size_t) (h0 + h) * p.q2) + 8 * c;
            qa[h] = *(const float4 *) qp;
            qb[h] = *(const float4 *) (qp + 4);
        }
        const int key0 = sp * (AO_CS / S) + wave * (NI * AO_KPI) + kq;
        const uint16_t * mrow = p.mask ? p.mask : (const uint16_t *) p.k;
        uint16_t mraw[NI];
        uint4 kr[NI], vr[NI];
#pragma unroll
        for (int t = 0; t < NI; ++t) mraw[t] = mrow[min(key0 + t * AO_KPI, p.n_kv - 1)];
#pragma unroll
        for (int t = 0; t < NI; ++t) kr[t] = *(const uint4 *) (kb + (size_t) min(key0 + t * AO_KPI, p.n_kv - 1) * p.k1);
#pragma unroll
        for (int t = 0; t < NI; ++t) vr[t] = *(const uint4 *) (vb + (size_t) min(key0 + t * AO_KPI, p.n_kv - 1) * p.v1);
        MX_TRACE(tr, 1);
        h2v qh[2][4];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            qh[h][0] = h2v{(_Float16) qa[h].x, (_Float16) qa[h].y}; qh[h][1] = h2v{(_Float16) qa[h].z, (_Float16) qa[h].w};
            qh[h][2] = h2v{(_Float16) qb[h].x, (_Float16) qb[h].y}; qh[h][3] = h2v{(_Float16) qb[h].z, (_Float16) qb[h].w};
        }
        float mk[NI];
#pragma unroll
        for (int t = 0; t < NI; ++t) mk[t] = key0 + t * AO_KPI < p.n_kv ? (p.mask ? h2f(mraw[t]) : 0.f) : -INFINITY;
        float s[2][NI];
#pragma unroll
        for (int t = 0; t < NI; ++t)
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                float a = __builtin_amdgcn_fdot2(__builtin_bit_cast(h2v, kr[t].x), qh[h][0], 0.f, false);
                a = __builtin_amdgcn_fdot2(__builtin_bit_cast(h2v, kr[t].y), qh[h][1], a, false);
                a = __builtin_amdgcn_fdot2(__builtin_bit_cast(h2v, kr[t].z), qh[h][2], a, false);
                a = __builtin_amdgcn_fdot2(__builtin_bit_cast(h2v, kr[t].w), qh[h][3], a, false);
                a = dpp_sum_group<AO_LPK>(a);
                s[h][t] = mk[t] == -INFINITY ? -INFINITY : (a * p.scale + mk[t]) * 1.4426950408889634f;
            }
        float (*wo)[2][AO_D] = (float (*)[2][AO_D]) smem;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            float mc = s[h][0];
#pragma unroll
            for (int t = 1; t < NI; ++t) mc = fmaxf(mc, s[h][t]);
            mc = ao_max4(mc);
            float pr_[NI], lc = 0.f;
#pragma unroll
            for (int t = 0; t < NI; ++t) { pr_[t] = mc == -INFINITY ? 0.f : __builtin_amdgcn_exp2f(s[h][t] - mc); lc += pr_[t]; }
            lc = ao_sum4(lc);
            float o[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) o[i] = 0.f;
#pragma unroll
            for (int t = 0; t < NI; ++t) {
                const uint32_t vw[4] = {vr[t].x, vr[t].y, vr[t].z, vr[t].w};
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    o[2 * i] += pr_[t] * h2f((uint16_t) (vw[i] & 0xFFFF));
                    o[2 * i + 1] += pr_[t] * h2f((uint16_t) (vw[i] >> 16));
                }
            }
#pragma unroll
            for (int i = 0; i < 8; ++i) o[i] = ao_sum4(o[i]);
            if (lane == 0) { wm[wave][h] = mc; wl[wave][h] = lc; }
            if (kq == 0) {
                *(float4 *) &wo[wave][h][8 * c] = make_float4(o[0], o[1], o[2], o[3]);
                *(float4 *) &wo[wave][h][8 * c + 4] = make_float4(o[4], o[5], o[6], o[7]);
            }
        }
        MX_TRACE(tr, 2);
        __syncthreads();
        if (tid < 2 * AO_D) {
            const int h = tid / AO_D, d = tid % AO_D;
            float Mw = wm[0][h];
#pragma unroll
            for (int w = 1; w < AO_NW; ++w) Mw = fmaxf(Mw, wm[w][h]);
            float Lw = 0.f, O = 0.f;
#pragma unroll
            for (int w = 0; w < AO_NW; ++w) {
                const float f = wm[w][h] == -INFINITY ? 0.f : __builtin_amdgcn_exp2f(wm[w][h] - Mw);
                Lw += wl[w][h] * f;
                O += wo[w][h][d] * f;
            }
            // element (head h0 + h, split sp, d) at ((h0 + h) S + sp) D + d; stats after the K S elements
            unsigned long long * gq = (unsigned long long *) p.part;
            auto put = [&](size_t i, float x) {
                __hip_atomic_store(gq + i, (unsigned long long) ((uint64_t) __float_as_uint(x) | ((uint64_t) tag << 32)),
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            };
            if constexpr (S == 1) put((size_t) h0 * AO_D + tid, Lw == 0.f ? 0.f : O / Lw);
            else {
                put((size_t) ((h0 + h) * S + sp) * AO_D + d, O);
                if (d < 2) put((size_t) K * S + (size_t) ((h0 + h) * S + sp) * 2 + d, d == 0 ? Mw : Lw);
            }
        }
        MX_TRACE(tr, 3);
        MX_TRACE_BLK(p.trace_blk, 1);
        return;
    }
    // ---- GEMV workgroup: 32 rows x the whole K (16 lanes per row, U units per lane)
    const int gw = L - NA;
    const int sub = lane & 15;
    const int row = 32 * gw + 4 * wave + (lane >> 4);
    const char * wrow = p.wo + (size_t) min(row, p.M - 1) * p.wo_row;
    W2<GGML_TYPE_Q4_K> wr[U];
    if (p.dbg & 4) {
#pragma unroll
        for (int j = 0; j < U; ++j) { wr[j].hd = make_int4(tid, 0, 0, 0); wr[j].w0 = make_int4(j, 0, 0, 0); wr[j].w1 = make_int4(0, j, 0, 0); }
    } else {
#pragma unroll
        for (int j = 0; j < U; ++j) w2_load<GGML_TYPE_Q4_K>(wrow, sub + 16 * j, wr[j]);
    }
    const float res = p.res[min(row, p.M - 1)];
    // poll this thread's granules (agent-scope loads, all in flight) for this launch's tag:
    // S == 1 the KPT outputs; S > 1 their S split partials and the head's S (max, sum)
    const unsigned long long * gp = (const unsigned long long *) p.part;
    const int e0 = KPT * tid, hh = e0 / AO_D, d0 = e0 % AO_D;
    constexpr int NGR = S == 1 ? KPT : S * KPT + 2 * S;
    unsigned long long v[NGR];
    bool lost = false;
    for (int it = 0;; ++it) {                   // bounded: a lost granule ends in NaN, not a hang
        if constexpr (S == 1) {
#pragma unroll
            for (int j = 0; j < KPT; ++j) v[j] = __hip_atomic_load(gp + e0 + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
#pragma unroll
            for (int q = 0; q < S; ++q)
#pragma unroll
                for (int j = 0; j < KPT; ++j)
                    v[q * KPT + j] = __hip_atomic_load(gp + (size_t) (hh * S + q) * AO_D + d0 + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
            for (int j = 0; j < 2 * S; ++j)
                v[S * KPT + j] = __hip_atomic_load(gp + (size_t) K * S + (size_t) hh * S * 2 + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        bool ok = true;
#pragma unroll
        for (int j = 0; j < NGR; ++j) ok &= (unsigned) (v[j] >> 32) == tag;
        if (ok || (p.dbg & 1)) break;
        if (it == (1 << 22)) { lost = true; break; }
        __builtin_amdgcn_s_sleep(1);
    }
    MX_TRACE(tr, 1);
    // q8_1 of this thread's KPT values (KPT = 8: four threads per 32-block, 16: two) — the
    // arithmetic of gemv.cuh q8_half (q8_scale / q8_round), so the int8 values are identical
    const LdsAct a = lds_act(smem, K);
    {
        float x[KPT];
        float amax = 0.f;
        if constexpr (S == 1) {
#pragma unroll
            for (int j = 0; j < KPT; ++j) x[j] = __uint_as_float((unsigned) v[j]);
        } else {
            // merge the splits (log2-domain maxima, as k_fattn_dec2_combine)
            float ms[S], w[S], Mx = -INFINITY, Ls = 0.f;
#pragma unroll
            for (int q = 0; q < S; ++q) { ms[q] = __uint_as_float((unsigned) v[S * KPT + 2 * q]); Mx = fmaxf(Mx, ms[q]); }
#pragma unroll
            for (int q = 0; q < S; ++q) {
                w[q] = ms[q] == -INFINITY ? 0.f : __builtin_amdgcn_exp2f(ms[q] - Mx);
                Ls += w[q] * __uint_as_float((unsigned) v[S * KPT + 2 * q + 1]);
            }
#pragma unroll
            for (int j = 0; j < KPT; ++j) {
                float o = 0.f;
#pragma unroll
                for (int q = 0; q < S; ++q) o += w[q] * __uint_as_float((unsigned) v[q * KPT + j]);
                x[j] = Ls == 0.f ? 0.f : o / Ls;
            }
        }
#pragma unroll
        for (int j = 0; j < KPT; ++j) amax = fmaxf(amax, fabsf(x[j]));
        amax = fmaxf(amax, dpp_f<0xB1>(-INFINITY, amax));
        if constexpr (KPT == 8) amax = fmaxf(amax, dpp_f<0x4E>(-INFINITY, amax));
        const Q8Scale qs = q8_scale(amax);
        int sum = 0, pk[KPT / 4];
#pragma unroll
        for (int j = 0; j < KPT / 4; ++j) {
            int w = 0;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int qi = q8_round(x[4 * j + k], qs.id);
                sum += qi;
                w |= (qi & 0xFF) << (8 * k);
            }
            pk[j] = w;
        }
        sum += dpp_i<0xB1>(0, sum);
        if constexpr (KPT == 8) sum += dpp_i<0x4E>(0, sum);
        if constexpr (KPT == 8) *(int2 *) (a.q + 8 * tid) = make_int2(pk[0], pk[1]);
        else *(int4 *) (a.q + 16 * tid) = make_int4(pk[0], pk[1], pk[2], pk[3]);
        constexpr int TPB = 32 / KPT;           // threads per 32-block
        if (tid % TPB == 0) { a.d[tid / TPB] = qs.d; a.s[tid / TPB] = qs.d * (float) sum; }
    }
    __syncthreads();
    MX_TRACE(tr, 2);
    float acc = 0.f;
#pragma unroll
    for (int j = 0; j < U; ++j) acc += w2_dot<GGML_TYPE_Q4_K>(wr[j], sub + 16 * j, a);
    acc = dpp_sum_group<16>(acc);
    if (sub == 0 && row < p.M) p.dst[row] = lost ? __int_as_float(0x7FC00000) : acc + res;
    MX_TRACE(tr, 3);
    if (tid == 0)   // this launch's share of the 2^16 count (workgroup 0 takes the remainder)
        __hip_atomic_fetch_add(p.cnt, gw == 0 ? 65536u - (unsigned) NG + 1u : 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    MX_TRACE_BLK(p.trace_blk, 1);
}

static bool ao_view(const ggml_tensor * t) {
    return t->op == GGML_OP_RESHAPE || t->op == GGML_OP_VIEW || t->op == GGML_OP_PERMUTE || t->op == GGML_OP_TRANSPOSE;
}

// Opt-in (measured slower than the two launches it replaces, DESIGN §3.3 / profiles/r03/
// attn_o_fusion_ab.txt): g_tune[27] = 64 (v2, + 32: one key split), 16 (v1); bits 2/4/8:
// timing experiments; GGML_MI355X_ATTN_O_FUSION=1 turns v2 on
static const bool g_attn_o_env = getenv("GGML_MI355X_ATTN_O_FUSION") != nullptr;

// returns the number of graph nodes consumed from i (0: no match)
int fuse_attn_oproj(OpCtx & c, ggml_cgraph * g, int i, const UseCount & uses) {
    if (!(g_tune[27] & (16 | 64)) && !g_attn_o_env) return 0;
    auto use = [&](const ggml_tensor * t) { auto it = uses.find(t); return it == uses.end() ? 0 : it->second; };
    ggml_tensor * fa = g->nodes[i];
    if (fa->op != GGML_OP_FLASH_ATTN_EXT) return 0;
    const ggml_tensor * q = fa->src[0], * k = fa->src[1], * v = fa->src[2], * m = fa->src[3];
    if (fa->src[4] || mx_op_param<float>(fa, 1) != 0.0f || mx_op_param<float>(fa, 2) != 0.0f) return 0;   // sinks, ALiBi, softcap
    if (q->type != GGML_TYPE_F32 || k->type != GGML_TYPE_F16 || v->type != GGML_TYPE_F16 || fa->type != GGML_TYPE_F32) return 0;
    const int D = (int) k->ne[0], H = (int) q->ne[2], Hkv = (int) k->ne[2], n_kv = (int) k->ne[1];
    if (D != AO_D || v->ne[0] != D || q->ne[0] != D || q->ne[1] != 1 || q->ne[3] != 1 || k->ne[3] != 1 || v->ne[3] != 1) return 0;
    if (H % Hkv || (H / Hkv) % 2 || H % 2 || n_kv < 1 || n_kv > AO_CS || v->ne[1] != n_kv || v->ne[2] != Hkv) return 0;
    if (q->nb[0] != 4 || q->nb[2] % 16 || (uintptr_t) q->data % 16) return 0;
    if (k->nb[0] != 2 || v->nb[0] != 2 || k->nb[1] % 16 || v->nb[1] % 16 || k->nb[2] % 16 || v->nb[2] % 16 ||
        (uintptr_t) k->data % 16 || (uintptr_t) v->data % 16) return 0;
    if (m && (m->type != GGML_TYPE_F16 || m->ne[0] < n_kv || m->ne[2] > 1 || m->ne[3] > 1 || m->nb[0] != 2)) return 0;
    if (!mx_is_contiguous(fa) || mx_nelements(fa) != (int64_t) D * H) return 0;
    // FA -> (views) -> MUL_MAT(wo, view of FA) -> ADD(mm, residual), nothing else in between
    ggml_tensor * mm = nullptr, * add = nullptr, * rs = nullptr;
    int last = i;
    for (int j = i + 1; j < g->n_nodes && j < i + 8; ++j) {
        ggml_tensor * n = g->nodes[j];
        if (ao_view(n)) {
            if (!rs && n->src[0] == fa) rs = n;
            continue;
        }
        if (!mm && n->op == GGML_OP_MUL_MAT && rs && n->src[1] == rs) { mm = n; last = j; continue; }
        if (mm && n->op == GGML_OP_ADD && (n->src[0] == mm || n->src[1] == mm)) { add = n; last = j; }
        break;
    }
    if (!mm || !add || !rs) return 0;
    const ggml_tensor * wo = mm->src[0];
    const ggml_tensor * res = add->src[0] == mm ? add->src[1] : add->src[0];
    if (rs->op != GGML_OP_RESHAPE || rs->ne[0] != (int64_t) D * H || rs->ne[1] != 1) return 0;
    if (wo->type != GGML_TYPE_Q4_K || wo->ne[0] != (int64_t) D * H || wo->ne[2] != 1 || wo->ne[3] != 1 || wo->nb[0] != 144 ||
        wo->nb[1] % 16 || (uintptr_t) wo->data % 16 || tensor_is_split(wo)) return 0;
    const int64_t M = wo->ne[1];
    if (mm->ne[0] != M || mm->ne[1] != 1 || res == mm || res->type != GGML_TYPE_F32 || add->type != GGML_TYPE_F32) return 0;
    if (!mx_is_contiguous(res) || !mx_is_contiguous(add) || mx_nelements(res) != M || mx_nelements(add) != M) return 0;
    if (use(fa) != 1 || use(rs) != 1 || use(mm) != 1 || ((fa->flags | rs->flags | mm->flags) & GGML_TENSOR_FLAG_OUTPUT)) return 0;
    for (int j = i + 1; j < last; ++j) if (g->nodes[j] != mm && !ao_view(g->nodes[j])) return 0;
    // the output is stored by each row chunk's last workgroup while other workgroups may
    // still read q and the mask: it must not overlap them (in place over the residual is fine)
    for (const ggml_tensor * t : {q, m, k, v, wo})
        if (t && t_overlaps_ext(t, add)) return 0;
    if (add->data != res->data && t_overlaps_ext(res, add)) return 0;
    const bool v1 = (g_tune[27] & 16) != 0;    // A/B: round-3 v1 (redundant attention per row chunk)
    constexpr int TPR = 2, RPW = AO_NT / TPR;
    const int NP = H / 2, NR = v1 ? (int) mx_ceil_div(M, RPW) : (int) mx_ceil_div(M, 32);
    const int S2 = D * H == 4096 && !(g_tune[27] & 32) ? 2 : 1;   // v2 key splits (k_attn_o2<4, 2> / <4, 1> / <8, 1>)
    if (v1 && NR > MX_FA_CNT / 2) return 0;
    if (!v1 && D * H != 4096 && D * H != 8192) return 0;   // k_attn_o2<U>: K = 1024 U
    const size_t part_bytes = (v1 ? (size_t) NP * M : (size_t) D * H * S2 + 2 * S2 * H) * sizeof(uint2) + 256;
    if (c.scratch->avail() < part_bytes) return 0;
    for (int j = i; j <= last; ++j) {
        deferred_guard_node_ext(c, g->nodes[j]);
        act_cache_invalidate(c.s, g->nodes[j]);
    }
    AoArgs a{};
    a.q = (const char *) q->data; a.q2 = q->nb[2];
    a.k = (const char *) k->data; a.k1 = k->nb[1]; a.k2 = k->nb[2];
    a.v = (const char *) v->data; a.v1 = v->nb[1]; a.v2 = v->nb[2];
    a.mask = m ? (const uint16_t *) m->data : nullptr;   // row 0: the one query token
    a.wo = (const char *) wo->data; a.wo_row = wo->nb[1];
    a.res = (const float *) res->data;
    a.dst = (float *) add->data;
    a.part = (uint2 *) c.scratch->take(part_bytes);
    a.cnt = v1 ? c.s->fa_cnt + MX_FA_CNT / 2 : c.s->fa_cnt + MX_FA_CNT - 1;
    a.n_kv = n_kv; a.H = H; a.Hkv = Hkv; a.M = (int) M; a.NP = NP; a.NR = NR;
    a.scale = mx_op_param<float>(fa, 0);
    a.dbg = (g_tune[27] >> 1) & 7;
    a.trace = mx_trace_slot(0);
    a.trace_blk = mx_trace_blocks();
    const unsigned T = v1 ? (unsigned) (NP * NR) : (unsigned) (NP * S2 + NR);
    unsigned npf = 0;
    a.pf_n = (T % 8 == 0) ? c.s->pf_n : 0;   // prefetch ids must start on XCD 0
    for (int r = 0; r < a.pf_n; ++r) {
        a.pf[r] = c.s->pf_ptr[r]; a.pf_eighth[r] = c.s->pf_len[r] / 8; a.pf_lines[r] = (unsigned) (c.s->pf_take[r] / 128);
    }
    // v2: the CUs the attention and GEMV workgroups leave free (g_tune[21] > 0 forces a count,
    // < 0 none); v1: opt-in (at 132 VGPRs a CU holds no second 8-wave workgroup)
    if (a.pf_n && g_tune[21] > 0) npf = (unsigned) g_tune[21] & ~7u;
    else if (a.pf_n && !v1 && g_tune[21] == 0 && T < 256) npf = (256u - T) & ~7u;
    if (!npf) a.pf_n = 0;
    MX_KLOG("attn_o v%d D=%d n_kv=%d H=%d Hkv=%d M=%lld NP=%d NR=%d pf=%d", v1 ? 1 : 2, D, n_kv, H, Hkv, (long long) M, NP, NR, a.pf_n ? (int) npf : 0);
    if (v1) k_attn_o<TPR><<<T + npf, AO_NT, 0, c.st>>>(a);
    else if (D * H == 4096 && S2 == 2) k_attn_o2<4, 2><<<T + npf, AO_NT, 0, c.st>>>(a);
    else if (D * H == 4096) k_attn_o2<4, 1><<<T + npf, AO_NT, 0, c.st>>>(a);
    else k_attn_o2<8, 1><<<T + npf, AO_NT, 0, c.st>>>(a);
    return last - i + 1;
}

}  // namespace mx
#endif  // MX_AB_VARIANTS
