// ops_gemv_nc.hip — multi-column decode GEMV (round 6): dst[:, c] = W · x_c for 2..8
// activation columns (llama-server's parallel slots, speculative drafts). Reference:
// mul_mat_vec_q templated on ncols_dst 1..8 (ggml-cuda/mmvq.cu:397-502, dispatch
// ggml-cuda.cu:2183-2266 for src1->ne[1] <= MMVQ_MAX_BATCH_SIZE); its perf case is
// tests/test-backend-ops.cpp:8429-8435 (4096 x bs x 14336, bs 1..8).
//
// MI355X design. The round-1 k_mmvq (ops_mmvq.hip) read every column's q8 activation from
// the vector-memory path for every weight unit — NC x (32 + 8) bytes per 18-36 weight bytes
// — so its load path, not HBM, set the time (bs 2 at 0.30 of HBM, bs 8 at 0.11). Here the
// columns' q8 images (k_quantize_act, shared through the act cache) are staged into LDS by
// LDS-DMA once per workgroup, behind the first batch of weight loads (the k_gemv2 order:
// activation DMA, weights, wait for the DMA only); each lane unpacks a weight unit once and
// dots it against all NC columns out of LDS (w2_dot per column: the unpacking is common
// subexpression, the activation reads are the only per-column loads).
#include "backend.h"
#include "gemv.cuh"
#include "mm.h"

#include <type_traits>

namespace mx {

struct GncArgs {
    const char * w; size_t w_row;
    float * dst; size_t d_col;           // dst column stride (floats)
    const int8_t * q; const float * d; const float * s; int64_t kp;   // ActQ columns
    int nrows, units, K, ncols;
};

// LDS: NC q8 images (K bytes each), then NC x K/32 scales d, then NC x K/32 sums s
__host__ __device__ constexpr size_t gnc_lds_bytes(int nc, int64_t K) { return (size_t) nc * ((size_t) K + (size_t) K / 4); }

template <int QT, int LPR, int UPL, int NC>
__global__ __launch_bounds__(256) void k_gemv_nc(GncArgs p) {
    extern __shared__ __align__(16) char smem[];
    constexpr int NT = 256, RPW = 64 / LPR, STEP = LPR * UPL;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int sub = lane % LPR;
    const int blk = xcd_block((int) blockIdx.x, (int) gridDim.x, true);
    const int row = (blk * 4 + wave) * RPW + lane / LPR;
    const bool valid = row < p.nrows;
    const char * rows[1] = {p.w + (int64_t) (valid ? row : p.nrows - 1) * p.w_row};
    const int K = p.K, nb = K / 32;
    int8_t * lq = (int8_t *) smem;
    float * ld = (float *) (smem + (size_t) NC * K);
    float * ls = ld + NC * nb;
    // the activation DMA first: it retires before the weight loads issued after it
#pragma unroll
    for (int c = 0; c < NC; ++c) {
        const int cc = min(c, p.ncols - 1);      // padding columns re-read the last one
        dma_to_lds<NT, 16>(p.q + (int64_t) cc * p.kp, lq + (size_t) c * K, K);
        dma_to_lds<NT, 4>(p.d + (int64_t) cc * (p.kp / 32), ld + c * nb, nb * 4);
        dma_to_lds<NT, 4>(p.s + (int64_t) cc * (p.kp / 32), ls + c * nb, nb * 4);
    }
    W2<QT> r[1][UPL], r2[1][UPL];
    __builtin_amdgcn_sched_barrier(0);
    w2_load_batch<QT, UPL, 1>(rows, sub, LPR, p.units, r);
    __builtin_amdgcn_sched_barrier(0);
    wait_vmcnt<UPL * w2_loads<QT>()>();          // the DMA has landed (loads retire in order)
    lds_barrier();
    LdsAct act[NC];
#pragma unroll
    for (int c = 0; c < NC; ++c) act[c] = LdsAct{lq + (size_t) c * K, ld + c * nb, ls + c * nb};
    float acc[NC];
#pragma unroll
    for (int c = 0; c < NC; ++c) acc[c] = 0.f;
    // two register stages: batch it + 1's weights are in flight while batch it is dotted
    // against the NC columns (the grids here run 1-2 waves per SIMD: with one stage every
    // batch paid the whole memory latency and then its VALU work in series)
    auto dots = [&](const W2<QT> (&w)[1][UPL], int it) {
#pragma unroll
        for (int j = 0; j < UPL; ++j) {
            const int u = it * STEP + sub + j * LPR;
            if (u < p.units) {
#pragma unroll
                for (int c = 0; c < NC; ++c) acc[c] += w2_dot<QT>(w[0][j], u, act[c]);
            }
            __builtin_amdgcn_sched_barrier(0);
        }
    };
    const int n_iter = (p.units + STEP - 1) / STEP;
    for (int it = 0; it < n_iter; it += 2) {
        if (it + 1 < n_iter) w2_load_batch<QT, UPL, 1>(rows, (it + 1) * STEP + sub, LPR, p.units, r2);
        __builtin_amdgcn_sched_barrier(0);
        dots(r, it);
        if (it + 2 < n_iter) w2_load_batch<QT, UPL, 1>(rows, (it + 2) * STEP + sub, LPR, p.units, r);
        __builtin_amdgcn_sched_barrier(0);
        if (it + 1 < n_iter) dots(r2, it + 1);
    }
#pragma unroll
    for (int c = 0; c < NC; ++c) acc[c] = dpp_sum_group<LPR>(acc[c]);
    if (sub == LPR - 1 && valid) {
#pragma unroll
        for (int c = 0; c < NC; ++c) if (c < p.ncols) p.dst[(size_t) c * p.d_col + row] = acc[c];
    }
}

template <int QT, int NC, int LPR>
static void gnc_launch_l(OpCtx & c, const GncArgs & p) {
    constexpr int UPL = QT == GGML_TYPE_Q6_K ? 2 : 4;
    constexpr int RPB = 4 * (64 / LPR);
    const size_t lds = gnc_lds_bytes(NC, p.K);
    if (lds > 65536) MX_LDS_OPTIN((k_gemv_nc<QT, LPR, UPL, NC>), 160 * 1024);
    MX_KLOG("gemv_nc qt=%d nc=%d ncols=%d K=%d M=%d lds=%zu lpr=%d", QT, NC, p.ncols, p.K, p.nrows, lds, LPR);
    k_gemv_nc<QT, LPR, UPL, NC><<<(unsigned) ((p.nrows + RPB - 1) / RPB), 256, lds, c.st>>>(p);
}

template <int QT, int NC>
static void gnc_launch(OpCtx & c, const GncArgs & p) {
    // 4 units per lane in flight (Q6_K: 2, its unit holds 5 loads). Up to 4 columns: 32 lanes
    // per row, 8 rows per workgroup — twice the workgroups of 16-row tiles, and their LDS images
    // still fit two or more per CU (the waves waited 0.55 of their time at one per SIMD,
    // pmc_gnc_sq.json); 6 / 8 columns: 16 lanes x 16 rows (at 72-143 KB of LDS per workgroup
    // smaller tiles only add staging). Test-backend-ops perf, 4096 x bs x 14336, same box
    // (profiles/r06/multicolumn_gemv_table.txt): Q4_K bs 2 9.1 -> 7.7 us, bs 4 14.2 -> 12.2, bs 8
    // 24.8 -> 30.7 with 8-row tiles. g_tune[47] = 16 / 32 forces one geometry (sweeps).
    if (g_tune[47] == 16) return gnc_launch_l<QT, NC, 16>(c, p);
    if (g_tune[47] == 32 || NC <= 4) return gnc_launch_l<QT, NC, 32>(c, p);
    gnc_launch_l<QT, NC, 16>(c, p);
}

template <int QT>
static void gnc_type(OpCtx & c, const GncArgs & p) {
    switch (p.ncols) {
        case 2: gnc_launch<QT, 2>(c, p); break;
        case 3: gnc_launch<QT, 3>(c, p); break;
        case 4: gnc_launch<QT, 4>(c, p); break;
        case 5: case 6: gnc_launch<QT, 6>(c, p); break;
        default: gnc_launch<QT, 8>(c, p); break;
    }
}

static int gnc_nc(int64_t ncols) { return ncols <= 4 ? (int) ncols : (ncols <= 6 ? 6 : 8); }

// 2..8 columns of one channel (x->ne[2] == x->ne[3] == 1), contiguous dst columns, the
// LDS images within one CU's 160 KB
bool gemv_nc_ok(const ggml_tensor * dst) {
    static const bool off = getenv("GGML_MI355X_GEMV_NC_OFF") != nullptr;   // A/B: the round-1 k_mmvq
    const ggml_tensor * w = dst->src[0], * x = dst->src[1];
    if (off || !g_gemv2 || !gemv2_type_ok(w->type) || x->type != GGML_TYPE_F32 || dst->type != GGML_TYPE_F32) return false;
    const int64_t K = w->ne[0];
    const int64_t qk = (w->type == GGML_TYPE_Q4_0 || w->type == GGML_TYPE_Q8_0) ? 32 : 256;
    if (K % qk || x->ne[0] != K || x->ne[1] < 2 || x->ne[1] > 8 || x->ne[2] != 1 || x->ne[3] != 1) return false;
    if (w->ne[2] != 1 || w->ne[3] != 1 || w->nb[0] != (size_t) mx_type(w->type).size || w->ne[1] > INT32_MAX) return false;
    if (x->nb[0] != 4 || dst->nb[0] != 4 || dst->ne[0] != w->ne[1] || dst->ne[1] != x->ne[1] || dst->nb[1] % 4) return false;
    return gnc_lds_bytes(gnc_nc(x->ne[1]), K) <= 160 * 1024;
}

void gemv_nc_run(OpCtx & c, ggml_tensor * dst) {
    const ggml_tensor * w = dst->src[0], * x = dst->src[1];
    const ActQ a = quantize_activations(c, x);
    GncArgs p{};
    p.w = (const char *) w->data; p.w_row = w->nb[1];
    p.dst = (float *) dst->data; p.d_col = dst->nb[1] / 4;
    p.q = a.q; p.d = a.d; p.s = a.s; p.kp = a.kp;
    p.nrows = (int) w->ne[1]; p.K = (int) w->ne[0]; p.ncols = (int) x->ne[1];
    p.units = (int) (w->ne[0] / ((w->type == GGML_TYPE_Q4_0 || w->type == GGML_TYPE_Q8_0) ? 32 : 64));
    MX_ASSERT(a.kp == p.K);
    switch (w->type) {
        case GGML_TYPE_Q4_K: gnc_type<GGML_TYPE_Q4_K>(c, p); break;
        case GGML_TYPE_Q5_K: gnc_type<GGML_TYPE_Q5_K>(c, p); break;
        case GGML_TYPE_Q6_K: gnc_type<GGML_TYPE_Q6_K>(c, p); break;
        case GGML_TYPE_Q4_0: gnc_type<GGML_TYPE_Q4_0>(c, p); break;
        case GGML_TYPE_Q8_0: gnc_type<GGML_TYPE_Q8_0>(c, p); break;
        default: MX_ABORT("gemv_nc type %d", (int) w->type);
    }
}

}  // namespace mx

namespace mx {

// ---------------------------------------------------------------------------
// MoE decode: the down projection's MUL_MAT_ID and the expert combine in one launch
// (round 6). build_moe_ffn (src/llama-graph.cpp:1201-1296) ends every MoE layer with
// experts = MUL_MAT_ID(down_exps, glu, ids) -> MUL(experts, weights) -> the ADDs of the
// per-slot views [-> ADD(residual)]; k_moe_combine ran that tail as its own ~5 us launch
// (profiles/r06/, Mixtral tg: 4.8 us per layer). Here a workgroup owns RPB rows of one
// token for EVERY slot: it stages the n_used q8 activations (the gate/up SwiGLU's q8 copy)
// into LDS, streams each slot's expert rows (expert id read on the device), and writes
// out[row] = sum_s w_s * (W_{e_s} x_s)[row] (+ residual) — the combine's arithmetic in its
// order (slot 0 first, then + each next slot, then + the residual).
// ---------------------------------------------------------------------------
struct GmcArgs {
    const char * w; size_t w_row, w_exp; int n_expert;
    const char * ids; size_t id0, id1;
    const int8_t * q; const float * d; const float * s; int64_t kp;   // q8 column t * n_used + slot
    const float * wt; size_t wt1, wt2;                                 // weights [1, n_used, n_tok] (floats)
    const float * res; size_t r1;
    float * out; size_t o1;
    int nrows, units, K;
};

template <int QT, int LPR, int UPL, int NU>
__global__ __launch_bounds__(256) void k_moe_down_comb(GmcArgs p) {
    extern __shared__ __align__(16) char smem[];
    constexpr int NT = 256, RPW = 64 / LPR, STEP = LPR * UPL;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int sub = lane % LPR;
    const int blk = xcd_block((int) blockIdx.x, (int) gridDim.x, true);
    const int row = (blk * 4 + wave) * RPW + lane / LPR;
    const bool valid = row < p.nrows;
    const int64_t rr = valid ? row : p.nrows - 1;
    const int t = blockIdx.y;
    const int K = p.K, nb = K / 32;
    int8_t * lq = (int8_t *) smem;
    float * ld = (float *) (smem + (size_t) NU * K);
    float * ls = ld + NU * nb;
    // expert ids, router weights and the residual first: the weight addresses wait for the ids
    int ex[NU];
    float wt[NU];
#pragma unroll
    for (int s = 0; s < NU; ++s) {
        ex[s] = *(const int32_t *) (p.ids + (size_t) s * p.id0 + (size_t) t * p.id1);
        wt[s] = p.wt[(size_t) t * p.wt2 + (size_t) s * p.wt1];
    }
    const float res = p.res ? p.res[(size_t) t * p.r1 + rr] : 0.f;
#pragma unroll
    for (int s = 0; s < NU; ++s) {
        const int64_t col = (int64_t) t * NU + s;
        dma_to_lds<NT, 16>(p.q + col * p.kp, lq + (size_t) s * K, K);
        dma_to_lds<NT, 4>(p.d + col * (p.kp / 32), ld + s * nb, nb * 4);
        dma_to_lds<NT, 4>(p.s + col * (p.kp / 32), ls + s * nb, nb * 4);
    }
    const char * rows[NU];
#pragma unroll
    for (int s = 0; s < NU; ++s) rows[s] = p.w + (size_t) min(max(ex[s], 0), p.n_expert - 1) * p.w_exp + (size_t) rr * p.w_row;
    W2<QT> r[NU][UPL];
    __builtin_amdgcn_sched_barrier(0);
    w2_load_batch<QT, UPL, NU>(rows, sub, LPR, p.units, r);
    __builtin_amdgcn_sched_barrier(0);
    wait_vmcnt<UPL * NU * w2_loads<QT>()>();      // the DMA has landed (loads retire in order)
    lds_barrier();
    LdsAct act[NU];
#pragma unroll
    for (int s = 0; s < NU; ++s) act[s] = LdsAct{lq + (size_t) s * K, ld + s * nb, ls + s * nb};
    float acc[NU];
#pragma unroll
    for (int s = 0; s < NU; ++s) acc[s] = 0.f;
    const int n_iter = (p.units + STEP - 1) / STEP;
    for (int it = 0; it < n_iter; ++it) {
        if (it) w2_load_batch<QT, UPL, NU>(rows, it * STEP + sub, LPR, p.units, r);
#pragma unroll
        for (int j = 0; j < UPL; ++j) {
            const int u = it * STEP + sub + j * LPR;
            if (u < p.units) {
#pragma unroll
                for (int s = 0; s < NU; ++s) acc[s] += w2_dot<QT>(r[s][j], u, act[s]);
            }
            __builtin_amdgcn_sched_barrier(0);
        }
    }
#pragma unroll
    for (int s = 0; s < NU; ++s) acc[s] = dpp_sum_group<LPR>(acc[s]);
    if (sub == LPR - 1 && valid) {
        float v = 0.f;
#pragma unroll
        for (int s = 0; s < NU; ++s) {
            const float e = ex[s] >= 0 && ex[s] < p.n_expert ? acc[s] * wt[s] : 0.f;
            v = s == 0 ? e : v + e;
        }
        if (p.res) v += res;
        p.out[(size_t) t * p.o1 + row] = v;
    }
}

bool moe_down_combine_ok(int type, int64_t K, int64_t M, int n_used, int n_tok) {
    if (!g_gemv2 || !gemv2_type_ok(type) || M > INT32_MAX || n_tok < 1 || n_tok > 8) return false;
    if (n_used != 2 && n_used != 4 && n_used != 8) return false;
    const int64_t qk = (type == GGML_TYPE_Q4_0 || type == GGML_TYPE_Q8_0) ? 32 : 256;
    return K % qk == 0 && K <= GEMV2_MAX_K && gnc_lds_bytes(n_used, K) <= 160 * 1024;
}

template <int QT, int NU>
static void gmc_launch(OpCtx & c, const GmcArgs & p, int n_tok) {
    constexpr int UPL = NU <= 2 ? 2 : 1;
    const size_t lds = gnc_lds_bytes(NU, p.K);
    auto go = [&](auto lpr) {
        constexpr int LPR = decltype(lpr)::value, RPB = 4 * (64 / LPR);
        if (lds > 65536) MX_LDS_OPTIN((k_moe_down_comb<QT, LPR, UPL, NU>), 160 * 1024);
        MX_KLOG("moe_down_comb qt=%d n_used=%d n_tok=%d lpr=%d K=%d M=%d res=%d", QT, NU, n_tok, LPR, p.K, p.nrows, p.res != nullptr);
        k_moe_down_comb<QT, LPR, UPL, NU><<<dim3((unsigned) ((p.nrows + RPB - 1) / RPB), (unsigned) n_tok), 256, lds, c.st>>>(p);
    };
    if (p.units >= 128) go(std::integral_constant<int, 32>());
    else go(std::integral_constant<int, 16>());
}

template <int QT>
static void gmc_type(OpCtx & c, const GmcArgs & p, int n_used, int n_tok) {
    if (n_used == 2) gmc_launch<QT, 2>(c, p, n_tok);
    else if (n_used == 4) gmc_launch<QT, 4>(c, p, n_tok);
    else gmc_launch<QT, 8>(c, p, n_tok);
}

void moe_down_combine_launch(OpCtx & c, const MoeDownComb & a) {
    const ggml_tensor * as = a.as;
    GmcArgs p{};
    p.w = (const char *) as->data; p.w_row = as->nb[1]; p.w_exp = as->nb[2]; p.n_expert = (int) as->ne[2];
    p.ids = a.ids; p.id0 = a.id0; p.id1 = a.id1;
    p.q = a.q; p.d = a.qd; p.s = a.qs; p.kp = a.kp;
    p.wt = a.wt; p.wt1 = a.wt1; p.wt2 = a.wt2;
    p.res = a.res; p.r1 = a.r1;
    p.out = a.out; p.o1 = a.o1;
    p.nrows = (int) as->ne[1]; p.K = (int) as->ne[0];
    p.units = (int) (as->ne[0] / ((as->type == GGML_TYPE_Q4_0 || as->type == GGML_TYPE_Q8_0) ? 32 : 64));
    MX_ASSERT(a.kp == p.K && moe_down_combine_ok(as->type, p.K, p.nrows, a.n_used, a.n_tok));
    switch (as->type) {
        case GGML_TYPE_Q4_K: gmc_type<GGML_TYPE_Q4_K>(c, p, a.n_used, a.n_tok); break;
        case GGML_TYPE_Q5_K: gmc_type<GGML_TYPE_Q5_K>(c, p, a.n_used, a.n_tok); break;
        case GGML_TYPE_Q6_K: gmc_type<GGML_TYPE_Q6_K>(c, p, a.n_used, a.n_tok); break;
        case GGML_TYPE_Q4_0: gmc_type<GGML_TYPE_Q4_0>(c, p, a.n_used, a.n_tok); break;
        case GGML_TYPE_Q8_0: gmc_type<GGML_TYPE_Q8_0>(c, p, a.n_used, a.n_tok); break;
        default: MX_ABORT("moe_down_comb type %d", (int) as->type);
    }
}

}  // namespace mx
