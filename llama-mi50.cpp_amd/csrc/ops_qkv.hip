// ops_qkv.hip — fused decode attention-input block: the Q, K and V projections of
// one token in ONE launch, with RoPE (NORMAL mode) on Q and K in the epilogue and
// the K/V rows written straight into the f16 KV cache.
//
// Replaces, for n_tokens == 1, the node chain libllama emits per layer
// (src/models/llama.cpp:44-79 + build_attn src/llama-graph.cpp:1918-1945 +
// llama_kv_cache::cpy_k/cpy_v src/llama-kv-cache.cpp:1072-1161):
//   MUL_MAT(wq,x) MUL_MAT(wk,x) MUL_MAT(wv,x) ROPE(q) ROPE(k) SET_ROWS(k) SET_ROWS(v)
// = 7 launches → 1. The reference CUDA backend fuses ROPE→SET_ROWS only
// (ggml-cuda.cu:3088-3122). Semantics per node are unchanged: GEMV as mmvq,
// RoPE as ops.cpp:5523-5800 (theta by repeated multiplication), f32→f16 RNE stores.
#include "backend.h"
#include "mm.h"
#include <functional>
#include "gemv.cuh"

namespace mx {

struct QkvArgs {
    const char * w[3];
    size_t w_row[3];
    int rows[3];
    int nblk_q, nblk_k;            // block ranges: [0,nq) q, [nq,nq+nk) k, rest v
    int units_a, units_k, units_v, K;
    XStage xs;
    float * q_out;                 // roped q, f32 [n_embd]
    char * kc; size_t kc_nb1; const char * kidx; int kidx64;
    char * vc; size_t vc_nb1; const char * vidx; int vidx64; int v_trans;
    const int32_t * pos; const float * ff;
    const float2 * tab;            // RoPE (cos, sin) per dimension pair, k_rope_table
    int n_dims;
    float theta_scale, freq_scale, ext_factor, attn_factor, corr0, corr1;
    unsigned long long * trace;    // debug (MX_TRACE), workgroup 0
    unsigned long long * trace_blk;
    float * kq8f; float * vq8f;    // q8_0 caches: roped K / V rows staged in f32 (k_kv_store_q8)
};

__device__ __forceinline__ int64_t read_idx(const char * p, int is64, int64_t i) {
    return is64 ? ((const int64_t *) p)[i] : (int64_t) ((const int32_t *) p)[i];
}

// Geometry: LA lanes x UA units per row for Q/K (LA <= 32: the RoPE pair, rows 2i and
// 2i+1, sits LA lanes apart in one wave), LV x UV for V (no pairing). Rows per block =
// 4 waves x 64/L. Weight types per matrix: QTA (q), QTK (k), QTV (v) — the recipes mix
// them (Q4_K_M: v Q6_K on the use_more_bits layers, Q5_K on the others at 70B; 8-expert
// Q4_K_M/Q5_K_M: k and v Q8_0, src/llama-quant.cpp:302-321).
// BAL (round 3): one workgroup per 16 q rows that also takes 4 k rows and 4 v rows (7 waves:
// 0-3 q, 4 k, 5-6 v at 32 lanes per row) — the 448-block grid of the split layout (q 256 +
// k 64 + v 128 blocks: 1.75 per CU, so 192 CUs streamed two blocks while 64 idled) becomes
// 256 equal blocks (59.5 KB each at Llama-3-8B), one per CU; wave-uniform matrix choice.
template <int QTA, int QTK, int QTV, int MODE, int LA = 16, int UA = 4, int LV = 16, int UV = 4, bool BAL = false>
__global__ __launch_bounds__(BAL ? 448 : 256) void k_qkv_rope_store(QkvArgs p) {
    static_assert(LA <= 32, "RoPE pairs must share a wave");
    static_assert(!BAL || (LA == 16 && LV == 32), "balanced layout: 4 q/k rows, 2 v rows per wave");
    constexpr int NT = BAL ? 448 : 256;
    extern __shared__ __align__(16) char smem[];
    constexpr int RBA = 4 * (64 / LA), RBV = 4 * (64 / LV);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    int m, bl, row;
    if constexpr (BAL) {
        m = wave < 4 ? 0 : (wave == 4 ? 1 : 2);
        bl = (gridDim.x & 7) == 0 ? xcd_block((int) blockIdx.x, (int) gridDim.x, p.xs.xcd) : (int) blockIdx.x;
        row = m == 0 ? bl * 16 + wave * 4 + lane / 16 : (m == 1 ? bl * 4 + lane / 16 : bl * 4 + (wave - 5) * 2 + lane / 32);
    } else {
        // XCD-contiguous order within each matrix's block range (gemv.cuh xcd_block): every
        // 128-B line of q_out and of the K/V cache rows is then written by one XCD's L2
        m = (int) blockIdx.x < p.nblk_q ? 0 : ((int) blockIdx.x < p.nblk_q + p.nblk_k ? 1 : 2);
        const int base = m == 0 ? 0 : (m == 1 ? p.nblk_q : p.nblk_q + p.nblk_k);
        const int nb = m == 0 ? p.nblk_q : (m == 1 ? p.nblk_k : (int) gridDim.x - p.nblk_q - p.nblk_k);
        bl = (base & 7) == 0 ? xcd_block((int) blockIdx.x - base, nb, p.xs.xcd) : (int) blockIdx.x - base;
        row = m == 2 ? bl * RBV + wave * (64 / LV) + lane / LV : bl * RBA + wave * (64 / LA) + lane / LA;
    }
    const int L = m == 2 ? LV : LA;
    const int sub = lane % L;
    const bool valid = row < p.rows[m];
    const char * rows[1] = {p.w[m] + (int64_t) (valid ? row : p.rows[m] - 1) * p.w_row[m]};
    const LdsAct a = lds_act(smem, p.K);
    float * red = gemv_lds_red(smem, p.K);
    float acc[1];
    unsigned long long * tr = blockIdx.x == 0 ? p.trace : nullptr;
    MX_TRACE(tr, 0);
    MX_TRACE_BLK(p.trace_blk, 0);
    // epilogue operands (position, KV-cache row) prefetched ahead of the weight stream:
    // loaded in the epilogue they were two dependent round trips after the dot products
    int pos = p.pos[0];
    // (I64 indices only, see fuse_qkv_rope_store: one branch-free load)
    int64_t kvrow = ((const int64_t *) (m == 2 ? p.vidx : p.kidx))[m == 2 && p.v_trans ? (valid ? row : 0) : 0];
    const int d = row % p.n_dims;
    const bool odd = d & 1;
    const int i0 = d & ~1;
    // RoPE cos/sin of this row's dimension pair from the per-token table (k_rope_table):
    // computed per lane (theta loop + libm sincos) it cost ~2 us per launch
    float2 csn = p.tab[i0 / 2];
    auto fence = [&] { asm volatile("" : "+v"(pos)); asm volatile("" : "+v"(kvrow)); asm volatile("" : "+v"(csn.x)); asm volatile("" : "+v"(csn.y)); };
    StageRegs<NT, MODE> sr;
    stage_issue<NT, MODE>(p.xs, p.K, a, sr);
    // block-uniform branch (BAL: wave-uniform; every arm reaches the same barriers)
    if (m == 2) gemv_rows_staged<QTV, LV, UV, 1, NT, MODE>(rows, p.units_v, sub, a, p.xs, p.K, red, sr, acc, fence);
    else if (QTK != QTA && m == 1) gemv_rows_staged<QTK, LA, UA, 1, NT, MODE>(rows, p.units_k, sub, a, p.xs, p.K, red, sr, acc, fence);
    else gemv_rows_staged<QTA, LA, UA, 1, NT, MODE>(rows, p.units_a, sub, a, p.xs, p.K, red, sr, acc, fence);
    MX_TRACE(tr, 3);
    MX_TRACE_BLK(p.trace_blk, 1);
    const float v = acc[0];   // row sum: in lane sub == L-1 (every lane of the row for L <= 16)
    const float pv = __shfl_xor(v, LA, 64);
    if (sub != L - 1 || !valid) return;
    if (MX_DBG(p.xs.dbg & 4)) { if (m == 0) p.q_out[row] = v; return; }
    if (MX_DBG(p.xs.dbg & 8) && m > 0) return;
    if (m == 2) {
        if (p.vq8f) { p.vq8f[row] = v; return; }
        const uint16_t h = f2h(v);
        if (p.v_trans) *(uint16_t *) (p.vc + kvrow * p.vc_nb1) = h;
        else *(uint16_t *) (p.vc + kvrow * p.vc_nb1 + row * 2) = h;
        return;
    }
    const float cs = csn.x, sn = csn.y;
    const float x0 = odd ? pv : v, x1 = odd ? v : pv;
    const float r = odd ? x0 * sn + x1 * cs : x0 * cs - x1 * sn;
    if (m == 0) p.q_out[row] = r;
    else if (p.kq8f) p.kq8f[row] = r;
    else *(uint16_t *) (p.kc + kvrow * p.kc_nb1 + row * 2) = f2h(r);
    MX_TRACE(tr, 4);
}

// q8_0 KV caches (-ctk/-ctv q8_0): the token's roped K row and V row, staged in f32 by
// k_qkv_rope_store, quantised into their cache rows (SET_ROWS to a q8_0 tensor: from_float
// = quantize_row_q8_0: quants.cuh quantize_block_q8_0's arithmetic), one lane per element,
// a 32-lane half-wave per block (a thread per block serialised 32 loads: 12 us)
__global__ __launch_bounds__(256) void k_kv_store_q8(QkvArgs p, int nk, int nv) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;   // element of K then V (nk, nv % 32 == 0)
    const bool isk = e < nk;
    const int i = isk ? e : e - nk;
    const bool on = e < nk + nv;
    const float x = on ? (isk ? p.kq8f[i] : p.vq8f[min(i, nv - 1)]) : 0.f;
    const int lane = threadIdx.x & 63;
    const float amax = __shfl(dpp_max_group<32>(fabsf(x)), (lane & 32) | 31, 64);
    const float d = amax / 127.0f;
    const float id = d != 0.0f ? 1.0f / d : 0.0f;
    if (!on) return;
    const int64_t kvrow = ((const int64_t *) (isk ? p.kidx : p.vidx))[0];
    char * blk = (isk ? p.kc + kvrow * p.kc_nb1 : p.vc + kvrow * p.vc_nb1) + 34 * (i >> 5);
    blk[2 + (i & 31)] = (char) (int8_t) roundf(__fmul_rn(x, id));
    if ((i & 31) == 0) *(uint16_t *) blk = f2h(d);
}

void kv_new_row_flush(OpCtx & c) {
    KvNewRow & r = c.s->kvnew;
    if (!r.on) return;
    r.on = false;
    QkvArgs p{};
    p.kq8f = const_cast<float *>(r.k); p.vq8f = const_cast<float *>(r.v);
    p.kc = r.kc; p.kc_nb1 = r.kc_nb1; p.vc = r.vc; p.vc_nb1 = r.vc_nb1;
    p.kidx = (const char *) r.kidx; p.vidx = (const char *) r.vidx;
    const int nk = r.k ? r.nk : 0, nv = r.v ? r.nv : 0;
    MX_KLOG("kv_store_q8 nk=%d nv=%d", nk, nv);
    k_kv_store_q8<<<(unsigned) mx_ceil_div(nk + nv, 256), 256, 0, c.st>>>(p, nk, nv);
}

// (cos θ·m, sin θ·m) for every dimension pair of one position: rope_yarn
// (ggml-cpu/ops.cpp:5529-5546) with theta by repeated multiplication as rope_cache_init
// (ops.cpp:5548-5566) — the per-pair values of op_rope, computed once per token.
__device__ __forceinline__ float2 qkv_rope_cs(const QkvArgs & p, float pf, int i) {
    float theta = pf;
    for (int k = 0; k < i; ++k) theta *= p.theta_scale;
    if (p.ff) theta /= p.ff[i];
    const float ti = p.freq_scale * theta;
    float th = ti, ms = p.attn_factor;
    if (p.ext_factor != 0.0f) {
        const float y = (i - p.corr0) / fmaxf(0.001f, p.corr1 - p.corr0);
        const float mix = (1.0f - fminf(1.0f, fmaxf(0.0f, y))) * p.ext_factor;
        th = ti * (1 - mix) + theta * mix;
        ms *= 1.0f + 0.1f * logf(1.0f / p.freq_scale);
    }
    return make_float2(cosf(th) * ms, sinf(th) * ms);
}

__global__ void k_rope_table(QkvArgs p, float2 * tab) {
    const int i = threadIdx.x + blockIdx.x * blockDim.x;   // pair index
    if (i >= p.n_dims / 2) return;
    tab[i] = qkv_rope_cs(p, (float) p.pos[0], i);
}

// Prefill (n_tokens > 1) epilogue of the q/k/v projections (round 3): ROPE(q) -> the rope
// output, ROPE(k) -> K cache rows, v -> V cache rows, in one launch after the grouped GEMM
// instead of 2 ROPE + 2 SET_ROWS launches (k_rope2 + k_set_rows: ~26 us per pp512 layer).
// One workgroup per token: its (cos, sin) table in LDS (qkv_rope_cs: the k_rope2 / CPU
// values, bit-identical), then every adjacent row pair of q, k and v (NORMAL rope pairs
// 2i, 2i+1); f32 -> f16 cache stores round to nearest even as SET_ROWS does.
struct QkvPpArgs {
    const float * q; const float * k; const float * v;   // projections [M, N] f32, contiguous
    const float * part; int part_ld, ks, N, row0[3];     // SPLIT: the GEMM's split-K partials instead (mm.h M4Split)
    float * rq;                                          // roped q [n_dims, heads, N], contiguous
    char * kc; size_t kc_nb1; const int64_t * kidx;      // K cache view rows (f16), row per token
    char * vc; size_t vc_nb1; const int64_t * vidx;
    int Mq, Mk, Mv;
    // round 6: caches the epilogue cannot store itself (q8_0 / q4_0 rows, the transposed V of
    // -fa 0) get their f32 rows here instead — roped K in the ROPE(k) output, V in the V
    // projection — for the graph's own SET_ROWS node right after; skip_v: V is materialised
    // already (the plain GEMM wrote it) and only that SET_ROWS runs
    float * kf32; float * vf32; int skip_v;
};
// KS: 0 = the plain projections; > 0 = the q/k/v GEMM ran split-K (KS planes; -1: any
// count) and left its partial planes, summed here in plane order as k_mmq4_reduce adds
// them — the reduce pass and its round trip are gone. Pairs are processed CH at a time
// with every load of a chunk issued before any store (a loop that consumed each load
// before the next was one memory round trip per pair: 11.7 us per pp512 layer).
template <int KS>
__device__ __forceinline__ float2 qkv_pp_ld(const QkvPpArgs & e, int seg, int t, int j) {
    if constexpr (KS == 0) {
        const float * x = seg == 0 ? e.q + (size_t) t * e.Mq : seg == 1 ? e.k + (size_t) t * e.Mk : e.v + (size_t) t * e.Mv;
        return ((const float2 *) x)[j];
    } else {
        const float * b = e.part + (size_t) t * e.part_ld + e.row0[seg] + 2 * j;
        const size_t pl = (size_t) e.N * e.part_ld;
        float2 v = *(const float2 *) b;
        if constexpr (KS > 0) {
#pragma unroll
            for (int z = 1; z < KS; ++z) { const float2 w = *(const float2 *) (b + z * pl); v.x += w.x; v.y += w.y; }
        } else {
            for (int z = 1; z < e.ks; ++z) { const float2 w = *(const float2 *) (b + z * pl); v.x += w.x; v.y += w.y; }
        }
        return v;
    }
}
template <int KS>
__global__ __launch_bounds__(256) void k_qkv_pp_epi(QkvArgs p, QkvPpArgs e) {
    __shared__ float2 tab[MX_ROPE_TAB];
    const int t = blockIdx.x;
    const int np = p.n_dims / 2;
    const float pf = (float) p.pos[t];
    for (int i = threadIdx.x; i < np; i += blockDim.x) tab[i] = qkv_rope_cs(p, pf, i);
    const int pq = e.Mq / 2, pk = e.Mk / 2, pv = e.skip_v ? 0 : e.Mv / 2, total = pq + pk + pv;
    float2 * rq = (float2 *) (e.rq + (size_t) t * e.Mq);
    uint32_t * kr = (uint32_t *) (e.kf32 ? nullptr : e.kc + (size_t) e.kidx[t] * e.kc_nb1);
    uint32_t * vr = (uint32_t *) (e.vf32 || e.skip_v ? nullptr : e.vc + (size_t) e.vidx[t] * e.vc_nb1);
    constexpr int CH = 6;
    auto load_chunk = [&](int j0, float2 (&x)[CH]) {
#pragma unroll
        for (int c = 0; c < CH; ++c) {
            const int j = min(j0 + 256 * c, total - 1);           // clamped: loads, not branches
            const int seg = j < pq ? 0 : j < pq + pk ? 1 : 2;
            x[c] = qkv_pp_ld<KS>(e, seg, t, seg == 0 ? j : seg == 1 ? j - pq : j - pq - pk);
        }
    };
    auto store_chunk = [&](int j0, const float2 (&x)[CH]) {
#pragma unroll
        for (int c = 0; c < CH; ++c) {
            const int j = j0 + 256 * c;
            if (j >= total) break;
            if (j < pq) {
                const float2 cs = tab[j % np];
                rq[j] = make_float2(x[c].x * cs.x - x[c].y * cs.y, x[c].x * cs.y + x[c].y * cs.x);
            } else if (j < pq + pk) {
                const int jj = j - pq;
                const float2 cs = tab[jj % np];
                const float2 r = make_float2(x[c].x * cs.x - x[c].y * cs.y, x[c].x * cs.y + x[c].y * cs.x);
                if (e.kf32) ((float2 *) (e.kf32 + (size_t) t * e.Mk))[jj] = r;
                else kr[jj] = (uint32_t) f2h(r.x) | ((uint32_t) f2h(r.y) << 16);
            } else {
                const int jj = j - pq - pk;
                if (e.vf32) ((float2 *) (e.vf32 + (size_t) t * e.Mv))[jj] = x[c];
                else vr[jj] = (uint32_t) f2h(x[c].x) | ((uint32_t) f2h(x[c].y) << 16);
            }
        }
    };
    float2 x[CH];
    load_chunk(threadIdx.x, x);                  // the first chunk's loads fly while the table is built
    __syncthreads();
    store_chunk(threadIdx.x, x);
    for (int j0 = threadIdx.x + CH * 256; j0 < total; j0 += CH * 256) {
        load_chunk(j0, x);
        store_chunk(j0, x);
    }
}

static const ggml_tensor * base_of(const ggml_tensor * t) {
    while (t && (t->op == GGML_OP_RESHAPE || t->op == GGML_OP_VIEW)) t = t->src[0];
    return t;
}

static float yarn_corr(int n_dims, int n_ctx_orig, float n_rot, float base) {
    return n_dims * logf(n_ctx_orig / (n_rot * 2 * (float) M_PI)) / (2 * logf(base));
}



// Prefill form of the match below (n_tokens > 8, f16 caches, V stored untransposed — the
// -fa 1 graph): the three projections as the grouped GEMM (k_mmq4 / k_mmq3m), then
// k_qkv_pp_epi for the two ROPEs and the two SET_ROWS. g_tune[27] bit 128 or
// GGML_MI355X_NO_QKV_PP=1: node by node (A/B).
static const bool g_no_qkv_pp = getenv("GGML_MI355X_NO_QKV_PP") != nullptr;
static int qkv_prefill(OpCtx & c, ggml_cgraph * g, int i, int last, const ggml_tensor * x, ggml_tensor * mq, ggml_tensor * mk,
                       ggml_tensor * mv, ggml_tensor * rq, ggml_tensor * rk, ggml_tensor * sk, ggml_tensor * sv,
                       const std::function<int(const ggml_tensor *)> & uses) {
    if (g_no_qkv_pp || (g_tune[27] & 128)) return 0;
    const int64_t N = x->ne[1];
    if (x->ne[2] != 1 || x->ne[3] != 1 || N > INT32_MAX) return 0;
    for (const ggml_tensor * r : {rq, rk}) {
        if (mx_op_param<int32_t>(r, 2) != GGML_ROPE_TYPE_NORMAL || r->type != GGML_TYPE_F32 || !mx_is_contiguous(r)) return 0;
        if (r->src[1]->type != GGML_TYPE_I32 || r->src[1]->ne[0] != N) return 0;
    }
    if (memcmp(rq->op_params, rk->op_params, 11 * sizeof(int32_t)) != 0 || rq->src[1] != rk->src[1] || rq->src[2] != rk->src[2]) return 0;
    const int n_dims = mx_op_param<int32_t>(rq, 1);
    if (n_dims != rq->ne[0] || n_dims != rk->ne[0] || n_dims % 2 || n_dims > 2 * MX_ROPE_TAB || (rq->src[2] && rq->src[2]->type != GGML_TYPE_F32)) return 0;
    const int64_t Mq = mq->ne[0], Mk = mk->ne[0], Mv = mv->ne[0];
    for (const ggml_tensor * m : {mq, mk, mv})
        if (m->type != GGML_TYPE_F32 || !mx_is_contiguous(m) || m->ne[1] != N || m->ne[2] != 1 || m->ne[3] != 1 || m->ne[0] % 2) return 0;
    if (mx_nelements(rq) != Mq * N || mx_nelements(rk) != Mk * N || Mq % n_dims || Mk % n_dims) return 0;
    if ((mq->flags | mk->flags | mv->flags | rk->flags) & GGML_TENSOR_FLAG_OUTPUT) return 0;
    if (uses(mq) != 1 || uses(mk) != 1 || uses(rk) != 1) return 0;
    // (mv: one use, or two for -fa 0's V — the reshape the transposed SET_ROWS reads and
    // nothing else: uses counts the graph's direct consumers)
    if (uses(mv) != 1) return 0;
    // SET_ROWS: f16 cache views stored by the epilogue (one row of the projection per token,
    // I64 indices); round 6: other caches keep their SET_ROWS node, fed f32 rows by the
    // epilogue (k_mode / v_mode 1: q8_0 / q4_0 rows; v_mode 2: -fa 0's transposed V, one index
    // per element) — the q/k/v GEMM stays grouped and the two ROPEs fused either way
    const ggml_tensor * kix = sk->src[1], * vix = sv->src[1];
    auto qcache = [](const ggml_tensor * t) { return t->type == GGML_TYPE_Q8_0 || t->type == GGML_TYPE_Q4_0; };
    int k_mode = 0, v_mode = 0;
    if (sk->type == GGML_TYPE_F16 && sk->nb[0] == 2) k_mode = 0;
    else if (qcache(sk) && sk->ne[0] == Mk) k_mode = 1;
    else return 0;
    if (sk->ne[0] != Mk || sk->src[0]->ne[0] != Mk || sk->src[0]->ne[1] != N || kix->ne[0] != N || kix->type != GGML_TYPE_I64) return 0;
    if (sv->type == GGML_TYPE_F16 && sv->nb[0] == 2 && sv->ne[0] == Mv && sv->src[0]->ne[0] == Mv && sv->src[0]->ne[1] == N && vix->ne[0] == N) v_mode = 0;
    else if (qcache(sv) && sv->ne[0] == Mv && sv->src[0]->ne[0] == Mv && sv->src[0]->ne[1] == N && vix->ne[0] == N) v_mode = 1;
    else if (sv->type == GGML_TYPE_F16 && sv->ne[0] == 1 && sv->src[0]->ne[0] == 1 && sv->src[0]->ne[1] == Mv * N &&
             vix->ne[0] == Mv * N) v_mode = 2;
    else return 0;
    if (vix->type != GGML_TYPE_I64 || !mx_is_contiguous(kix) || !mx_is_contiguous(vix)) return 0;
    if (k_mode == 0 && (sk->nb[1] % 4 || (uintptr_t) sk->data % 4)) return 0;
    if (v_mode == 0 && (sv->nb[1] % 4 || (uintptr_t) sv->data % 4)) return 0;
    // f32 rows for the SET_ROWS nodes: where those nodes read (the ROPE(k) output, the V
    // projection), contiguous [M, N]; kept in place only (no scratch copies below)
    if (k_mode && (base_of(sk->src[0]) != rk || !mx_is_contiguous(rk) || (rk->flags & GGML_TENSOR_FLAG_OUTPUT))) return 0;
    if (v_mode && (base_of(sv->src[0]) != mv || (mv->flags & GGML_TENSOR_FLAG_OUTPUT))) return 0;
    for (int j = i; j <= last; ++j) {
        deferred_guard_node_ext(c, g->nodes[j]);
        act_cache_invalidate(c.s, g->nodes[j]);
    }
    // The fused launch moves mk / mv (and the stores) ahead of the nodes between the
    // members; libllama's order (q, RoPE(q), v, k, RoPE(k): build_attn's expansion) lets the
    // allocator place a later projection over one that has died in between (mv over mq).
    // Overlapping outputs go to scratch copies instead (shallow tensor copies, data moved);
    // the rope output may sit exactly on mq (each thread reads its pair before writing it).
    const bool disjoint = !t_overlaps_ext(mq, mk) && !t_overlaps_ext(mq, mv) && !t_overlaps_ext(mk, mv) &&
                          !t_overlaps_ext(x, mq) && !t_overlaps_ext(x, mk) && !t_overlaps_ext(x, mv) &&
                          !t_overlaps_ext(rq, mk) && !t_overlaps_ext(rq, mv) && (rq->data == mq->data || !t_overlaps_ext(rq, mq));
    ggml_tensor tcp[3];
    ggml_tensor * mms[3] = {mq, mk, mv};
    // The epilogue's f32 rows for the SET_ROWS nodes go where those nodes read them (rk, mv);
    // with them, the outputs the epilogue writes (rq, rk, mv) must be distinct memory. libllama's
    // allocator puts a later projection over one that died in between (mv over mq: not
    // disjoint), so then the GEMM writes scratch copies below and only rq / rk / mv are written
    // in place. (ROPE may run in place: rk exactly on mk is fine, each thread reads its pair
    // before writing it.)
    if (k_mode && (t_overlaps_ext(rk, rq) || (v_mode && t_overlaps_ext(rk, mv)) ||
                   (disjoint && ((t_overlaps_ext(rk, mk) && rk->data != mk->data) || t_overlaps_ext(rk, mq) || t_overlaps_ext(rk, mv) ||
                                 t_overlaps_ext(rk, x))))) return 0;
    if (v_mode && t_overlaps_ext(mv, rq)) return 0;
    if (!disjoint) {
        const size_t need = (size_t) (Mq + Mk + Mv) * N * sizeof(float) + 3 * 256;
        if (c.scratch->avail() < need) return 0;
        for (int k = 0; k < 3; ++k) {
            tcp[k] = *mms[k];
            tcp[k].data = c.scratch->take((size_t) mms[k]->ne[0] * N * sizeof(float));
            mms[k] = &tcp[k];
        }
    }
    M4Split sp{};
    g_m4_split = (g_tune[27] & 256) ? nullptr : &sp;   // bit 256: keep the reduce pass (A/B)
    const bool grouped = mmq_group_run(c, mms, 3);
    g_m4_split = nullptr;
    if (!grouped) { sp.ks = 0; op_mul_mat(c, mms[0]); op_mul_mat(c, mms[1]); op_mul_mat(c, mms[2]); }
    QkvArgs p{};
    p.pos = (const int32_t *) rq->src[1]->data;
    p.ff = rq->src[2] ? (const float *) rq->src[2]->data : nullptr;
    p.n_dims = n_dims;
    const int n_ctx_orig = mx_op_param<int32_t>(rq, 4);
    const float base = mx_op_param<float>(rq, 5);
    p.freq_scale = mx_op_param<float>(rq, 6);
    p.ext_factor = mx_op_param<float>(rq, 7);
    p.attn_factor = mx_op_param<float>(rq, 8);
    p.theta_scale = powf(base, -2.0f / n_dims);
    p.corr0 = std::max(0.0f, floorf(yarn_corr(n_dims, n_ctx_orig, mx_op_param<float>(rq, 9), base)));
    p.corr1 = std::min((float) (n_dims - 1), ceilf(yarn_corr(n_dims, n_ctx_orig, mx_op_param<float>(rq, 10), base)));
    QkvPpArgs e{};
    e.q = (const float *) mms[0]->data; e.k = (const float *) mms[1]->data; e.v = (const float *) mms[2]->data;
    e.rq = (float *) rq->data;
    e.kc = (char *) sk->data; e.kc_nb1 = sk->nb[1]; e.kidx = (const int64_t *) kix->data;
    e.vc = (char *) sv->data; e.vc_nb1 = sv->nb[1]; e.vidx = (const int64_t *) vix->data;
    e.Mq = (int) Mq; e.Mk = (int) Mk; e.Mv = (int) Mv;
    if (k_mode) e.kf32 = (float *) rk->data;
    if (v_mode) {
        // the split-K planes summed (or the scratch copy moved) into the V projection; else
        // the plain GEMM wrote it in place
        if (sp.ks > 1 || mms[2] != mv) e.vf32 = (float *) mv->data;
        else e.skip_v = 1;
    }
    MX_KLOG("qkv_pp N=%lld Mq=%lld Mk=%lld Mv=%lld n_dims=%d ks=%d disjoint=%d k_mode=%d v_mode=%d", (long long) N, (long long) Mq,
            (long long) Mk, (long long) Mv, n_dims, sp.ks, (int) disjoint, k_mode, v_mode);
    if (sp.ks > 1) {
        e.part = sp.part; e.part_ld = sp.part_ld; e.ks = sp.ks; e.N = (int) N;
        for (int k = 0; k < 3; ++k) e.row0[k] = sp.row0[k];
        if (sp.ks == 2) k_qkv_pp_epi<2><<<(unsigned) N, 256, 0, c.st>>>(p, e);
        else k_qkv_pp_epi<-1><<<(unsigned) N, 256, 0, c.st>>>(p, e);
    } else k_qkv_pp_epi<0><<<(unsigned) N, 256, 0, c.st>>>(p, e);
    // the SET_ROWS nodes of the caches the epilogue did not store (q8_0 / q4_0 rows, the
    // transposed V) — their sources now hold the f32 rows
    if (k_mode) op_set_rows(c, sk);
    if (v_mode) op_set_rows(c, sv);
    return last - i + 1;
}

// Returns the number of graph nodes consumed starting at i (0 = not fused).
int fuse_qkv_rope_store(OpCtx & c, ggml_cgraph * g, int i, const UseCount & use_map) {
    auto uses = [&](const ggml_tensor * t) { auto it = use_map.find(t); return it == use_map.end() ? 0 : it->second; };
    // Collect the 7 member nodes from i on, skipping views. Any other node in the
    // window aborts the match, so running the fused kernel at position i cannot
    // reorder anything but the members. Order-independent: matches both this
    // runner's order and libllama's (q, v, k expansion, build_attn).
    ggml_tensor * mm[3] = {}, * rope[2] = {}, * sr[2] = {};
    int n_mm = 0, n_rope = 0, n_sr = 0, last = -1;
    const ggml_tensor * x = g->nodes[i]->src[1];
    if (g->nodes[i]->op != GGML_OP_MUL_MAT || !x) return 0;
    auto is_mm = [&](const ggml_tensor * t) { for (int k = 0; k < n_mm; ++k) if (mm[k] == t) return true; return false; };
    auto is_rope = [&](const ggml_tensor * t) { for (int k = 0; k < n_rope; ++k) if (rope[k] == t) return true; return false; };
    for (int j = i; j < g->n_nodes && j < i + 32; ++j) {
        ggml_tensor * n = g->nodes[j];
        if (n->op == GGML_OP_RESHAPE || n->op == GGML_OP_VIEW) continue;
        if (n->op == GGML_OP_MUL_MAT && n->src[1] == x && n_mm < 3) mm[n_mm++] = n;
        else if (n->op == GGML_OP_ROPE && n_rope < 2 && is_mm(base_of(n->src[0]))) rope[n_rope++] = n;
        else if (n->op == GGML_OP_SET_ROWS && n_sr < 2 && (is_rope(base_of(n->src[0])) || is_mm(base_of(n->src[0])))) sr[n_sr++] = n;
        else return 0;
        last = j;
        if (n_mm == 3 && n_rope == 2 && n_sr == 2) break;
    }
    if (n_mm != 3 || n_rope != 2 || n_sr != 2) return 0;
    // classify: K is the roped projection that is stored, Q the roped one that is not,
    // V the projection stored without rope
    ggml_tensor * rq = nullptr, * rk = nullptr, * sk = nullptr, * sv = nullptr;
    for (ggml_tensor * r : sr) {
        const ggml_tensor * src = base_of(r->src[0]);
        if (src == rope[0] || src == rope[1]) { if (sk) return 0; sk = r; rk = (ggml_tensor *) src; }
        else { if (sv) return 0; sv = r; }
    }
    if (!sk || !sv) return 0;
    rq = rope[0] == rk ? rope[1] : rope[0];
    ggml_tensor * mq = (ggml_tensor *) base_of(rq->src[0]), * mk = (ggml_tensor *) base_of(rk->src[0]);
    ggml_tensor * mv = (ggml_tensor *) base_of(sv->src[0]);
    if (mq == mk || mq == mv || mk == mv) return 0;
    if (x->ne[1] > 8) return qkv_prefill(c, g, i, last, x, mq, mk, mv, rq, rk, sk, sv, uses);
    if (x->ne[1] != 1 || x->ne[2] != 1 || x->ne[3] != 1) return 0;
    if (!g_gemv2 || !gemv2_ok(mq->src[0], x, mq) || !gemv2_ok(mk->src[0], x, mk) || !gemv2_ok(mv->src[0], x, mv)) return 0;
    const ggml_tensor * wq = mq->src[0], * wk = mk->src[0], * wv = mv->src[0];
    if (wq->ne[0] != wk->ne[0] || wq->ne[0] != wv->ne[0]) return 0;
    for (const ggml_tensor * r : {rq, rk}) {
        if (mx_op_param<int32_t>(r, 2) != GGML_ROPE_TYPE_NORMAL || r->type != GGML_TYPE_F32 || !mx_is_contiguous(r)) return 0;
        if (r->src[1]->type != GGML_TYPE_I32 || r->src[1]->ne[0] != 1) return 0;
    }
    if (memcmp(rq->op_params, rk->op_params, 11 * sizeof(int32_t)) != 0 || rq->src[1] != rk->src[1] || rq->src[2] != rk->src[2]) return 0;
    const int n_dims = mx_op_param<int32_t>(rq, 1);
    if (n_dims != rq->ne[0] || n_dims % 2 || n_dims > 2 * MX_ROPE_TAB || (rq->src[2] && rq->src[2]->type != GGML_TYPE_F32)) return 0;
    // only the fused consumers may read the intermediate results
    if ((mq->flags | mk->flags | mv->flags | rk->flags) & GGML_TENSOR_FLAG_OUTPUT) return 0;
    if (uses(mq) != 1 || uses(mk) != 1 || uses(mv) != 1 || uses(rk) != 1) return 0;
    // KV stores: f16 or q8_0 caches (q8_0 rows quantised by k_kv_store_q8), K and V types
    // independent (round 6: -ctk q8_0 -ctv f16, the fork's own line), one token
    const bool kq8 = sk->type == GGML_TYPE_Q8_0, vq8 = sv->type == GGML_TYPE_Q8_0;
    if ((!kq8 && sk->type != GGML_TYPE_F16) || (!vq8 && sv->type != GGML_TYPE_F16)) return 0;
    const size_t eszk = kq8 ? 34 : 2, eszv = vq8 ? 34 : 2;
    const ggml_tensor * kix = sk->src[1], * vix = sv->src[1];
    if (sk->src[0]->ne[0] != wk->ne[1] || sk->src[0]->ne[1] != 1 || kix->ne[0] != 1 || sk->nb[0] != eszk) return 0;
    int v_trans;
    if (sv->src[0]->ne[0] == wv->ne[1] && sv->src[0]->ne[1] == 1 && vix->ne[0] == 1 && sv->nb[0] == eszv) v_trans = 0;
    else if (!vq8 && sv->src[0]->ne[0] == 1 && sv->src[0]->ne[1] == wv->ne[1] && vix->ne[0] == wv->ne[1] && sv->ne[0] == 1) v_trans = 1;
    else return 0;
    const bool anyq8 = kq8 || vq8;
    if ((kq8 && wk->ne[1] % 32) || (vq8 && wv->ne[1] % 32) || (anyq8 && c.scratch->avail() < (size_t) 4 * (wk->ne[1] + wv->ne[1]) + 512)) return 0;
    for (const ggml_tensor * ix : {kix, vix}) if (ix->type != GGML_TYPE_I64) return 0;   // llama's KV indices
    // Round 5, row-split weights (-sm row): q, k and v split alike, at head boundaries (the
    // 256-row slice granule is a multiple of n_dims): one fused launch per slice on the
    // slice device's own stream (split_fork / split_join), writing its q rows, its K / V
    // cache columns and its RoPE on the main device through peer access — instead of 3
    // GEMVs + 2 ROPE + 2 SET_ROWS launches per slice pair
    const bool split = tensor_is_split(wq) || tensor_is_split(wk) || tensor_is_split(wv);
    void * sd[3][MX_MAX_DEVICES];
    int64_t slo[3][MX_MAX_DEVICES], shi[3][MX_MAX_DEVICES];
    int sdev[3][MX_MAX_DEVICES], ns = 0;
    if (split) {
        const int n_dims_q = mx_op_param<int32_t>(rq, 1);
        if (anyq8 || !tensor_is_split(wq) || !tensor_is_split(wk) || !tensor_is_split(wv) || n_dims_q <= 0) return 0;
        for (int t = 0; t < 3; ++t) {
            const int n = split_slices(c.s, t == 0 ? wq : t == 1 ? wk : wv, sd[t], slo[t], shi[t], sdev[t]);
            if (!n || (t && n != ns)) return 0;
            ns = n;
        }
        for (int k = 0; k < ns; ++k) {
            if (sdev[1][k] != sdev[0][k] || sdev[2][k] != sdev[0][k]) return 0;
            if (slo[0][k] % n_dims_q || slo[1][k] % n_dims_q || (shi[0][k] - slo[0][k]) % 2 || (shi[1][k] - slo[1][k]) % 2) return 0;
        }
    }

    QkvArgs p{};
    const ggml_tensor * ws[3] = {wq, wk, wv};
    for (int t = 0; t < 3; ++t) { p.w[t] = (const char *) ws[t]->data; p.w_row[t] = ws[t]->nb[1]; p.rows[t] = ws[t]->ne[1]; }
    // geometry (g_tune[12] sweeps; opbench attn_in + decode bench on MI355X,
    // profiles/r01/opbench_qkv_geometry.txt): Q/K 16 lanes x 2 units (two batches over
    // K = 4096), V 32 x 2 — 6.9 us vs 8.3 for the 16 x 4 / 16 x 4 of the first version:
    // half the per-lane dot tail
    int cfg = g_tune[12] ? g_tune[12] - 1 : 5;
    static const int GEO[6][4] = {{16, 4, 16, 4}, {16, 4, 64, 1}, {32, 2, 64, 1}, {32, 2, 32, 2}, {32, 1, 32, 1}, {16, 2, 32, 2}};
    if (cfg < 0 || cfg > 5) cfg = 5;
    const int rba = 4 * (64 / GEO[cfg][0]), rbv = 4 * (64 / GEO[cfg][2]);
    p.nblk_q = (int) mx_ceil_div(wq->ne[1], rba);
    p.K = (int) wq->ne[0];
    auto units = [](const ggml_tensor * w) { return (int) (w->ne[0] / ((w->type == GGML_TYPE_Q4_0 || w->type == GGML_TYPE_Q8_0) ? 32 : 64)); };
    p.units_a = units(wq); p.units_k = units(wk); p.units_v = units(wv);
    p.nblk_k = (int) mx_ceil_div(wk->ne[1], rba);
    const int nblk_v = (int) mx_ceil_div(wv->ne[1], rbv);
    p.q_out = (float *) rq->data;
    p.kc = (char *) sk->data; p.kc_nb1 = sk->nb[1]; p.kidx = (const char *) kix->data; p.kidx64 = kix->type == GGML_TYPE_I64;
    p.vc = (char *) sv->data; p.vc_nb1 = sv->nb[1]; p.vidx = (const char *) vix->data; p.vidx64 = vix->type == GGML_TYPE_I64;
    p.v_trans = v_trans;
    p.pos = (const int32_t *) rq->src[1]->data;
    p.ff = rq->src[2] ? (const float *) rq->src[2]->data : nullptr;
    p.n_dims = n_dims;
    p.trace = mx_trace_slot(2);
    p.trace_blk = mx_trace_blocks();
    const int n_ctx_orig = mx_op_param<int32_t>(rq, 4);
    const float base = mx_op_param<float>(rq, 5);
    p.freq_scale = mx_op_param<float>(rq, 6);
    p.ext_factor = mx_op_param<float>(rq, 7);
    p.attn_factor = mx_op_param<float>(rq, 8);
    p.theta_scale = powf(base, -2.0f / n_dims);
    p.corr0 = std::max(0.0f, floorf(yarn_corr(n_dims, n_ctx_orig, mx_op_param<float>(rq, 9), base)));
    p.corr1 = std::min((float) (n_dims - 1), ceilf(yarn_corr(n_dims, n_ctx_orig, mx_op_param<float>(rq, 10), base)));

    const int ta = wq->type, tk = wk->type, tv = wv->type;
    void (*kern)(QkvArgs) = nullptr;
    // the (q, k, v) weight-type triples of the recipes: Q4_K_M / Q5_K_M (v Q6_K on the
    // use_more_bits layers; v Q5_K at 70B; k and v Q8_0 for 8 experts), Q4_0, Q8_0, Q6_K.
    // The Llama-3-8B Q4_K_M mixes get every geometry; the others the default one.
#define QKV_TYPES(X) X(GGML_TYPE_Q4_K, GGML_TYPE_Q4_K, GGML_TYPE_Q4_K) X(GGML_TYPE_Q4_K, GGML_TYPE_Q4_K, GGML_TYPE_Q6_K) \
    X(GGML_TYPE_Q4_K, GGML_TYPE_Q4_K, GGML_TYPE_Q5_K) X(GGML_TYPE_Q4_K, GGML_TYPE_Q4_K, GGML_TYPE_Q8_0) \
    X(GGML_TYPE_Q4_K, GGML_TYPE_Q8_0, GGML_TYPE_Q8_0) X(GGML_TYPE_Q5_K, GGML_TYPE_Q5_K, GGML_TYPE_Q5_K) \
    X(GGML_TYPE_Q5_K, GGML_TYPE_Q5_K, GGML_TYPE_Q6_K) X(GGML_TYPE_Q5_K, GGML_TYPE_Q5_K, GGML_TYPE_Q8_0) \
    X(GGML_TYPE_Q5_K, GGML_TYPE_Q8_0, GGML_TYPE_Q8_0) X(GGML_TYPE_Q6_K, GGML_TYPE_Q6_K, GGML_TYPE_Q6_K) \
    X(GGML_TYPE_Q4_0, GGML_TYPE_Q4_0, GGML_TYPE_Q4_0) X(GGML_TYPE_Q8_0, GGML_TYPE_Q8_0, GGML_TYPE_Q8_0)
#define GEOS(TA, TV, M) if (ta == TA && tk == TA && tv == TV) kern = cfg == 0 ? k_qkv_rope_store<TA, TA, TV, M, 16, 4, 16, 4> : \
        cfg == 1 ? k_qkv_rope_store<TA, TA, TV, M, 16, 4, 64, 1> : cfg == 2 ? k_qkv_rope_store<TA, TA, TV, M, 32, 2, 64, 1> : \
        cfg == 3 ? k_qkv_rope_store<TA, TA, TV, M, 32, 2, 32, 2> : cfg == 4 ? k_qkv_rope_store<TA, TA, TV, M, 32, 1, 32, 1> : \
        k_qkv_rope_store<TA, TA, TV, M, 16, 2, 32, 2>;
#define QKV(TA, TK, TV) if (ta == TA && tk == TK && tv == TV) kern = k_qkv_rope_store<TA, TK, TV, XS_NORM, 16, 2, 32, 2>;
    QKV_TYPES(QKV)
#undef QKV
    GEOS(GGML_TYPE_Q4_K, GGML_TYPE_Q4_K, XS_NORM) GEOS(GGML_TYPE_Q4_K, GGML_TYPE_Q6_K, XS_NORM)
    if (!kern) return 0;
    if (!fused_io_ok({rq, sk, sv}, {rq->src[1], rq->src[2], kix, vix})) return 0;
    if (!gemv2_stage(c, x, {rq, sk, sv}, {}, &p.xs, 3)) return 0;
    const int mode = gemv_mode(p.xs, p.K, 0);
    if (mode != XS_NORM) {   // the fused block normally follows attn_norm; other sources
#define QKV(TA, TK, TV) if (ta == TA && tk == TK && tv == TV) kern = mode == XS_Q8 ? k_qkv_rope_store<TA, TK, TV, XS_Q8, 16, 2, 32, 2> : \
        mode == XS_NORM_H2 ? k_qkv_rope_store<TA, TK, TV, XS_NORM_H2, 16, 2, 32, 2> : k_qkv_rope_store<TA, TK, TV, XS_F32_H2, 16, 2, 32, 2>;
        QKV_TYPES(QKV)
#undef QKV
    }
#undef QKV_TYPES
    // the per-token RoPE table: once per graph pass for a (position, params, factors) key
    Stream * S = c.s;
    if (!S->rope_valid || S->rope_pos != (const void *) p.pos || S->rope_ff != (const void *) p.ff ||
        memcmp(S->rope_params, rq->op_params, sizeof(S->rope_params)) != 0) {
        k_rope_table<<<(n_dims / 2 + 63) / 64, 64, 0, c.st>>>(p, (float2 *) S->rope_tab);
        S->rope_valid = true; S->rope_pos = p.pos; S->rope_ff = p.ff;
        memcpy(S->rope_params, rq->op_params, sizeof(S->rope_params));
    }
    p.tab = (const float2 *) S->rope_tab;
    for (int j = i; j <= last; ++j) act_cache_invalidate(c.s, g->nodes[j]);
#undef GEOS
    if (mode != XS_NORM && cfg != 5) return 0;   // the other sources exist in the default geometry only
    dim3 grid((unsigned) (p.nblk_q + p.nblk_k + nblk_v));
    unsigned nthr = 256;
    // balanced layout (GQA 4: q rows = 4 x k rows = 4 x v rows, one block per 16 q rows),
    // default geometry, the norm / f32 / q8 sources a 448-thread block stages in one pass.
    // Opt-in (g_tune[30] = 1): measured 7.12 vs 6.71 us alone (opbench attn_in) and within
    // the noise in tg128 (584 vs 582 tok/s), profiles/r03/qkv_balanced_ab.txt
    const bool bal = MX_AB_VARIANTS && g_tune[30] == 1 && cfg == 5 && wq->ne[1] % 16 == 0 && wq->ne[1] == 4 * wk->ne[1] && wq->ne[1] == 4 * wv->ne[1] &&
                     p.K <= 16 * 448 && (mode == XS_NORM || mode == XS_Q8 || mode == XS_F32);
    if (bal) {
        void (*kb)(QkvArgs) = nullptr;
#define QKB(TA, TK, TV) if (ta == TA && tk == TK && tv == TV) kb = mode == XS_Q8 ? k_qkv_rope_store<TA, TK, TV, XS_Q8, 16, 2, 32, 2, true> : \
        mode == XS_F32 ? k_qkv_rope_store<TA, TK, TV, XS_F32, 16, 2, 32, 2, true> : k_qkv_rope_store<TA, TK, TV, XS_NORM, 16, 2, 32, 2, true>;
        QKB(GGML_TYPE_Q4_K, GGML_TYPE_Q4_K, GGML_TYPE_Q4_K) QKB(GGML_TYPE_Q4_K, GGML_TYPE_Q4_K, GGML_TYPE_Q6_K)
        QKB(GGML_TYPE_Q4_K, GGML_TYPE_Q8_0, GGML_TYPE_Q8_0) QKB(GGML_TYPE_Q5_K, GGML_TYPE_Q8_0, GGML_TYPE_Q8_0)
        QKB(GGML_TYPE_Q4_0, GGML_TYPE_Q4_0, GGML_TYPE_Q4_0) QKB(GGML_TYPE_Q8_0, GGML_TYPE_Q8_0, GGML_TYPE_Q8_0)
#undef QKB
        if (kb) { kern = kb; grid = dim3((unsigned) (wq->ne[1] / 16)); nthr = 448; }
    }
    // round 6: the q8_0 rows go to the stream's persistent stage and are left to the decode
    // attention (KvNewRow) unless GGML_MI355X_NO_KV_DEFER / g_tune[40] = 1 (A/B: a
    // k_kv_store_q8 launch right after this one, the round-5 form)
    static const bool no_defer = getenv("GGML_MI355X_NO_KV_DEFER") != nullptr;
    const bool defer = anyq8 && !no_defer && g_tune[40] != 1 && wk->ne[1] + wv->ne[1] <= MX_KVQ8_STAGE;
    if (defer) {
        if (kq8) p.kq8f = c.s->kvq8_stage;
        if (vq8) p.vq8f = c.s->kvq8_stage + wk->ne[1];
    } else {
        if (kq8) p.kq8f = (float *) c.scratch->take(4 * wk->ne[1]);
        if (vq8) p.vq8f = (float *) c.scratch->take(4 * wv->ne[1]);
    }
    if (split) {
        int remote = 0;
        for (int k = 0; k < ns; ++k) remote += !split_on_main(c.s, wq, sdev[0][k]);
        MX_KLOG("qkv_split qta=%d qtk=%d qtv=%d mode=%d K=%d slices=%d remote=%d", ta, tk, tv, mode, p.K, ns, remote);
        for (int k = 0; k < ns; ++k) {
            QkvArgs ps = p;
            for (int t = 0; t < 3; ++t) { ps.w[t] = (const char *) sd[t][k]; ps.rows[t] = (int) (shi[t][k] - slo[t][k]); }
            ps.nblk_q = (int) mx_ceil_div(ps.rows[0], rba);
            ps.nblk_k = (int) mx_ceil_div(ps.rows[1], rba);
            const int nbv = (int) mx_ceil_div(ps.rows[2], rbv);
            ps.q_out = p.q_out + slo[0][k];
            ps.kc = p.kc + slo[1][k] * 2;
            if (v_trans) ps.vidx = p.vidx + slo[2][k] * 8;      // one I64 cache index per V element
            else ps.vc = p.vc + slo[2][k] * 2;
            const dim3 gs((unsigned) (ps.nblk_q + ps.nblk_k + nbv));
            if (split_on_main(c.s, wq, sdev[0][k])) {
                hipLaunchKernelGGL(kern, gs, dim3(nthr), gemv_lds_bytes(p.K, mode), c.st, ps);
                continue;
            }
            OpCtx dc = split_fork(c, sdev[0][k]);
            size_t moved = 0;   // (round 6) x and the norm weight copied to the slice device once
            ps.xs = split_local_xs(dc, c.s, sdev[0][k], p.xs, p.K, &moved);
            hipLaunchKernelGGL(kern, gs, dim3(nthr), gemv_lds_bytes(p.K, mode), dc.st, ps);
        }
        for (int k = 0; k < ns; ++k) if (!split_on_main(c.s, wq, sdev[0][k])) split_join(c, sdev[0][k]);
        HIP_CHECK(hipSetDevice(c.s->device));
        return last - i + 1;
    }
    MX_KLOG("qkv qta=%d qtk=%d qtv=%d mode=%d cfg=%d K=%d kq8=%d vq8=%d bal=%d", ta, tk, tv, mode, cfg, p.K, (int) kq8, (int) vq8,
            (int) (nthr == 448));
    hipLaunchKernelGGL(kern, grid, dim3(nthr), gemv_lds_bytes(p.K, mode), c.st, p);
    if (anyq8) {   // the q8_0 rows (nk / nv = 0: that cache took its f16 row in the launch above)
        const int nk = kq8 ? (int) wk->ne[1] : 0, nv = vq8 ? (int) wv->ne[1] : 0;
        if (defer) {
            KvNewRow & r = c.s->kvnew;
            r.on = true;
            r.k = p.kq8f; r.v = p.vq8f;
            r.kc = p.kc; r.kc_nb1 = p.kc_nb1; r.vc = p.vc; r.vc_nb1 = p.vc_nb1;
            r.kidx = (const int64_t *) kix->data; r.vidx = (const int64_t *) vix->data;
            r.nk = nk; r.nv = nv;
        } else {
            k_kv_store_q8<<<(unsigned) mx_ceil_div(nk + nv, 256), 256, 0, c.st>>>(p, nk, nv);
        }
    }
    return last - i + 1;
}

}  // namespace mx
