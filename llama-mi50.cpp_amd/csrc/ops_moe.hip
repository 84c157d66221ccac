// ops_moe.hip — MUL_MAT_ID (MoE expert matmul) on gfx950.
//
// Semantics (ggml_mul_mat_id, ggml.c; CPU ggml-cpu.c:1503): as = [K, M, n_expert],
// b = [K, ne11, n_tok], ids = [n_used, n_tok] i32; for every token t and slot e,
// dst[:, e, t] = as[:, :, ids[e, t]] · b[:, e % ne11, t].
// Reference GPU: ggml_cuda_mul_mat_id (ggml-cuda.cu:2268-2420) — its generic path
// copies ids to the host and synchronises (:2333-2356). Here expert selection is
// resolved on the device inside the kernel (the id is read per block), so the
// whole MoE layer stays capturable in a HIP graph.
#include "backend.h"
#include "mm.h"
#include "gemv.h"

namespace mx {

struct MoeArgs {
    const char * w; size_t w_row, w_exp;
    const char * ids; size_t id0, id1;
    float * dst; size_t d1, d2;           // floats
    int64_t M, K, units, n_used, ne11, n_expert;
};

template <int QT, int LPR>
__global__ __launch_bounds__(256) void k_moe_mmvq(MoeArgs p, ActQ a) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    constexpr int RPW = 64 / LPR;
    const int64_t row = ((int64_t) blockIdx.x * 4 + wave) * RPW + lane / LPR;
    const int sub = lane % LPR;
    const int64_t item = blockIdx.y;   // (e, t)
    const int64_t e = item % p.n_used, t = item / p.n_used;
    const int32_t ex = *(const int32_t *) (p.ids + e * p.id0 + t * p.id1);
    if (ex < 0 || ex >= p.n_expert) return;
    const int64_t col = t * p.ne11 + (e % p.ne11);
    ActQ ac = a;
    ac.q += col * a.kp; ac.d += col * (a.kp / 32); ac.s += col * (a.kp / 32);
    float acc[1] = {0.f};
    if (row < p.M) {
        const char * r = p.w + (size_t) ex * p.w_exp + (size_t) row * p.w_row;
        for (int u = sub; u < p.units; u += LPR) unit_dot<QT, 1>(r, u, ac, acc);
    }
#pragma unroll
    for (int o = LPR / 2; o > 0; o >>= 1) acc[0] += __shfl_xor(acc[0], o, 64);
    if (sub == 0 && row < p.M) p.dst[e * p.d1 + t * p.d2 + row] = acc[0];
}

template <int QT>
__device__ __forceinline__ float moe_w_elem(const char * row, int64_t k) {
    if constexpr (QT == GGML_TYPE_F32) return ((const float *) row)[k];
    else if constexpr (QT == GGML_TYPE_F16) return h2f(((const uint16_t *) row)[k]);
    else return dequant_one<QT>(row + (k / qk_of<QT>()) * qsize_of<QT>(), (int) (k % qk_of<QT>()));
}

// generic: one wave per (row, item), f32 activations, exact dequant
template <int QT>
__global__ __launch_bounds__(256) void k_moe_generic(MoeArgs p, const char * b, size_t b1, size_t b2) {
    const int lane = threadIdx.x & 63;
    const int64_t row = (int64_t) blockIdx.x * 4 + (threadIdx.x >> 6);
    const int64_t item = blockIdx.y;
    const int64_t e = item % p.n_used, t = item / p.n_used;
    const int32_t ex = *(const int32_t *) (p.ids + e * p.id0 + t * p.id1);
    if (row >= p.M || ex < 0 || ex >= p.n_expert) return;
    const char * wr = p.w + (size_t) ex * p.w_exp + (size_t) row * p.w_row;
    const float * x = (const float *) (b + (e % p.ne11) * b1 + t * b2);
    float acc = 0.f;
    for (int64_t k = lane; k < p.K; k += 64) acc += moe_w_elem<QT>(wr, k) * x[k];
    acc = wave_sum(acc);
    if (lane == 0) p.dst[e * p.d1 + t * p.d2 + row] = acc;
}

bool mul_mat_id_supported(const ggml_tensor * dst) {
    const ggml_tensor * as = dst->src[0];
    const ggml_tensor * b = dst->src[1];
    const ggml_tensor * ids = dst->src[2];
    if (dst->type != GGML_TYPE_F32 || b->type != GGML_TYPE_F32 || ids->type != GGML_TYPE_I32) return false;
    if (as->ne[3] != 1 || b->ne[3] != 1) return false;
    if (b->nb[0] != 4 || dst->nb[0] != 4) return false;
    switch (as->type) {
        case GGML_TYPE_F32: case GGML_TYPE_F16:
        case GGML_TYPE_Q4_0: case GGML_TYPE_Q4_1: case GGML_TYPE_Q5_0: case GGML_TYPE_Q5_1: case GGML_TYPE_Q8_0:
        case GGML_TYPE_Q4_K: case GGML_TYPE_Q5_K: case GGML_TYPE_Q6_K:
            return as->nb[0] == (size_t) mx_type(as->type).size;
        default: return false;
    }
}

size_t mul_mat_id_scratch(const ggml_tensor * dst) {
    const ggml_tensor * as = dst->src[0];
    if (const size_t g = mmq4_moe_scratch(dst)) return g;
    if (mmvq_type_ok(as->type) && as->ne[0] % qk_of_type(as->type) == 0) return quantize_scratch(dst->src[1]);
    return 0;
}

template <int QT>
static void moe_launch_q(OpCtx & c, const MoeArgs & p, const ActQ & a, int64_t items) {
    MX_KLOG("moe_mmvq qt=%d K=%d M=%d items=%lld", QT, (int) p.K, (int) p.M, (long long) items);
    if (p.K <= 2048) k_moe_mmvq<QT, 16><<<dim3((unsigned) mx_ceil_div(p.M, 16), (unsigned) items), 256, 0, c.st>>>(p, a);
    else if (p.K <= 8192) k_moe_mmvq<QT, 32><<<dim3((unsigned) mx_ceil_div(p.M, 8), (unsigned) items), 256, 0, c.st>>>(p, a);
    else k_moe_mmvq<QT, 64><<<dim3((unsigned) mx_ceil_div(p.M, 4), (unsigned) items), 256, 0, c.st>>>(p, a);
}

void op_mul_mat_id(OpCtx & c, ggml_tensor * dst) {
    const ggml_tensor * as = dst->src[0];
    const ggml_tensor * b = dst->src[1];
    const ggml_tensor * ids = dst->src[2];
    MoeArgs p{};
    p.w = (const char *) as->data; p.w_row = as->nb[1]; p.w_exp = as->nb[2];
    p.ids = (const char *) ids->data; p.id0 = ids->nb[0]; p.id1 = ids->nb[1];
    p.dst = (float *) dst->data; p.d1 = dst->nb[1] / 4; p.d2 = dst->nb[2] / 4;
    p.M = as->ne[1]; p.K = as->ne[0]; p.units = as->ne[0] / 32;
    p.n_used = ids->ne[0]; p.ne11 = b->ne[1]; p.n_expert = as->ne[2];
    const int64_t items = ids->ne[0] * ids->ne[1];
    if (items == 0) return;
    if (mmq4_moe(c, dst)) return;     // prefill: expert-grouped MFMA GEMM (ops_mmq4.hip)
    if (gemv2_moe(c, dst, nullptr, dst)) return;   // decode: v2 GEMV per (slot, token) item
    if (mmvq_type_ok(as->type) && as->ne[0] % qk_of_type(as->type) == 0) {
        ActQ a = quantize_activations(c, b);
        switch (as->type) {
            case GGML_TYPE_Q4_K: moe_launch_q<GGML_TYPE_Q4_K>(c, p, a, items); break;
            case GGML_TYPE_Q5_K: moe_launch_q<GGML_TYPE_Q5_K>(c, p, a, items); break;
            case GGML_TYPE_Q6_K: moe_launch_q<GGML_TYPE_Q6_K>(c, p, a, items); break;
            case GGML_TYPE_Q4_0: moe_launch_q<GGML_TYPE_Q4_0>(c, p, a, items); break;
            case GGML_TYPE_Q8_0: moe_launch_q<GGML_TYPE_Q8_0>(c, p, a, items); break;
            default: break;
        }
        return;
    }
    dim3 grid((unsigned) mx_ceil_div(p.M, 4), (unsigned) items);
    MX_KLOG("moe_generic type=%d K=%d M=%d items=%lld", (int) as->type, (int) p.K, (int) p.M, (long long) items);
    const char * pb = (const char *) b->data;
    switch (as->type) {
#define MG(T) case T: k_moe_generic<T><<<grid, 256, 0, c.st>>>(p, pb, b->nb[1], b->nb[2]); break;
        MG(GGML_TYPE_F32) MG(GGML_TYPE_F16) MG(GGML_TYPE_Q4_0) MG(GGML_TYPE_Q4_1) MG(GGML_TYPE_Q5_0) MG(GGML_TYPE_Q5_1)
        MG(GGML_TYPE_Q8_0) MG(GGML_TYPE_Q4_K) MG(GGML_TYPE_Q5_K) MG(GGML_TYPE_Q6_K)
#undef MG
        default: MX_ABORT("mul_mat_id type %d", (int) as->type);
    }
}

}  // namespace mx

namespace mx {

extern int g_tune[48];

// ---------------------------------------------------------------------------
// MoE router in one launch (reference fusion: ggml-cuda/topk-moe.cu): the node chain
// SOFT_MAX(logits) -> ARGSORT(desc) [-> top-k view] -> GET_ROWS(probs, top-k)
// [-> SUM_ROWS -> CLAMP -> DIV] of llama's build_moe_ffn (src/llama-graph.cpp:1201-1296).
// One wave per token, one lane per expert (n_expert <= 64); every node of the chain still
// gets its output written (they are tiny), so any other reader stays correct.
// ---------------------------------------------------------------------------
struct TopkArgs {
    const float * logits; size_t l1;        // [n_exp, n_tok], row stride in floats
    float * probs; size_t p1;
    int32_t * order; size_t o1;              // argsort output [n_exp, n_tok]
    float * w; size_t w1;                    // get_rows output [1, k, n_tok]: stride per token (floats)
    float * sum; float * clamped;            // [1, n_tok] (nullable)
    float * wn; size_t wn1;                  // div output [k, n_tok] (nullable)
    float cmin, cmax, scale;
    int n_exp, k;
};

// one wave; lane e holds expert e's logit (before the soft_max scale) in `lg`
__device__ __forceinline__ void topk_chain(const TopkArgs & a, int t, int lane, float lg) {
    const bool on = lane < a.n_exp;
    const float x = on ? lg * a.scale : -INFINITY;
    const float m = wave_max(x);
    const float e = on ? expf(x - m) : 0.0f;
    const float s = wave_sum(e);
    const float p = on ? e / s : -INFINITY;
    if (on) a.probs[(size_t) t * a.p1 + lane] = p;
    // descending rank, ties to the lower index
    int rank = 0;
    for (int j = 0; j < a.n_exp; ++j) {
        const float pj = __shfl(p, j, 64);
        rank += (pj > p) || (pj == p && j < lane);
    }
    if (on) a.order[(size_t) t * a.o1 + rank] = lane;
    const bool top = on && rank < a.k;
    if (top) a.w[(size_t) t * a.w1 + rank] = p;
    if (a.sum) {
        // sum in rank order (the CPU's SUM_ROWS adds the selected weights in that order)
        float ws = 0.f;
        for (int r = 0; r < a.k; ++r) {
            float v = 0.f;
            for (int j = 0; j < a.n_exp; ++j) {
                const int rj = __shfl(rank, j, 64);
                const float pj = __shfl(p, j, 64);
                if (rj == r) v = pj;
            }
            ws += v;
        }
        const float cl = fminf(fmaxf(ws, a.cmin), a.cmax);
        if (lane == 0) { a.sum[t] = ws; a.clamped[t] = cl; }
        if (top) a.wn[(size_t) t * a.wn1 + rank] = p / cl;
    }
}

__global__ __launch_bounds__(64) void k_topk_moe(TopkArgs a) {
    const int lane = threadIdx.x, t = blockIdx.x;
    topk_chain(a, t, lane, lane < a.n_exp ? a.logits[(size_t) t * a.l1 + lane] : 0.f);
}

// A fused chain runs its nodes at once, one workgroup per token (per row tile): a thread's
// outputs must not land on data another thread still reads or writes. ggml-alloc gives
// dead tensors' memory to later nodes and runs SOFT_MAX / DIV / CLAMP / ADD / MUL in
// place, so e.g. SUM_ROWS can sit inside the logits. Two regions may overlap only when
// they start at the same address with the same per-token stride (an in-place op: the
// thread that reads an element is the one that overwrites it); with one token the
// stride does not matter.
struct ChainReg { const void * p; size_t n, stride; };

static bool chain_alias_ok(const ChainReg * r, int n, bool one_tok) {
    for (int x = 0; x < n; ++x)
        for (int y = x + 1; y < n; ++y) {
            const char * up = (const char *) r[x].p, * vp = (const char *) r[y].p;
            if (!up || !vp || !(up < vp + r[y].n && vp < up + r[x].n)) continue;
            if (up == vp && (one_tok || r[x].stride == r[y].stride)) continue;
            return false;
        }
    return true;
}

static ChainReg chain_reg(const ggml_tensor * t, int tok_dim) {
    return t ? ChainReg{t->data, mx_nbytes(t), t->nb[tok_dim]} : ChainReg{nullptr, 0, 0};
}

static const ggml_tensor * view_base(const ggml_tensor * t) {
    while (t && (t->op == GGML_OP_RESHAPE || t->op == GGML_OP_VIEW || t->op == GGML_OP_PERMUTE || t->op == GGML_OP_TRANSPOSE))
        t = t->src[0];
    return t;
}

// The SOFT_MAX -> ARGSORT -> GET_ROWS [-> SUM_ROWS -> CLAMP -> DIV] chain starting at node i:
// its arguments in *out and the index of its last node (0: no match)
static int match_topk_moe(ggml_cgraph * g, int i, TopkArgs * out) {
    ggml_tensor * sm = g->nodes[i];
    if (sm->op != GGML_OP_SOFT_MAX || sm->src[1] || sm->type != GGML_TYPE_F32 || sm->src[0]->type != GGML_TYPE_F32) return 0;
    if (mx_op_param<float>(sm, 1) != 0.0f || sm->ne[0] > 64 || sm->ne[2] != 1 || sm->ne[3] != 1) return 0;
    if (!mx_is_contiguous(sm) || sm->src[0]->nb[0] != 4) return 0;
    ggml_tensor * as = nullptr, * gr = nullptr, * sr = nullptr, * cl = nullptr, * dv = nullptr;
    int last = i;
    for (int j = i + 1; j < g->n_nodes && j < i + 16; ++j) {
        ggml_tensor * n = g->nodes[j];
        if (n->op == GGML_OP_RESHAPE || n->op == GGML_OP_VIEW || n->op == GGML_OP_PERMUTE || n->op == GGML_OP_TRANSPOSE) continue;
        if (!as && n->op == GGML_OP_ARGSORT && view_base(n->src[0]) == sm) { as = n; last = j; continue; }
        if (as && !gr && n->op == GGML_OP_GET_ROWS && view_base(n->src[0]) == sm && view_base(n->src[1]) == as) { gr = n; last = j; continue; }
        if (gr && !sr && n->op == GGML_OP_SUM_ROWS && view_base(n->src[0]) == gr) { sr = n; last = j; continue; }
        if (sr && !cl && n->op == GGML_OP_CLAMP && n->src[0] == sr) { cl = n; last = j; continue; }
        if (cl && !dv && n->op == GGML_OP_DIV && view_base(n->src[0]) == gr && n->src[1] == cl) { dv = n; last = j; continue; }
        break;
    }
    if (!as || !gr) return 0;
    if (sr && (!cl || !dv)) { sr = cl = dv = nullptr; }
    // shapes: argsort [n_exp, n_tok] desc; get_rows [1, k, n_tok] of probs [1, n_exp, n_tok]
    const int n_exp = (int) sm->ne[0], n_tok = (int) sm->ne[1];
    if (mx_op_param<int32_t>(as, 0) != GGML_SORT_ORDER_DESC || as->type != GGML_TYPE_I32 || !mx_is_contiguous(as)) return 0;
    if (as->ne[0] != n_exp || as->ne[1] != n_tok) return 0;
    const ggml_tensor * idx = gr->src[1];
    const int k = (int) idx->ne[0];
    if (gr->type != GGML_TYPE_F32 || gr->ne[0] != 1 || gr->ne[1] != k || gr->ne[2] != n_tok || !mx_is_contiguous(gr)) return 0;
    if (idx->ne[1] != n_tok || idx->nb[0] != 4 || idx->nb[1] != as->nb[1] || idx->data != as->data) return 0;
    if (dv && (dv->type != GGML_TYPE_F32 || mx_nelements(dv) != (int64_t) k * n_tok || !mx_is_contiguous(dv) ||
               sr->type != GGML_TYPE_F32 || cl->type != GGML_TYPE_F32 || mx_nelements(sr) != n_tok || mx_nelements(cl) != n_tok))
        return 0;
    // nothing between i and last may be a different node (the fused launch runs them at i)
    for (int j = i + 1; j <= last; ++j) {
        ggml_tensor * n = g->nodes[j];
        if (n == as || n == gr || n == sr || n == cl || n == dv) continue;
        if (n->op != GGML_OP_RESHAPE && n->op != GGML_OP_VIEW && n->op != GGML_OP_PERMUTE && n->op != GGML_OP_TRANSPOSE) return 0;
    }
    // one token is one wave that reads its logits before any store, and stores in the
    // chain's order: any aliasing is then harmless
    const ChainReg regs[] = {chain_reg(sm->src[0], 1), chain_reg(sm, 1), chain_reg(as, 1), chain_reg(gr, 2),
                             chain_reg(sr, 1), chain_reg(cl, 1), chain_reg(dv, 1)};
    if (n_tok > 1 && !chain_alias_ok(regs, 7, false)) return 0;
    TopkArgs & a = *out;
    a = TopkArgs{};
    a.logits = (const float *) sm->src[0]->data; a.l1 = sm->src[0]->nb[1] / 4;
    a.probs = (float *) sm->data; a.p1 = sm->nb[1] / 4;
    a.order = (int32_t *) as->data; a.o1 = as->nb[1] / 4;
    a.w = (float *) gr->data; a.w1 = gr->nb[2] / 4;
    a.scale = mx_op_param<float>(sm, 0);
    a.n_exp = n_exp; a.k = k;
    if (dv) {
        a.sum = (float *) sr->data; a.clamped = (float *) cl->data;
        a.cmin = mx_op_param<float>(cl, 0); a.cmax = mx_op_param<float>(cl, 1);
        a.wn = (float *) dv->data; a.wn1 = (size_t) k;
    }
    return last;
}

// returns the number of graph nodes consumed from i (0: no match)
int fuse_topk_moe(OpCtx & c, ggml_cgraph * g, int i) {
    TopkArgs a;
    const int last = match_topk_moe(g, i, &a);
    if (!last) return 0;
    const int n_tok = (int) g->nodes[i]->ne[1];
    for (int j = i; j <= last; ++j) {
        deferred_guard_node_ext(c, g->nodes[j]);
        act_cache_invalidate(c.s, g->nodes[j]);
    }
    MX_KLOG("topk_moe n_exp=%d k=%d n_tok=%d norm=%d", a.n_exp, a.k, n_tok, a.wn != nullptr);
    k_topk_moe<<<(unsigned) n_tok, 64, 0, c.st>>>(a);
    return last - i + 1;
}

// ---------------------------------------------------------------------------
// Round 5: the MoE block's head in ONE launch for a decoded token — ffn_norm (RMS_NORM ->
// MUL(w), the f32 output and its q8 copy for the expert GEMVs, k_rms_norm_q8's
// arithmetic), the router MUL_MAT(gate_inp [K, n_exp] f32/f16, cur) and the top-k chain
// above (build_moe_ffn, src/llama-graph.cpp:1183-1296). The Mixtral decode profile
// (profiles/r05/) ran them as three ~5 us launches per layer (rms_norm_q8 4.8-5.1,
// mmv_dense 4.8, topk_moe 4.6: 470 us of a 3,078 us token); one workgroup doing all of it
// took 13.1 us (160 KB through one CU). Now one workgroup per expert: each normalises the
// whole row (thread t holds 32-chunk t of x, the norm weight and of its expert's router row,
// all loads issued together), writes its 1/n_exp share of cur and the q8 copy, and its
// logit; the last workgroup to arrive (agent-scope write-through logit stores + one
// device-scope counter, reset by it for the next launch / graph replay: the protocol of
// k_fattn_dec2's in-launch split merge) runs the top-k chain.
// ---------------------------------------------------------------------------
struct RouterArgs {
    const float * x; const float * nw; float eps; int K;
    float * cur; int8_t * q; float * qd; float * qs;          // MUL output, its q8 copy (act cache)
    const char * wr; size_t wr1; int wf16;                       // router weights, row (expert) stride in bytes
    float * logits;                                               // MUL_MAT output [n_exp]
    unsigned int * cnt;                                           // arrival counter, zero between launches
    TopkArgs tk;
};

__global__ __launch_bounds__(256) void k_moe_router(RouterArgs p) {
    __shared__ float red[16];
    __shared__ int s_last;
    const int tid = threadIdx.x, lane = tid & 63, e = blockIdx.x;
    const int K = p.K, nch = K / 32;
    const bool on = tid < nch;                                    // K <= 32 x 256
    const int ch = on ? tid : 0;
    float xr[32], wn[32], wv[32];
#pragma unroll
    for (int j = 0; j < 32; j += 4) {
        const float4 a = *(const float4 *) (p.x + 32 * ch + j), b = *(const float4 *) (p.nw + 32 * ch + j);
        xr[j] = a.x; xr[j + 1] = a.y; xr[j + 2] = a.z; xr[j + 3] = a.w;
        wn[j] = b.x; wn[j + 1] = b.y; wn[j + 2] = b.z; wn[j + 3] = b.w;
    }
    const char * row = p.wr + (size_t) e * p.wr1;
    if (p.wf16) {
#pragma unroll
        for (int j = 0; j < 32; j += 8) {
            const uint4 h = *(const uint4 *) (row + 2 * (size_t) (32 * ch + j));
            const uint32_t hw[4] = {h.x, h.y, h.z, h.w};
#pragma unroll
            for (int k = 0; k < 4; ++k) { wv[j + 2 * k] = h2f((uint16_t) (hw[k] & 0xFFFF)); wv[j + 2 * k + 1] = h2f((uint16_t) (hw[k] >> 16)); }
        }
    } else {
#pragma unroll
        for (int j = 0; j < 32; j += 4) {
            const float4 c = *(const float4 *) (row + 4 * (size_t) (32 * ch + j));
            wv[j] = c.x; wv[j + 1] = c.y; wv[j + 2] = c.z; wv[j + 3] = c.w;
        }
    }
    float ss = 0.f;
    if (on) {
#pragma unroll
        for (int j = 0; j < 32; ++j) ss += xr[j] * xr[j];
    }
    ss = block_sum(ss, red);
    const float scale = 1.0f / sqrtf(ss / (float) K + p.eps);
    float v[32], acc = 0.f;
#pragma unroll
    for (int j = 0; j < 32; ++j) {
        v[j] = (xr[j] * scale) * wn[j];
        acc += wv[j] * v[j];
    }
    // this workgroup's share of cur and of its q8 copy: chunks [e * per, (e + 1) * per)
    const int per = (nch + gridDim.x - 1) / gridDim.x;
    if (on && tid >= e * per && tid < (e + 1) * per) {
#pragma unroll
        for (int j = 0; j < 32; j += 4) *(float4 *) (p.cur + 32 * tid + j) = make_float4(v[j], v[j + 1], v[j + 2], v[j + 3]);
        float amax = 0.f;
#pragma unroll
        for (int j = 0; j < 32; ++j) amax = fmaxf(amax, fabsf(v[j]));
        const Q8Scale qsc = q8_scale(amax);
        int sum = 0, packed[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            int wq = 0;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int qi = q8_round(v[4 * j + k], qsc.id);
                sum += qi;
                wq |= (qi & 0xFF) << (8 * k);
            }
            packed[j] = wq;
        }
        int4 * o = (int4 *) (p.q + 32 * tid);
        o[0] = make_int4(packed[0], packed[1], packed[2], packed[3]);
        o[1] = make_int4(packed[4], packed[5], packed[6], packed[7]);
        p.qd[tid] = qsc.d;
        p.qs[tid] = qsc.d * (float) sum;
    }
    acc = block_sum(on ? acc : 0.f, red);
    if (tid == 0) __hip_atomic_store(&p.logits[e], acc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // write-through
    // ---- the last workgroup to arrive runs the top-k chain
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    if (tid == 0) s_last = __hip_atomic_fetch_add(p.cnt, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1;
    __syncthreads();
    if (!s_last) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    if (tid < 64) {
        const float lg = lane < p.tk.n_exp ? __hip_atomic_load(&p.logits[lane], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0.f;
        topk_chain(p.tk, 0, lane, lg);
    }
    if (tid == 0) __hip_atomic_store(p.cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Round 6: the same block as ONE 1024-thread workgroup for routers of <= 8 experts (Mixtral):
// thread t holds 4-float groups t (+ 1024) of x, the norm weight and of EVERY expert's router
// row — all (2 + n_exp) x G 16-byte loads issued together, one memory round trip — then one
// barrier for the sum of squares, one for the n_exp partial logits, and wave 0 runs the
// top-k chain. The 8-workgroup form above paid, after its own loads and reductions, a
// write-through logit store, a device-scope arrival, an acquire and the logits' reload in
// the last workgroup: 8.3-8.7 us per layer (profiles/r06/). The norm's sum of squares and
// the logits are summed in another order than there (per-thread groups of 4 instead of 32).
template <int G, bool F16>
__global__ __launch_bounds__(1024) void k_moe_router1(RouterArgs p) {
    constexpr int NE = 8, NW = 16;
    __shared__ float red[NW][NE + 1];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int K = p.K, ng = K / 4;
    float4 xv[G], wv[G], rv[G][NE];
#pragma unroll
    for (int g = 0; g < G; ++g) {
        const int gi = min(tid + 1024 * g, ng - 1);
        xv[g] = *(const float4 *) (p.x + 4 * gi);
        wv[g] = *(const float4 *) (p.nw + 4 * gi);
#pragma unroll
        for (int e = 0; e < NE; ++e) {
            const int ee = min(e, p.tk.n_exp - 1);
            const char * row = p.wr + (size_t) ee * p.wr1;
            if constexpr (F16) {
                const uint2 h = *(const uint2 *) (row + 8 * (size_t) gi);
                rv[g][e] = make_float4(h2f((uint16_t) (h.x & 0xFFFF)), h2f((uint16_t) (h.x >> 16)),
                                       h2f((uint16_t) (h.y & 0xFFFF)), h2f((uint16_t) (h.y >> 16)));
            } else {
                rv[g][e] = *(const float4 *) (row + 16 * (size_t) gi);
            }
        }
    }
    float ss = 0.f;
#pragma unroll
    for (int g = 0; g < G; ++g)
        if (tid + 1024 * g < ng) ss += xv[g].x * xv[g].x + xv[g].y * xv[g].y + xv[g].z * xv[g].z + xv[g].w * xv[g].w;
    ss = wave_sum(ss);
    if (lane == 0) red[wave][NE] = ss;
    __syncthreads();
    ss = 0.f;
#pragma unroll
    for (int w = 0; w < NW; ++w) ss += red[w][NE];
    const float scale = 1.0f / sqrtf(ss / (float) K + p.eps);
    float acc[NE];
#pragma unroll
    for (int e = 0; e < NE; ++e) acc[e] = 0.f;
#pragma unroll
    for (int g = 0; g < G; ++g) {
        const int gi = tid + 1024 * g;
        const bool on = gi < ng;
        const float v[4] = {(xv[g].x * scale) * wv[g].x, (xv[g].y * scale) * wv[g].y,
                            (xv[g].z * scale) * wv[g].z, (xv[g].w * scale) * wv[g].w};
#pragma unroll
        for (int e = 0; e < NE; ++e)
            if (on) acc[e] += rv[g][e].x * v[0] + rv[g][e].y * v[1] + rv[g][e].z * v[2] + rv[g][e].w * v[3];
        // cur and its q8 copy: 8 threads (32 values) per block, the block's amax and sum by DPP
        float amax = on ? fmaxf(fmaxf(fabsf(v[0]), fabsf(v[1])), fmaxf(fabsf(v[2]), fabsf(v[3]))) : 0.f;
        amax = dpp_max_group<8>(amax);                 // (groups of <= 16 lanes: in every lane)
        const Q8Scale qsc = q8_scale(amax);
        int qi[4], sum = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) { qi[j] = q8_round(v[j], qsc.id); sum += qi[j]; }
        sum = dpp_sum_group_i<8>(sum);
        if (on) {
            *(float4 *) (p.cur + 4 * gi) = make_float4(v[0], v[1], v[2], v[3]);
            *(int *) (p.q + 4 * gi) = (qi[0] & 0xFF) | ((qi[1] & 0xFF) << 8) | ((qi[2] & 0xFF) << 16) | ((qi[3] & 0xFF) << 24);
            if ((lane & 7) == 0) { p.qd[gi >> 3] = qsc.d; p.qs[gi >> 3] = qsc.d * (float) sum; }
        }
    }
#pragma unroll
    for (int e = 0; e < NE; ++e) {
        const float a = wave_sum(acc[e]);
        if (lane == 0) red[wave][e] = a;
    }
    __syncthreads();
    if (wave == 0) {
        float lg = 0.f;
        if (lane < p.tk.n_exp) {
#pragma unroll
            for (int w = 0; w < NW; ++w) lg += red[w][lane];
            p.logits[lane] = lg;
        }
        topk_chain(p.tk, 0, lane, lg);
    }
}

// RMS_NORM at node i -> MUL(w) -> MUL_MAT(gate_inp, cur) -> the top-k chain, one token.
// Returns the nodes consumed (0: no match).
int fuse_moe_router(OpCtx & c, ggml_cgraph * g, int i, const UseCount & use_map) {
    static const bool off = getenv("GGML_MI355X_NO_MOE_ROUTER_FUSION") != nullptr;   // A/B
    if (off || g_tune[34] == 1 || i + 3 >= g->n_nodes) return 0;
    ggml_tensor * norm = g->nodes[i], * mul = g->nodes[i + 1];
    if (norm->op != GGML_OP_RMS_NORM || mul->op != GGML_OP_MUL || norm->type != GGML_TYPE_F32 || mul->type != GGML_TYPE_F32) return 0;
    const ggml_tensor * x = norm->src[0];
    const ggml_tensor * w = mul->src[0] == norm ? mul->src[1] : (mul->src[1] == norm ? mul->src[0] : nullptr);
    const int64_t K = x->ne[0];
    if (!w || mx_nrows(x) != 1 || K % 32 || K > 32 * 256 || !mx_is_contiguous(x) || !mx_are_same_shape(mul, norm)) return 0;
    if (w->type != GGML_TYPE_F32 || mx_nelements(w) != K || !mx_is_contiguous(w) || !mx_is_contiguous(mul)) return 0;
    if (((uintptr_t) x->data | (uintptr_t) w->data | (uintptr_t) mul->data) & 15) return 0;
    auto uses = [&](const ggml_tensor * t) { auto it = use_map.find(t); return it == use_map.end() ? 0 : it->second; };
    if (uses(norm) != 1 || (norm->flags & GGML_TENSOR_FLAG_OUTPUT)) return 0;
    // the router MUL_MAT, then the soft_max chain right after it
    int jm = i + 2;
    while (jm < g->n_nodes && (g->nodes[jm]->op == GGML_OP_RESHAPE || g->nodes[jm]->op == GGML_OP_VIEW)) ++jm;
    if (jm + 1 >= g->n_nodes) return 0;
    ggml_tensor * mm = g->nodes[jm];
    if (mm->op != GGML_OP_MUL_MAT || mm->src[1] != mul || mm->type != GGML_TYPE_F32 || !mx_is_contiguous(mm)) return 0;
    const ggml_tensor * gi = mm->src[0];
    const int n_exp = (int) gi->ne[1];
    if ((gi->type != GGML_TYPE_F32 && gi->type != GGML_TYPE_F16) || gi->ne[0] != K || gi->ne[2] != 1 || gi->ne[3] != 1 ||
        gi->nb[0] != (size_t) mx_type(gi->type).size || gi->nb[1] % 16 || (uintptr_t) gi->data % 16 || n_exp > 64) return 0;
    if (mm->ne[0] != n_exp || mm->ne[1] != 1) return 0;
    int js = jm + 1;
    while (js < g->n_nodes && (g->nodes[js]->op == GGML_OP_RESHAPE || g->nodes[js]->op == GGML_OP_VIEW)) ++js;
    if (js >= g->n_nodes || g->nodes[js]->op != GGML_OP_SOFT_MAX || g->nodes[js]->src[0] != mm) return 0;
    TopkArgs tk;
    const int last = match_topk_moe(g, js, &tk);
    if (!last || tk.n_exp != n_exp) return 0;
    for (int j = i + 2; j < js; ++j) if (g->nodes[j] != mm && g->nodes[j]->op != GGML_OP_RESHAPE && g->nodes[j]->op != GGML_OP_VIEW) return 0;
    // written before the top-k chain reads anything: cur and logits must not overlap what
    // the launch reads (x, w, the router rows) or each other; the chain's own outputs are
    // one wave's, written after every read (fuse_topk_moe)
    for (const ggml_tensor * o : {(const ggml_tensor *) mul, (const ggml_tensor *) mm})
        for (const ggml_tensor * in : {x, w, gi})
            if (t_overlaps_ext(o, in)) return 0;
    if (t_overlaps_ext(mul, mm)) return 0;
    for (const void * tkout : {(const void *) tk.probs, (const void *) tk.order, (const void *) tk.w, (const void *) tk.sum,
                               (const void *) tk.clamped, (const void *) tk.wn}) {
        // the chain's outputs may lie over the logits (in place) but not over cur or the inputs
        if (!tkout) continue;
        const char * p0 = (const char *) tkout;
        for (const ggml_tensor * t : {(const ggml_tensor *) mul, x, w, gi})
            if (p0 >= (const char *) t->data && p0 < (const char *) t->data + mx_nbytes(t)) return 0;
    }
    for (int j = i; j <= last; ++j) {
        deferred_guard_node_ext(c, g->nodes[j]);
        act_cache_invalidate(c.s, g->nodes[j]);
    }
    ActQ * a = act_cache_alloc(c.s, mul);
    if (!a) return 0;
    RouterArgs r{};
    r.x = (const float *) x->data; r.nw = (const float *) w->data; r.eps = mx_op_param<float>(norm, 0); r.K = (int) K;
    r.cur = (float *) mul->data; r.q = (int8_t *) a->q; r.qd = (float *) a->d; r.qs = (float *) a->s;
    r.wr = (const char *) gi->data; r.wr1 = gi->nb[1]; r.wf16 = gi->type == GGML_TYPE_F16;
    r.logits = (float *) mm->data;
    r.tk = tk;
    r.cnt = c.s->fa_cnt + MX_FA_CNT - 2;        // (a slot of its own above the decode attention's counters)
    // round 6: <= 8 experts and K <= 8192 in one 1024-thread workgroup (k_moe_router1);
    // GGML_MI355X_MOE_ROUTER_WG=1 or g_tune[46] = 1 keeps one workgroup per expert (A/B)
    static const bool per_expert = getenv("GGML_MI355X_MOE_ROUTER_WG") != nullptr;
    if (!per_expert && g_tune[46] != 1 && n_exp <= 8 && K % 128 == 0 && K <= 8192) {
        MX_KLOG("moe_router1 K=%d n_exp=%d k=%d norm=%d wf16=%d", (int) K, n_exp, tk.k, tk.wn != nullptr, r.wf16);
        if (K <= 4096) { if (r.wf16) k_moe_router1<1, true><<<1, 1024, 0, c.st>>>(r); else k_moe_router1<1, false><<<1, 1024, 0, c.st>>>(r); }
        else { if (r.wf16) k_moe_router1<2, true><<<1, 1024, 0, c.st>>>(r); else k_moe_router1<2, false><<<1, 1024, 0, c.st>>>(r); }
        return last - i + 1;
    }
    MX_KLOG("moe_router K=%d n_exp=%d k=%d norm=%d wf16=%d", (int) K, n_exp, tk.k, tk.wn != nullptr, r.wf16);
    k_moe_router<<<(unsigned) n_exp, 256, 0, c.st>>>(r);
    return last - i + 1;
}

// ---------------------------------------------------------------------------
// expert combine: MUL(experts [M, n_used, n_tok], weights [1, n_used, n_tok]), the ADDs of
// its per-slot views (llama's "aggregate experts" loop), optionally + the residual —
// one elementwise launch instead of n_used + 1
// ---------------------------------------------------------------------------
__global__ void k_moe_combine(const float * ex, size_t e1, size_t e2, const float * w, size_t w1, size_t w2, int n_used,
                              const float * res, size_t r1, float * mulout, float * out, size_t o1, int M) {
    const int row = blockIdx.x * blockDim.x + threadIdx.x, t = blockIdx.y;
    if (row >= M) return;
    float acc = 0.f;
    for (int e = 0; e < n_used; ++e) {
        const float v = ex[(size_t) t * e2 + (size_t) e * e1 + row] * w[(size_t) t * w2 + (size_t) e * w1];
        if (mulout) mulout[(size_t) t * e2 + (size_t) e * e1 + row] = v;
        acc = e == 0 ? v : acc + v;
    }
    if (res) acc += res[(size_t) t * r1 + row];
    out[(size_t) t * o1 + row] = acc;
}

// The combine chain starting at the MUL node i: MUL(experts, weights), the ADDs of its
// per-slot views [, ADD(residual)], with every alias check the fused launches need.
// Returns the index of its last node (0: no match).
struct CombineMatch {
    ggml_tensor * mul = nullptr, * out = nullptr;
    const ggml_tensor * ex = nullptr, * w = nullptr;
    const float * res = nullptr; size_t r1 = 0;
    bool mul_needed = false;
    int M = 0, n_used = 0, n_tok = 0;
};
static int match_moe_combine(ggml_cgraph * g, int i, const UseCount & use_map, CombineMatch & m) {
    auto uses = [&](const ggml_tensor * t) { auto it = use_map.find(t); return it == use_map.end() ? 0 : it->second; };
    ggml_tensor * mul = g->nodes[i];
    if (mul->op != GGML_OP_MUL || mul->type != GGML_TYPE_F32) return 0;
    const ggml_tensor * ex = mul->src[0], * w = mul->src[1];
    if (!ex || !w || ex->op != GGML_OP_MUL_MAT_ID || ex->type != GGML_TYPE_F32 || w->type != GGML_TYPE_F32) return 0;
    const int M = (int) ex->ne[0], n_used = (int) ex->ne[1], n_tok = (int) ex->ne[2];
    if (n_used < 2 || n_used > 16 || w->ne[0] != 1 || w->ne[1] != n_used || w->ne[2] != n_tok || ex->nb[0] != 4) return 0;
    if (!mx_are_same_shape(mul, ex) || !mx_is_contiguous(mul)) return 0;
    // the chain: ADD(view(mul, 0), view(mul, 1)), ADD(prev, view(mul, 2)), ... [, ADD(prev, residual)]
    ggml_tensor * prev = nullptr;
    int last = i, found = 1;
    std::vector<ggml_tensor *> chain;
    for (int j = i + 1; j < g->n_nodes && j < i + 8 + 2 * n_used && found < n_used; ++j) {
        ggml_tensor * n = g->nodes[j];
        if (n->op == GGML_OP_VIEW || n->op == GGML_OP_RESHAPE) continue;
        if (n->op != GGML_OP_ADD || n->type != GGML_TYPE_F32) return 0;
        const ggml_tensor * a0 = n->src[0], * a1 = n->src[1];
        // slot views: [M, n_tok] at offset slot * nb1 with the token stride of mul
        auto slot_view = [&](const ggml_tensor * v, int slot) {
            return v->op == GGML_OP_VIEW && v->src[0] == mul && v->view_offs == (size_t) slot * mul->nb[1] && v->ne[0] == M &&
                   v->ne[1] == n_tok && v->nb[1] == mul->nb[2] && v->nb[0] == 4;
        };
        if (!slot_view(a1, found) || !(prev ? a0 == prev : slot_view(a0, 0))) return 0;
        prev = n; last = j; ++found; chain.push_back(n);
    }
    if (found != n_used || !prev || prev->ne[0] != M || prev->ne[1] != n_tok || prev->nb[0] != 4) return 0;
    // every intermediate read only inside the chain
    for (size_t k = 0; k + 1 < chain.size(); ++k) if (uses(chain[k]) != 1) return 0;
    // optional residual add right after
    ggml_tensor * out = prev;
    const float * res = nullptr;
    size_t r1 = 0;
    for (int j = last + 1; j < g->n_nodes && j < last + 4; ++j) {
        ggml_tensor * n = g->nodes[j];
        if (n->op == GGML_OP_VIEW || n->op == GGML_OP_RESHAPE) continue;
        if (n->op == GGML_OP_ADD && n->type == GGML_TYPE_F32 && uses(prev) == 1 && !(prev->flags & GGML_TENSOR_FLAG_OUTPUT) &&
            (n->src[0] == prev || n->src[1] == prev) && mx_are_same_shape(n, prev) && n->nb[0] == 4) {
            const ggml_tensor * r = n->src[0] == prev ? n->src[1] : n->src[0];
            if (r->type == GGML_TYPE_F32 && r->nb[0] == 4 && mx_are_same_shape(r, prev)) {
                bool between_ok = true;
                for (int q = last + 1; q < j; ++q) {
                    const int op = g->nodes[q]->op;
                    if (op != GGML_OP_VIEW && op != GGML_OP_RESHAPE) between_ok = false;
                }
                if (between_ok) { res = (const float *) r->data; r1 = r->nb[1] / 4; out = n; last = j; }
            }
        }
        break;
    }
    const bool mul_needed = uses(mul) != n_used || (mul->flags & GGML_TENSOR_FLAG_OUTPUT);
    {
        // the weights are read by every thread of a token: nothing written may touch them
        const ChainReg regs[] = {chain_reg(ex, 2), chain_reg(mul_needed ? mul : nullptr, 2), chain_reg(out, 1),
                                 {res, res ? mx_nbytes(out) : 0, res ? r1 * 4 : 0}};
        const ChainReg wr[] = {chain_reg(w, 2), regs[1], regs[2]};
        if (!chain_alias_ok(regs, 4, n_tok == 1)) return 0;
        if (!chain_alias_ok(wr, 3, false) || (wr[1].p && wr[1].p == wr[0].p) || wr[2].p == wr[0].p) return 0;
    }
    m.mul = mul; m.out = out; m.ex = ex; m.w = w; m.res = res; m.r1 = r1; m.mul_needed = mul_needed;
    m.M = M; m.n_used = n_used; m.n_tok = n_tok;
    return last;
}

int fuse_moe_combine(OpCtx & c, ggml_cgraph * g, int i, const UseCount & use_map) {
    CombineMatch m;
    const int last = match_moe_combine(g, i, use_map, m);
    if (!last) return 0;
    for (int j = i; j <= last; ++j) {
        deferred_guard_node_ext(c, g->nodes[j]);
        act_cache_invalidate(c.s, g->nodes[j]);
    }
    const ggml_tensor * ex = m.ex, * w = m.w;
    MX_KLOG("moe_combine M=%d n_used=%d n_tok=%d res=%d", m.M, m.n_used, m.n_tok, m.res != nullptr);
    const dim3 grid((unsigned) mx_ceil_div(m.M, 256), (unsigned) m.n_tok);
    k_moe_combine<<<grid, 256, 0, c.st>>>((const float *) ex->data, ex->nb[1] / 4, ex->nb[2] / 4, (const float *) w->data,
                                          w->nb[1] / 4, w->nb[2] / 4, m.n_used, m.res, m.r1,
                                          m.mul_needed ? (float *) m.mul->data : nullptr, (float *) m.out->data, m.out->nb[1] / 4, m.M);
    return last - i + 1;
}

// Round 6: the down projection's MUL_MAT_ID at node i together with the combine chain that
// follows it (moe_down_combine_launch, ops_gemv_nc.hip): the experts' outputs are never
// written, so nothing else may read them (the MUL is their only consumer and needs no
// output of its own). GGML_MI355X_NO_MOE_DOWN_COMBINE=1: the two launches (A/B).
int fuse_moe_down_combine(OpCtx & c, ggml_cgraph * g, int i, const UseCount & use_map) {
    static const bool off = getenv("GGML_MI355X_NO_MOE_DOWN_COMBINE") != nullptr;
    auto uses = [&](const ggml_tensor * t) { auto it = use_map.find(t); return it == use_map.end() ? 0 : it->second; };
    ggml_tensor * dst = g->nodes[i];
    if (off || dst->op != GGML_OP_MUL_MAT_ID || uses(dst) != 1 || (dst->flags & GGML_TENSOR_FLAG_OUTPUT)) return 0;
    int j = i + 1;
    while (j < g->n_nodes && (g->nodes[j]->op == GGML_OP_VIEW || g->nodes[j]->op == GGML_OP_RESHAPE)) ++j;
    if (j >= g->n_nodes || g->nodes[j]->op != GGML_OP_MUL || g->nodes[j]->src[0] != dst) return 0;
    CombineMatch m;
    const int last = match_moe_combine(g, j, use_map, m);
    if (!last || m.mul_needed || m.ex != dst) return 0;
    const ggml_tensor * as = dst->src[0], * b = dst->src[1], * ids = dst->src[2];
    const int64_t K = as->ne[0];
    if (as->ne[3] != 1 || as->nb[0] != (size_t) mx_type(as->type).size || b->type != GGML_TYPE_F32 || ids->type != GGML_TYPE_I32) return 0;
    if (!moe_down_combine_ok(as->type, K, as->ne[1], m.n_used, m.n_tok)) return 0;
    if (b->ne[0] != K || b->ne[1] != m.n_used || b->ne[2] != m.n_tok || !mx_is_contiguous(b)) return 0;
    if (ids->ne[0] != m.n_used || ids->ne[1] != m.n_tok || dst->ne[0] != as->ne[1]) return 0;
    // the combined output is written while ids, the weights, b and its q8 copy are read
    for (const ggml_tensor * in : {b, ids, m.w})
        if (t_overlaps_ext(m.out, in)) return 0;
    ActQ a{};
    if (const ActQ * q = act_cache_find(c.s, b)) a = *q;
    if (!a.q || a.kp != K) {
        if (!mmvq_type_ok(as->type)) return 0;
        a = quantize_activations(c, b);   // (the SwiGLU's q8 copy is normally in the act cache)
    }
    if (a.kp != K) return 0;
    for (int k = i; k <= last; ++k) {
        deferred_guard_node_ext(c, g->nodes[k]);
        if (k != i) act_cache_invalidate(c.s, g->nodes[k]);
    }
    MoeDownComb d{};
    d.as = as;
    d.ids = (const char *) ids->data; d.id0 = ids->nb[0]; d.id1 = ids->nb[1];
    d.q = a.q; d.qd = a.d; d.qs = a.s; d.kp = a.kp;
    d.wt = (const float *) m.w->data; d.wt1 = m.w->nb[1] / 4; d.wt2 = m.w->nb[2] / 4;
    d.res = m.res; d.r1 = m.r1;
    d.out = (float *) m.out->data; d.o1 = m.out->nb[1] / 4;
    d.n_used = m.n_used; d.n_tok = m.n_tok;
    moe_down_combine_launch(c, d);
    return last - i + 1;
}

}  // namespace mx
