// exec.cpp — graph executor behind backend_i.graph_compute.
//
// Reference behaviour (ggml-cuda.cu:3394-3977): walk the cgraph in order, skip
// view-only nodes, fuse short node chains, and replay a captured device graph when
// consecutive cgraphs are identical (the decode loop builds the same graph every
// token: src/llama-context.cpp:1131 graph reuse + KV padding to 256 cells,
// src/llama-kv-cache.cpp:1003-1017).
//
// MI355X design: one HIP stream per backend; a cgraph signature (op, shape,
// strides, data pointers, op params) decides replay; capture happens only on the
// second sighting of a signature so one-shot prefill graphs run eagerly.
#include "backend.h"
#include <chrono>
#include "gemv.h"

#include <algorithm>
#include <atomic>
#include <unordered_map>

namespace mx {

static bool is_view_op(int op) {
    return op == GGML_OP_NONE || op == GGML_OP_RESHAPE || op == GGML_OP_VIEW ||
           op == GGML_OP_PERMUTE || op == GGML_OP_TRANSPOSE;
}

size_t nofa_long_scratch(const ggml_tensor * sm);   // ops_fattn_dec.hip: the long -fa 0 decode chain

size_t scratch_bytes(const ggml_tensor * n, bool add_norm) {
    switch (n->op) {
        case GGML_OP_SOFT_MAX:       return nofa_long_scratch(n);
        case GGML_OP_MUL_MAT:        return mul_mat_scratch(n, add_norm);
        case GGML_OP_MUL_MAT_ID:     return mul_mat_id_scratch(n);
        case GGML_OP_FLASH_ATTN_EXT: return flash_attn_scratch(n);
        default:                     return 0;
    }
}

// The cgraph signature (every node's op, type, shape, strides, data pointer and op params,
// and the same of its sources) decides whether the captured hipGraph still applies. It is
// compared against the stored one in place, word by word, overwriting where it differs:
// no per-call vector, one pass (the decode graph is ~1,000 nodes and this runs on the
// host between tokens, with the GPU idle).
struct SigCursor {
    std::vector<uint64_t> & k;
    size_t pos = 0;
    bool same = true;
    inline void put(uint64_t v) {
        if (pos < k.size()) {
            if (k[pos] != v) { same = false; k[pos] = v; }
        } else {
            k.push_back(v);
            same = false;
        }
        ++pos;
    }
};

static inline void sig_tensor(SigCursor & c, const ggml_tensor * t) {
    c.put(((uint64_t) t->op << 32) | (uint64_t) t->type);
    for (int i = 0; i < 4; ++i) { c.put((uint64_t) t->ne[i]); c.put((uint64_t) t->nb[i]); }
    c.put((uint64_t) (uintptr_t) t->data);
}

// returns true when g's signature equals the stored key (which is updated to g's)
extern unsigned g_tune_gen;   // backend.cpp: bumped by every changed ggml_backend_mi355x_set_tune
// Round 4: a node's sources enter by pointer, data pointer, row stride and the first two
// extents (packed) — 4 words instead of 10 (a source that is itself a node of this graph
// is signed in full as that node; a scheduler split's graph view has no leafs, so sources
// from outside it are covered by these four), ~29 words per node instead of ~55 (the walk
// was ~27 us of host time per drop-in token, with the GPU idle).
static bool graph_signature_same(const ggml_cgraph * g, std::vector<uint64_t> & key) {
    SigCursor c{key};
    c.put((uint64_t) g->n_nodes | ((uint64_t) g_tune_gen << 32));
    c.put((uint64_t) g->n_leafs);
    for (int i = 0; i < g->n_nodes; ++i) {
        const ggml_tensor * n = g->nodes[i];
        sig_tensor(c, n);
        const uint64_t * p = (const uint64_t *) n->op_params;
        for (int j = 0; j < GGML_MAX_OP_PARAMS / 8; ++j) c.put(p[j]);
        uint64_t ns = 0;
        for (int j = 0; j < GGML_MAX_SRC; ++j) {
            const ggml_tensor * s = n->src[j];
            if (!s) continue;
            c.put((uint64_t) (uintptr_t) s ^ ((uint64_t) j << 58));
            c.put((uint64_t) (uintptr_t) s->data);
            c.put((uint64_t) s->nb[1] ^ ((uint64_t) s->type << 56) ^ ((uint64_t) s->op << 48));
            c.put((uint64_t) (uint32_t) s->ne[0] | ((uint64_t) (uint32_t) s->ne[1] << 32));
            // round 5: the outer extents and strides as one mixed word, so a
            // source from outside a split's view that changes only there re-captures
            c.put(((uint64_t) s->ne[2] * 0x9E3779B97F4A7C15ull) ^ ((uint64_t) s->ne[3] * 0xC2B2AE3D27D4EB4Full) ^
                  ((uint64_t) s->nb[2] * 0x165667B19E3779F9ull) ^ ((uint64_t) s->nb[3] * 0xD6E8FEB86659FD93ull));
            ++ns;
        }
        c.put(ns | ((uint64_t) n->flags << 8));
    }
    for (int i = 0; i < g->n_leafs; ++i) {
        sig_tensor(c, g->leafs[i]);
        c.put((uint64_t) (uintptr_t) g->leafs[i]);
    }
    if (c.pos != key.size()) { key.resize(c.pos); c.same = false; }
    return c.same;
}

// ---- fusion ---------------------------------------------------------------
// RMS_NORM → MUL(norm, w): the build_norm pair (src/llama-graph.cpp build_norm;
// reference fusion gate ggml-cuda.cu:3844-3854).
using UseMap = UseCount;
static bool g_no_qkv = getenv("GGML_MI355X_NO_QKV_FUSION") != nullptr;
static bool g_no_moe_fusion = getenv("GGML_MI355X_NO_MOE_FUSION") != nullptr;   // A/B
static bool g_no_topk = getenv("GGML_MI355X_NO_TOPK_FUSION") != nullptr;
static bool g_no_combine = getenv("GGML_MI355X_NO_COMBINE_FUSION") != nullptr;
static bool g_no_attn_nofa = getenv("GGML_MI355X_NO_ATTN_FUSION") != nullptr;   // -fa 0 decode chain

// ---- deferred RMS norm --------------------------------------------------------
// An attn_norm / ffn_norm pair whose every consumer is a single-token GEMV is not
// run: each GEMV workgroup recomputes rms_norm(x)·w in its prologue (gemv.cuh).
// The pair is materialised after all if anything else reads its output or writes
// the memory it depends on before the consumers ran.
static bool overlaps(const void * a, size_t na, const void * b, size_t nb) {
    const char * pa = (const char *) a, * pb = (const char *) b;
    return pa < pb + nb && pb < pa + na;
}
static bool t_overlaps(const ggml_tensor * a, const ggml_tensor * b) {
    return a && b && a->data && b->data && overlaps(a->data, mx_nbytes(a), b->data, mx_nbytes(b));
}
bool t_overlaps_ext(const ggml_tensor * a, const ggml_tensor * b) { return t_overlaps(a, b); }
bool split_graph_capturable(int main_hip);   // split.cpp

// General output-overlap guard of a fused launch (round 4). ggml-alloc hands a node the
// memory of tensors that died earlier in node order (and runs ADD/MUL/SOFT_MAX/ROPE in
// place), so an unfused chain may legally write a later member's output over an input an
// earlier member already consumed; one fused grid reads and writes in no such order (two
// allocator-aliasing bugs came from exactly this: the MoE chain, r02, and the prefill q/k/v
// epilogue, r03). A fusion runs only if no output overlaps an input it reads or another
// output — except the (output, input) pairs the caller names as element-wise in place:
// the same start address, every element read before it is written by the same thread.
bool fused_io_ok(std::initializer_list<const ggml_tensor *> outs, std::initializer_list<const ggml_tensor *> ins,
                 std::initializer_list<std::pair<const ggml_tensor *, const ggml_tensor *>> inplace) {
    for (const ggml_tensor * o : outs) {
        if (!o) continue;
        for (const ggml_tensor * o2 : outs)
            if (o2 && o2 != o && t_overlaps(o, o2)) return false;
        for (const ggml_tensor * in : ins) {
            if (!in || !t_overlaps(o, in)) continue;
            bool ok = false;
            for (const auto & pr : inplace) ok = ok || (pr.first == o && pr.second == in && o->data == in->data);
            if (!ok) return false;
        }
    }
    return true;
}

XStage xstage_of(Stream * s, const ggml_tensor * x) {
    for (const DeferredNorm & d : s->deferred)
        if (x->data == d.mul->data && mx_nelements(x) == mx_nelements(d.mul) && mx_is_contiguous(x)) {
            XStage xs{(const float *) d.norm->src[0]->data, (const float *) d.w->data, mx_op_param<float>(d.norm, 0), 1};
            xs.dbg = MX_AB_VARIANTS ? g_tune[11] : 0;
            xs.xcd = g_tune[15] != 1;
            xs.drain = g_tune[14] == 1;
            xs.postscale = g_tune[42] != 1;
            return xs;
        }
    XStage xs{(const float *) x->data, nullptr, 0.0f, 0};
    xs.dbg = MX_AB_VARIANTS ? g_tune[11] : 0;
    xs.xcd = g_tune[15] != 1;
    xs.drain = g_tune[14] == 1;
    if (const ActQ * a = act_cache_find(s, x)) {
        if (a->kp == x->ne[0]) { xs.q8 = a->q; xs.q8d = a->d; xs.q8s = a->s; }
    }
    return xs;
}

static void materialize(OpCtx & c, size_t k) {
    const DeferredNorm d = c.s->deferred[k];
    c.s->deferred.erase(c.s->deferred.begin() + k);
    act_cache_invalidate(c.s, d.mul);
    op_rms_norm(c, d.norm, d.w, d.mul);
}

void deferred_guard_write(OpCtx & c, const ggml_tensor * t) {
    for (size_t k = 0; k < c.s->deferred.size();) {
        const DeferredNorm & d = c.s->deferred[k];
        if (t_overlaps(t, d.norm->src[0]) || t_overlaps(t, d.w) || t_overlaps(t, d.mul)) materialize(c, k);
        else ++k;
    }
}

void deferred_guard_read(OpCtx & c, const ggml_tensor * t) {
    for (size_t k = 0; k < c.s->deferred.size();) {
        if (t_overlaps(t, c.s->deferred[k].mul)) materialize(c, k);
        else ++k;
    }
}

bool gemv2_stage(OpCtx & c, const ggml_tensor * x, std::initializer_list<const ggml_tensor *> outs,
                 std::initializer_list<const ggml_tensor *> reads, XStage * xs, int absorbs) {
    for (const ggml_tensor * t : reads) deferred_guard_read(c, t);
    // A deferred norm this launch absorbs for its last pending consumers is never
    // materialised: its output's memory is dead, and libllama's allocator hands it to this
    // launch's own output once the gate/up MUL_MATs are its last readers (the GLU lands over
    // the normed x whenever the graph's layout puts it there — at llama-bench -d 16384 in
    // 30 of 32 layers). Writing there must not materialise the norm (round 4 did: an
    // RMS-norm launch, then the q8 path, 30 us per layer)
    for (const ggml_tensor * t : outs) {
        for (size_t k = 0; k < c.s->deferred.size();) {
            const DeferredNorm & d = c.s->deferred[k];
            const bool absorbed = x->data == d.mul->data && mx_nelements(x) == mx_nelements(d.mul) && d.pending <= absorbs;
            if (t_overlaps(t, d.norm->src[0]) || t_overlaps(t, d.w) || (!absorbed && t_overlaps(t, d.mul))) materialize(c, k);
            else ++k;
        }
    }
    *xs = xstage_of(c.s, x);
    const size_t xb = (size_t) x->ne[0] * sizeof(float);
    for (const ggml_tensor * t : outs) {
        if (overlaps(t->data, mx_nbytes(t), xs->x, xb)) return false;
        if (xs->norm && overlaps(t->data, mx_nbytes(t), xs->nw, xb)) return false;
    }
    return true;
}

// before an ordinary node: it reads nothing deferred (except a GEMV's src1, which the
// GEMV absorbs) and overwrites nothing a deferred norm still needs
static void deferred_guard_node(OpCtx & c, const ggml_tensor * n) {
    if (c.s->deferred.empty()) return;
    // (a row-split MUL_MAT's slices run through op_mul_mat on other streams, which see no
    // deferred norm: it absorbs nothing; the fused per-slice launches stage x on this stream)
    const bool absorbs = n->op == GGML_OP_MUL_MAT && g_gemv2 && gemv2_ok(n->src[0], n->src[1], n) && !tensor_is_split(n->src[0]);
    for (size_t k = 0; k < c.s->deferred.size();) {
        bool hit = false;
        for (int j = 0; j < GGML_MAX_SRC && !hit; ++j) {
            if (!n->src[j] || (absorbs && j == 1)) continue;
            hit = t_overlaps(n->src[j], c.s->deferred[k].mul);
        }
        if (hit) materialize(c, k);
        else ++k;
    }
    deferred_guard_write(c, n);
}

void deferred_guard_node_ext(OpCtx & c, const ggml_tensor * n) { deferred_guard_node(c, n); }

static bool try_defer_norm(OpCtx & c, ggml_cgraph * g, int i, UseMap & uses) {
    if (!g_gemv2 || i + 1 >= g->n_nodes) return false;
    ggml_tensor * norm = g->nodes[i];
    ggml_tensor * mul = g->nodes[i + 1];
    if (mul->op != GGML_OP_MUL || norm->type != GGML_TYPE_F32 || mul->type != GGML_TYPE_F32) return false;
    const ggml_tensor * w = mul->src[0] == norm ? mul->src[1] : (mul->src[1] == norm ? mul->src[0] : nullptr);
    const ggml_tensor * x = norm->src[0];
    if (!w || !mx_are_same_shape(mul, norm) || uses[norm] != 1) return false;
    if ((norm->flags | mul->flags) & GGML_TENSOR_FLAG_OUTPUT) return false;
    const int64_t K = x->ne[0];
    if (x->type != GGML_TYPE_F32 || mx_nelements(x) != K || !mx_is_contiguous(x) || K % 32 || K > GEMV2_MAX_NORM_K) return false;
    if (w->type != GGML_TYPE_F32 || mx_nelements(w) != K || !mx_is_contiguous(w)) return false;
    if (((uintptr_t) x->data | (uintptr_t) w->data) & 15) return false;
    const int need = uses[mul];
    if (need < 1) return false;   // a graph result, not an intermediate
    int found = 0;
    for (int j = i + 2; j < g->n_nodes && j < i + 66 && found < need; ++j) {
        const ggml_tensor * m = g->nodes[j];
        for (int k = 0; k < GGML_MAX_SRC; ++k) {
            if (m->src[k] != mul) continue;
            if (m->op != GGML_OP_MUL_MAT || k != 1 || !gemv2_ok(m->src[0], mul, m)) return false;
            // the lm_head (128256 rows = 8016 workgroups): each workgroup would stage 32 KB
            // (x and the norm weight) and normalise / quantise 4096 values again; one
            // RMS_NORM+MUL+q8 launch and q8 staging measured 76.5 + 5.7 us against 86.8
            // (decode profiles, r02). g_tune[22] = 1 keeps the deferral (A/B)
            if (m->src[0]->ne[1] > 65536 && g_tune[22] != 1) return false;
            ++found;
        }
    }
    if (found != need) return false;
    c.s->deferred.push_back(DeferredNorm{norm, w, mul, need});
    return true;
}

// Nodes [first, last] of the graph have run: a deferred norm whose last consumer was
// among them is retired. Its output is dead from here on, so the allocator may hand its
// memory (or its input's) to later tensors — without retirement their writes would
// materialise the norm for nobody (libllama's allocation does exactly that: two wasted
// RMS-norm launches per layer in the drop-in decode, profiles/r02/dropin_decode_v1).
static void deferred_retire(Stream * s, ggml_cgraph * g, int first, int last) {
    if (s->deferred.empty()) return;
    for (int j = first; j <= last && j < g->n_nodes; ++j) {
        const ggml_tensor * n = g->nodes[j];
        if (n->op != GGML_OP_MUL_MAT) continue;
        for (DeferredNorm & d : s->deferred)
            if (n->src[1] == d.mul) --d.pending;
    }
    for (size_t k = 0; k < s->deferred.size();) {
        if (s->deferred[k].pending <= 0) s->deferred.erase(s->deferred.begin() + k);
        else ++k;
    }
}

static bool try_fuse_rms_mul(OpCtx & c, ggml_cgraph * g, int i, UseMap & uses) {
    if (i + 1 >= g->n_nodes) return false;
    ggml_tensor * norm = g->nodes[i];
    ggml_tensor * mul = g->nodes[i + 1];
    if (mul->op != GGML_OP_MUL || norm->type != GGML_TYPE_F32 || mul->type != GGML_TYPE_F32) return false;
    const ggml_tensor * w = mul->src[0] == norm ? mul->src[1] : (mul->src[1] == norm ? mul->src[0] : nullptr);
    if (!w || w->type != GGML_TYPE_F32 || w->ne[0] != norm->ne[0] || !mx_is_contiguous_rows(w)) return false;
    if (!mx_are_same_shape(mul, norm)) return false;
    // one row per workgroup, read whole before it is written: in place over x is safe, any
    // other overlap is not
    const ggml_tensor * x = norm->src[0];
    const bool same_rows = mx_are_same_shape(mul, x) && mul->nb[1] == x->nb[1] && mul->nb[2] == x->nb[2] && mul->nb[3] == x->nb[3];
    if (!fused_io_ok({mul}, {x, w}, {{mul, same_rows ? x : nullptr}})) return false;
    // the norm output must be consumed only by the MUL (it is a graph-internal temporary)
    if (uses[norm] != 1 || (norm->flags & GGML_TENSOR_FLAG_OUTPUT)) return false;
    act_cache_invalidate(c.s, mul);
    // decode rows: also emit the q8 activation the following GEMVs read
    if (!rms_norm_mul_q8(c, norm, w, mul)) op_rms_norm(c, norm, w, mul);
    return true;
}

// MUL_MAT → ADD(mm, residual): the GEMV epilogue adds the residual
// (attention output projection and FFN down projection of every layer). Prefill, when the
// next pair is RMS_NORM(add) → MUL(norm, w) (ffn_norm / the next attn_norm): the reduce,
// the residual and the norm in one pass after the GEMM (ops_mm.hip mm_add_rms_norm).
// Returns the number of nodes consumed (0: no match).
bool mm_add_rms_norm(OpCtx & c, ggml_tensor * mm, const ggml_tensor * res, ggml_tensor * add, const ggml_tensor * norm,
                     const ggml_tensor * w, ggml_tensor * mul);   // ops_mm.hip
static int try_fuse_mm_add(OpCtx & c, ggml_cgraph * g, int i, UseMap & uses) {
    if (i + 1 >= g->n_nodes) return 0;
    ggml_tensor * mm = g->nodes[i];
    ggml_tensor * add = g->nodes[i + 1];
    if (add->op != GGML_OP_ADD) return 0;
    const ggml_tensor * res = add->src[0] == mm ? add->src[1] : (add->src[1] == mm ? add->src[0] : nullptr);
    if (!res || res == mm || uses[mm] != 1 || (mm->flags & GGML_TENSOR_FLAG_OUTPUT)) return 0;
    // the epilogue reads each residual element and writes the sum from the same thread: in
    // place (same start and strides) is safe, a shifted overlap is not
    const bool same = res->nb[1] == add->nb[1] && res->nb[2] == add->nb[2] && res->nb[3] == add->nb[3];
    if (!fused_io_ok({add}, {res}, {{add, same ? res : nullptr}})) return 0;
    act_cache_invalidate(c.s, add);
    if (mmvq_small_batch_ok(mm)) return mmvq_fused_add(c, mm, res, add) ? 2 : 0;
    if (i + 3 < g->n_nodes) {
        ggml_tensor * norm = g->nodes[i + 2], * mul = g->nodes[i + 3];
        const ggml_tensor * w = mul->op == GGML_OP_MUL ? (mul->src[0] == norm ? mul->src[1] : (mul->src[1] == norm ? mul->src[0] : nullptr)) : nullptr;
        if (norm->op == GGML_OP_RMS_NORM && norm->src[0] == add && w && uses[norm] == 1 && mx_are_same_shape(mul, norm) &&
            !((norm->flags | mul->flags) & GGML_TENSOR_FLAG_OUTPUT)) {
            if (mm_add_rms_norm(c, mm, res, add, norm, w, mul)) return 4;   // (invalidates mul's cached forms itself)
        }
    }
    return mmq_fused_add(c, mm, res, add) ? 2 : 0;
}

// The last layer of a decoded token (src/models/llama.cpp: inp_out_ids): MUL_MAT(wo, x) ->
// GET_ROWS(mm, ids) , GET_ROWS(inpSA, ids) -> ADD. With one token both GET_ROWS select the
// only row (ids holds 0: libllama never asks for a row that is not there), so the chain is
// MUL_MAT -> ADD(inpSA): the GEMV with the residual epilogue writing the ADD's output — one
// launch instead of four (drop-in decode profile, profiles/r04/: two k_get_rows + one ADD
// per token beside the GEMV). Returns the nodes consumed (0: no match).
static int try_fuse_mm_rows_add(OpCtx & c, ggml_cgraph * g, int i, UseMap & uses) {
    ggml_tensor * mm = g->nodes[i];
    if (mm->src[1]->ne[1] != 1 || mx_nrows(mm) != 1 || uses[mm] != 1 || (mm->flags & GGML_TENSOR_FLAG_OUTPUT)) return 0;
    ggml_tensor * g1 = nullptr, * g2 = nullptr, * add = nullptr;
    int last = i;
    for (int j = i + 1; j < g->n_nodes && j <= i + 4; ++j) {
        ggml_tensor * n = g->nodes[j];
        if (is_view_op(n->op)) continue;
        if (n->op == GGML_OP_GET_ROWS && !g1 && n->src[0] == mm) { g1 = n; last = j; continue; }
        if (n->op == GGML_OP_GET_ROWS && !g2 && n->src[0] != mm) { g2 = n; last = j; continue; }
        if (n->op == GGML_OP_ADD && g1 && g2 && ((n->src[0] == g1 && n->src[1] == g2) || (n->src[0] == g2 && n->src[1] == g1))) {
            add = n; last = j;
        }
        break;
    }
    if (!add) return 0;
    const ggml_tensor * res = g2->src[0];
    for (const ggml_tensor * gr : {g1, g2}) {
        const ggml_tensor * ids = gr->src[1];
        if (gr->type != GGML_TYPE_F32 || gr->src[0]->type != GGML_TYPE_F32 || mx_nrows(gr->src[0]) != 1 || mx_nrows(gr) != 1 ||
            mx_nelements(ids) != 1 || uses[gr] != 1 || (gr->flags & GGML_TENSOR_FLAG_OUTPUT)) return 0;
    }
    if (!mx_are_same_shape(res, mm) || !mx_are_same_shape(add, mm) || !mx_is_contiguous(res) || !mx_is_contiguous(add)) return 0;
    const bool same = res->nb[1] == add->nb[1];
    if (!fused_io_ok({add}, {res}, {{add, same ? res : nullptr}})) return 0;
    act_cache_invalidate(c.s, add);
    if (!mmvq_fused_add(c, mm, res, add)) return 0;
    return last - i + 1;
}

// Round 5: FLASH_ATTN_EXT of one decode token -> RESHAPE -> MUL_MAT(wo) -> ADD(residual)
// (build_attn + the residual, src/models/llama.cpp; or the last layer's MUL_MAT ->
// GET_ROWS x2 -> ADD chain above). The attention runs as split partials into scratch
// (fa_dec2_partials: 4 x more workgroups, a quarter of the K/V each) and the residual GEMV
// merges them in its prologue (XStage::fap) instead of a combine launch: the attention's
// output tensor is never written. Returns the nodes consumed (0: no match).
int fa_dec2_partials_nsplit(const ggml_tensor * fa);           // ops_fattn_dec.hip
void fa_dec2_partials(OpCtx & c, ggml_tensor * dst, float * part, int nsplit);
static const bool g_no_fa_split_o = getenv("GGML_MI355X_NO_FA_SPLIT_O") != nullptr;   // A/B
int fuse_moe_router(OpCtx & c, ggml_cgraph * g, int i, const UseCount & uses);   // ops_moe.hip
static const bool g_fa_dec1_env = getenv("GGML_MI355X_FA_DEC1") != nullptr;
static int fuse_attn_split_o(OpCtx & c, ggml_cgraph * g, int i, UseMap & uses) {
    // g_tune[32] = 1 (or GGML_MI355X_NO_FA_SPLIT_O): the round-4 path (one-split attention, O from x)
    if (g_no_fa_split_o || g_tune[32] == 1 || g_fa_dec1_env || g_tune[10] == 1 || !g_gemv2) return 0;
    ggml_tensor * fa = g->nodes[i];
    const int ns = fa_dec2_partials_nsplit(fa);
    if (!ns) return 0;
    const ggml_tensor * q = fa->src[0];
    const int64_t D = fa->src[1]->ne[0], H = q->ne[2];
    if (fa->type != GGML_TYPE_F32 || !mx_is_contiguous(fa) || mx_nelements(fa) != D * H) return 0;
    if (uses[fa] != 1 || (fa->flags & GGML_TENSOR_FLAG_OUTPUT)) return 0;
    ggml_tensor * rs = nullptr, * mm = nullptr;
    int jm = -1;
    for (int j = i + 1; j < g->n_nodes && j < i + 8; ++j) {
        ggml_tensor * n = g->nodes[j];
        if (is_view_op(n->op)) {
            if (!rs && n->src[0] == fa) rs = n;
            continue;
        }
        if (n->op == GGML_OP_MUL_MAT && rs && n->src[1] == rs) { mm = n; jm = j; }
        break;
    }
    if (!mm || rs->op != GGML_OP_RESHAPE || rs->ne[0] != D * H || mx_nrows(rs) != 1 || uses[rs] != 1 || (rs->flags & GGML_TENSOR_FLAG_OUTPUT)) return 0;
    const ggml_tensor * wo = mm->src[0];
    if (!gemv2_fap_o_ok(c.s, wo, rs, mm)) return 0;
    if (uses[mm] != 1 || (mm->flags & GGML_TENSOR_FLAG_OUTPUT)) return 0;
    // the tail: ADD(mm, res) right after, or GET_ROWS(mm) , GET_ROWS(res) -> ADD
    const ggml_tensor * res = nullptr;
    ggml_tensor * add = nullptr, * g1 = nullptr, * g2 = nullptr;
    int last = -1;
    if (jm + 1 < g->n_nodes && g->nodes[jm + 1]->op == GGML_OP_ADD) {
        add = g->nodes[jm + 1];
        res = add->src[0] == mm ? add->src[1] : (add->src[1] == mm ? add->src[0] : nullptr);
        last = jm + 1;
    } else {
        for (int j = jm + 1; j < g->n_nodes && j <= jm + 4; ++j) {
            ggml_tensor * n = g->nodes[j];
            if (is_view_op(n->op)) continue;
            if (n->op == GGML_OP_GET_ROWS && !g1 && n->src[0] == mm) { g1 = n; continue; }
            if (n->op == GGML_OP_GET_ROWS && !g2 && n->src[0] != mm) { g2 = n; continue; }
            if (n->op == GGML_OP_ADD && g1 && g2 && ((n->src[0] == g1 && n->src[1] == g2) || (n->src[0] == g2 && n->src[1] == g1))) {
                add = n; last = j;
            }
            break;
        }
        if (!add) return 0;
        for (const ggml_tensor * gr : {g1, g2}) {   // one token: both GET_ROWS are the identity
            if (gr->type != GGML_TYPE_F32 || gr->src[0]->type != GGML_TYPE_F32 || mx_nrows(gr->src[0]) != 1 || mx_nrows(gr) != 1 ||
                mx_nelements(gr->src[1]) != 1 || uses[gr] != 1 || (gr->flags & GGML_TENSOR_FLAG_OUTPUT)) return 0;
        }
        res = g2->src[0];
    }
    if (!res || res == mm || add->type != GGML_TYPE_F32 || res->type != GGML_TYPE_F32) return 0;
    if (!mx_are_same_shape(res, mm) || !mx_are_same_shape(add, mm) || !mx_is_contiguous(res) || !mx_is_contiguous(add)) return 0;
    // the epilogue reads each residual element and writes the sum from the same thread
    const bool same = res->nb[1] == add->nb[1];
    if (!fused_io_ok({add}, {res}, {{add, same ? res : nullptr}})) return 0;
    const size_t part_bytes = (size_t) H * ns * (D + 2) * sizeof(float) + 256;
    if (c.scratch->avail() < part_bytes) return 0;
    for (int j = i; j <= last; ++j) {
        deferred_guard_node(c, g->nodes[j]);
        act_cache_invalidate(c.s, g->nodes[j]);
    }
    float * part = (float *) c.scratch->take(part_bytes);
    fa_dec2_partials(c, fa, part, ns);
    XStage xs{nullptr, nullptr, 0.0f, 0};
    xs.xcd = g_tune[15] != 1;
    xs.fap = part; xs.fap_ns = ns; xs.fap_d = (int) D;
    c.s->gpf_armed = c.s->gpf_node && c.s->gpf_node == mm && !tensor_is_split(wo);   // the second prefetch stage rides on this GEMV
    gemv2_fap_o_launch(c, wo, xs, (float *) add->data, (const float *) res->data);
    return last - i + 1;
}

// MUL_MAT(gate) , MUL_MAT(up) , GLU(gate, up) with one activation column:
// one pass over the activation, two weight streams (ggml-cuda.cu:2145-2181).
static bool try_fuse_glu(OpCtx & c, ggml_cgraph * g, int i, UseMap & uses, bool gemv_only = false) {
    if (i + 2 >= g->n_nodes) return false;
    ggml_tensor * a = g->nodes[i];
    ggml_tensor * b = g->nodes[i + 1];
    ggml_tensor * glu = g->nodes[i + 2];
    if (a->op != GGML_OP_MUL_MAT || b->op != GGML_OP_MUL_MAT || glu->op != GGML_OP_GLU) return false;
    if (!glu->src[1]) return false;
    const ggml_tensor * gate = nullptr, * up = nullptr;
    const bool swapped = mx_op_param<int32_t>(glu, 1) != 0;
    if (swapped) return false;
    if (glu->src[0] == a && glu->src[1] == b) { gate = a; up = b; }
    else if (glu->src[0] == b && glu->src[1] == a) { gate = b; up = a; }
    else return false;
    if (uses[a] != 1 || uses[b] != 1 || ((a->flags | b->flags) & GGML_TENSOR_FLAG_OUTPUT)) return false;
    act_cache_invalidate(c.s, glu);
    return mmvq_fused_glu(c, gate, up, glu) || (!gemv_only && mmq_fused_glu(c, gate, up, glu));
}

// MUL_MAT_ID(gate), MUL_MAT_ID(up), GLU of a decode step (llama build_moe_ffn): one v2
// GEMV over both expert streams per (slot, token) item, SwiGLU epilogue, and the q8 of
// the result for the down projection's prologue
bool mmq4_moe_glu(OpCtx & c, const ggml_tensor * gate, const ggml_tensor * up, ggml_tensor * glu);   // ops_mmq4.hip
static const bool g_no_moe_glu_mm = getenv("GGML_MI355X_NO_MOE_GLU_MM") != nullptr;   // A/B

static bool try_fuse_moe_glu(OpCtx & c, ggml_cgraph * g, int i, UseMap & uses) {
    if (i + 2 >= g->n_nodes) return false;
    ggml_tensor * a = g->nodes[i];
    ggml_tensor * b = g->nodes[i + 1];
    ggml_tensor * glu = g->nodes[i + 2];
    if (a->op != GGML_OP_MUL_MAT_ID || b->op != GGML_OP_MUL_MAT_ID || glu->op != GGML_OP_GLU || !glu->src[1]) return false;
    if (mx_op_param<int32_t>(glu, 0) != GGML_GLU_OP_SWIGLU || mx_op_param<int32_t>(glu, 1) != 0) return false;
    const ggml_tensor * gate = glu->src[0] == a && glu->src[1] == b ? a : (glu->src[0] == b && glu->src[1] == a ? b : nullptr);
    if (!gate) return false;
    const ggml_tensor * up = gate == a ? b : a;
    if (gate->src[1] != up->src[1] || gate->src[2] != up->src[2]) return false;
    if (uses[a] != 1 || uses[b] != 1 || ((a->flags | b->flags) & GGML_TENSOR_FLAG_OUTPUT)) return false;
    if (!mx_are_same_shape(glu, gate) || glu->type != GGML_TYPE_F32 || !mx_is_contiguous(glu)) return false;
    for (const ggml_tensor * t : {gate->src[1], gate->src[2], gate->src[0], up->src[0]})
        if (t_overlaps(t, glu)) return false;
    deferred_guard_read(c, gate->src[1]);
    deferred_guard_write(c, glu);
    act_cache_invalidate(c.s, glu);
    // prefill (round 5): the expert-grouped gate/up GEMM with the SwiGLU epilogue (k_mmq4 EPI 3)
    if (up->src[2]->ne[1] > 8) return !g_no_moe_glu_mm && mmq4_moe_glu(c, gate, up, glu);
    ActQ * q8 = glu->ne[0] % 32 == 0 ? act_cache_alloc(c.s, glu) : nullptr;
    if (!gemv2_moe(c, gate, up->src[0], glu, q8)) {
        if (q8) act_cache_invalidate(c.s, glu);
        return false;
    }
    return true;
}

static void run_node(OpCtx & c, ggml_tensor * n) {
    switch (n->op) {
        case GGML_OP_GET_ROWS:   op_get_rows(c, n); break;
        case GGML_OP_SET_ROWS:   op_set_rows(c, n); break;
        case GGML_OP_DUP:
        case GGML_OP_CONT:
        case GGML_OP_CPY:        op_cpy(c, n->src[0], n); break;
        case GGML_OP_ADD:
        case GGML_OP_SUB:
        case GGML_OP_MUL:
        case GGML_OP_DIV:        op_binary(c, n); break;
        case GGML_OP_SCALE:      op_scale(c, n); break;
        case GGML_OP_CLAMP:      op_clamp(c, n); break;
        case GGML_OP_UNARY:      op_unary(c, n); break;
        case GGML_OP_GLU:        op_glu(c, n); break;
        case GGML_OP_RMS_NORM:   op_rms_norm(c, n, nullptr, n); break;
        case GGML_OP_NORM:       op_norm(c, n); break;
        case GGML_OP_ROPE:       op_rope(c, n); break;
        case GGML_OP_SOFT_MAX:   op_soft_max(c, n); break;
        case GGML_OP_SUM_ROWS:   op_sum_rows(c, n); break;
        case GGML_OP_ARGSORT:    op_argsort(c, n); break;
        case GGML_OP_MUL_MAT:    if (tensor_is_split(n->src[0])) op_mul_mat_split(c, n); else op_mul_mat(c, n); break;
        case GGML_OP_MUL_MAT_ID: op_mul_mat_id(c, n); break;
        case GGML_OP_FLASH_ATTN_EXT: op_flash_attn_ext(c, n); break;
        default: MX_ABORT("unsupported op %d on node %s", (int) n->op, n->name);
    }
}

static bool g_sync_debug = getenv("GGML_MI355X_SYNC_DEBUG") != nullptr;

// Prefill q/k/v: the MUL_MATs that share this one's src1 within the next few nodes run
// in one launch here (mmq_group_run). The later members move ahead of the nodes between
// (q's RoPE in libllama's order), so those must not touch their outputs — the allocator
// may place a later member's output over a tensor that dies in between — nor write x or
// the weights.
static bool try_group_mm(OpCtx & c, ggml_cgraph * g, int i, std::unordered_map<const ggml_tensor *, int> & done) {
    ggml_tensor * n0 = g->nodes[i];
    const ggml_tensor * x = n0->src[1];
    if (!x || x->ne[1] <= 8 || g_no_qkv) return false;
    ggml_tensor * mm[3] = {n0};
    int pos[3] = {i}, nm = 1;
    std::vector<int> between;
    for (int j = i + 1; j < g->n_nodes && j < i + 24 && nm < 3; ++j) {
        ggml_tensor * n = g->nodes[j];
        if (is_view_op(n->op) || mx_is_empty(n)) continue;
        if (n->op == GGML_OP_MUL_MAT && n->src[1] == x) { mm[nm] = n; pos[nm++] = j; continue; }
        between.push_back(j);
        if (between.size() > 6) break;
    }
    if (nm < 2) return false;
    for (int k = 1; k < nm; ++k)
        for (int j : between) {
            if (j > pos[k]) continue;
            const ggml_tensor * b = g->nodes[j];
            if (t_overlaps(b, mm[k]) || t_overlaps(b, x) || t_overlaps(b, mm[k]->src[0])) return false;
            for (int s = 0; s < GGML_MAX_SRC; ++s) if (b->src[s] && t_overlaps(b->src[s], mm[k])) return false;
        }
    for (int k = 0; k < nm; ++k) { deferred_guard_node(c, mm[k]); act_cache_invalidate(c.s, mm[k]); }
    if (!mmq_group_run(c, mm, nm)) return false;
    for (int k = 1; k < nm; ++k) done[mm[k]] = 1;
    c.s->n_fused += nm - 1;
    c.s->n_nodes_run += nm;
    return true;
}

// Decode attention is latency-bound (one K/V round trip over 32 CUs, ~6 us per layer) and
// leaves HBM idle. Its launch carries extra workgroups that touch one dword per 128-B line
// of the weights the next streaming GEMV reads (gate/up: the first MUL_MATs after the
// attention whose weights are >= 16 MB, sharing one activation), from the XCD whose
// blocks will read them (gemv.cuh xcd_block gives XCD x the x-th eighth of a matrix's
// rows, starting at its head), so that GEMV starts on L2 / Infinity-Cache hits.
// Measured on the Llama-3-8B decode (tg128 603 -> 617 tok/s, same box): 16 MB over gate
// and up took 1.3 us off the SwiGLU launch per 6.6 MB; the 9.4 MB output projection
// (latency-bound at ~2 TB/s) gained nothing, and budgets past ~24 MB outlast the
// attention itself. Budget: g_tune[23] MB (> 0), else GGML_MI355X_FA_PREFETCH_MB
// (default 16; 0 = off); minimum matrix size g_tune[24] KB (-1 = none).
extern int g_tune[48];
static int g_pf_mb_env = getenv("GGML_MI355X_FA_PREFETCH_MB") ? atoi(getenv("GGML_MI355X_FA_PREFETCH_MB")) : 16;
static int g_gpf_mb_env = getenv("GGML_MI355X_GEMV_PREFETCH_MB") ? atoi(getenv("GGML_MI355X_GEMV_PREFETCH_MB")) : 0;
static void fa_prefetch_plan(Stream * s, ggml_cgraph * g, int i, int64_t n_q, bool nofa) {
    s->pf_n = 0;
    // the non-FA chain's kernel is shorter than the 16 MB stream: measured 554 -> 546 tok/s
    // with it (bench tg128 --no-fa, same box), so there it is opt-in (g_tune[26] MB)
    const int mb = nofa ? g_tune[26] : (g_tune[23] ? g_tune[23] : g_pf_mb_env);
    if (mb <= 0 || n_q > 4) return;                            // decode rows only
    const size_t min_len = g_tune[24] ? (size_t) std::max(0, g_tune[24]) << 10 : (size_t) 16 << 20;   // tune 24 in KB
    const ggml_tensor * x = nullptr;
    for (int j = i + 1; j < g->n_nodes && j < i + 64 && s->pf_n < 4; ++j) {
        const ggml_tensor * n = g->nodes[j];
        if (n->op == GGML_OP_FLASH_ATTN_EXT || n->op == GGML_OP_MUL_MAT_ID) break;
        if (n->op != GGML_OP_MUL_MAT || !n->src[0]->data || tensor_is_split(n->src[0]) || n->src[1]->ne[1] > 4) continue;
        if (mx_nbytes(n->src[0]) < min_len) continue;
        if (x && n->src[1] != x) break;       // the next GEMV only
        x = n->src[1];
        s->pf_ptr[s->pf_n] = (const char *) n->src[0]->data;
        s->pf_len[s->pf_n++] = mx_nbytes(n->src[0]);
    }
    const size_t per = ((size_t) mb << 20) / std::max(1, s->pf_n);   // even split: one kernel reads them together
    for (int r = 0; r < s->pf_n; ++r) s->pf_take[r] = std::min(s->pf_len[r], per) / 8;
    // second stage (g_tune[25] MB, else GGML_MI355X_GEMV_PREFETCH_MB): carried by the first
    // MUL_MAT after the attention when it is a small latency-bound GEMV (under min_len)
    s->gpf_node = nullptr;
    const int mb2 = g_tune[25] ? g_tune[25] : g_gpf_mb_env;
    if (mb2 <= 0 || !s->pf_n) return;
    for (int j = i + 1; j < g->n_nodes && j < i + 16; ++j) {
        const ggml_tensor * n = g->nodes[j];
        if (n->op != GGML_OP_MUL_MAT || n->src[0]->type == GGML_TYPE_F16 || n->src[0]->type == GGML_TYPE_F32) continue;   // attention mul_mats
        if (mx_nbytes(n->src[0]) < min_len && n->src[1]->ne[1] == 1) s->gpf_node = n;
        break;
    }
    s->gpf_off = s->pf_take[0];
    const size_t per2 = ((size_t) mb2 << 20) / s->pf_n;
    s->gpf_take = std::min(s->pf_len[0] / 8 - std::min(s->pf_len[0] / 8, s->gpf_off), per2 / 8);
    for (int r = 1; r < s->pf_n; ++r) if (s->pf_take[r] != s->gpf_off) s->gpf_node = nullptr;   // one offset for all
}

// bumped whenever any stream's scratch / activation buffers move: a captured graph whose
// row-split slices ran on other streams (their buffers are not the capturing stream's)
// must not replay over freed memory
static std::atomic<unsigned> g_buf_gen{0};
void exec_bump_buf_gen() { ++g_buf_gen; }   // a stream buffer a capture may reference moved (ops_fattn_mma.hip mask16)

// row split: MUL_MATs right after node i (views between) that share its src1 and whose
// split weights have the same non-empty slices, all reachable directly: run as one group
static int try_split_group(OpCtx & c, ggml_cgraph * g, int i, std::unordered_map<const ggml_tensor *, int> & done) {
    ggml_tensor * n = g->nodes[i];
    void * dt[MX_MAX_DEVICES];
    int64_t lo[MX_MAX_DEVICES], hi[MX_MAX_DEVICES];
    int dv0[MX_MAX_DEVICES], dv[MX_MAX_DEVICES];
    const int ns = split_slices(c.s, n->src[0], dt, lo, hi, dv0);
    if (!ns || n->type != GGML_TYPE_F32 || !mx_is_contiguous(n)) return 0;
    ggml_tensor * grp[3] = {n, nullptr, nullptr};
    int ng = 1;
    for (int j = i + 1; j < g->n_nodes && ng < 3; ++j) {
        ggml_tensor * m = g->nodes[j];
        if (is_view_op(m->op) || mx_is_empty(m)) continue;
        if (m->op != GGML_OP_MUL_MAT || m->src[1] != n->src[1] || !tensor_is_split(m->src[0]) || m->type != GGML_TYPE_F32 ||
            !mx_is_contiguous(m)) break;
        if (split_slices(c.s, m->src[0], dt, lo, hi, dv) != ns || memcmp(dv, dv0, sizeof(int) * ns)) break;
        bool reads_group = false;   // (never: a MUL_MAT of the group reading another's output)
        for (int k = 0; k < ng; ++k) reads_group = reads_group || m->src[0] == grp[k] || t_overlaps(m->src[1], grp[k]);
        if (reads_group) break;
        grp[ng++] = m;
    }
    if (ng < 2) return 0;
    for (int k = 0; k < ng; ++k) {
        deferred_guard_node(c, grp[k]);
        act_cache_invalidate(c.s, grp[k]);
        if (k) done[grp[k]] = 1;
    }
    op_mul_mat_split_n(c, grp, ng);
    return ng;
}

// nodes that may read a pending q8_0 KV row (KvNewRow): every view of a quantised cache is
// q8_0 / q4_0 typed, so any node with such an operand (conservatively: quantised weights too),
// and any attention. Others (libllama's mask cast between the QKV block and the first
// attention) leave the row pending.
static bool kvnew_touches(const ggml_tensor * n) {
    auto qt = [](const ggml_tensor * t) { return t && (t->type == GGML_TYPE_Q8_0 || t->type == GGML_TYPE_Q4_0); };
    if (qt(n) || n->op == GGML_OP_FLASH_ATTN_EXT) return true;
    for (int k = 0; k < GGML_MAX_SRC; ++k) if (qt(n->src[k])) return true;
    return false;
}

static void run_nodes(Stream * s, ggml_cgraph * g) {
    OpCtx c{s, s->stream, &s->scratch};
    static thread_local UseMap uses;
    uses.clear();
    if (s->use_fusion) {
        for (int i = 0; i < g->n_nodes; ++i)
            for (int k = 0; k < GGML_MAX_SRC; ++k)
                if (g->nodes[i]->src[k]) uses[g->nodes[i]->src[k]]++;
    }
    act_cache_reset(s);
    s->deferred.clear();
    s->rope_valid = false;
    s->mask16_src = nullptr;
    s->kvnew.on = false;
    static thread_local std::unordered_map<const ggml_tensor *, int> done;   // run ahead by a group
    done.clear();
    for (int i = 0; i < g->n_nodes; ++i) {
        ggml_tensor * n = g->nodes[i];
        if (is_view_op(n->op) || mx_is_empty(n)) continue;
        if (!done.empty() && done.count(n)) continue;
        s->scratch.reset();
        // a q8_0 KV row the fused QKV launch left pending: stored now by a node that may read
        // the cache, unless it is the decode attention that takes the row (KvNewRow, backend.h)
        if (s->kvnew.on && kvnew_touches(n) && !fa_takes_new_row(s, n)) kv_new_row_flush(c);
        // (pf_n read by the attention launch and gpf_node; the non-FA chain starts at
        // MUL_MAT(k, q) and is matched by fuse_attn_nofa below)
        if (n->op == GGML_OP_FLASH_ATTN_EXT) fa_prefetch_plan(s, g, i, n->src[0]->ne[1], false);
        else if (n->op == GGML_OP_MUL_MAT && n->src[0]->type == GGML_TYPE_F16 && n->src[1]->ne[1] == 1) fa_prefetch_plan(s, g, i, 1, true);
        s->gpf_armed = s->gpf_node && n == s->gpf_node;
        if (s->use_fusion && s->split_graph) {
            // row-split weights: the RMS norm deferred into the fused per-slice launches that
            // consume it (QKV, SwiGLU: their x staging runs on this stream and goes to every
            // slice); any other consumer materialises it first (deferred_guard_node: a split
            // MUL_MAT absorbs nothing). GGML_MI355X_NO_SPLIT_DEFER=1: the round-5 first form
            // (RMS_NORM + MUL materialised by one launch)
            static const bool no_split_defer = getenv("GGML_MI355X_NO_SPLIT_DEFER") != nullptr;
            const int i0 = i;
            if (!no_split_defer && n->op == GGML_OP_RMS_NORM && try_defer_norm(c, g, i, uses)) { i += 1; s->n_fused += 2; s->n_nodes_run += 2; continue; }
            if (n->op == GGML_OP_RMS_NORM && try_fuse_rms_mul(c, g, i, uses)) { i += 1; s->n_fused += 1; s->n_nodes_run += 2; continue; }
            // decode gate/up/SwiGLU and MUL_MAT -> ADD over row-split weights whose slices are
            // on this GPU: the SwiGLU / residual GEMV per slice (mmvq_fused_glu / _add)
            static const bool no_split_fusion = getenv("GGML_MI355X_NO_SPLIT_FUSION") != nullptr;   // A/B
            if (!no_split_fusion && n->op == GGML_OP_MUL_MAT && tensor_is_split(n->src[0]) && mmvq_small_batch_ok(n)) {
                if (try_fuse_glu(c, g, i, uses, true)) { i += 2; s->n_fused += 2; s->n_nodes_run += 3; deferred_retire(s, g, i0, i); continue; }
                const int k = try_fuse_mm_add(c, g, i, uses);
                if (k) { i += k - 1; s->n_fused += k - 1; s->n_nodes_run += k; deferred_retire(s, g, i0, i); continue; }
            }
            // decode attention as split partials merged in each O-projection slice's prologue
            // (-fa 1: fuse_attn_split_o; -fa 0: the chain's split partials, ops_fattn_dec.hip)
            if (!no_split_fusion && n->op == GGML_OP_FLASH_ATTN_EXT) {
                const int k = fuse_attn_split_o(c, g, i, uses);
                if (k > 0) { i += k - 1; s->n_fused += 2; s->n_nodes_run += 3; deferred_retire(s, g, i0, i); continue; }
            }
            if (!no_split_fusion && !g_no_attn_nofa && n->op == GGML_OP_MUL_MAT && !tensor_is_split(n->src[0])) {
                const int k = fuse_attn_nofa(c, g, i, uses);
                if (k > 0) { i += k - 1; s->n_fused += 3; s->n_nodes_run += 4; deferred_retire(s, g, i0, i); continue; }
            }
            // q / k / v + RoPE + K/V stores of one token: one fused launch per slice (ops_qkv.hip)
            if (!no_split_fusion && !g_no_qkv && n->op == GGML_OP_MUL_MAT && tensor_is_split(n->src[0]) && n->src[1]->ne[1] == 1) {
                const int k = fuse_qkv_rope_store(c, g, i, uses);
                if (k > 0) { i += k - 1; s->n_fused += 6; s->n_nodes_run += 7; deferred_retire(s, g, i0, i); continue; }
            }
            // q / k / v (split MUL_MATs sharing src1, only views between): one fork / join
            if (!no_split_fusion && n->op == GGML_OP_MUL_MAT && tensor_is_split(n->src[0])) {
                const int ng = try_split_group(c, g, i, done);
                if (ng > 1) { s->n_nodes_run += ng; deferred_retire(s, g, i0, i); continue; }
            }
        } else if (s->use_fusion) {
            const int i0 = i;
            if (n->op == GGML_OP_RMS_NORM && !g_no_moe_fusion) {   // the MoE block's norm + router + top-k (ops_moe.hip)
                const int k = fuse_moe_router(c, g, i, uses);
                if (k > 0) { i += k - 1; s->n_fused += k - 1; s->n_nodes_run += k; deferred_retire(s, g, i0, i); continue; }
            }
            if (n->op == GGML_OP_RMS_NORM && try_defer_norm(c, g, i, uses)) { i += 1; s->n_fused += 2; s->n_nodes_run += 2; continue; }
            if (n->op == GGML_OP_RMS_NORM && try_fuse_rms_mul(c, g, i, uses)) { i += 1; s->n_fused += 1; s->n_nodes_run += 2; continue; }
            if (n->op == GGML_OP_MUL_MAT && !g_no_qkv) {
                const int k = fuse_qkv_rope_store(c, g, i, uses);
                if (k > 0) { i += k - 1; s->n_fused += 6; s->n_nodes_run += 7; deferred_retire(s, g, i0, i); continue; }
            }
            if (n->op == GGML_OP_MUL_MAT && !g_no_attn_nofa) {
                const int k = fuse_attn_nofa(c, g, i, uses);
                if (k > 0) { i += k - 1; s->n_fused += 3; s->n_nodes_run += 4; deferred_retire(s, g, i0, i); continue; }
            }
            if (n->op == GGML_OP_FLASH_ATTN_EXT) {
                const int k = fuse_attn_split_o(c, g, i, uses);
                if (k > 0) { i += k - 1; s->n_fused += 2; s->n_nodes_run += 3; deferred_retire(s, g, i0, i); continue; }
            }
            if (n->op == GGML_OP_MUL_MAT_ID && !g_no_moe_fusion && !g_no_combine) {   // down projection + combine
                const int k = fuse_moe_down_combine(c, g, i, uses);
                if (k > 0) { i += k - 1; s->n_fused += k - 1; s->n_nodes_run += k; deferred_retire(s, g, i0, i); continue; }
            }
            if (n->op == GGML_OP_MUL_MAT_ID && try_fuse_moe_glu(c, g, i, uses)) { i += 2; s->n_fused += 2; s->n_nodes_run += 3; continue; }
            if (n->op == GGML_OP_SOFT_MAX && !g_no_moe_fusion && !g_no_topk) {
                const int k = fuse_topk_moe(c, g, i);
                if (k > 0) { i += k - 1; s->n_fused += 3; s->n_nodes_run += 4; deferred_retire(s, g, i0, i); continue; }
            }
            if (n->op == GGML_OP_MUL && !g_no_moe_fusion && !g_no_combine) {
                const int k = fuse_moe_combine(c, g, i, uses);
                if (k > 0) { i += k - 1; s->n_fused += 2; s->n_nodes_run += 3; deferred_retire(s, g, i0, i); continue; }
            }
            if (n->op == GGML_OP_MUL_MAT && try_fuse_glu(c, g, i, uses)) { i += 2; s->n_fused += 2; s->n_nodes_run += 3; deferred_retire(s, g, i0, i); continue; }
            if (n->op == GGML_OP_MUL_MAT && try_group_mm(c, g, i, done)) continue;
            if (n->op == GGML_OP_MUL_MAT) {
                int k = try_fuse_mm_add(c, g, i, uses);
                if (k == 0) k = try_fuse_mm_rows_add(c, g, i, uses);
                if (k > 0) { i += k - 1; s->n_fused += k - 1; s->n_nodes_run += k; deferred_retire(s, g, i0, i); continue; }
            }
        }
        deferred_guard_node(c, n);
        act_cache_invalidate(s, n);
        run_node(c, n);
        deferred_retire(s, g, i, i);
        s->n_nodes_run++;
        if (g_sync_debug) {
            hipError_t e = hipStreamSynchronize(s->stream);
            if (e != hipSuccess) MX_ABORT("node %d (%s, op %d) failed: %s", i, n->name, (int) n->op, hipGetErrorString(e));
        }
    }
    // every consumer of a deferred norm has run by now; nothing is left pending
    s->deferred.clear();
    kv_new_row_flush(c);
    HIP_CHECK(hipGetLastError());
}

// grow a stream's scratch arena, activation ring and f16 slots to the given sizes
void graph_cache_forget(Stream * s) {
    for (GraphCache & gc : s->gslots) gc.key.clear();
}

// (never inside a capture)
static void stream_reserve(Stream * s, size_t need, size_t slot, size_t f16need) {
    if (slot > s->act_slot || f16need > s->f16.cap || need > s->scratch.cap) ++g_buf_gen;
    if (slot > s->act_slot) {
        HIP_CHECK(hipStreamSynchronize(s->stream));
        if (s->act.base) HIP_CHECK(hipFree(s->act.base));
        s->act_slot = (slot + 4095) & ~(size_t) 4095;
        HIP_CHECK(hipMalloc((void **) &s->act.base, 4 * s->act_slot));
        s->act.cap = 4 * s->act_slot;
        graph_cache_forget(s);
    }
    if (f16need > s->f16.cap) {
        HIP_CHECK(hipStreamSynchronize(s->stream));
        if (s->f16.base) HIP_CHECK(hipFree(s->f16.base));
        HIP_CHECK(hipMalloc((void **) &s->f16.base, 2 * f16need));
        s->f16.cap = f16need;
        s->f16_src[0] = s->f16_src[1] = nullptr;
        graph_cache_forget(s);
    }
    if (need > s->scratch.cap) {
        HIP_CHECK(hipStreamSynchronize(s->stream));
        if (s->scratch.base) HIP_CHECK(hipFree(s->scratch.base));
        size_t cap = std::max<size_t>(need + need / 4, 16u << 20);
        HIP_CHECK(hipMalloc((void **) &s->scratch.base, cap));
        s->scratch.cap = cap;
        graph_cache_forget(s);  // captured kernels point at the old arena
    }
}

// the buffers one MUL_MAT node needs on stream s (the row split's per-device slices)
void stream_reserve_node(Stream * s, const ggml_tensor * n) {
    size_t slot = 0;
    if (mmvq_small_batch_ok(n)) slot = act_slot_bytes(n->src[1]);
    stream_reserve(s, scratch_bytes(n), slot, mmq_act_bytes(n));
}

void graph_compute_impl(Stream * s, ggml_cgraph * g, ggml_status * status) {
    HIP_CHECK(hipSetDevice(s->device));
    staged_writes_wait(s->device, s->stream);
    s->n_graph_compute++;
    if (s->abort_cb && s->abort_cb(s->abort_data)) { *status = GGML_STATUS_ABORTED; return; }

    // A graph identical to the last one (the decode steps of libllama and of our runner)
    // replays its capture before anything else: the per-node buffer sizing below cost
    // ~100 us of host time per token while the GPU waited (drop-in stats, round 2).
    // Round 4: kGraphSlots captures per stream, found by signature (LRU), so graphs that
    // alternate — a pp2048 prompt's four ubatches (n_kv 512 .. 2048), a prompt and its
    // decode — replay too instead of each evicting the other's capture (the eager form of a
    // prefill graph ran ~8 % behind its replay: the host's per-node work does not stay
    // ahead of the GPU).
    const bool graphs = s->use_graphs && !g_sync_debug;
    static const int nslots = [] {   // GGML_MI355X_GRAPH_SLOTS=1: the round-3 single capture (A/B)
        const char * v = getenv("GGML_MI355X_GRAPH_SLOTS");
        return v && *v ? std::max(1, std::min(kGraphSlots, atoi(v))) : kGraphSlots;
    }();
    bool seen = false;   // this signature was computed before (second sighting or later)
    bool evicted = false;   // a first sighting that pushed another signature's graph out
    if (graphs) {
        const auto t0 = std::chrono::steady_clock::now();
        const bool same_prev = graph_signature_same(g, s->gsig);   // s->gsig now holds g's signature
        int k = -1;
        if (same_prev && s->gslots[s->gcur].key.size() == s->gsig.size() && !s->gsig.empty() &&
            s->gslots[s->gcur].key.data() != nullptr && !s->gslots[s->gcur].key.empty())
            k = s->gcur;                                            // (the slot holds gsig by construction)
        for (int j = 0; j < nslots && k < 0; ++j) {
            const std::vector<uint64_t> & kk = s->gslots[j].key;
            if (kk.size() == s->gsig.size() && !kk.empty() && memcmp(kk.data(), s->gsig.data(), kk.size() * 8) == 0) k = j;
        }
        const auto t1 = std::chrono::steady_clock::now();
        s->us_sig += std::chrono::duration<double, std::micro>(t1 - t0).count();
        if (k >= 0) {
            GraphCache & gc = s->gslots[k];
            s->gcur = k;
            gc.last_use = ++s->gtick;
            if (gc.exec && gc.buf_gen == g_buf_gen.load()) {
                HIP_CHECK(hipGraphLaunch(gc.exec, s->stream));
                s->us_launch += std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t1).count();
                s->n_graph_replay++;
                return;
            }
            if (gc.exec) { HIP_CHECK(hipGraphExecDestroy(gc.exec)); gc.exec = nullptr; }   // moved buffers: stale
            if (gc.graph) { HIP_CHECK(hipGraphDestroy(gc.graph)); gc.graph = nullptr; }
            seen = true;
        } else {
            // first sighting: the least recently used slot (an empty one first) takes it
            int v = 0;
            for (int j = 1; j < nslots; ++j) {
                const GraphCache & a = s->gslots[j], & b = s->gslots[v];
                if ((a.key.empty() && !b.key.empty()) || (a.key.empty() == b.key.empty() && a.last_use < b.last_use)) v = j;
            }
            GraphCache & gc = s->gslots[v];
            evicted = !gc.key.empty();
            if (gc.exec) { HIP_CHECK(hipGraphExecDestroy(gc.exec)); gc.exec = nullptr; }
            if (gc.graph) { HIP_CHECK(hipGraphDestroy(gc.graph)); gc.graph = nullptr; }
            gc.key = s->gsig;
            gc.hits = 0;
            gc.last_use = ++s->gtick;
            s->gcur = v;
        }
    }
    GraphCache & gc = s->gslots[s->gcur];

    size_t need = 0, slot = 0, f16need = 0;
    for (int i = 0; i < g->n_nodes; ++i) {
        // (the prefill GEMM -> ADD -> RMS_NORM chain keeps its product in scratch: try_fuse_mm_add)
        const bool add_norm = g->nodes[i]->op == GGML_OP_MUL_MAT && i + 2 < g->n_nodes && g->nodes[i + 1]->op == GGML_OP_ADD &&
                              g->nodes[i + 2]->op == GGML_OP_RMS_NORM && g->nodes[i + 2]->src[0] == g->nodes[i + 1];
        need = std::max(need, scratch_bytes(g->nodes[i], add_norm));
        if (g->nodes[i]->op == GGML_OP_MUL_MAT || g->nodes[i]->op == GGML_OP_MUL_MAT_ID) f16need = std::max(f16need, mmq_act_bytes(g->nodes[i]));
        if (g->nodes[i]->op == GGML_OP_MUL_MAT && mmvq_small_batch_ok(g->nodes[i])) slot = std::max(slot, act_slot_bytes(g->nodes[i]->src[1]));
        if (g->nodes[i]->op == GGML_OP_MUL && mx_nrows(g->nodes[i]) <= 8) slot = std::max(slot, act_slot_bytes(g->nodes[i]));
        // MoE decode: the q8 copy of the gate/up SwiGLU output (= this node's shape) and of src1
        if (g->nodes[i]->op == GGML_OP_MUL_MAT_ID && g->nodes[i]->src[2]->ne[1] <= 8)
            slot = std::max({slot, act_slot_bytes(g->nodes[i]), act_slot_bytes(g->nodes[i]->src[1])});
    }
    stream_reserve(s, need, slot, f16need);   // a reallocation clears every key: no capture of old buffers replays
    if (graphs && gc.key.empty()) { gc.key = s->gsig; seen = false; }   // (counts as a first sighting again)

    // row-split weights (split.cpp): every device works on the node, the slices fork off
    // onto the devices' own streams and join back by events; only the fusions without a
    // MUL_MAT apply. Captured like any graph when the slice devices are this GPU (the fork /
    // join events pull the slice streams into the capture), eager across GPUs.
    bool split = false;
    for (int i = 0; i < g->n_nodes && !split; ++i) split = g->nodes[i]->op == GGML_OP_MUL_MAT && tensor_is_split(g->nodes[i]->src[0]);
    s->split_graph = split;
    if (split && !split_graph_capturable(s->device)) {
        gc.key.clear();   // never captured: the next sighting must not count as a repeat
        run_nodes(s, g);
        s->split_graph = false;
        return;
    }
    if (!graphs || gc.key.empty()) { run_nodes(s, g); s->split_graph = false; return; }
    if (!seen) {
        // first sighting: eager. Round 5: the capture is recorded and instantiated right
        // behind the eager launches (the GPU is still executing them, so the host's capture
        // time is mostly hidden), and the SECOND sighting already replays. Capturing only at
        // the second sighting made it pay capture + instantiate with the GPU idle: llama-bench's
        // first timed pp512 repetition ran 33.0k against 35.3-35.8k tok/s for the later ones
        // (its warmup run is the first sighting; profiles/r05/trace_pp512_gaps.txt).
        // GGML_MI355X_CAPTURE_SECOND=1 restores the round-4 order (A/B).
        // only while a slot is free — once every slot holds a graph, a first sighting
        // (the changing ubatch shapes of a long prompt, one-off graphs) would pay the capture
        // and evict a graph that does repeat; there the capture waits for a second sighting.
        static const bool second = getenv("GGML_MI355X_CAPTURE_SECOND") != nullptr;
        run_nodes(s, g);
        if (second || evicted) { s->split_graph = false; return; }
        HIP_CHECK(hipStreamBeginCapture(s->stream, hipStreamCaptureModeThreadLocal));
        // (the kernel-choice log and the executor counters record the eager pass only: the
        // capture repeats its choices)
        const int klog_on = g_klog;
        const uint64_t nf = s->n_fused, nr = s->n_nodes_run;
        g_klog = 0;
        run_nodes(s, g);
        g_klog = klog_on;
        s->n_fused = nf; s->n_nodes_run = nr;
        s->split_graph = false;
        hipGraph_t graph = nullptr;
        HIP_CHECK(hipStreamEndCapture(s->stream, &graph));
        HIP_CHECK(hipGraphInstantiate(&gc.exec, graph, nullptr, nullptr, 0));
        static const bool upload = getenv("GGML_MI355X_GRAPH_UPLOAD") != nullptr;
        if (upload) HIP_CHECK(hipGraphUpload(gc.exec, s->stream));
        gc.graph = graph;
        gc.buf_gen = g_buf_gen.load();
        return;
    }
    // second sighting of the same signature: capture and launch. (Recording it on a side
    // stream behind an eager run instead measured no better for the prompt and slower for the
    // first decode repetition: profiles/r04/graph_slots_ab.txt)
    HIP_CHECK(hipStreamBeginCapture(s->stream, hipStreamCaptureModeThreadLocal));
    run_nodes(s, g);
    s->split_graph = false;
    hipGraph_t graph = nullptr;
    HIP_CHECK(hipStreamEndCapture(s->stream, &graph));
    HIP_CHECK(hipGraphInstantiate(&gc.exec, graph, nullptr, nullptr, 0));
    gc.graph = graph;
    gc.buf_gen = g_buf_gen.load();
    HIP_CHECK(hipGraphLaunch(gc.exec, s->stream));
}

}  // namespace mx
