// host_graph.cpp — ggml-compatible graph construction, allocation and compute over
// the backend C-ABI (see include/mx_graph.h). Each constructor reproduces the shape,
// strides, op and op_params that the corresponding ggml.c constructor produces, so
// the backend receives exactly what the reference's libllama would hand it.
#include "mx_graph.h"
#include "common.h"

#include <deque>
#include <vector>
#include <unordered_set>
#include <cmath>

struct mxg_context {
    std::deque<ggml_tensor> tensors;
    std::vector<ggml_backend_buffer_t> buffers;
    std::deque<ggml_cgraph> graphs;
    std::deque<std::vector<ggml_tensor *>> node_store;
};

namespace {

ggml_tensor * new_impl(mxg_context * ctx, ggml_type type, int n_dims, const int64_t * ne, ggml_tensor * view_src, size_t view_offs) {
    if (view_src && view_src->view_src) {  // ggml_new_tensor_impl: views of views point at the base
        view_offs += view_src->view_offs;
        view_src = view_src->view_src;
    }
    ctx->tensors.emplace_back();
    ggml_tensor * t = &ctx->tensors.back();
    memset(t, 0, sizeof(*t));
    t->type = type;
    for (int i = 0; i < 4; ++i) t->ne[i] = i < n_dims ? ne[i] : 1;
    const mx_type_info ti = mx_type(type);
    t->nb[0] = ti.size;
    t->nb[1] = t->nb[0] * (t->ne[0] / ti.blck);
    for (int i = 2; i < 4; ++i) t->nb[i] = t->nb[i - 1] * t->ne[i - 1];
    t->view_src = view_src;
    t->view_offs = view_offs;
    if (view_src && view_src->data) {
        t->data = (char *) view_src->data + view_offs;
        t->buffer = view_src->buffer;
    }
    return t;
}

ggml_tensor * dup_tensor(mxg_context * ctx, const ggml_tensor * a) { return new_impl(ctx, a->type, 4, a->ne, nullptr, 0); }

ggml_tensor * view_tensor(mxg_context * ctx, ggml_tensor * a) {
    ggml_tensor * r = new_impl(ctx, a->type, 4, a->ne, a, 0);
    for (int i = 0; i < 4; ++i) r->nb[i] = a->nb[i];
    return r;
}

void set_params(ggml_tensor * t, const void * p, size_t n) { memcpy(t->op_params, p, n); }

bool is_contiguous(const ggml_tensor * t) { return mx_is_contiguous(t); }

}  // namespace

extern "C" {

mxg_context * mxg_init(void) { return new mxg_context(); }

void mxg_free(mxg_context * ctx) {
    if (!ctx) return;
    for (auto b : ctx->buffers) {
        if (b->iface.free_buffer) b->iface.free_buffer(b);
        delete b;
    }
    delete ctx;
}

ggml_tensor * mxg_new_tensor(mxg_context * ctx, ggml_type type, int n_dims, const int64_t * ne) {
    return new_impl(ctx, type, n_dims, ne, nullptr, 0);
}
ggml_tensor * mxg_new_tensor_4d(mxg_context * ctx, ggml_type type, int64_t ne0, int64_t ne1, int64_t ne2, int64_t ne3) {
    const int64_t ne[4] = {ne0, ne1, ne2, ne3};
    return new_impl(ctx, type, 4, ne, nullptr, 0);
}
void mxg_set_name(ggml_tensor * t, const char * name) { strncpy(t->name, name, GGML_MAX_NAME - 1); }
void mxg_set_input(ggml_tensor * t) { t->flags |= GGML_TENSOR_FLAG_INPUT; }
void mxg_set_output(ggml_tensor * t) { t->flags |= GGML_TENSOR_FLAG_OUTPUT; }

ggml_tensor * mxg_reshape_4d(mxg_context * ctx, ggml_tensor * a, int64_t ne0, int64_t ne1, int64_t ne2, int64_t ne3) {
    MX_ASSERT(is_contiguous(a) && ne0 * ne1 * ne2 * ne3 == mx_nelements(a));
    const int64_t ne[4] = {ne0, ne1, ne2, ne3};
    ggml_tensor * r = new_impl(ctx, a->type, 4, ne, a, 0);
    r->op = GGML_OP_RESHAPE;
    r->src[0] = a;
    return r;
}

ggml_tensor * mxg_view_4d(mxg_context * ctx, ggml_tensor * a, int64_t ne0, int64_t ne1, int64_t ne2, int64_t ne3,
                          size_t nb1, size_t nb2, size_t nb3, size_t offset) {
    const int64_t ne[4] = {ne0, ne1, ne2, ne3};
    ggml_tensor * r = new_impl(ctx, a->type, 4, ne, a, offset);
    set_params(r, &offset, sizeof(offset));
    r->nb[1] = nb1; r->nb[2] = nb2; r->nb[3] = nb3;
    r->op = GGML_OP_VIEW;
    r->src[0] = a;
    return r;
}

ggml_tensor * mxg_permute(mxg_context * ctx, ggml_tensor * a, int ax0, int ax1, int ax2, int ax3) {
    ggml_tensor * r = view_tensor(ctx, a);
    const int ax[4] = {ax0, ax1, ax2, ax3};
    int64_t ne[4];
    size_t nb[4];
    for (int i = 0; i < 4; ++i) { ne[ax[i]] = a->ne[i]; nb[ax[i]] = a->nb[i]; }
    for (int i = 0; i < 4; ++i) { r->ne[i] = ne[i]; r->nb[i] = nb[i]; }
    r->op = GGML_OP_PERMUTE;
    r->src[0] = a;
    set_params(r, ax, sizeof(ax));
    return r;
}

ggml_tensor * mxg_transpose(mxg_context * ctx, ggml_tensor * a) {
    ggml_tensor * r = view_tensor(ctx, a);
    r->ne[0] = a->ne[1]; r->ne[1] = a->ne[0];
    r->nb[0] = a->nb[1]; r->nb[1] = a->nb[0];
    r->op = GGML_OP_TRANSPOSE;
    r->src[0] = a;
    return r;
}

ggml_tensor * mxg_cont(mxg_context * ctx, ggml_tensor * a) {
    return mxg_cont_4d(ctx, a, a->ne[0], a->ne[1], a->ne[2], a->ne[3]);
}

ggml_tensor * mxg_cont_4d(mxg_context * ctx, ggml_tensor * a, int64_t ne0, int64_t ne1, int64_t ne2, int64_t ne3) {
    MX_ASSERT(mx_nelements(a) == ne0 * ne1 * ne2 * ne3);
    ggml_tensor * r = mxg_new_tensor_4d(ctx, a->type, ne0, ne1, ne2, ne3);
    r->op = GGML_OP_CONT;
    r->src[0] = a;
    return r;
}

ggml_tensor * mxg_cpy(mxg_context * ctx, ggml_tensor * a, ggml_tensor * b) {
    MX_ASSERT(mx_nelements(a) == mx_nelements(b));
    ggml_tensor * r = view_tensor(ctx, b);
    r->op = GGML_OP_CPY;
    r->src[0] = a;
    r->src[1] = b;
    return r;
}

ggml_tensor * mxg_cast(mxg_context * ctx, ggml_tensor * a, ggml_type type) {
    ggml_tensor * r = new_impl(ctx, type, 4, a->ne, nullptr, 0);
    r->op = GGML_OP_CPY;
    r->src[0] = a;
    r->src[1] = r;
    return r;
}

ggml_tensor * mxg_get_rows(mxg_context * ctx, ggml_tensor * a, ggml_tensor * b) {
    MX_ASSERT(a->ne[2] == b->ne[1] && a->ne[3] == b->ne[2] && b->type == GGML_TYPE_I32);
    const ggml_type t = a->type == GGML_TYPE_I32 ? GGML_TYPE_I32 : GGML_TYPE_F32;
    ggml_tensor * r = mxg_new_tensor_4d(ctx, t, a->ne[0], b->ne[0], b->ne[1], b->ne[2]);
    r->op = GGML_OP_GET_ROWS;
    r->src[0] = a;
    r->src[1] = b;
    return r;
}

ggml_tensor * mxg_set_rows(mxg_context * ctx, ggml_tensor * a, ggml_tensor * b, ggml_tensor * c) {
    MX_ASSERT(a->ne[0] == b->ne[0] && b->ne[1] == c->ne[0] && b->type == GGML_TYPE_F32);
    ggml_tensor * r = view_tensor(ctx, a);
    r->op = GGML_OP_SET_ROWS;
    r->src[0] = b;
    r->src[1] = c;
    r->src[2] = a;
    return r;
}

ggml_tensor * mxg_mul_mat(mxg_context * ctx, ggml_tensor * a, ggml_tensor * b) {
    MX_ASSERT(a->ne[0] == b->ne[0] && b->ne[2] % a->ne[2] == 0 && b->ne[3] % a->ne[3] == 0);
    ggml_tensor * r = mxg_new_tensor_4d(ctx, GGML_TYPE_F32, a->ne[1], b->ne[1], b->ne[2], b->ne[3]);
    r->op = GGML_OP_MUL_MAT;
    r->src[0] = a;
    r->src[1] = b;
    return r;
}

ggml_tensor * mxg_mul_mat_id(mxg_context * ctx, ggml_tensor * as, ggml_tensor * b, ggml_tensor * ids) {
    MX_ASSERT(ids->type == GGML_TYPE_I32 && as->ne[0] == b->ne[0]);
    ggml_tensor * r = mxg_new_tensor_4d(ctx, GGML_TYPE_F32, as->ne[1], ids->ne[0], b->ne[2], 1);
    r->op = GGML_OP_MUL_MAT_ID;
    r->src[0] = as;
    r->src[1] = b;
    r->src[2] = ids;
    return r;
}

ggml_tensor * mxg_binary(mxg_context * ctx, ggml_op op, ggml_tensor * a, ggml_tensor * b) {
    ggml_tensor * r = dup_tensor(ctx, a);
    r->op = op;
    r->src[0] = a;
    r->src[1] = b;
    return r;
}

ggml_tensor * mxg_scale(mxg_context * ctx, ggml_tensor * a, float s) {
    ggml_tensor * r = dup_tensor(ctx, a);
    const float p[2] = {s, 0.0f};
    set_params(r, p, sizeof(p));
    r->op = GGML_OP_SCALE;
    r->src[0] = a;
    return r;
}

ggml_tensor * mxg_clamp(mxg_context * ctx, ggml_tensor * a, float mn, float mxv) {
    ggml_tensor * r = view_tensor(ctx, a);
    const float p[2] = {mn, mxv};
    set_params(r, p, sizeof(p));
    r->op = GGML_OP_CLAMP;
    r->src[0] = a;
    return r;
}

ggml_tensor * mxg_unary(mxg_context * ctx, ggml_tensor * a, ggml_unary_op op) {
    ggml_tensor * r = dup_tensor(ctx, a);
    const int32_t p = (int32_t) op;
    set_params(r, &p, sizeof(p));
    r->op = GGML_OP_UNARY;
    r->src[0] = a;
    return r;
}

ggml_tensor * mxg_glu_split(mxg_context * ctx, ggml_tensor * a, ggml_tensor * b, ggml_glu_op op) {
    ggml_tensor * r = new_impl(ctx, a->type, 4, a->ne, nullptr, 0);
    const int32_t p[2] = {(int32_t) op, 0};
    set_params(r, p, sizeof(p));
    r->op = GGML_OP_GLU;
    r->src[0] = a;
    r->src[1] = b;
    return r;
}

ggml_tensor * mxg_rms_norm(mxg_context * ctx, ggml_tensor * a, float eps) {
    ggml_tensor * r = dup_tensor(ctx, a);
    set_params(r, &eps, sizeof(eps));
    r->op = GGML_OP_RMS_NORM;
    r->src[0] = a;
    return r;
}

ggml_tensor * mxg_rope_ext(mxg_context * ctx, ggml_tensor * a, ggml_tensor * pos, ggml_tensor * ff, int n_dims, int mode,
                           int n_ctx_orig, float freq_base, float freq_scale, float ext_factor, float attn_factor,
                           float beta_fast, float beta_slow) {
    MX_ASSERT(pos->type == GGML_TYPE_I32 && a->ne[2] == pos->ne[0]);
    ggml_tensor * r = dup_tensor(ctx, a);
    int32_t p[15] = {0, n_dims, mode, 0, n_ctx_orig};
    memcpy(p + 5, &freq_base, 4);
    memcpy(p + 6, &freq_scale, 4);
    memcpy(p + 7, &ext_factor, 4);
    memcpy(p + 8, &attn_factor, 4);
    memcpy(p + 9, &beta_fast, 4);
    memcpy(p + 10, &beta_slow, 4);
    set_params(r, p, sizeof(p));
    r->op = GGML_OP_ROPE;
    r->src[0] = a;
    r->src[1] = pos;
    r->src[2] = ff;
    return r;
}

ggml_tensor * mxg_soft_max_ext(mxg_context * ctx, ggml_tensor * a, ggml_tensor * mask, float scale, float max_bias) {
    ggml_tensor * r = dup_tensor(ctx, a);
    const float p[2] = {scale, max_bias};
    set_params(r, p, sizeof(p));
    r->op = GGML_OP_SOFT_MAX;
    r->src[0] = a;
    r->src[1] = mask;
    return r;
}

ggml_tensor * mxg_flash_attn_ext(mxg_context * ctx, ggml_tensor * q, ggml_tensor * k, ggml_tensor * v, ggml_tensor * mask,
                                 float scale, float max_bias, float softcap) {
    ggml_tensor * r = mxg_new_tensor_4d(ctx, GGML_TYPE_F32, v->ne[0], q->ne[2], q->ne[1], q->ne[3]);
    const float p[3] = {scale, max_bias, softcap};
    set_params(r, p, sizeof(p));
    r->op_params[3] = GGML_PREC_F32;  // ggml_flash_attn_ext_set_prec(GGML_PREC_F32), llama-graph.cpp
    r->op = GGML_OP_FLASH_ATTN_EXT;
    r->src[0] = q;
    r->src[1] = k;
    r->src[2] = v;
    r->src[3] = mask;
    return r;
}

ggml_tensor * mxg_argsort(mxg_context * ctx, ggml_tensor * a, ggml_sort_order order) {
    ggml_tensor * r = new_impl(ctx, GGML_TYPE_I32, 4, a->ne, nullptr, 0);
    const int32_t p = (int32_t) order;
    set_params(r, &p, sizeof(p));
    r->op = GGML_OP_ARGSORT;
    r->src[0] = a;
    return r;
}

ggml_tensor * mxg_sum_rows(mxg_context * ctx, ggml_tensor * a) {
    ggml_tensor * r = mxg_new_tensor_4d(ctx, a->type, 1, a->ne[1], a->ne[2], a->ne[3]);
    r->op = GGML_OP_SUM_ROWS;
    r->src[0] = a;
    return r;
}

// ---- graph ------------------------------------------------------------------
static void visit(ggml_tensor * t, std::unordered_set<ggml_tensor *> & seen, std::vector<ggml_tensor *> & nodes,
                  std::vector<ggml_tensor *> & leafs) {
    if (!t || seen.count(t)) return;
    seen.insert(t);
    for (int i = 0; i < GGML_MAX_SRC; ++i) if (t->src[i] && t->src[i] != t) visit(t->src[i], seen, nodes, leafs);
    if (t->op == GGML_OP_NONE && !(t->flags & GGML_TENSOR_FLAG_PARAM)) leafs.push_back(t);
    else nodes.push_back(t);
}

struct GraphStore {
    std::unordered_set<ggml_tensor *> seen;
    std::vector<ggml_tensor *> nodes, leafs;
};

ggml_cgraph * mxg_build(mxg_context * ctx, ggml_tensor * out) {
    ctx->graphs.emplace_back();
    ggml_cgraph * g = &ctx->graphs.back();
    memset(g, 0, sizeof(*g));
    mxg_expand(ctx, g, out);
    return g;
}

void mxg_expand(mxg_context * ctx, ggml_cgraph * g, ggml_tensor * out) {
    // rebuild node list including previous nodes (ggml_build_forward_expand appends)
    std::unordered_set<ggml_tensor *> seen;
    std::vector<ggml_tensor *> nodes, leafs;
    for (int i = 0; i < g->n_nodes; ++i) { seen.insert(g->nodes[i]); nodes.push_back(g->nodes[i]); }
    for (int i = 0; i < g->n_leafs; ++i) { seen.insert(g->leafs[i]); leafs.push_back(g->leafs[i]); }
    visit(out, seen, nodes, leafs);
    ctx->node_store.emplace_back(nodes);
    ctx->node_store.emplace_back(leafs);
    auto & ns = ctx->node_store[ctx->node_store.size() - 2];
    auto & ls = ctx->node_store.back();
    g->nodes = ns.data();
    g->leafs = ls.data();
    g->n_nodes = (int) ns.size();
    g->n_leafs = (int) ls.size();
    g->size = (int) (ns.size() + ls.size());
}

size_t mxg_nbytes(const ggml_tensor * t) { return mx_nbytes(t); }

int mxg_alloc(mxg_context * ctx, ggml_backend_buffer_type_t buft) {
    const size_t align = buft->iface.get_alignment(buft);
    size_t total = 0;
    std::vector<std::pair<ggml_tensor *, size_t>> plan;
    for (auto & t : ctx->tensors) {
        if (t.data || t.view_src) continue;
        const size_t sz = buft->iface.get_alloc_size ? buft->iface.get_alloc_size(buft, &t) : mx_nbytes(&t);
        plan.push_back({&t, total});
        total += (sz + align - 1) / align * align;
    }
    if (!plan.empty()) {
        ggml_backend_buffer_t buf = buft->iface.alloc_buffer(buft, total);
        if (!buf) return -1;
        ctx->buffers.push_back(buf);
        char * base = (char *) buf->iface.get_base(buf);
        for (auto & p : plan) {
            p.first->data = base + p.second;
            p.first->buffer = buf;
            if (buf->iface.init_tensor) buf->iface.init_tensor(buf, p.first);
        }
    }
    // resolve views (ggml_backend_view_init)
    for (auto & t : ctx->tensors) {
        if (t.view_src && !t.data && t.view_src->data) {
            t.data = (char *) t.view_src->data + t.view_offs;
            t.buffer = t.view_src->buffer;
        }
    }
    return 0;
}

size_t mxg_alloc_bytes(const mxg_context * ctx) {
    size_t n = 0;
    for (auto b : ctx->buffers) n += b->size;
    return n;
}

void mxg_tensor_set(ggml_tensor * t, const void * data, size_t offset, size_t size) {
    MX_ASSERT(t->buffer && t->data);
    t->buffer->iface.set_tensor(t->buffer, t, data, offset, size);
}

void mxg_tensor_get(const ggml_tensor * t, void * data, size_t offset, size_t size) {
    MX_ASSERT(t->buffer && t->data);
    t->buffer->iface.get_tensor(t->buffer, t, data, offset, size);
}

ggml_status mxg_compute(ggml_backend_t backend, ggml_cgraph * g) {
    ggml_status st = backend->iface.graph_compute(backend, g);
    if (backend->iface.synchronize) backend->iface.synchronize(backend);
    return st;
}

void mxg_synchronize(ggml_backend_t backend) { if (backend->iface.synchronize) backend->iface.synchronize(backend); }
void mxg_backend_free(ggml_backend_t backend) { backend->iface.free(backend); }

}  // extern "C"
