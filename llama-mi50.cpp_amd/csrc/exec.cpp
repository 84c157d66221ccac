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

#include <algorithm>
#include <unordered_map>

namespace mx {

static bool is_view_op(int op) {
    return op == GGML_OP_NONE || op == GGML_OP_RESHAPE || op == GGML_OP_VIEW ||
           op == GGML_OP_PERMUTE || op == GGML_OP_TRANSPOSE;
}

size_t scratch_bytes(const ggml_tensor * n) {
    switch (n->op) {
        case GGML_OP_MUL_MAT:        return mul_mat_scratch(n);
        case GGML_OP_MUL_MAT_ID:     return mul_mat_id_scratch(n);
        case GGML_OP_FLASH_ATTN_EXT: return flash_attn_scratch(n);
        default:                     return 0;
    }
}

static void sig_tensor(std::vector<uint64_t> & k, const ggml_tensor * t) {
    k.push_back(((uint64_t) t->op << 32) | (uint64_t) t->type);
    for (int i = 0; i < 4; ++i) { k.push_back((uint64_t) t->ne[i]); k.push_back((uint64_t) t->nb[i]); }
    k.push_back((uint64_t) (uintptr_t) t->data);
}

static void graph_signature(const ggml_cgraph * g, std::vector<uint64_t> & k) {
    k.clear();
    k.push_back((uint64_t) g->n_nodes);
    for (int i = 0; i < g->n_nodes; ++i) {
        const ggml_tensor * n = g->nodes[i];
        sig_tensor(k, n);
        const uint64_t * p = (const uint64_t *) n->op_params;
        for (int j = 0; j < GGML_MAX_OP_PARAMS / 8; ++j) k.push_back(p[j]);
        for (int j = 0; j < GGML_MAX_SRC; ++j) {
            const ggml_tensor * s = n->src[j];
            if (!s) { k.push_back(0); continue; }
            sig_tensor(k, s);
        }
    }
}

// ---- fusion ---------------------------------------------------------------
// RMS_NORM → MUL(norm, w): the build_norm pair (src/llama-graph.cpp build_norm;
// reference fusion gate ggml-cuda.cu:3844-3854).
using UseMap = std::unordered_map<const ggml_tensor *, int>;

static bool try_fuse_rms_mul(OpCtx & c, ggml_cgraph * g, int i, UseMap & uses) {
    if (i + 1 >= g->n_nodes) return false;
    ggml_tensor * norm = g->nodes[i];
    ggml_tensor * mul = g->nodes[i + 1];
    if (mul->op != GGML_OP_MUL || norm->type != GGML_TYPE_F32 || mul->type != GGML_TYPE_F32) return false;
    const ggml_tensor * w = mul->src[0] == norm ? mul->src[1] : (mul->src[1] == norm ? mul->src[0] : nullptr);
    if (!w || w->type != GGML_TYPE_F32 || w->ne[0] != norm->ne[0] || !mx_is_contiguous_rows(w)) return false;
    if (!mx_are_same_shape(mul, norm)) return false;
    // the norm output must be consumed only by the MUL (it is a graph-internal temporary)
    if (uses[norm] != 1 || (norm->flags & GGML_TENSOR_FLAG_OUTPUT)) return false;
    op_rms_norm(c, norm, w, mul);
    return true;
}

// MUL_MAT(gate) , MUL_MAT(up) , GLU(gate, up) with one activation column:
// one pass over the activation, two weight streams (ggml-cuda.cu:2145-2181).
static bool try_fuse_glu(OpCtx & c, ggml_cgraph * g, int i, UseMap & uses) {
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
    return mmvq_fused_glu(c, gate, up, glu);
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
        case GGML_OP_MUL_MAT:    op_mul_mat(c, n); break;
        case GGML_OP_MUL_MAT_ID: op_mul_mat_id(c, n); break;
        case GGML_OP_FLASH_ATTN_EXT: op_flash_attn_ext(c, n); break;
        default: MX_ABORT("unsupported op %d on node %s", (int) n->op, n->name);
    }
}

static bool g_sync_debug = getenv("GGML_MI355X_SYNC_DEBUG") != nullptr;

static void run_nodes(Stream * s, ggml_cgraph * g) {
    OpCtx c{s, s->stream, &s->scratch};
    static thread_local UseMap uses;
    uses.clear();
    if (s->use_fusion) {
        for (int i = 0; i < g->n_nodes; ++i)
            for (int k = 0; k < GGML_MAX_SRC; ++k)
                if (g->nodes[i]->src[k]) uses[g->nodes[i]->src[k]]++;
    }
    for (int i = 0; i < g->n_nodes; ++i) {
        ggml_tensor * n = g->nodes[i];
        if (is_view_op(n->op) || mx_is_empty(n)) continue;
        s->scratch.reset();
        if (s->use_fusion) {
            if (n->op == GGML_OP_RMS_NORM && try_fuse_rms_mul(c, g, i, uses)) { i += 1; s->n_fused += 1; s->n_nodes_run += 2; continue; }
            if (n->op == GGML_OP_MUL_MAT && try_fuse_glu(c, g, i, uses)) { i += 2; s->n_fused += 2; s->n_nodes_run += 3; continue; }
        }
        run_node(c, n);
        s->n_nodes_run++;
        if (g_sync_debug) {
            hipError_t e = hipStreamSynchronize(s->stream);
            if (e != hipSuccess) MX_ABORT("node %d (%s, op %d) failed: %s", i, n->name, (int) n->op, hipGetErrorString(e));
        }
    }
    HIP_CHECK(hipGetLastError());
}

void graph_compute_impl(Stream * s, ggml_cgraph * g, ggml_status * status) {
    HIP_CHECK(hipSetDevice(s->device));
    s->n_graph_compute++;
    if (s->abort_cb && s->abort_cb(s->abort_data)) { *status = GGML_STATUS_ABORTED; return; }

    size_t need = 0;
    for (int i = 0; i < g->n_nodes; ++i) need = std::max(need, scratch_bytes(g->nodes[i]));
    if (need > s->scratch.cap) {
        HIP_CHECK(hipStreamSynchronize(s->stream));
        if (s->scratch.base) HIP_CHECK(hipFree(s->scratch.base));
        size_t cap = std::max<size_t>(need + need / 4, 16u << 20);
        HIP_CHECK(hipMalloc((void **) &s->scratch.base, cap));
        s->scratch.cap = cap;
        s->gcache.key.clear();  // captured kernels point at the old arena
    }

    if (!s->use_graphs || g_sync_debug) { run_nodes(s, g); return; }

    static thread_local std::vector<uint64_t> key;
    graph_signature(g, key);
    GraphCache & gc = s->gcache;
    if (gc.exec && key == gc.key) {
        HIP_CHECK(hipGraphLaunch(gc.exec, s->stream));
        s->n_graph_replay++;
        return;
    }
    if (key != gc.key) {  // first sighting: run eagerly, remember the signature
        gc.key = key;
        gc.hits = 0;
        if (gc.exec) { HIP_CHECK(hipGraphExecDestroy(gc.exec)); gc.exec = nullptr; }
        if (gc.graph) { HIP_CHECK(hipGraphDestroy(gc.graph)); gc.graph = nullptr; }
        run_nodes(s, g);
        return;
    }
    // second sighting of the same signature: capture and launch
    HIP_CHECK(hipStreamBeginCapture(s->stream, hipStreamCaptureModeThreadLocal));
    run_nodes(s, g);
    hipGraph_t graph = nullptr;
    HIP_CHECK(hipStreamEndCapture(s->stream, &graph));
    HIP_CHECK(hipGraphInstantiate(&gc.exec, graph, nullptr, nullptr, 0));
    gc.graph = graph;
    HIP_CHECK(hipGraphLaunch(gc.exec, s->stream));
}

}  // namespace mx
