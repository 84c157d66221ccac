// backend.h — internal state of the MI355X ggml backend (one object per device
// and per stream) and the op-dispatch contract between the executor and kernels.
#pragma once

#include "common.h"
#include <string>
#include <vector>
#include <unordered_map>

namespace mx {

struct Device {
    int id = 0;
    std::string name, description, pci_bus_id;
    size_t total_mem = 0;
    int n_cu = 0;
    ggml_backend_device dev{};
    ggml_backend_buffer_type buft{};
    ggml_backend_buffer_type host_buft{};
};

struct BufferCtx {
    int device = 0;
    void * base = nullptr;
    size_t size = 0;
    std::string name;
};

// Stream-ordered scratch arena. Sized before a graph runs (never inside a
// capture), reset per node: kernels on one stream execute in order, so every
// node may reuse the whole arena.
struct Scratch {
    char * base = nullptr;
    size_t cap = 0, off = 0;
    void * take(size_t bytes) {
        size_t a = (off + 255) & ~(size_t) 255;
        MX_ASSERT(a + bytes <= cap);
        off = a + bytes;
        return base + a;
    }
    void reset() { off = 0; }
};

struct GraphCache {
    std::vector<uint64_t> key;    // signature of the captured cgraph
    hipGraph_t graph = nullptr;
    hipGraphExec_t exec = nullptr;
    int hits = 0;
};

struct Stream {
    int device = 0;
    hipStream_t stream = nullptr;
    Scratch scratch;
    GraphCache gcache;
    bool use_graphs = true;
    bool use_fusion = true;
    std::string name;
    ggml_backend backend{};
    ggml_abort_callback abort_cb = nullptr;
    void * abort_data = nullptr;
    // profiling counters (read through mx_backend_stats)
    uint64_t n_graph_compute = 0, n_graph_replay = 0, n_nodes_run = 0, n_fused = 0;
};

// ---------------------------------------------------------------------------
// op dispatch (implemented in ops_*.hip)
// ---------------------------------------------------------------------------
struct OpCtx {
    Stream * s;
    hipStream_t st;
    Scratch * scratch;
};

// returns true when the backend can execute `op` (supports_op contract,
// ggml-backend-impl.h:171)
bool supports_op(const ggml_tensor * op);
// scratch bytes a node needs (upper bound)
size_t scratch_bytes(const ggml_tensor * node);

// kernels: each computes `dst` from dst->src[] on the stream
void op_get_rows(OpCtx & c, ggml_tensor * dst);
void op_set_rows(OpCtx & c, ggml_tensor * dst);
void op_cpy(OpCtx & c, const ggml_tensor * src, ggml_tensor * dst);
void op_binary(OpCtx & c, ggml_tensor * dst);          // ADD SUB MUL DIV
void op_scale(OpCtx & c, ggml_tensor * dst);
void op_clamp(OpCtx & c, ggml_tensor * dst);
void op_unary(OpCtx & c, ggml_tensor * dst);
void op_glu(OpCtx & c, ggml_tensor * dst);
void op_rms_norm(OpCtx & c, ggml_tensor * dst, const ggml_tensor * mul /*nullable*/, ggml_tensor * out /*fused dst*/);
void op_norm(OpCtx & c, ggml_tensor * dst);
void op_rope(OpCtx & c, ggml_tensor * dst);
void op_soft_max(OpCtx & c, ggml_tensor * dst);
void op_sum_rows(OpCtx & c, ggml_tensor * dst);
void op_argsort(OpCtx & c, ggml_tensor * dst);
void op_mul_mat(OpCtx & c, ggml_tensor * dst);
void op_mul_mat_id(OpCtx & c, ggml_tensor * dst);
void op_flash_attn_ext(OpCtx & c, ggml_tensor * dst);

size_t mul_mat_scratch(const ggml_tensor * dst);
size_t mul_mat_id_scratch(const ggml_tensor * dst);
size_t flash_attn_scratch(const ggml_tensor * dst);
bool mul_mat_supported(const ggml_tensor * dst);
bool mul_mat_id_supported(const ggml_tensor * dst);
bool flash_attn_supported(const ggml_tensor * dst);

// fused decode helpers (fusion.cpp decides, kernels live in ops_mmvq.hip)
// y_gate/up = W·x ; out = act(gate) * up   (ggml-cuda.cu:2145-2181 semantics)
bool mmvq_fused_glu(OpCtx & c, const ggml_tensor * gate_mm, const ggml_tensor * up_mm, ggml_tensor * glu);

Stream * stream_of(ggml_backend_t b);

}  // namespace mx
