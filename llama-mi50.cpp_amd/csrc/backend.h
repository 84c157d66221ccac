// backend.h — internal state of the MI355X ggml backend (one object per device
// and per stream) and the op-dispatch contract between the executor and kernels.
#pragma once

#include "common.h"
#include <string>
#include <vector>
#include <unordered_map>
#include <initializer_list>
#include <utility>

namespace mx {

constexpr int MX_MAX_DEVICES = 16;
// row split (split.cpp)
bool buft_is_split(ggml_backend_buffer_type_t t);
int split_main_device(ggml_backend_buffer_type_t t);
bool tensor_is_split(const ggml_tensor * t);
bool mx_force_peer();   // GGML_MI355X_FORCE_PEER: cross-device copy branches on one GPU (split.cpp)
ggml_backend_buffer_type_t split_buffer_type(int main_device, const float * tensor_split);
// order `stream` after the device's staged small buffer writes (backend.cpp)
void staged_writes_wait(int dev, hipStream_t stream);

struct Device {
    int id = 0;                      // HIP device (GGML_MI355X_VIRTUAL_DEVICES may map several here)
    int index = 0;                   // logical device index in the registry
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
    size_t avail() const { const size_t a = (off + 255) & ~(size_t) 255; return a < cap ? cap - a : 0; }
};

// quantised activation columns: int8 values + per-32 f32 scale d and d·Σq
// staged small writes (backend.cpp): queued ranges of the pinned ring copied by one
// k_stage_flush launch (ops_misc.hip)
struct StageEntry { const char * src; char * dst; uint32_t n, chunk0; };
constexpr int kFlushMax = 16;                  // ranges per flush launch
// bytes per workgroup: one 16-B load per thread, i.e. ONE round trip over PCIe per workgroup
// (16 KB per workgroup took four: the decoded token's 16 KB embedding row made the flush
// 10.4 us, profiles/r05/)
constexpr uint32_t kFlushChunk = 4096;
struct StageFlushArgs { StageEntry e[kFlushMax]; int n; };
void stage_flush_launch(const StageFlushArgs & a, unsigned chunks, hipStream_t st);
void exec_bump_buf_gen();   // exec.cpp: captured graphs re-capture before their next replay

struct ActQ {
    const int8_t * q;    // [ncols][kp]
    const float * d;     // [ncols][kp/32]
    const float * s;     // [ncols][kp/32]
    int64_t kp;          // padded K (multiple of 32)
};

// A MUL_MAT src1 quantised once per graph pass and shared by every GEMV that reads
// it (Q/K/V share the attn-norm output, gate/up share the ffn-norm output).
// Keyed by the memory it was quantised from (data, row length, column count), so a
// reshape/view of the producer's output (e.g. the flash-attn result reshaped to
// [n_embd, n_tokens]) finds it too.
struct ActCacheEntry {
    const void * data = nullptr;
    int64_t ne0 = 0, ncols = 0;
    size_t bytes = 0;
    ActQ a{};
};

struct GraphCache {
    std::vector<uint64_t> key;    // signature of the captured cgraph
    unsigned buf_gen = 0;         // g_buf_gen at capture (a row split's slice streams' buffers)
    hipGraph_t graph = nullptr;
    hipGraphExec_t exec = nullptr;
    int hits = 0;
    uint64_t last_use = 0;        // LRU among the stream's slots
};
constexpr int kGraphSlots = 8;    // captured cgraphs kept per stream (a pp2048 prompt: 4 ubatch shapes)

// RMS_NORM → MUL(w) whose only consumers are single-token GEMVs: not materialised,
// the GEMV prologues recompute it from x (exec.cpp run_nodes)
struct DeferredNorm {
    ggml_tensor * norm;
    const ggml_tensor * w;
    ggml_tensor * mul;
    int pending;      // consumers (GEMVs) that have not run yet; 0: retired, never materialised
};

constexpr int MX_ROPE_TAB = 512;   // RoPE dimension pairs the per-token table holds
constexpr int MX_KVQ8_STAGE = 32768;   // floats of Stream::kvq8_stage (a K + a V row of one token)

// Round 6: this token's q8_0 K / V cache row(s), staged in f32 by the fused decode QKV launch
// (ops_qkv.hip) and not yet in the cache: the next decode attention over those caches
// quantises and stores them (k_fattn_dec2, FaDecArgs::nr_*) — one k_kv_store_q8 launch per
// layer less; any other consumer first runs that launch (kv_new_row_flush)
struct KvNewRow {
    bool on = false;
    const float * k = nullptr, * v = nullptr;   // staged rows (null: that cache took its row already)
    char * kc = nullptr, * vc = nullptr;        // cache (view) bases, row strides
    size_t kc_nb1 = 0, vc_nb1 = 0;
    const int64_t * kidx = nullptr, * vidx = nullptr;
    int nk = 0, nv = 0;                          // row lengths (elements)
};
constexpr int MX_FA_CNT = 4096;    // decode flash-attn split counters (q rows x KV heads)

struct Stream {
    int device = 0;
    std::vector<DeferredNorm> deferred;
    hipStream_t stream = nullptr;
    hipEvent_t cpy_ev = nullptr;       // cpy_tensor_async ordering event (one per stream, reused)
    Scratch scratch;
    Scratch act;                       // ring of quantised activations (act_cache)
    ActCacheEntry act_cache[4];
    // f16 copies of prefill GEMM activations (q/k/v and gate/up share one), two slots of
    // f16.cap bytes each: a kernel can read one while writing the next GEMM's input to the
    // other (fused SwiGLU -> down projection); f16_last = the slot used most recently
    Scratch f16;
    const void * f16_src[2] = {nullptr, nullptr};
    int64_t f16_key[2][4] = {{0, 0, 0, 0}, {0, 0, 0, 0}};   // K, ncols, nb1, kp
    int f16_last = 0;
    int act_next = 0;
    size_t act_slot = 0;               // bytes per ring slot
    GraphCache gslots[kGraphSlots];
    int gcur = 0;                      // slot of the last graph computed
    uint64_t gtick = 0;
    std::vector<uint64_t> gsig;        // signature of the last graph computed
    // RoPE cos/sin table of the current token (ops_qkv.hip): computed once per graph
    // pass by the first fused QKV block, read by all layers' (same position, same params)
    float * rope_tab = nullptr;        // device, float2 [MX_ROPE_TAB]
    unsigned int * fa_cnt = nullptr;   // device, zeroed; each decode FA launch leaves it zero
    float * kvq8_stage = nullptr;      // device, MX_KVQ8_STAGE floats (KvNewRow's staged rows)
    KvNewRow kvnew;
    // weight ranges the next decode attention launch touches while HBM is otherwise idle
    // (fa_prefetch_plan in exec.cpp; consumed by fa_dec2_run)
    const char * pf_ptr[4] = {};
    size_t pf_len[4] = {}, pf_take[4] = {};   // bytes; bytes taken from the head of each eighth
    int pf_n = 0;
    // second stage: the GEMV right after the attention (output projection, ~2 TB/s) warms
    // the next part of each eighth (gpf_off .. + gpf_take) while its own stream runs
    const ggml_tensor * gpf_node = nullptr;   // the MUL_MAT that carries it
    bool gpf_armed = false;                   // set while that node runs
    size_t gpf_off = 0, gpf_take = 0;
    bool rope_valid = false;
    // -fa 0 prefill (round 6): the f16 copy of the graph's f32 KQ mask, converted by the first
    // layer's attention and reused by the others of the same graph pass (every layer reads the
    // same input mask); valid while mask16_src matches (reset at each pass)
    uint16_t * mask16 = nullptr; size_t mask16_cap = 0;
    const void * mask16_src = nullptr; int64_t mask16_key[3] = {0, 0, 0};
    const void * rope_pos = nullptr, * rope_ff = nullptr;
    int32_t rope_params[11] = {};
    bool use_graphs = true;
    bool use_fusion = true;
    bool split_graph = false;        // the graph holds row-split weights: only fusions without a split matrix
    std::string name;
    ggml_backend backend{};
    ggml_abort_callback abort_cb = nullptr;
    void * abort_data = nullptr;
    // profiling counters (read through mx_backend_stats)
    uint64_t n_graph_compute = 0, n_graph_replay = 0, n_nodes_run = 0, n_fused = 0;
    // host-side cost of the backend entry points libllama calls per token (GGML_MI355X_STATS):
    // microseconds spent inside graph_compute / set_async / get_async / synchronize, and
    // the calls and bytes of the copies
    double us_compute = 0, us_set = 0, us_get = 0, us_sync = 0;
    double us_sig = 0, us_launch = 0;   // inside graph_compute: signature compare, hipGraphLaunch
    uint64_t n_set = 0, n_get = 0, b_set = 0, b_get = 0;
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
// scratch bytes a node needs (upper bound; add_norm: the MUL_MAT feeds an ADD -> RMS_NORM pair)
size_t scratch_bytes(const ggml_tensor * node, bool add_norm = false);

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
void op_mul_mat_split(OpCtx & c, ggml_tensor * dst);
void op_mul_mat_split_n(OpCtx & c, ggml_tensor * const * dsts, int n);   // 1-3 sharing src1, one fork / join
int split_local_slices(const Stream * s, const ggml_tensor * w, void ** data, int64_t * lo, int64_t * hi);
// every non-empty slice of a row-split weight whose device reads the main device's memory
// directly (same GPU or peer access): data, rows, logical device; 0 when any slice cannot
int split_slices(const Stream * s, const ggml_tensor * w, void ** data, int64_t * lo, int64_t * hi, int * dev);
bool split_on_main(const Stream * s, const ggml_tensor * w, int dev);   // slice of w runs on the main stream itself
OpCtx split_fork(OpCtx & c, int dev);             // the slice device's stream, after the main stream's work so far
struct XStage;
// (round 6) the activation of a fused per-slice launch copied to the slice device once (split.cpp)
XStage split_local_xs(OpCtx & dc, const Stream * main, int dev, const XStage & xs, int64_t K, size_t * bytes);
void split_join(OpCtx & c, int dev);              // the main stream, after the slice stream's work so far
void split_stream_free(const Stream * main);   // be_free: drop the freed stream's row-split staging
void op_mul_mat_id(OpCtx & c, ggml_tensor * dst);
void op_flash_attn_ext(OpCtx & c, ggml_tensor * dst);

size_t mul_mat_scratch(const ggml_tensor * dst, bool add_norm = false);   // add_norm: an ADD -> RMS_NORM follows
size_t mul_mat_id_scratch(const ggml_tensor * dst);
size_t flash_attn_scratch(const ggml_tensor * dst);
bool mul_mat_supported(const ggml_tensor * dst);
bool mul_mat_id_supported(const ggml_tensor * dst);
bool flash_attn_supported(const ggml_tensor * dst);

// fused decode helpers (exec.cpp decides, kernels live in ops_mmvq.hip / ops_misc.hip)
// y_gate/up = W·x ; out = act(gate) * up   (ggml-cuda.cu:2145-2181 semantics)
bool mmvq_fused_glu(OpCtx & c, const ggml_tensor * gate_mm, const ggml_tensor * up_mm, ggml_tensor * glu);
// the same node triple for a prefill ubatch on MFMA (k_mmq3g, ops_mm.hip)
bool mmq_fused_glu(OpCtx & c, const ggml_tensor * gate_mm, const ggml_tensor * up_mm, ggml_tensor * glu);
bool mmq_fused_add(OpCtx & c, const ggml_tensor * mm, const ggml_tensor * res, ggml_tensor * add);
// 2-3 prefill GEMMs sharing src1 (q/k/v) in one launch (k_mmq3m); false if not eligible (nothing run)
bool mmq_group_run(OpCtx & c, ggml_tensor * const * mms, int n);
#if defined(__HIPCC__)
// f16 act-cache slot for a producer's f32 output rows (ops_mm.hip); null if it does not fit
_Float16 * mmq_act_claim(OpCtx & c, const void * data, int64_t K, int64_t ncols, size_t row_bytes);
#endif
// out = W·x + residual (MUL_MAT followed by ADD)
bool mmvq_fused_add(OpCtx & c, const ggml_tensor * mm, const ggml_tensor * residual, ggml_tensor * add);
// RMS_NORM → MUL(w) that also emits the quantised activation of its output
bool rms_norm_mul_q8(OpCtx & c, ggml_tensor * norm, const ggml_tensor * w, ggml_tensor * out);
// activation-cache management (ops_mmvq.hip)
size_t act_slot_bytes(const ggml_tensor * src1);
void act_cache_reset(Stream * s);
void graph_cache_forget(Stream * s);   // buffers moved: no captured graph may replay
void act_cache_invalidate(Stream * s, const ggml_tensor * written);
ActQ * act_cache_alloc(Stream * s, const ggml_tensor * t);   // reserve a slot for t (caller fills it)
ActQ * act_cache_alloc_raw(Stream * s, const void * data, int64_t ne0, int64_t ncols, size_t bytes);
const ActQ * act_cache_find(Stream * s, const ggml_tensor * t);   // q8 form of t, if cached
bool mmvq_small_batch_ok(const ggml_tensor * mm);             // MUL_MAT runs on the GEMV path
size_t mmq_act_bytes(const ggml_tensor * mm);                 // f16 activation bytes of a prefill GEMM (0: none)
// consumer count of every tensor in the graph being executed
using UseCount = std::unordered_map<const ggml_tensor *, int>;
// decode Q/K/V projections + RoPE + KV-cache stores in one launch; returns nodes consumed
int fuse_qkv_rope_store(OpCtx & c, ggml_cgraph * g, int i, const UseCount & uses);
// MoE router chain / expert combine in one launch each (ops_moe.hip); nodes consumed
int fuse_topk_moe(OpCtx & c, ggml_cgraph * g, int i);
// the pending q8_0 KV row(s) of KvNewRow: stored by one k_kv_store_q8 launch (ops_qkv.hip)
void kv_new_row_flush(OpCtx & c);
// the decode attention `fa` will consume Stream::kvnew itself (ops_fattn_dec.hip)
bool fa_takes_new_row(const Stream * s, const ggml_tensor * fa);
// -fa 0 decode attention chain (ops_fattn_dec.hip)
int fuse_attn_nofa(OpCtx & c, ggml_cgraph * g, int i, const UseCount & uses);
bool t_overlaps_ext(const ggml_tensor * a, const ggml_tensor * b);
// no output of a fused launch overlaps its inputs or another output, except the named
// element-wise in-place (output, input) pairs at the same start (exec.cpp)
bool fused_io_ok(std::initializer_list<const ggml_tensor *> outs, std::initializer_list<const ggml_tensor *> ins,
                 std::initializer_list<std::pair<const ggml_tensor *, const ggml_tensor *>> inplace = {});
int fuse_moe_combine(OpCtx & c, ggml_cgraph * g, int i, const UseCount & uses);
int fuse_moe_down_combine(OpCtx & c, ggml_cgraph * g, int i, const UseCount & uses);   // MUL_MAT_ID + combine
// the executor's guard for a node about to run (deferred norms it reads or overwrites)
void deferred_guard_node_ext(OpCtx & c, const ggml_tensor * n);

Stream * stream_of(ggml_backend_t b);

}  // namespace mx
