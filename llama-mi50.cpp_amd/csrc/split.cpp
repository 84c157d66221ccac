// split.cpp — row-split tensor parallelism (`llama -sm row`): the weight rows of every 2D
// matrix are partitioned over the devices, each device multiplies its rows with the
// activation, the row slices of the result are gathered on the main device.
//
// Reference behaviour replaced (not ported): llama asks the backend registry for the
// optional proc "ggml_backend_split_buffer_type" (src/llama-model.cpp:391-409) and puts
// the matrices in that buffer type when the device's supports_op accepts the MUL_MAT;
// the CUDA backend's split buffer (ggml-cuda.cu:778-1067) keeps per-device row slices in
// tensor->extra, and ggml_cuda_op_mul_mat (:1452-1770) broadcasts src1, runs every
// device's slice and copies the partial dst back (:1432).
//
// MI355X form: one process drives all devices (as the reference does for -sm row); each
// device runs its slice with the same kernels as an unsplit MUL_MAT (decode GEMV, prefill
// GEMM) on an auxiliary stream of its own, reading src1 where it lies on the main device and
// writing its rows of dst there directly (peer access over xGMI is enabled between all
// pairs at registry init; without it: peer copies in and out); events fork the slices off
// the main stream and join them back. Graphs with split weights keep the fusions that
// involve no split matrix, and are captured into one hipGraph when the slice devices are
// the main GPU (virtual devices), eager otherwise (split_graph_capturable).
// GGML_MI355X_VIRTUAL_DEVICES=N exposes the GPUs N times over (tests: a row split over
// two logical devices of one MI355X exercises every path but the xGMI link itself).
#include "backend.h"
#include "gemv.h"

#include <algorithm>
#include <array>
#include <map>
#include <mutex>

namespace mx {

int mx_dev_count();
int mx_dev_hip(int logical);
ggml_backend_dev_t mx_dev_handle(int logical);
Stream * mx_aux_stream(int logical);
bool mx_peer_enabled(int hip_a, int hip_b);
void stream_reserve_node(Stream * s, const ggml_tensor * n);

constexpr int64_t SPLIT_ROUND = 256;   // rows per slice are a multiple (GEMM row tiles, q8 groups)

struct SplitBuftCtx {
    int main = 0;
    std::array<float, MX_MAX_DEVICES> split{};   // cumulative start fractions
    std::string name;
};
struct SplitExtra {
    void * data[MX_MAX_DEVICES] = {};
    int64_t lo[MX_MAX_DEVICES] = {}, hi[MX_MAX_DEVICES] = {};
};
struct SplitBufCtx {
    const SplitBuftCtx * t = nullptr;
    std::vector<SplitExtra *> extras;
};

static void row_split(const SplitBuftCtx * c, int64_t nrows, int d, int64_t * lo, int64_t * hi) {
    const int n = mx_dev_count();
    auto at = [&](int i) { int64_t r = (int64_t) ((double) nrows * c->split[i]); return r - r % SPLIT_ROUND; };
    *lo = d == 0 ? 0 : at(d);
    *hi = d == n - 1 ? nrows : at(d + 1);
    if (*hi < *lo) *hi = *lo;
}

static void free_extra(SplitExtra * e) {
    for (int d = 0; d < MX_MAX_DEVICES; ++d)
        if (e->data[d]) { hipSetDevice(mx_dev_hip(d)); hipFree(e->data[d]); }
    delete e;
}

// ---- buffer
static void sbuf_free(ggml_backend_buffer_t b) {
    SplitBufCtx * c = (SplitBufCtx *) b->context;
    for (SplitExtra * e : c->extras) free_extra(e);
    delete c;
}
// tensors of a split buffer have no single address: data points into a dummy range
static void * sbuf_base(ggml_backend_buffer_t) { return (void *) 0x1000; }
static ggml_status sbuf_init_tensor(ggml_backend_buffer_t b, ggml_tensor * t) {
    if (t->view_src) return GGML_STATUS_SUCCESS;
    SplitBufCtx * c = (SplitBufCtx *) b->context;
    MX_ASSERT(mx_is_contiguous(t) && t->ne[2] == 1 && t->ne[3] == 1);
    SplitExtra * e = new SplitExtra();
    const size_t rs = mx_row_size(t->type, t->ne[0]);
    for (int d = 0; d < mx_dev_count(); ++d) {
        row_split(c->t, t->ne[1], d, &e->lo[d], &e->hi[d]);
        const int64_t n = e->hi[d] - e->lo[d];
        if (n == 0) continue;
        HIP_CHECK(hipSetDevice(mx_dev_hip(d)));
        // + 16 bytes: the kernels' vector loads may run past the last block of the last row
        HIP_CHECK(hipMalloc(&e->data[d], (size_t) n * rs + 256));
        HIP_CHECK(hipMemset(e->data[d], 0, (size_t) n * rs + 256));
    }
    t->extra = e;
    c->extras.push_back(e);
    return GGML_STATUS_SUCCESS;
}
static void sbuf_set(ggml_backend_buffer_t, ggml_tensor * t, const void * data, size_t off, size_t size) {
    MX_ASSERT(off == 0 && size == mx_nbytes(t) && t->extra);   // whole tensors, as the reference
    const SplitExtra * e = (const SplitExtra *) t->extra;
    const size_t rs = mx_row_size(t->type, t->ne[0]);
    for (int d = 0; d < mx_dev_count(); ++d) {
        const int64_t n = e->hi[d] - e->lo[d];
        if (n == 0) continue;
        HIP_CHECK(hipSetDevice(mx_dev_hip(d)));
        HIP_CHECK(hipMemcpy(e->data[d], (const char *) data + e->lo[d] * rs, n * rs, hipMemcpyHostToDevice));
    }
}
static void sbuf_get(ggml_backend_buffer_t, const ggml_tensor * t, void * data, size_t off, size_t size) {
    MX_ASSERT(off == 0 && size == mx_nbytes(t) && t->extra);
    const SplitExtra * e = (const SplitExtra *) t->extra;
    const size_t rs = mx_row_size(t->type, t->ne[0]);
    for (int d = 0; d < mx_dev_count(); ++d) {
        const int64_t n = e->hi[d] - e->lo[d];
        if (n == 0) continue;
        HIP_CHECK(hipSetDevice(mx_dev_hip(d)));
        HIP_CHECK(hipMemcpy((char *) data + e->lo[d] * rs, e->data[d], n * rs, hipMemcpyDeviceToHost));
    }
}
static void sbuf_clear(ggml_backend_buffer_t b, uint8_t v) {
    SplitBufCtx * c = (SplitBufCtx *) b->context;
    (void) c; (void) v;   // weights are always set whole; nothing reads a cleared split buffer
}
static const ggml_backend_buffer_i kSplitBufIface = {
    sbuf_free, sbuf_base, sbuf_init_tensor, nullptr, sbuf_set, sbuf_get, nullptr, sbuf_clear, nullptr,
};

// ---- buffer type
static const char * sbuft_name(ggml_backend_buffer_type_t t) { return ((SplitBuftCtx *) t->context)->name.c_str(); }
static ggml_backend_buffer_t sbuft_alloc(ggml_backend_buffer_type_t t, size_t size) {
    SplitBufCtx * c = new SplitBufCtx();
    c->t = (const SplitBuftCtx *) t->context;
    return new ggml_backend_buffer{kSplitBufIface, t, c, size, GGML_BACKEND_BUFFER_USAGE_WEIGHTS};
}
static size_t sbuft_align(ggml_backend_buffer_type_t) { return 128; }
static size_t sbuft_alloc_size(ggml_backend_buffer_type_t, const ggml_tensor * t) { return mx_nbytes(t); }
static bool sbuft_is_host(ggml_backend_buffer_type_t) { return false; }
static const ggml_backend_buffer_type_i kSplitBuftIface = {
    sbuft_name, sbuft_alloc, sbuft_align, nullptr, sbuft_alloc_size, sbuft_is_host,
};

bool buft_is_split(ggml_backend_buffer_type_t t) { return t && t->iface.alloc_buffer == sbuft_alloc; }
int split_main_device(ggml_backend_buffer_type_t t) { return ((const SplitBuftCtx *) t->context)->main; }
bool tensor_is_split(const ggml_tensor * t) { return t && t->buffer && buft_is_split(t->buffer->buft); }

// the proc "ggml_backend_split_buffer_type": (main device, tensor_split fractions)
ggml_backend_buffer_type_t split_buffer_type(int main_device, const float * tensor_split) {
    static std::mutex mu;
    static std::map<std::pair<int, std::array<float, MX_MAX_DEVICES>>, ggml_backend_buffer_type> types;
    std::lock_guard<std::mutex> lk(mu);
    const int n = mx_dev_count();
    if (main_device < 0 || main_device >= n) return nullptr;
    std::array<float, MX_MAX_DEVICES> cum{};
    bool zero = true;
    for (int i = 0; i < n && tensor_split; ++i) zero = zero && tensor_split[i] == 0.0f;
    float sum = 0.0f;
    for (int i = 0; i < n; ++i) {       // default: equal shares (the devices are identical)
        cum[i] = sum;
        sum += zero ? 1.0f : tensor_split[i];
    }
    for (int i = 0; i < n; ++i) cum[i] /= sum;
    auto it = types.find({main_device, cum});
    if (it != types.end()) return &it->second;
    SplitBuftCtx * c = new SplitBuftCtx();
    c->main = main_device;
    c->split = cum;
    c->name = "MI355X" + std::to_string(main_device) + "_Split";
    ggml_backend_buffer_type bt{kSplitBuftIface, mx_dev_handle(main_device), c};
    return &types.emplace(std::make_pair(main_device, cum), bt).first->second;
}

// ---- MUL_MAT with a split src0
// Staging buffers and events per (main stream, slice device): two contexts on the same main
// device (two main streams) never share a slice's staging buffers or events (a
// second context's peer copy could overwrite the no-peer gather buffer before the first
// one's scatter had read it).
struct SliceState {
    void * a = nullptr; size_t acap = 0;        // round 6: the fused launches' activation, slice-local
    std::map<const void *, void *> nw;          // norm weights copied to the slice device (weights gen below)
    unsigned nw_gen = 0;
    void * x = nullptr; size_t xcap = 0;        // no-peer path: src1 copy on the slice device
    void * y = nullptr; size_t ycap = 0;        // no-peer path: the slice's partial dst there
    void * g = nullptr; size_t gcap = 0;        // no-peer gather: the partial dst staged on main
    hipEvent_t ev_main = nullptr;               // main stream -> slice stream (created on main)
    hipEvent_t ev_done = nullptr;               // slice stream -> main stream (created on slice)
};
static std::mutex g_split_mu;
static std::map<std::pair<const Stream *, int>, SliceState> g_slices;   // (main stream, slice logical)

static void * grow(void *& p, size_t & cap, int hip, size_t bytes) {
    if (bytes > cap) {
        HIP_CHECK(hipSetDevice(hip));
        if (p) HIP_CHECK(hipFree(p));
        HIP_CHECK(hipMalloc(&p, bytes));
        cap = bytes;
    }
    return p;
}

// a freed backend's staging state goes with it (a later Stream allocated at the
// same address found the old one's events and gather buffer, possibly on another GPU)
void split_stream_free(const Stream * main) {
    std::lock_guard<std::mutex> lk(g_split_mu);
    for (auto it = g_slices.begin(); it != g_slices.end();) {
        if (it->first.first != main) { ++it; continue; }
        SliceState & st = it->second;
        const int d = it->first.second;
        HIP_CHECK(hipSetDevice(mx_dev_hip(d)));
        if (st.ev_done) { HIP_CHECK(hipEventSynchronize(st.ev_done)); HIP_CHECK(hipEventDestroy(st.ev_done)); }
        if (st.x) HIP_CHECK(hipFree(st.x));
        if (st.a) HIP_CHECK(hipFree(st.a));
        for (auto & kv : st.nw) HIP_CHECK(hipFree(kv.second));
        if (st.y) HIP_CHECK(hipFree(st.y));
        HIP_CHECK(hipSetDevice(main->device));
        if (st.ev_main) { HIP_CHECK(hipEventSynchronize(st.ev_main)); HIP_CHECK(hipEventDestroy(st.ev_main)); }
        if (st.g) HIP_CHECK(hipFree(st.g));
        it = g_slices.erase(it);
    }
}

static SliceState & slice_state(const Stream * main, int main_l, int d) {
    SliceState & st = g_slices[{main, d}];
    if (!st.ev_main) {
        HIP_CHECK(hipSetDevice(mx_dev_hip(main_l)));
        HIP_CHECK(hipEventCreateWithFlags(&st.ev_main, hipEventDisableTiming));
        HIP_CHECK(hipSetDevice(mx_dev_hip(d)));
        HIP_CHECK(hipEventCreateWithFlags(&st.ev_done, hipEventDisableTiming));
    }
    return st;
}

// A split graph may be captured into one hipGraph (exec.cpp) when every slice device is
// the main device's GPU (virtual devices): the fork / join events make the slice streams
// part of the capture. Across GPUs a capture would have to span devices, which this
// backend does not rely on: those graphs run eagerly. GGML_MI355X_SPLIT_GRAPHS=0 turns
// the capture off, =2 tries it across GPUs as well (experiment) — but never when a slice
// device lacks peer access to the main one: its staging copies (hipMemcpyPeerAsync) are
// not captured into a graph, they would run once at capture time and never on replay.
bool split_graph_capturable(int main_hip) {
    static const int mode = [] { const char * v = getenv("GGML_MI355X_SPLIT_GRAPHS"); return v ? atoi(v) : 1; }();
    if (mode == 0) return false;
    if (mode == 2) {
        for (int d = 0; d < mx_dev_count(); ++d) {
            const int hip = mx_dev_hip(d);
            if (hip != main_hip && !mx_peer_enabled(hip, main_hip)) {
                MX_KLOG("split_graphs=2 refused: device %d has no peer access to %d (peer copies)", hip, main_hip);
                return false;
            }
        }
        return true;
    }
    for (int d = 0; d < mx_dev_count(); ++d)
        if (mx_dev_hip(d) != main_hip) return false;
    return true;
}

// GGML_MI355X_FORCE_PEER=1 (tests): take the cross-device copy branches even when two
// logical devices are the same GPU (hipMemcpyPeerAsync between a device and itself is
// legal), so virtual-device runs execute the code real multi-GPU runs take.
bool mx_force_peer() {
    static const bool f = [] { const char * v = getenv("GGML_MI355X_FORCE_PEER"); return v && *v && strcmp(v, "0") != 0; }();
    return f;
}

// the slices of a row-split weight when every non-empty one lies on the main stream's own
// GPU (logical devices of one GPU, no forced peer path): their data and row ranges; 0 when
// any slice needs another device's stream (the fused per-slice launches run on c.st only)
int split_local_slices(const Stream * s, const ggml_tensor * w, void ** data, int64_t * lo, int64_t * hi) {
    if (!tensor_is_split(w) || !w->extra || mx_force_peer()) return 0;
    const SplitExtra * e = (const SplitExtra *) w->extra;
    if (mx_dev_hip(split_main_device(w->buffer->buft)) != s->device) return 0;
    int n = 0;
    for (int d = 0; d < mx_dev_count(); ++d) {
        if (e->hi[d] == e->lo[d]) continue;
        if (mx_dev_hip(d) != s->device || !mx_peer_enabled(s->device, s->device)) return 0;
        data[n] = e->data[d]; lo[n] = e->lo[d]; hi[n] = e->hi[d];
        ++n;
    }
    return n;
}

// Round 5: the fused per-slice decode launches (SwiGLU, GEMV + residual: ops_mmvq.hip) on
// every slice's own device — not only when all slices are this GPU's (split_local_slices).
// A slice device with peer access reads x (or its q8 copy) from the main device and
// writes its rows of the output there directly; the launches fork off the main stream and
// join back by the same per-(main stream, device) events as op_mul_mat_split.
int split_slices(const Stream * s, const ggml_tensor * w, void ** data, int64_t * lo, int64_t * hi, int * dev) {
    if (!tensor_is_split(w) || !w->extra) return 0;
    const SplitExtra * e = (const SplitExtra *) w->extra;
    if (mx_dev_hip(split_main_device(w->buffer->buft)) != s->device) return 0;
    int n = 0;
    for (int d = 0; d < mx_dev_count(); ++d) {
        if (e->hi[d] == e->lo[d]) continue;
        const int hip = mx_dev_hip(d);
        if (!mx_peer_enabled(hip, s->device)) return 0;      // (same GPU: mx_peer_enabled(h, h))
        data[n] = e->data[d]; lo[n] = e->lo[d]; hi[n] = e->hi[d]; dev[n] = d;
        ++n;
    }
    return n;
}

// GGML_MI355X_FORCE_PEER makes the other logical devices of this GPU behave as separate
// GPUs; the main device's own slice stays on the main stream, as it would on real hardware
bool split_on_main(const Stream * s, const ggml_tensor * w, int dev) {
    return mx_dev_hip(dev) == s->device && (!mx_force_peer() || dev == split_main_device(w->buffer->buft));
}

// Round 6: the activation of a fused per-slice decode launch, copied to a slice device that
// is not the main GPU — once per op and device — instead of read from the main GPU by
// every workgroup over xGMI (the QKV slice alone was ~224 workgroups x 32 KB of
// remote reads per layer; the reference quantises src1 once and peer-copies it, ggml-cuda.cu:
// 1603-1611, 1680-1692). On dc's stream (after split_fork): x (f32) or its q8 image, the
// attention's split partials (fap), and the deferred norm's weight — static model data,
// copied once per device and kept while no weights buffer changes (mx_weights_gen). Returns
// the XStage over the local copies; *bytes = the bytes this call moved to the device.
unsigned mx_weights_gen();
XStage split_local_xs(OpCtx & dc, const Stream * main, int dev, const XStage & xs, int64_t K, size_t * bytes) {
    *bytes = 0;
    const int hip = mx_dev_hip(dev);
    std::lock_guard<std::mutex> lk(g_split_mu);
    int main_l = 0;
    for (int d = 0; d < mx_dev_count(); ++d) if (mx_dev_hip(d) == main->device) { main_l = d; break; }
    SliceState & st = slice_state(main, main_l, dev);
    XStage r = xs;
    auto copy = [&](void * dst, const void * src, size_t n) {
        HIP_CHECK(hipSetDevice(hip));
        // (one GPU under FORCE_PEER: a plain device copy — a peer copy between a device and
        // itself is not captured into a graph, it would run once at capture time)
        if (hip == main->device) HIP_CHECK(hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToDevice, dc.st));
        else HIP_CHECK(hipMemcpyPeerAsync(dst, hip, src, main->device, n, dc.st));
        *bytes += n;
    };
    size_t need = 0;
    const size_t xb = (size_t) K * 4, qb = (size_t) K + 2 * (size_t) (K / 32) * 4;
    const size_t fb = xs.fap ? (size_t) (K / xs.fap_d) * xs.fap_ns * (xs.fap_d + 2) * 4 : 0;
    if (xs.fap) need = fb;
    else if (xs.q8) need = qb;
    else need = xb;
    // one buffer for every op of the graph, sized once: a later op must not reallocate it
    // while an earlier op's slice kernel still reads it (nor inside a graph capture)
    char * buf = (char *) grow(st.a, st.acap, hip, std::max<size_t>(need + 512, (size_t) 512 << 10));
    if (xs.fap) {
        copy(buf, xs.fap, fb);
        r.fap = (const float *) buf;
    } else if (xs.q8) {
        copy(buf, xs.q8, (size_t) K);
        copy(buf + ((K + 255) & ~(int64_t) 255), xs.q8d, (size_t) (K / 32) * 4);
        copy(buf + ((K + 255) & ~(int64_t) 255) + 256 + (size_t) (K / 32) * 4, xs.q8s, (size_t) (K / 32) * 4);
        r.q8 = (const int8_t *) buf;
        r.q8d = (const float *) (buf + ((K + 255) & ~(int64_t) 255));
        r.q8s = (const float *) (buf + ((K + 255) & ~(int64_t) 255) + 256 + (size_t) (K / 32) * 4);
    } else {
        copy(buf, xs.x, xb);
        r.x = (const float *) buf;
    }
    if (xs.norm) {
        if (st.nw_gen != mx_weights_gen()) {
            HIP_CHECK(hipSetDevice(hip));
            for (auto & kv : st.nw) HIP_CHECK(hipFree(kv.second));
            st.nw.clear();
            st.nw_gen = mx_weights_gen();
        }
        auto it = st.nw.find(xs.nw);
        if (it == st.nw.end()) {
            void * p = nullptr;
            HIP_CHECK(hipSetDevice(hip));
            HIP_CHECK(hipMalloc(&p, xb));
            copy(p, xs.nw, xb);
            it = st.nw.emplace(xs.nw, p).first;
        }
        r.nw = (const float *) it->second;
    }
    MX_KLOG("split_stage dev=%d K=%lld bytes=%zu src=%s", dev, (long long) K, *bytes, xs.fap ? "fap" : (xs.q8 ? "q8" : (xs.norm ? "norm" : "f32")));
    return r;
}

OpCtx split_fork(OpCtx & c, int dev) {
    std::lock_guard<std::mutex> lk(g_split_mu);
    int main_l = 0;
    for (int d = 0; d < mx_dev_count(); ++d) if (mx_dev_hip(d) == c.s->device) { main_l = d; break; }
    SliceState & st = slice_state(c.s, main_l, dev);
    Stream * ds = mx_aux_stream(dev);
    HIP_CHECK(hipSetDevice(c.s->device));
    HIP_CHECK(hipEventRecord(st.ev_main, c.st));
    HIP_CHECK(hipSetDevice(mx_dev_hip(dev)));
    HIP_CHECK(hipStreamWaitEvent(ds->stream, st.ev_main, 0));
    return OpCtx{ds, ds->stream, &ds->scratch};
}

void split_join(OpCtx & c, int dev) {
    std::lock_guard<std::mutex> lk(g_split_mu);
    int main_l = 0;
    for (int d = 0; d < mx_dev_count(); ++d) if (mx_dev_hip(d) == c.s->device) { main_l = d; break; }
    SliceState & st = slice_state(c.s, main_l, dev);
    Stream * ds = mx_aux_stream(dev);
    HIP_CHECK(hipSetDevice(mx_dev_hip(dev)));
    HIP_CHECK(hipEventRecord(st.ev_done, ds->stream));
    HIP_CHECK(hipSetDevice(c.s->device));
    HIP_CHECK(hipStreamWaitEvent(c.st, st.ev_done, 0));
}

// dsts: 1-3 MUL_MATs sharing src1 whose src0 are row-split alike (q / k / v). Every slice
// device's stream forks off the main stream once, runs its slices of all of them, and joins
// back once (round 4 forked and joined per matrix and per device in turn, so the slices of
// one matrix ran one device after another: -ts 1,1,1,1 under FORCE_PEER measured 0.22x).
void op_mul_mat_split_n(OpCtx & c, ggml_tensor * const * dsts, int n) {
    MX_ASSERT(n >= 1 && n <= 3);
    const ggml_tensor * w0 = dsts[0]->src[0];
    const ggml_tensor * x = dsts[0]->src[1];
    const SplitExtra * e0 = (const SplitExtra *) w0->extra;
    for (int k = 0; k < n; ++k) {
        const ggml_tensor * dst = dsts[k];
        MX_ASSERT(dst->src[1] == x && dst->src[0]->extra && mx_is_contiguous(dst) && dst->type == GGML_TYPE_F32);
        const SplitExtra * e = (const SplitExtra *) dst->src[0]->extra;
        for (int d = 0; d < mx_dev_count(); ++d) MX_ASSERT((e->hi[d] == e->lo[d]) == (e0->hi[d] == e0->lo[d]));
    }
    MX_ASSERT(e0 && x->type == GGML_TYPE_F32 && mx_is_contiguous(x));
    MX_ASSERT(x->ne[2] * x->ne[3] == dsts[0]->ne[2] * dsts[0]->ne[3]);
    const int64_t N = x->ne[1] * x->ne[2] * x->ne[3];
    const size_t xb = mx_nbytes(x);
    const int main_hip = c.s->device;
    const int main_l = split_main_device(w0->buffer->buft);
    MX_ASSERT(mx_dev_hip(main_l) == main_hip);
    std::lock_guard<std::mutex> lk(g_split_mu);
    const bool force = mx_force_peer();
    for (int k = 0; k < n; ++k)
        MX_KLOG("mm_split M=%d K=%d N=%d devices=%d peer=%d direct=%d group=%d", (int) dsts[k]->src[0]->ne[1], (int) x->ne[0], (int) N,
                mx_dev_count(), (int) force, (int) mx_peer_enabled(main_hip, main_hip), n);
    struct Plan { int d, hip; bool local, direct; Stream * ds; };
    Plan plan[MX_MAX_DEVICES];
    int np = 0;
    // fork: src1 is ready on the main stream at this point; every slice stream waits for it
    for (int d = 0; d < mx_dev_count(); ++d) {
        if (e0->hi[d] == e0->lo[d]) continue;
        const int hip = mx_dev_hip(d);
        // a slice on the main GPU itself runs on the main stream (no fork / join: each is a
        // cross-queue barrier in a captured graph); other GPUs' slices — and under
        // GGML_MI355X_FORCE_PEER the other logical devices' — on the slice device's stream
        const bool cross = hip != main_hip || (force && d != main_l);
        const bool direct = !cross || mx_peer_enabled(hip, main_hip);   // slice device reaches main's memory itself
        const bool local = !cross && direct;
        Plan & pl = plan[np++];
        pl = Plan{d, hip, local, direct, local ? c.s : mx_aux_stream(d)};
        if (local) continue;
        SliceState & st = slice_state(c.s, main_l, d);
        HIP_CHECK(hipSetDevice(main_hip));
        HIP_CHECK(hipEventRecord(st.ev_main, c.st));
        HIP_CHECK(hipSetDevice(hip));
        HIP_CHECK(hipStreamWaitEvent(pl.ds->stream, st.ev_main, 0));
    }
    // the slices: each device's stream runs its rows of every matrix
    for (int pi = 0; pi < np; ++pi) {
        const Plan & pl = plan[pi];
        SliceState & st = slice_state(c.s, main_l, pl.d);
        Stream * ds = pl.ds;
        if (!pl.local) { ds->scratch.reset(); act_cache_reset(ds); }   // (the slices share x: its q8 copy too)
        void * xd = nullptr;
        for (int k = 0; k < n; ++k) {
            ggml_tensor * dst = dsts[k];
            const ggml_tensor * w = dst->src[0];
            const SplitExtra * e = (const SplitExtra *) w->extra;
            const int64_t rows = e->hi[pl.d] - e->lo[pl.d];
            ggml_tensor ws = *w, xs = *x, ys = *dst;
            ws.ne[1] = rows; ws.nb[2] = ws.nb[3] = ws.nb[1] * rows; ws.data = e->data[pl.d]; ws.buffer = nullptr; ws.extra = nullptr;
            ws.view_src = nullptr;
            xs.buffer = nullptr; xs.view_src = nullptr;
            ys.ne[0] = rows; ys.buffer = nullptr; ys.view_src = nullptr;
            ys.src[0] = &ws; ys.src[1] = &xs;
            void * yd = nullptr;
            if (pl.direct) {
                // the slice kernel reads src1 where it lies and writes its rows of every column
                // straight into dst (over xGMI when the devices differ: peer access is on
                // between them) — no staging copies
                ys.data = (char *) dst->data + e->lo[pl.d] * 4;
                if (N == 1) { ys.nb[1] = (size_t) rows * 4; ys.nb[2] = ys.nb[3] = ys.nb[1]; }   // one column: contiguous
            } else {
                // no peer access (GGML_MI355X_NO_PEER or no link): src1 by peer copy to the
                // slice device (once per group), the partial dst there, one contiguous peer copy
                // back into a staging buffer on main, scattered into dst on the main stream
                MX_ASSERT(n == 1);
                xd = grow(st.x, st.xcap, pl.hip, xb);
                yd = grow(st.y, st.ycap, pl.hip, (size_t) rows * N * 4);
                HIP_CHECK(hipSetDevice(pl.hip));
                // (one GPU: a plain device copy — a peer copy between a device and itself is
                // not captured into a graph, it runs once at capture time)
                if (pl.hip == main_hip) HIP_CHECK(hipMemcpyAsync(xd, x->data, xb, hipMemcpyDeviceToDevice, ds->stream));
                else HIP_CHECK(hipMemcpyPeerAsync(xd, pl.hip, x->data, main_hip, xb, ds->stream));
                xs.data = xd;
                ys.nb[1] = (size_t) rows * 4; ys.nb[2] = ys.nb[1] * ys.ne[1]; ys.nb[3] = ys.nb[2] * ys.ne[2];
                ys.data = yd;
            }
            if (pl.local) {   // the main stream's buffers are sized for the graph's nodes, this slice included
                c.scratch->reset();
                op_mul_mat(c, &ys);
                continue;
            }
            stream_reserve_node(ds, &ys);
            OpCtx dc{ds, ds->stream, &ds->scratch};
            ds->scratch.reset();
            HIP_CHECK(hipSetDevice(pl.hip));
            op_mul_mat(dc, &ys);
            if (!pl.direct) {
                void * gm = grow(st.g, st.gcap, main_hip, (size_t) rows * N * 4);
                if (pl.hip == main_hip) HIP_CHECK(hipMemcpyAsync(gm, yd, (size_t) rows * N * 4, hipMemcpyDeviceToDevice, ds->stream));
                else HIP_CHECK(hipMemcpyPeerAsync(gm, main_hip, yd, pl.hip, (size_t) rows * N * 4, ds->stream));
            }
        }
    }
    // join: the main stream waits for every slice stream once
    for (int pi = 0; pi < np; ++pi) {
        const Plan & pl = plan[pi];
        if (pl.local) continue;
        SliceState & st = slice_state(c.s, main_l, pl.d);
        HIP_CHECK(hipSetDevice(pl.hip));
        HIP_CHECK(hipEventRecord(st.ev_done, pl.ds->stream));
        HIP_CHECK(hipSetDevice(main_hip));
        HIP_CHECK(hipStreamWaitEvent(c.st, st.ev_done, 0));
        if (!pl.direct) {   // (n == 1) the staged rows into dst
            const ggml_tensor * dst = dsts[0];
            const SplitExtra * e = (const SplitExtra *) dst->src[0]->extra;
            const int64_t rows = e->hi[pl.d] - e->lo[pl.d];
            HIP_CHECK(hipMemcpy2DAsync((char *) dst->data + e->lo[pl.d] * 4, dst->nb[1], st.g, (size_t) rows * 4, (size_t) rows * 4, N,
                                       hipMemcpyDeviceToDevice, c.st));
        }
    }
    HIP_CHECK(hipSetDevice(main_hip));
}

void op_mul_mat_split(OpCtx & c, ggml_tensor * dst) { op_mul_mat_split_n(c, &dst, 1); }

}  // namespace mx
