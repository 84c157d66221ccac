// backend.cpp — the MI355X ggml backend object model behind the reference's
// backend C-ABI (ggml/src/ggml-backend-impl.h:17-251): registry, devices,
// device/pinned buffer types, buffers, streams and events.
//
// Behavioural spec followed (the reference CUDA/HIP backend, replaced not ported):
//   registry/device enumeration  ggml-cuda.cu:5024-5075
//   buffer set/get/cpy           ggml-cuda.cu:600-700
//   async copies + events        ggml-cuda.cu:2760-2860
//   offload_op batch threshold   ggml-cuda.cu:4872-4891
#include "backend.h"
#include "ggml_mi355x.h"

#include <algorithm>
#include <chrono>
#include <cstdarg>
#include <mutex>
#include <memory>

#include <dlfcn.h>
#include <execinfo.h>
#include <fcntl.h>
#include <signal.h>
#include <ucontext.h>
#include <unistd.h>

namespace mx {

void graph_compute_impl(Stream * s, ggml_cgraph * g, ggml_status * status);  // exec.cpp

static std::vector<std::unique_ptr<Device>> g_devices;
static ggml_backend_reg g_reg{};
static std::once_flag g_once;

static const uint8_t kGuid[16] = {0x6d, 0x69, 0x33, 0x35, 0x35, 0x78, 0x2d, 0x67,
                                  0x66, 0x78, 0x39, 0x35, 0x30, 0x2d, 0x76, 0x31};

static Device * dev_ctx(ggml_backend_dev_t d) { return (Device *) d->context; }

// ---------------------------------------------------------------------------
// staged small writes. libllama writes each graph input through the buffer interface
// (set_input: token ids, positions, KQ mask, KV-cache row indices, output ids —
// src/llama-graph.cpp), about six per decoded token; a synchronous hipMemcpy each left
// the GPU idle between tokens. Writes up to 64 KB are copied into a pinned ring and
// sent asynchronously on the device's compute stream (the stream of the first backend
// created on it), so they are ordered before that backend's next graph; `ev` marks the
// latest one for every other path that touches device memory (buffer reads, memsets,
// copies, another stream's graph), which waits for it first.
// ---------------------------------------------------------------------------
// Round 4: a staged write no longer issues its own copy. Each one only lands in the pinned
// ring and is queued; the queue is flushed — ONE kernel on the compute stream copying every
// queued range from the ring (zero-copy reads of pinned host memory), then one event — when
// anything needs device memory ordered: graph_compute, every other buffer path, a
// synchronize. Per decoded token libllama writes ~6 inputs: 6 x (hipMemcpyAsync +
// hipEventRecord) of host time on the critical path between tokens, and 6 blit launches on
// the GPU (drop-in profile, profiles/r04/), became one launch.
// (StageEntry / StageFlushArgs and the flush kernel k_stage_flush: backend.h, ops_misc.hip)

struct Staging {
    std::mutex mu;
    Stream * s = nullptr;          // compute stream the writes go to (null: synchronous writes)
    char * host = nullptr;         // pinned ring
    size_t cap = 0, off = 0;
    hipEvent_t ev = nullptr;
    bool pending = false;          // a flushed write may still be in flight (ev marks the last)
    std::vector<StageEntry> queued;   // in the ring, not yet copied
    uint64_t n = 0;                // staged writes (GGML_MI355X_STATS)
    uint64_t n_flush = 0;          // flush launches
    uint64_t n_dropped = 0;        // queued writes dropped because their buffer was freed
};
static Staging g_stage[MX_MAX_DEVICES];
static bool env_flag(const char * name) { const char * v = getenv(name); return v && *v && strcmp(v, "0") != 0; }
static constexpr size_t kStageMax = 4 << 20, kStageRing = 32 << 20;

static void stage_flush_locked(Staging & st) {
    if (st.queued.empty()) return;
    int cur = 0;
    HIP_CHECK(hipGetDevice(&cur));
    if (cur != st.s->device) HIP_CHECK(hipSetDevice(st.s->device));
    for (size_t b = 0; b < st.queued.size(); b += kFlushMax) {
        StageFlushArgs a{};
        uint32_t chunks = 0;
        a.n = (int) std::min<size_t>(kFlushMax, st.queued.size() - b);
        for (int k = 0; k < a.n; ++k) {
            a.e[k] = st.queued[b + k];
            a.e[k].chunk0 = chunks;
            chunks += (a.e[k].n + kFlushChunk - 1) / kFlushChunk;
        }
        stage_flush_launch(a, chunks, st.s->stream);
        st.n_flush++;
    }
    HIP_CHECK(hipEventRecord(st.ev, st.s->stream));
    st.pending = true;
    st.queued.clear();
    if (cur != st.s->device) HIP_CHECK(hipSetDevice(cur));
}

static bool stage_write(int dev, void * dst, const void * data, size_t size) {
    if (dev < 0 || dev >= MX_MAX_DEVICES || size > kStageMax || size == 0) return false;
    Staging & st = g_stage[dev];
    std::lock_guard<std::mutex> lk(st.mu);
    if (!st.s) return false;
    if (!st.host) {
        if (hipHostMalloc((void **) &st.host, kStageRing, hipHostMallocPortable) != hipSuccess) { (void) hipGetLastError(); st.host = nullptr; return false; }
        HIP_CHECK(hipEventCreateWithFlags(&st.ev, hipEventDisableTiming));
        st.cap = kStageRing;
    }
    // a queued range this one overlaps is copied first (the ranges of one flush run in
    // parallel: the later write must not race the earlier)
    const char * lo = (const char *) dst, * hi = lo + size;
    for (const StageEntry & e : st.queued)
        if (e.dst < hi && lo < e.dst + e.n) { stage_flush_locked(st); break; }
    size_t a = (st.off + 255) & ~(size_t) 255;
    if (a + size > st.cap) {       // wrap: every earlier range has to be copied and done reading
        stage_flush_locked(st);
        HIP_CHECK(hipStreamSynchronize(st.s->stream));
        a = 0;
    }
    memcpy(st.host + a, data, size);
    st.queued.push_back(StageEntry{st.host + a, (char *) dst, (uint32_t) size, 0});
    st.off = a + size;
    st.n++;
    static const bool immediate = getenv("GGML_MI355X_STAGE_IMMEDIATE") != nullptr;   // A/B: one flush per write
    if (immediate) stage_flush_locked(st);
    return true;
}

// make `stream` wait for the device's staged writes (no-op when none or on their stream);
// queued ones are flushed first
void staged_writes_wait(int dev, hipStream_t stream) {
    if (dev < 0 || dev >= MX_MAX_DEVICES) return;
    Staging & st = g_stage[dev];
    std::lock_guard<std::mutex> lk(st.mu);
    if (st.s) stage_flush_locked(st);
    if (!st.pending || (st.s && st.s->stream == stream)) return;
    HIP_CHECK(hipStreamWaitEvent(stream, st.ev, 0));
}
// the same without flushing the queue: only writes already sent are ordered before `stream`
static void staged_writes_pending_wait(int dev, hipStream_t stream) {
    if (dev < 0 || dev >= MX_MAX_DEVICES) return;
    Staging & st = g_stage[dev];
    std::lock_guard<std::mutex> lk(st.mu);
    if (!st.pending || (st.s && st.s->stream == stream)) return;
    HIP_CHECK(hipStreamWaitEvent(stream, st.ev, 0));
}

// ---------------------------------------------------------------------------
// device buffers
// ---------------------------------------------------------------------------
// Round 6: a generation count of the model weights — bumped by any buffer free and by every
// write into a weights buffer (ggml_backend_buffer_set_usage(WEIGHTS), which libllama sets
// on its model buffers): copies of weights kept elsewhere (split.cpp's slice-local norm
// weights) are valid while it is unchanged
static std::atomic<unsigned> g_weights_gen{1};
unsigned mx_weights_gen() { return g_weights_gen.load(std::memory_order_relaxed); }
static void weights_touched(ggml_backend_buffer_t b) {
    if (b && b->usage == GGML_BACKEND_BUFFER_USAGE_WEIGHTS) g_weights_gen.fetch_add(1, std::memory_order_relaxed);
}
// Staged writes into this buffer that are still queued (be_sync no longer flushes, round 5)
// or flushed but in flight must land before the memory goes back: otherwise the later
// k_stage_flush writes into a freed range — or into the next allocation at that address.
// Queued ranges inside the buffer are dropped (the buffer's contents die with it); any in
// flight are waited for.
static void stage_release_range(int dev, const char * lo, const char * hi) {
    if (dev < 0 || dev >= MX_MAX_DEVICES) return;
    Staging & st = g_stage[dev];
    std::lock_guard<std::mutex> lk(st.mu);
    const size_t n0 = st.queued.size();
    st.queued.erase(std::remove_if(st.queued.begin(), st.queued.end(),
                                   [&](const StageEntry & e) { return e.dst >= lo && e.dst + e.n <= hi; }),
                    st.queued.end());
    st.n_dropped += n0 - st.queued.size();
    bool overlap = false;   // (a range straddling the buffer's edge: flush it, it writes a neighbour too)
    for (const StageEntry & e : st.queued) overlap |= e.dst < hi && lo < e.dst + e.n;
    if (overlap) stage_flush_locked(st);
    if (st.pending) {
        HIP_CHECK(hipEventSynchronize(st.ev));
        st.pending = false;
    }
}
static void buf_free(ggml_backend_buffer_t b) {
    g_weights_gen.fetch_add(1, std::memory_order_relaxed);
    BufferCtx * c = (BufferCtx *) b->context;
    if (c->base) {
        hipSetDevice(c->device);
        stage_release_range(c->device, (const char *) c->base, (const char *) c->base + c->size);
        hipFree(c->base);
    }
    delete c;
}
static void * buf_base(ggml_backend_buffer_t b) { return ((BufferCtx *) b->context)->base; }
static ggml_status buf_init_tensor(ggml_backend_buffer_t, ggml_tensor *) { return GGML_STATUS_SUCCESS; }

static void buf_memset(ggml_backend_buffer_t b, ggml_tensor * t, uint8_t v, size_t off, size_t size) {
    weights_touched(b);
    BufferCtx * c = (BufferCtx *) b->context;
    HIP_CHECK(hipSetDevice(c->device));
    staged_writes_wait(c->device, hipStreamPerThread);
    HIP_CHECK(hipMemsetAsync((char *) t->data + off, v, size, hipStreamPerThread));
    HIP_CHECK(hipStreamSynchronize(hipStreamPerThread));
}
static void buf_set(ggml_backend_buffer_t b, ggml_tensor * t, const void * data, size_t off, size_t size) {
    weights_touched(b);
    BufferCtx * c = (BufferCtx *) b->context;
    HIP_CHECK(hipSetDevice(c->device));
    if (stage_write(c->device, (char *) t->data + off, data, size)) return;
    staged_writes_wait(c->device, hipStreamPerThread);
    HIP_CHECK(hipMemcpyAsync((char *) t->data + off, data, size, hipMemcpyHostToDevice, hipStreamPerThread));
    HIP_CHECK(hipStreamSynchronize(hipStreamPerThread));
}
static void buf_get(ggml_backend_buffer_t b, const ggml_tensor * t, void * data, size_t off, size_t size) {
    BufferCtx * c = (BufferCtx *) b->context;
    HIP_CHECK(hipSetDevice(c->device));
    staged_writes_wait(c->device, hipStreamPerThread);
    HIP_CHECK(hipMemcpyAsync(data, (const char *) t->data + off, size, hipMemcpyDeviceToHost, hipStreamPerThread));
    HIP_CHECK(hipStreamSynchronize(hipStreamPerThread));
}
static bool buf_is_ours(ggml_backend_buffer_t b);
static bool buf_cpy(ggml_backend_buffer_t b, const ggml_tensor * src, ggml_tensor * dst) {
    if (!src->buffer || !buf_is_ours(src->buffer)) return false;
    BufferCtx * sc = (BufferCtx *) src->buffer->context;
    BufferCtx * dc = (BufferCtx *) b->context;
    const size_t n = mx_nbytes(src);
    HIP_CHECK(hipSetDevice(dc->device));
    staged_writes_wait(dc->device, hipStreamPerThread);
    staged_writes_wait(sc->device, hipStreamPerThread);
    if (sc->device == dc->device) {
        HIP_CHECK(hipMemcpyAsync(dst->data, src->data, n, hipMemcpyDeviceToDevice, hipStreamPerThread));
    } else {
        HIP_CHECK(hipMemcpyPeerAsync(dst->data, dc->device, src->data, sc->device, n, hipStreamPerThread));
    }
    HIP_CHECK(hipStreamSynchronize(hipStreamPerThread));
    return true;
}
static void buf_clear(ggml_backend_buffer_t b, uint8_t v) {
    weights_touched(b);
    BufferCtx * c = (BufferCtx *) b->context;
    HIP_CHECK(hipSetDevice(c->device));
    staged_writes_wait(c->device, hipStreamPerThread);
    HIP_CHECK(hipMemsetAsync(c->base, v, c->size, hipStreamPerThread));
    HIP_CHECK(hipStreamSynchronize(hipStreamPerThread));
}

static const ggml_backend_buffer_i kBufIface = {
    buf_free, buf_base, buf_init_tensor, buf_memset, buf_set, buf_get, buf_cpy, buf_clear, nullptr,
};
static bool buf_is_ours(ggml_backend_buffer_t b) { return b->iface.get_base == buf_base; }

static const char * buft_name(ggml_backend_buffer_type_t t) { return dev_ctx(t->device)->name.c_str(); }
static ggml_backend_buffer_t buft_alloc(ggml_backend_buffer_type_t t, size_t size) {
    Device * d = dev_ctx(t->device);
    HIP_CHECK(hipSetDevice(d->id));
    void * p = nullptr;
    size = std::max<size_t>(size, 1);
    if (hipMalloc(&p, size) != hipSuccess) {
        (void) hipGetLastError();
        fprintf(stderr, "%s: failed to allocate %.2f MiB on %s\n", __func__, size / 1048576.0, d->name.c_str());
        return nullptr;
    }
    BufferCtx * c = new BufferCtx{d->id, p, size, d->name};
    // ggml_backend_buffer_free (ggml-backend.cpp) releases the struct with delete
    return new ggml_backend_buffer{kBufIface, t, c, size, GGML_BACKEND_BUFFER_USAGE_ANY};
}
static size_t buft_align(ggml_backend_buffer_type_t) { return 256; }
static size_t buft_max(ggml_backend_buffer_type_t) { return SIZE_MAX; }
// Tail padding of quantised tensors: 16 bytes lets vector loads run past the last
// block of the last row without faulting (the kernels mask the values).
static size_t buft_alloc_size(ggml_backend_buffer_type_t, const ggml_tensor * t) {
    size_t n = mx_nbytes(t);
    if (mx_type(t->type).quant) n += 64;
    return n;
}
static bool buft_is_host(ggml_backend_buffer_type_t) { return false; }

static const ggml_backend_buffer_type_i kBuftIface = {
    buft_name, buft_alloc, buft_align, buft_max, buft_alloc_size, buft_is_host,
};

// ---------------------------------------------------------------------------
// pinned host buffers (get_host_buffer_type; ggml-cuda.cu:1120-1190 behaviour)
// ---------------------------------------------------------------------------
static void hbuf_free(ggml_backend_buffer_t b) { HIP_CHECK(hipHostFree(b->context)); }
static void * hbuf_base(ggml_backend_buffer_t b) { return b->context; }
static void hbuf_memset(ggml_backend_buffer_t, ggml_tensor * t, uint8_t v, size_t off, size_t size) { memset((char *) t->data + off, v, size); }
static void hbuf_set(ggml_backend_buffer_t, ggml_tensor * t, const void * d, size_t off, size_t size) { memcpy((char *) t->data + off, d, size); }
static void hbuf_get(ggml_backend_buffer_t, const ggml_tensor * t, void * d, size_t off, size_t size) { memcpy(d, (const char *) t->data + off, size); }
static bool hbuf_cpy(ggml_backend_buffer_t, const ggml_tensor * src, ggml_tensor * dst) {
    if (src->buffer && src->buffer->buft->iface.is_host && src->buffer->buft->iface.is_host(src->buffer->buft)) {
        memcpy(dst->data, src->data, mx_nbytes(src));
        return true;
    }
    return false;
}
static void hbuf_clear(ggml_backend_buffer_t b, uint8_t v) { memset(b->context, v, b->size); }
static const ggml_backend_buffer_i kHostBufIface = {
    hbuf_free, hbuf_base, nullptr, hbuf_memset, hbuf_set, hbuf_get, hbuf_cpy, hbuf_clear, nullptr,
};
static const char * hbuft_name(ggml_backend_buffer_type_t) { return "MI355X_Host"; }
static ggml_backend_buffer_t hbuft_alloc(ggml_backend_buffer_type_t t, size_t size) {
    void * p = nullptr;
    if (hipHostMalloc(&p, std::max<size_t>(size, 1), hipHostMallocPortable) != hipSuccess) {
        (void) hipGetLastError();
        return nullptr;
    }
    return new ggml_backend_buffer{kHostBufIface, t, p, size, GGML_BACKEND_BUFFER_USAGE_ANY};
}
static size_t hbuft_align(ggml_backend_buffer_type_t) { return 64; }
static bool hbuft_is_host(ggml_backend_buffer_type_t) { return true; }
static const ggml_backend_buffer_type_i kHostBuftIface = {
    hbuft_name, hbuft_alloc, hbuft_align, nullptr, nullptr, hbuft_is_host,
};

// ---------------------------------------------------------------------------
// backend (stream)
// ---------------------------------------------------------------------------
Stream * stream_of(ggml_backend_t b) { return (Stream *) b->context; }

static const char * be_name(ggml_backend_t b) { return stream_of(b)->name.c_str(); }
static double now_us() { return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count(); }
void klog_dump(const char * path);
static void be_free(ggml_backend_t b) {
    Stream * s = stream_of(b);
    hipSetDevice(s->device);
    if (s->device >= 0 && s->device < MX_MAX_DEVICES) {   // queued writes land before the stream goes
        Staging & st = g_stage[s->device];
        std::lock_guard<std::mutex> lk(st.mu);
        if (st.s == s) stage_flush_locked(st);
    }
    hipStreamSynchronize(s->stream);
    if (s->device >= 0 && s->device < MX_MAX_DEVICES) {   // later small writes go synchronous again
        Staging & st = g_stage[s->device];
        std::lock_guard<std::mutex> lk(st.mu);
        if (st.s == s) { st.s = nullptr; st.pending = false; }
    }
    // GGML_MI355X_STATS=1: executor counters of this backend on stderr when libllama frees
    // it (drop-in runs: shows the fusions fired on the reference's own node order)
    if (getenv("GGML_MI355X_STATS"))
        fprintf(stderr, "[mi355x] stats {\"backend\": \"%s\", \"graph_compute\": %llu, \"graph_replay\": %llu, "
                "\"nodes_run\": %llu, \"nodes_fused\": %llu, \"host_us\": {\"graph_compute\": %.0f, \"set_async\": %.0f, "
                "\"get_async\": %.0f, \"synchronize\": %.0f, \"signature\": %.0f, \"graph_launch\": %.0f}, \"n_set\": %llu, \"bytes_set\": %llu, \"n_get\": %llu, "
                "\"bytes_get\": %llu, \"n_staged\": %llu, \"n_stage_flush\": %llu}\n", s->name.c_str(), (unsigned long long) s->n_graph_compute,
                (unsigned long long) s->n_graph_replay, (unsigned long long) s->n_nodes_run, (unsigned long long) s->n_fused,
                s->us_compute, s->us_set, s->us_get, s->us_sync, s->us_sig, s->us_launch, (unsigned long long) s->n_set, (unsigned long long) s->b_set,
                (unsigned long long) s->n_get, (unsigned long long) s->b_get,
                (unsigned long long) (s->device >= 0 && s->device < MX_MAX_DEVICES ? g_stage[s->device].n : 0),
                (unsigned long long) (s->device >= 0 && s->device < MX_MAX_DEVICES ? g_stage[s->device].n_flush : 0));
    if (const char * kp = getenv("GGML_MI355X_KLOG")) klog_dump(kp);
    split_stream_free(s);
    hipSetDevice(s->device);
    for (GraphCache & gc : s->gslots) {
        if (gc.exec) hipGraphExecDestroy(gc.exec);
        if (gc.graph) hipGraphDestroy(gc.graph);
    }
    if (s->scratch.base) hipFree(s->scratch.base);
    if (s->act.base) hipFree(s->act.base);
    if (s->f16.base) hipFree(s->f16.base);
    if (s->rope_tab) hipFree(s->rope_tab);
    if (s->fa_cnt) hipFree(s->fa_cnt);
    if (s->kvq8_stage) hipFree(s->kvq8_stage);
    if (s->mask16) hipFree(s->mask16);
    if (s->cpy_ev) hipEventDestroy(s->cpy_ev);
    hipStreamDestroy(s->stream);
    delete s;  // the ggml_backend struct lives inside Stream
}
static void be_set_async(ggml_backend_t b, ggml_tensor * t, const void * data, size_t off, size_t size) {
    weights_touched(t->buffer);
    Stream * s = stream_of(b);
    const double t0 = now_us();
    HIP_CHECK(hipSetDevice(s->device));
    staged_writes_wait(s->device, s->stream);   // no-op on the staging stream itself
    HIP_CHECK(hipMemcpyAsync((char *) t->data + off, data, size, hipMemcpyHostToDevice, s->stream));
    s->us_set += now_us() - t0; s->n_set++; s->b_set += size;
}
static void be_get_async(ggml_backend_t b, const ggml_tensor * t, void * data, size_t off, size_t size) {
    Stream * s = stream_of(b);
    const double t0 = now_us();
    HIP_CHECK(hipSetDevice(s->device));
    staged_writes_wait(s->device, s->stream);
    HIP_CHECK(hipMemcpyAsync(data, (const char *) t->data + off, size, hipMemcpyDeviceToHost, s->stream));
    s->us_get += now_us() - t0; s->n_get++; s->b_get += size;
}
static bool is_our_backend(ggml_backend_t b);
// Layer-split hand-off (ggml-backend.cpp:1568 → reference ggml-cuda.cu:2799-2852):
// peer copy on the source stream over xGMI, ordered for the destination by an event.
static bool be_cpy_async(ggml_backend_t bsrc, ggml_backend_t bdst, const ggml_tensor * src, ggml_tensor * dst) {
    if (!is_our_backend(bsrc) || !is_our_backend(bdst)) return false;
    if (!src->buffer || !dst->buffer || !buf_is_ours(src->buffer) || !buf_is_ours(dst->buffer)) return false;
    Stream * ss = stream_of(bsrc);
    Stream * ds = stream_of(bdst);
    const size_t n = mx_nbytes(dst);
    HIP_CHECK(hipSetDevice(ss->device));
    staged_writes_wait(ss->device, ss->stream);   // a staged write to src (or to dst) lands first
    if (ds->device != ss->device) staged_writes_wait(ds->device, ss->stream);
    MX_KLOG("cpy_async %s -> %s bytes=%zu peer=%d", ss->name.c_str(), ds->name.c_str(), n,
            (int) (ss->device != ds->device || mx_force_peer()));
    if (ss->device == ds->device && !mx_force_peer()) {
        HIP_CHECK(hipMemcpyAsync(dst->data, src->data, n, hipMemcpyDeviceToDevice, ss->stream));
    } else {
        HIP_CHECK(hipMemcpyPeerAsync(dst->data, ds->device, src->data, ss->device, n, ss->stream));
    }
    if (ss != ds) {
        // the source stream's persistent event (re-recording it is legal once the wait
        // below has been enqueued: the waiter captured the earlier record)
        HIP_CHECK(hipEventRecord(ss->cpy_ev, ss->stream));
        HIP_CHECK(hipSetDevice(ds->device));
        HIP_CHECK(hipStreamWaitEvent(ds->stream, ss->cpy_ev, 0));
    }
    return true;
}
// Round 5: synchronize leaves queued staged writes queued. The scheduler synchronizes the
// backend before EVERY graph input it copies (ggml-backend.cpp:1464-1471, no events with
// one GPU), so flushing here made each of the ~6 inputs of a decoded token its own flush
// launch plus a host wait for it (BENCH_r04: n_stage_flush == n_staged). A queued write
// already holds its bytes in the pinned ring (the caller's buffer is free to reuse), and
// every path that reads or orders device memory flushes first (staged_writes_wait), so
// the token's inputs now go out in the one flush graph_compute issues.
static void be_sync(ggml_backend_t b) {
    Stream * s = stream_of(b);
    const double t0 = now_us();
    HIP_CHECK(hipSetDevice(s->device));
    static const bool flush_on_sync = env_flag("GGML_MI355X_SYNC_FLUSH");   // A/B: the round-4 behaviour
    if (flush_on_sync) staged_writes_wait(s->device, s->stream);
    else staged_writes_pending_wait(s->device, s->stream);   // flushed writes on another stream: ordered
    HIP_CHECK(hipStreamSynchronize(s->stream));
    s->us_sync += now_us() - t0;
}
static ggml_status be_graph_compute(ggml_backend_t b, ggml_cgraph * g) {
    Stream * s = stream_of(b);
    const double t0 = now_us();
    ggml_status st = GGML_STATUS_SUCCESS;
    graph_compute_impl(s, g, &st);
    s->us_compute += now_us() - t0;
    return st;
}
static void be_event_record(ggml_backend_t b, ggml_backend_event_t e) {
    Stream * s = stream_of(b);
    HIP_CHECK(hipSetDevice(s->device));
    HIP_CHECK(hipEventRecord((hipEvent_t) e->context, s->stream));
}
static void be_event_wait(ggml_backend_t b, ggml_backend_event_t e) {
    Stream * s = stream_of(b);
    HIP_CHECK(hipSetDevice(s->device));
    HIP_CHECK(hipStreamWaitEvent(s->stream, (hipEvent_t) e->context, 0));
}

static const ggml_backend_i kBackendIface = {
    be_name, be_free, be_set_async, be_get_async, be_cpy_async, be_sync,
    nullptr, nullptr, nullptr, nullptr,
    be_graph_compute, be_event_record, be_event_wait, nullptr,
};
static bool is_our_backend(ggml_backend_t b) { return b && b->iface.graph_compute == be_graph_compute; }


static ggml_backend_t make_backend(Device * d) {
    HIP_CHECK(hipSetDevice(d->id));
    Stream * s = new Stream();
    s->device = d->id;
    s->name = d->name;
    HIP_CHECK(hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking));
    HIP_CHECK(hipEventCreateWithFlags(&s->cpy_ev, hipEventDisableTiming));
    HIP_CHECK(hipMalloc((void **) &s->rope_tab, MX_ROPE_TAB * sizeof(float2)));   // never inside a capture
    HIP_CHECK(hipMalloc((void **) &s->fa_cnt, MX_FA_CNT * sizeof(unsigned int)));
    HIP_CHECK(hipMemset(s->fa_cnt, 0, MX_FA_CNT * sizeof(unsigned int)));
    HIP_CHECK(hipMalloc((void **) &s->kvq8_stage, MX_KVQ8_STAGE * sizeof(float)));
    s->use_graphs = !env_flag("GGML_MI355X_DISABLE_GRAPHS");
    s->use_fusion = !env_flag("GGML_MI355X_DISABLE_FUSION");
    s->backend.guid = (ggml_guid_t) kGuid;
    s->backend.iface = kBackendIface;
    s->backend.device = &d->dev;
    s->backend.context = s;
    if (d->id >= 0 && d->id < MX_MAX_DEVICES && !env_flag("GGML_MI355X_SYNC_SET")) {
        Staging & st = g_stage[d->id];
        std::lock_guard<std::mutex> lk(st.mu);
        if (!st.s) st.s = s;
    }
    return &s->backend;
}

// ---------------------------------------------------------------------------
// device
// ---------------------------------------------------------------------------
static const char * dv_name(ggml_backend_dev_t d) { return dev_ctx(d)->name.c_str(); }
static const char * dv_desc(ggml_backend_dev_t d) { return dev_ctx(d)->description.c_str(); }
static void dv_memory(ggml_backend_dev_t d, size_t * free, size_t * total) {
    HIP_CHECK(hipSetDevice(dev_ctx(d)->id));
    HIP_CHECK(hipMemGetInfo(free, total));
}
static ggml_backend_dev_type dv_type(ggml_backend_dev_t) { return GGML_BACKEND_DEVICE_TYPE_GPU; }
static void dv_props(ggml_backend_dev_t d, ggml_backend_dev_props * p) {
    p->name = dv_name(d);
    p->description = dv_desc(d);
    p->type = GGML_BACKEND_DEVICE_TYPE_GPU;
    p->device_id = dev_ctx(d)->pci_bus_id.c_str();
    dv_memory(d, &p->memory_free, &p->memory_total);
    p->caps.async = true;
    p->caps.host_buffer = !env_flag("GGML_MI355X_NO_PINNED");
    p->caps.buffer_from_host_ptr = false;
    p->caps.events = true;
}
static ggml_backend_t dv_init(ggml_backend_dev_t d, const char *) { return make_backend(dev_ctx(d)); }
static ggml_backend_buffer_type_t dv_buft(ggml_backend_dev_t d) { return &dev_ctx(d)->buft; }
static ggml_backend_buffer_type_t dv_host_buft(ggml_backend_dev_t d) { return &dev_ctx(d)->host_buft; }
// Row-split weights (split.cpp) serve one op only: MUL_MAT's src0, a 2D matrix, run from
// the split's main device with an f32 activation (the reference's CUDA rule,
// ggml_backend_cuda_device_supports_op).
// GGML_MI355X_REFUSE_OP=<op name> (ggml_op_name, e.g. FLASH_ATTN_EXT): report that op as
// unsupported — test infrastructure for the graph-split assertions of the drop-in tests
// (the scheduler then runs it on the CPU backend, which must show as extra splits)
static bool refused_op(const ggml_tensor * op) {
    static const int refuse = [] {
        const char * r = getenv("GGML_MI355X_REFUSE_OP");
        if (!r || !*r) return -1;
        static const struct { const char * name; int op; } names[] = {
            {"FLASH_ATTN_EXT", GGML_OP_FLASH_ATTN_EXT}, {"MUL_MAT", GGML_OP_MUL_MAT}, {"MUL_MAT_ID", GGML_OP_MUL_MAT_ID},
            {"ROPE", GGML_OP_ROPE}, {"RMS_NORM", GGML_OP_RMS_NORM}, {"SOFT_MAX", GGML_OP_SOFT_MAX}, {"SET_ROWS", GGML_OP_SET_ROWS},
        };
        for (const auto & n : names) if (strcmp(r, n.name) == 0) return n.op;
        return atoi(r);   // or the ggml_op enum value
    }();
    return refuse >= 0 && (int) op->op == refuse;
}
static bool dv_supports_op(ggml_backend_dev_t d, const ggml_tensor * op) {
    if (refused_op(op)) return false;
    for (int i = 0; i < GGML_MAX_SRC; ++i) {
        const ggml_tensor * s = op->src[i];
        if (!s || !s->buffer || !buft_is_split(s->buffer->buft)) continue;
        if (op->op != GGML_OP_MUL_MAT || i != 0 || s->ne[2] != 1 || s->ne[3] != 1) return false;
        if (split_main_device(s->buffer->buft) != dev_ctx(d)->index) return false;
        if (op->src[1]->type != GGML_TYPE_F32 || op->type != GGML_TYPE_F32) return false;
    }
    return supports_op(op);
}
static bool dv_supports_buft(ggml_backend_dev_t d, ggml_backend_buffer_type_t t) {
    if (buft_is_split(t)) return split_main_device(t) == dev_ctx(d)->index;
    return t->iface.alloc_buffer == buft_alloc && t->device == d;
}
static int64_t op_batch(const ggml_tensor * op) {
    switch (op->op) {
        case GGML_OP_GET_ROWS: return 0;
        case GGML_OP_MUL_MAT: return op->ne[1];
        case GGML_OP_MUL_MAT_ID: case GGML_OP_ROPE: case GGML_OP_ROPE_BACK: return op->ne[2];
        default: return mx_nrows(op);
    }
}
static bool dv_offload_op(ggml_backend_dev_t, const ggml_tensor * op) {
    static const int64_t min_batch = [] { const char * v = getenv("GGML_OP_OFFLOAD_MIN_BATCH"); return v ? atoll(v) : 32LL; }();
    return op_batch(op) >= min_batch;
}
static ggml_backend_event_t dv_event_new(ggml_backend_dev_t d) {
    HIP_CHECK(hipSetDevice(dev_ctx(d)->id));
    hipEvent_t e;
    HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    return new ggml_backend_event{d, e};
}
static void dv_event_free(ggml_backend_dev_t, ggml_backend_event_t e) {
    hipEventDestroy((hipEvent_t) e->context);
    delete e;
}
static void dv_event_sync(ggml_backend_dev_t, ggml_backend_event_t e) { HIP_CHECK(hipEventSynchronize((hipEvent_t) e->context)); }

static const ggml_backend_device_i kDevIface = {
    dv_name, dv_desc, dv_memory, dv_type, dv_props, dv_init, dv_buft, dv_host_buft, nullptr,
    dv_supports_op, dv_supports_buft, dv_offload_op, dv_event_new, dv_event_free, dv_event_sync,
};

// ---------------------------------------------------------------------------
// registry
// ---------------------------------------------------------------------------
static const char * rg_name(ggml_backend_reg_t) { return "MI355X"; }
static size_t rg_count(ggml_backend_reg_t) { return g_devices.size(); }
static ggml_backend_dev_t rg_get(ggml_backend_reg_t, size_t i) { return i < g_devices.size() ? &g_devices[i]->dev : nullptr; }

static ggml_backend_feature * rg_features(ggml_backend_reg_t) {
    static ggml_backend_feature f[] = {
        {"ARCH", "gfx950"}, {"WAVE", "64"}, {"MFMA", "f16"}, {"DOT", "v_dot4_i32_i8,v_dot2_f32_f16"}, {"HIP_GRAPHS", "1"}, {nullptr, nullptr},
    };
    return f;
}
static void rg_set_abort(ggml_backend_t b, ggml_abort_callback cb, void * data) {
    if (!is_our_backend(b)) return;
    stream_of(b)->abort_cb = cb;
    stream_of(b)->abort_data = data;
}
static void * rg_proc(ggml_backend_reg_t, const char * name) {
    if (strcmp(name, "ggml_backend_get_features") == 0) return (void *) rg_features;
    if (strcmp(name, "ggml_backend_set_abort_callback") == 0) return (void *) rg_set_abort;
    if (strcmp(name, "ggml_backend_split_buffer_type") == 0) return (void *) split_buffer_type;
    return nullptr;
}

static const ggml_backend_reg_i kRegIface = { rg_name, rg_count, rg_get, rg_proc };

// logical devices for the row split (split.cpp)
static bool g_peer[MX_MAX_DEVICES][MX_MAX_DEVICES];   // peer access enabled a -> b (HIP ids)
// (GGML_MI355X_NO_PEER: never, also between logical devices of one GPU, so the row split's
// staged gather runs in one-GPU tests)
bool mx_peer_enabled(int a, int b) {
    static const bool no_peer = env_flag("GGML_MI355X_NO_PEER");
    if (no_peer) return false;
    return a == b || (a >= 0 && b >= 0 && a < MX_MAX_DEVICES && b < MX_MAX_DEVICES && g_peer[a][b] && g_peer[b][a]);
}
int mx_dev_count() { return (int) g_devices.size(); }
int mx_dev_hip(int logical) { return g_devices[logical]->id; }
ggml_backend_dev_t mx_dev_handle(int logical) { return &g_devices[logical]->dev; }
// one auxiliary stream per logical device runs that device's row slices
Stream * mx_aux_stream(int logical) {
    static std::mutex mu;
    static Stream * aux[MX_MAX_DEVICES] = {};
    std::lock_guard<std::mutex> lk(mu);
    if (!aux[logical]) aux[logical] = stream_of(make_backend(g_devices[logical].get()));
    return aux[logical];
}

// GGML_MI355X_SEGV_TRACE=<file>|1: on SIGSEGV/SIGBUS write the faulting PC and address, every
// frame as module+offset (dladdr: stripped ROCm libraries still resolve to a module and an
// offset that addr2line / llvm-symbolizer can turn into a symbol offline) and the
// /proc/self/maps lines, then hand the signal to the handler that was installed before
// (a profiler's, say: restored and re-raised) or to the default action. Diagnostics only
// (the handler is not strictly async-signal-safe).
static int g_segv_fd = 2;
static struct sigaction g_segv_prev[2];   // SIGSEGV, SIGBUS
static void segv_write(const char * s) { if (write(g_segv_fd, s, strlen(s)) < 0) {} }
static void segv_handler(int sig, siginfo_t * si, void * uc) {
    char line[512];
    const ucontext_t * u = (const ucontext_t *) uc;
    const void * pc = (const void *) u->uc_mcontext.gregs[REG_RIP];
    snprintf(line, sizeof line, "[mi355x] signal %d addr %p pc %p\n", sig, si->si_addr, pc);
    segv_write(line);
    void * fr[64];
    const int nf = backtrace(fr, 64);
    for (int i = 0; i < nf + 1; ++i) {
        const void * a = i == 0 ? pc : fr[i - 1];
        Dl_info di{};
        if (dladdr(a, &di) && di.dli_fname)
            snprintf(line, sizeof line, "  #%02d %p %s+0x%lx %s+0x%lx\n", i, a, di.dli_fname,
                     (unsigned long) ((const char *) a - (const char *) di.dli_fbase), di.dli_sname ? di.dli_sname : "?",
                     di.dli_saddr ? (unsigned long) ((const char *) a - (const char *) di.dli_saddr) : 0ul);
        else snprintf(line, sizeof line, "  #%02d %p ?\n", i, a);
        segv_write(line);
    }
    segv_write("[mi355x] maps:\n");
    const int mf = open("/proc/self/maps", O_RDONLY);
    if (mf >= 0) {
        char buf[4096];
        ssize_t k;
        while ((k = read(mf, buf, sizeof buf)) > 0) if (write(g_segv_fd, buf, (size_t) k) < 0) break;
        close(mf);
    }
    // chain: put back what was installed before this handler and re-raise (the fault
    // re-triggers on return for a synchronous SIGSEGV; raise covers the rest)
    sigaction(sig, &g_segv_prev[sig == SIGBUS], nullptr);
    raise(sig);
}
static void segv_trace_install() {
    const char * v = getenv("GGML_MI355X_SEGV_TRACE");
    if (!v || !*v || strcmp(v, "0") == 0) return;
    if (strcmp(v, "1") != 0) { const int fd = open(v, O_WRONLY | O_CREAT | O_TRUNC, 0644); if (fd >= 0) g_segv_fd = fd; }
    struct sigaction sa{};
    sa.sa_sigaction = segv_handler;
    sa.sa_flags = SA_SIGINFO;
    sigemptyset(&sa.sa_mask);
    sigaction(SIGSEGV, &sa, &g_segv_prev[0]);
    sigaction(SIGBUS, &sa, &g_segv_prev[1]);
}

void klog_env_init();
static void init_registry() {
    segv_trace_install();
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) { (void) hipGetLastError(); n = 0; }
    // GGML_MI355X_VIRTUAL_DEVICES=V (tests): V logical devices over the n GPUs, round robin
    int nl = n;
    if (const char * v = getenv("GGML_MI355X_VIRTUAL_DEVICES")) if (n > 0 && atoi(v) > 0) nl = std::min(atoi(v), MX_MAX_DEVICES);
    for (int li = 0; li < nl; ++li) {
        const int i = li % std::max(n, 1);
        hipDeviceProp_t p;
        if (hipGetDeviceProperties(&p, i) != hipSuccess) continue;
        auto d = std::make_unique<Device>();
        d->id = i;
        d->index = (int) g_devices.size();
        d->name = "MI355X" + std::to_string(d->index);
        d->description = std::string(p.name[0] ? p.name : "AMD Instinct MI355X") + " (" + p.gcnArchName + ")";
        d->total_mem = p.totalGlobalMem;
        d->n_cu = p.multiProcessorCount;
        char pci[32] = {0};
        if (hipDeviceGetPCIBusId(pci, sizeof(pci), i) == hipSuccess) d->pci_bus_id = pci;
        for (auto & ch : d->pci_bus_id) ch = (char) tolower(ch);
        if (li >= n) d->pci_bus_id += "-v" + std::to_string(li);   // libllama skips devices with equal ids
        d->dev = ggml_backend_device{kDevIface, &g_reg, d.get()};
        d->buft = ggml_backend_buffer_type{kBuftIface, &d->dev, d.get()};
        d->host_buft = ggml_backend_buffer_type{kHostBuftIface, &d->dev, d.get()};
        g_devices.push_back(std::move(d));
    }
    // peer access between every pair of devices (reference: ggml_cuda_set_peer_access,
    // ggml-cuda.cu:1374): the layer split's hipMemcpyPeerAsync then goes device to device
    // over xGMI instead of staging through host memory. GGML_MI355X_NO_PEER=1 skips it.
    if (n > 1 && !getenv("GGML_MI355X_NO_PEER")) {
        for (int i = 0; i < n; ++i)
            for (int j = 0; j < n; ++j) {
                int ok = 0;
                if (i == j || hipDeviceCanAccessPeer(&ok, i, j) != hipSuccess || !ok) continue;
                hipSetDevice(i);
                const hipError_t e = hipDeviceEnablePeerAccess(j, 0);
                if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) (void) hipGetLastError();
                else if (i < MX_MAX_DEVICES && j < MX_MAX_DEVICES) g_peer[i][j] = true;
            }
        hipSetDevice(0);
    }
    klog_env_init();
    g_reg.api_version = GGML_BACKEND_API_VERSION;
    g_reg.iface = kRegIface;
    g_reg.context = nullptr;
}

}  // namespace mx

void mx_abort(const char * file, int line, const char * fmt, ...) {
    fprintf(stderr, "[mi355x] %s:%d: ", file, line);
    va_list ap;
    va_start(ap, fmt);
    vfprintf(stderr, fmt, ap);
    va_end(ap);
    fprintf(stderr, "\n");
    fflush(stderr);
    abort();
}

extern "C" {

ggml_backend_reg_t ggml_backend_mi355x_reg(void) {
    std::call_once(mx::g_once, mx::init_registry);
    return &mx::g_reg;
}

ggml_backend_reg_t ggml_backend_init(void) { return ggml_backend_mi355x_reg(); }

int ggml_backend_score(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) { (void) hipGetLastError(); return 0; }
    return n > 0 ? 200 : 0;
}

ggml_backend_t ggml_backend_mi355x_init(int device) {
    ggml_backend_reg_t r = ggml_backend_mi355x_reg();
    if (device < 0 || (size_t) device >= mx::g_devices.size()) return nullptr;
    return mx::make_backend(mx::g_devices[device].get());
    (void) r;
}

int ggml_backend_mi355x_get_device_count(void) {
    ggml_backend_mi355x_reg();
    return (int) mx::g_devices.size();
}

bool ggml_backend_is_mi355x(ggml_backend_t b) { return mx::is_our_backend(b); }

ggml_backend_buffer_type_t ggml_backend_mi355x_buffer_type(int device) {
    ggml_backend_mi355x_reg();
    if (device < 0 || (size_t) device >= mx::g_devices.size()) return nullptr;
    return &mx::g_devices[device]->buft;
}

void ggml_backend_mi355x_stats(ggml_backend_t b, uint64_t out[4]) {
    mx::Stream * s = mx::stream_of(b);
    out[0] = s->n_graph_compute; out[1] = s->n_graph_replay; out[2] = s->n_nodes_run; out[3] = s->n_fused;
}

void ggml_backend_mi355x_stage_stats(int device, uint64_t out[3]) {
    out[0] = out[1] = out[2] = 0;
    if (device < 0 || device >= mx::MX_MAX_DEVICES) return;
    mx::Staging & st = mx::g_stage[device];
    std::lock_guard<std::mutex> lk(st.mu);
    out[0] = st.n; out[1] = st.n_flush; out[2] = st.n_dropped;
}

}  // extern "C"

namespace mx {
double time_mmvq(Stream * s, const ggml_tensor * const * w, const ggml_tensor * const * w2, int nw,
                 const ggml_tensor * x, ggml_tensor * dst, int iters);
extern int g_tune[48];
}

extern "C" double ggml_backend_mi355x_time_mmvq(ggml_backend_t b, const ggml_tensor * const * w, const ggml_tensor * const * w2,
                                                int n_w, const ggml_tensor * x, ggml_tensor * dst, int iters) {
    mx::Stream * s = mx::stream_of(b);
    HIP_CHECK(hipSetDevice(s->device));
    return mx::time_mmvq(s, w, w2, n_w, x, dst, iters);
}

namespace mx {
static unsigned long long * g_trace_dev = nullptr;
unsigned long long * mx_trace_slot(int slot) {
    if (!g_tune[6]) return nullptr;
    if (!g_trace_dev) {
        HIP_CHECK(hipMalloc((void **) &g_trace_dev, 16 * 128 * sizeof(unsigned long long)));
        HIP_CHECK(hipMemset(g_trace_dev, 0, 16 * 128 * sizeof(unsigned long long)));
    }
    return g_trace_dev + slot * 128;
}
}

namespace mx {
static unsigned long long * g_trace_blk = nullptr;
unsigned long long * mx_trace_blocks() {
    if (g_tune[6] != 2) return nullptr;
    if (!g_trace_blk) HIP_CHECK(hipMalloc((void **) &g_trace_blk, 2 * 65536 * sizeof(unsigned long long)));
    return g_trace_blk;
}
}

extern "C" int ggml_backend_mi355x_trace_blocks_read(unsigned long long * out, int n) {
    if (!mx::g_trace_blk) return -1;
    if (n > 2 * 65536) n = 2 * 65536;
    HIP_CHECK(hipDeviceSynchronize());
    HIP_CHECK(hipMemcpy(out, mx::g_trace_blk, n * sizeof(unsigned long long), hipMemcpyDeviceToHost));
    HIP_CHECK(hipMemset(mx::g_trace_blk, 0, 2 * 65536 * sizeof(unsigned long long)));
    return n;
}

extern "C" int ggml_backend_mi355x_trace_read(unsigned long long * out, int n) {
    if (!mx::g_trace_dev) return -1;
    if (n > 16 * 128) n = 16 * 128;
    HIP_CHECK(hipDeviceSynchronize());
    HIP_CHECK(hipMemcpy(out, mx::g_trace_dev, n * sizeof(unsigned long long), hipMemcpyDeviceToHost));
    HIP_CHECK(hipMemset(mx::g_trace_dev, 0, 16 * 128 * sizeof(unsigned long long)));   // read-and-clear
    return n;
}

namespace mx {
int g_klog = 0;
static std::mutex g_klog_mu;
static std::string g_klog_buf;
void klog_add(const char * fmt, ...) {
    char line[256];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(line, sizeof(line), fmt, ap);
    va_end(ap);
    std::lock_guard<std::mutex> lk(g_klog_mu);
    if (g_klog_buf.size() < (1u << 22)) { g_klog_buf += line; g_klog_buf += '\n'; }
}

// GGML_MI355X_KLOG=<path>: record from registry init, written to <path> when a backend
// is freed (appended: one block per backend)
void klog_dump(const char * path) {
    std::lock_guard<std::mutex> lk(g_klog_mu);
    if (FILE * f = fopen(path, "a")) { fwrite(g_klog_buf.data(), 1, g_klog_buf.size(), f); fclose(f); }
    g_klog_buf.clear();
}
void klog_env_init() { if (getenv("GGML_MI355X_KLOG")) g_klog = 1; }
}

// on != 0: start recording kernel choices (clears the log); 0: stop
extern "C" void ggml_backend_mi355x_klog(int on) {
    std::lock_guard<std::mutex> lk(mx::g_klog_mu);
    mx::g_klog_buf.clear();
    mx::g_klog = on;
}
// copies the log (NUL-terminated, truncated to n - 1 bytes); returns its full length
extern "C" size_t ggml_backend_mi355x_klog_read(char * out, size_t n) {
    std::lock_guard<std::mutex> lk(mx::g_klog_mu);
    if (out && n) {
        const size_t k = std::min(n - 1, mx::g_klog_buf.size());
        memcpy(out, mx::g_klog_buf.data(), k);
        out[k] = 0;
    }
    return mx::g_klog_buf.size();
}

namespace mx { unsigned g_tune_gen = 0; }   // part of every cgraph signature (exec.cpp)
// a changed knob changes the launches a graph makes: captured graphs must not replay
extern "C" void ggml_backend_mi355x_set_tune(int idx, int value) {
    if (idx >= 0 && idx < 48 && mx::g_tune[idx] != value) { mx::g_tune[idx] = value; ++mx::g_tune_gen; }
}

extern "C" int ggml_backend_mi355x_ab_variants(void) { return MX_AB_VARIANTS; }
