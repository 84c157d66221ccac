// oracle/cpy_async_probe.cpp — TEST INFRASTRUCTURE ONLY. The layer-split hand-off as
// libllama's scheduler performs it (ggml-backend.cpp ggml_backend_sched_compute_splits:
// ggml_backend_tensor_copy_async between the split backends, then the next split's
// graph on the destination backend), driven through the reference's own ggml-backend
// code (libggml-ref.so) against libggml-mi355x.so loaded by path:
//   two backends (streams) of MI355X0 -> tensor on backend A, async copy to backend B's
//   buffer, a graph on B that reads it immediately (no host sync in between), read back.
// The copy must be ordered before B's graph by the backend's own event (be_cpy_async).
// Usage: cpy-async-probe <libggml-mi355x.so>; prints one JSON line, exit 0 on success.
#include "ggml.h"
#include "ggml-alloc.h"
#include "ggml-backend.h"

#include <cmath>
#include <cstdio>
#include <vector>

int main(int argc, char ** argv) {
    if (argc < 2) return 2;
    ggml_backend_reg_t reg = ggml_backend_load(argv[1]);
    if (!reg || ggml_backend_reg_dev_count(reg) < 1) { printf("{\"error\": \"load\"}\n"); return 3; }
    ggml_backend_dev_t dev = ggml_backend_reg_dev_get(reg, 0);
    ggml_backend_t ba = ggml_backend_dev_init(dev, nullptr);
    ggml_backend_t bb = ggml_backend_dev_init(dev, nullptr);
    const int64_t n = 1 << 22;   // 16 MB: long enough that an unordered graph would read stale data
    ggml_init_params ip = {ggml_tensor_overhead() * 8 + 8 * ggml_graph_overhead(), nullptr, true};
    ggml_context * ca = ggml_init(ip);
    ggml_context * cb = ggml_init(ip);
    ggml_tensor * src = ggml_new_tensor_1d(ca, GGML_TYPE_F32, n);
    ggml_tensor * dst = ggml_new_tensor_1d(cb, GGML_TYPE_F32, n);
    ggml_tensor * out = ggml_scale(cb, dst, 2.0f);
    ggml_backend_buffer_t bufa = ggml_backend_alloc_ctx_tensors(ca, ba);
    ggml_backend_buffer_t bufb = ggml_backend_alloc_ctx_tensors(cb, bb);
    std::vector<float> h(n), r(n);
    int bad = 0;
    for (int it = 0; it < 4; ++it) {
        for (int64_t i = 0; i < n; ++i) h[i] = (float) (i % 1000) + it;
        ggml_backend_tensor_set(src, h.data(), 0, n * 4);
        std::vector<float> z(n, -1.0f);
        ggml_backend_tensor_set(dst, z.data(), 0, n * 4);
        ggml_backend_tensor_copy_async(ba, bb, src, dst);
        ggml_cgraph * gf = ggml_new_graph(cb);
        ggml_build_forward_expand(gf, out);
        if (ggml_backend_graph_compute_async(bb, gf) != GGML_STATUS_SUCCESS) { printf("{\"error\": \"compute\"}\n"); return 4; }
        ggml_backend_synchronize(bb);
        ggml_backend_tensor_get(out, r.data(), 0, n * 4);
        for (int64_t i = 0; i < n; ++i) bad += r[i] != 2.0f * h[i];
    }
    printf("{\"backend\": \"%s\", \"elements\": %lld, \"mismatches\": %d}\n", ggml_backend_name(bb), (long long) n, bad);
    ggml_backend_buffer_free(bufa);
    ggml_backend_buffer_free(bufb);
    ggml_free(ca);
    ggml_free(cb);
    ggml_backend_free(ba);
    ggml_backend_free(bb);
    return bad == 0 ? 0 : 1;
}
