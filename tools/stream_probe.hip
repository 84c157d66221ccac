// stream_probe.hip — floors of the decode GEMV on this MI355X: how long a kernel that
// only streams S bytes of cold weights (and writes one word per workgroup) takes, for
// the Llama-3-8B decode matrix sizes, as (a) one-shot grids (every workgroup loads its
// slice once) and (b) persistent grid-stride loops at 1-4 workgroups per CU.
// Build: hipcc -O3 --offload-arch=gfx950 tools/stream_probe.hip -o tools/stream_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef int v4i __attribute__((ext_vector_type(4)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); exit(1); } } while (0)

// one-shot: each thread loads U v4i at stride blockDim*16 B
template <int U, bool NT>
__global__ __launch_bounds__(256) void k_oneshot(const v4i * __restrict__ p, size_t n16, int * out) {
    const size_t base = (size_t) blockIdx.x * 256 * U + threadIdx.x;
    v4i v[U];
#pragma unroll
    for (int j = 0; j < U; ++j) {
        const size_t i = base + (size_t) j * 256;
        if constexpr (NT) v[j] = i < n16 ? __builtin_nontemporal_load(p + i) : v4i{0, 0, 0, 0};
        else v[j] = i < n16 ? p[i] : v4i{0, 0, 0, 0};
    }
    int acc = 0;
#pragma unroll
    for (int j = 0; j < U; ++j) acc ^= v[j].x ^ v[j].y ^ v[j].z ^ v[j].w;
    if (acc == 0x12345678) out[blockIdx.x] = acc;
}

// persistent: chunks of 256*U v4i per workgroup iteration, two chunks in flight
template <int U>
__global__ __launch_bounds__(256) void k_persist(const v4i * __restrict__ p, size_t n16, int * out) {
    int acc = 0;
    const size_t chunk = (size_t) 256 * U;
    for (size_t c = blockIdx.x; c * chunk < n16; c += gridDim.x) {
        v4i v[U];
#pragma unroll
        for (int j = 0; j < U; ++j) {
            const size_t i = c * chunk + (size_t) j * 256 + threadIdx.x;
            v[j] = i < n16 ? __builtin_nontemporal_load(p + i) : v4i{0, 0, 0, 0};
        }
#pragma unroll
        for (int j = 0; j < U; ++j) acc ^= v[j].x ^ v[j].y ^ v[j].z ^ v[j].w;
    }
    if (acc == 0x12345678) out[blockIdx.x] = acc;
}


// the v2 GEMV's access pattern (Q4_K, K = 4096, 16 lanes per row, 4 units per lane,
// 3 loads per unit: header, two 16-B quarter-qs) without any compute
template <bool NT>
__global__ __launch_bounds__(256) void k_gemv_pattern(const char * __restrict__ w, int rows, int * out) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, sub = lane & 15;
    const int row = min((int) blockIdx.x * 16 + wave * 4 + (lane >> 4), rows - 1);
    const char * rp = w + (size_t) row * 2304;
    v4i v[12];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int u = sub + 16 * j;
        const char * b = rp + (u >> 2) * 144;
        const int g = u & 3;
        if constexpr (NT) {
            v[3 * j] = __builtin_nontemporal_load((const v4i *) b);
            v[3 * j + 1] = __builtin_nontemporal_load((const v4i *) (b + 16 + 32 * g));
            v[3 * j + 2] = __builtin_nontemporal_load((const v4i *) (b + 32 + 32 * g));
        } else {
            v[3 * j] = *(const v4i *) b;
            v[3 * j + 1] = *(const v4i *) (b + 16 + 32 * g);
            v[3 * j + 2] = *(const v4i *) (b + 32 + 32 * g);
        }
    }
    int acc = 0;
#pragma unroll
    for (int j = 0; j < 12; ++j) acc ^= v[j].x ^ v[j].y ^ v[j].z ^ v[j].w;
    if (acc == 0x12345678) out[blockIdx.x] = acc;
}

// coalesced: RPW rows per wave, the row's 144 16-B chunks spread over the lanes
template <int RPW>
__global__ __launch_bounds__(256) void k_row_coalesced(const char * __restrict__ w, int rows, int * out) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int row0 = ((int) blockIdx.x * 4 + wave) * RPW;
    constexpr int NC = 144 * RPW, NL = (NC + 63) / 64;
    const v4i * rp = (const v4i *) (w + (size_t) row0 * 2304);
    v4i v[NL];
#pragma unroll
    for (int j = 0; j < NL; ++j) {
        const int c = lane + 64 * j;
        v[j] = (c < NC && row0 + c / 144 < rows) ? __builtin_nontemporal_load(rp + c) : v4i{0, 0, 0, 0};
    }
    int acc = 0;
#pragma unroll
    for (int j = 0; j < NL; ++j) acc ^= v[j].x ^ v[j].y ^ v[j].z ^ v[j].w;
    if (acc == 0x12345678) out[blockIdx.x] = acc;
}

__global__ void k_empty(int * out) { if (threadIdx.x == 1023) out[0] = 1; }

int main() {
    const size_t POOL = (size_t) 2 << 30;
    char * buf; int * out;
    CK(hipMalloc(&buf, POOL));
    CK(hipMalloc(&out, 1 << 20));
    CK(hipMemset(buf, 1, POOL));
    hipStream_t st; CK(hipStreamCreate(&st));
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    const size_t sizes[] = {2359296, 9437184, 14155776, 33030144, 48168960, 66060288, 430940160};
    const char * names[] = {"k 1024x4096 q4k", "o 4096x4096 q4k", "qkv 6144x4096 q4k", "down 4096x14336 q4k",
                            "down q6k", "gate+up q4k", "lm_head q6k"};
    const int ITERS = 60;
    auto run = [&](const char * label, size_t S, auto launch) {
        const int ncopy = (int) std::min<size_t>(64, POOL / S);
        for (int i = 0; i < 4; ++i) launch((const v4i *) (buf + (size_t) (i % ncopy) * S), S / 16);
        CK(hipStreamSynchronize(st));
        CK(hipEventRecord(e0, st));
        for (int i = 0; i < ITERS; ++i) launch((const v4i *) (buf + (size_t) (i % ncopy) * S), S / 16);
        CK(hipEventRecord(e1, st));
        CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1));
        const double us = ms * 1000.0 / ITERS;
        printf("%-22s %-28s %9.2f us  %7.0f GB/s\n", label, "", us, S / us / 1e3);
    };
    // launch floor
    {
        CK(hipEventRecord(e0, st));
        for (int i = 0; i < 200; ++i) k_empty<<<256, 256, 0, st>>>(out);
        CK(hipEventRecord(e1, st));
        CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1));
        printf("empty kernel 256x256 back-to-back: %.2f us\n", ms * 1000 / 200);
    }
    for (int si = 0; si < 7; si += 2) {
        const size_t S = sizes[si];
        printf("== %s  %.1f MB\n", names[si], S / 1e6);
#define ONE(U, NT) run(NT ? "oneshot nt U" #U : "oneshot U" #U, S, [&](const v4i * p, size_t n) { \
            const unsigned g = (unsigned) ((n + 256 * U - 1) / (256 * U)); k_oneshot<U, NT><<<g, 256, 0, st>>>(p, n, out); });
        ONE(2, false) ONE(4, false) ONE(8, false) ONE(4, true) ONE(8, true) ONE(16, true)
#undef ONE
#define PER(U, BPC) run("persist U" #U " bpc" #BPC, S, [&](const v4i * p, size_t n) { \
            k_persist<U><<<256 * BPC, 256, 0, st>>>(p, n, out); });
        PER(4, 2) PER(8, 2) PER(4, 4) PER(8, 4) PER(8, 8)
#undef PER
    }

    const int prow[] = {6144, 4096, 28672, 187072};
    for (int R : prow) {
        const size_t S = (size_t) R * 2304;
        printf("== pattern rows=%d  %.1f MB\n", R, S / 1e6);
        run("gemv v2 pattern", S, [&](const v4i * p, size_t) { k_gemv_pattern<false><<<(R + 15) / 16, 256, 0, st>>>((const char *) p, R, out); });
        run("gemv v2 pattern nt", S, [&](const v4i * p, size_t) { k_gemv_pattern<true><<<(R + 15) / 16, 256, 0, st>>>((const char *) p, R, out); });
        run("row coalesced 1/wave", S, [&](const v4i * p, size_t) { k_row_coalesced<1><<<(R + 3) / 4, 256, 0, st>>>((const char *) p, R, out); });
        run("row coalesced 2/wave", S, [&](const v4i * p, size_t) { k_row_coalesced<2><<<(R + 7) / 8, 256, 0, st>>>((const char *) p, R, out); });
        run("row coalesced 4/wave", S, [&](const v4i * p, size_t) { k_row_coalesced<4><<<(R + 15) / 16, 256, 0, st>>>((const char *) p, R, out); });
    }
    return 0;
}
