// ops_fattn.hip — FLASH_ATTN_EXT on gfx950.
//
// Semantics: ggml_compute_forward_flash_attn_ext_f16_one_chunk
// (ggml-cpu/ops.cpp:8045-8260): Q is rounded to the K vec-dot type (f16),
// s = (q·k)·scale [softcap·tanh(s)] + slope·mask, keys whose mask is −inf are
// skipped, online softmax over keys, sinks enter once, empty rows give 0.
// Reference GPU: fattn.cu:280-482 (vec/tile kernels + split-KV combine).
//
// MI355X design: one block = (query row, KV head, KV split). The G = H/Hkv query
// heads that share a KV head are processed together, so each K/V byte is read
// once per query row (GQA 32/8 → 4× less KV traffic than per-head kernels).
// Per 256-key tile: lane-per-key scores for the G heads (q in LDS, broadcast
// reads), block softmax update, then threads over (head, dim) accumulate P·V with
// coalesced V row reads. Splits are merged by a combine kernel.
#include "backend.h"

namespace mx {

constexpr int FA_TILE = 256;
constexpr int FA_MAXG = 8;

struct FaArgs {
    const char * q; size_t q1, q2, q3;     // q strides (row, head, seq)
    const char * k; size_t k1, k2, k3;
    const char * v; size_t v1, v2, v3;
    const char * mask; size_t m1, m2, m3; int64_t mne2, mne3;
    float * opart; float * mpart; float * lpart;
    int64_t n_q, n_kv, H, Hkv, ns, nsplit, chunk;
    float scale, softcap, max_bias, m0, m1f;
    uint32_t n_head_log2;
    int k_aligned;                          // K rows 16-byte aligned → vector loads
};

template <typename T> __device__ __forceinline__ float ldkv(const T * p);
template <> __device__ __forceinline__ float ldkv<uint16_t>(const uint16_t * p) { return h2f(*p); }
template <> __device__ __forceinline__ float ldkv<float>(const float * p) { return *p; }

template <typename TK, typename TV, int D>
__global__ __launch_bounds__(256) void k_fattn(FaArgs p) {
    __shared__ float qs[FA_MAXG][D];
    __shared__ float sc[FA_MAXG][FA_TILE];
    __shared__ float red[FA_MAXG][4];
    __shared__ float mrun[FA_MAXG], lrun[FA_MAXG], alpha[FA_MAXG];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int64_t bx = blockIdx.x;
    const int64_t hk = bx % p.Hkv;
    const int64_t iq1 = (bx / p.Hkv) % p.n_q;
    const int64_t iq3 = bx / (p.Hkv * p.n_q);
    const int64_t split = blockIdx.y;
    const int G = (int) (p.H / p.Hkv);
    const int64_t kbeg = split * p.chunk, kend = min(p.n_kv, kbeg + p.chunk);

    // q rows of the G heads, rounded to f16 like the CPU vec-dot conversion
    for (int i = tid; i < G * D; i += blockDim.x) {
        const int g = i / D, d = i % D;
        const int64_t h = hk * G + g;
        const float x = *(const float *) (p.q + iq1 * p.q1 + h * p.q2 + iq3 * p.q3 + d * 4);
        qs[g][d] = (float) (_Float16) x;
    }
    if (tid < G) { mrun[tid] = -INFINITY; lrun[tid] = 0.f; }
    float slope[FA_MAXG];
#pragma unroll
    for (int g = 0; g < FA_MAXG; ++g) {
        const uint32_t h = (uint32_t) (hk * G + g);
        slope[g] = p.max_bias > 0.0f ? (h < p.n_head_log2 ? powf(p.m0, h + 1) : powf(p.m1f, 2 * (h - p.n_head_log2) + 1)) : 1.0f;
    }
    // output accumulators: thread owns (g, d) pairs o = tid + 256*j
    constexpr int NO = (FA_MAXG * D + 255) / 256;
    float oacc[NO];
#pragma unroll
    for (int j = 0; j < NO; ++j) oacc[j] = 0.f;
    __syncthreads();

    const char * kb = p.k + (hk) * p.k2 + (iq3 % p.ns) * p.k3;
    const char * vb = p.v + (hk) * p.v2 + (iq3 % p.ns) * p.v3;
    const char * mrow = p.mask ? p.mask + iq1 * p.m1 + ((hk * G) % p.mne2) * p.m2 + (iq3 % p.mne3) * p.m3 : nullptr;
    const bool mask_per_head = p.mask && p.mne2 > 1;

    for (int64_t t0 = kbeg; t0 < kend; t0 += FA_TILE) {
        // ---- scores: lane per key
        {
            const int64_t key = t0 + tid;
            float s[FA_MAXG];
#pragma unroll
            for (int g = 0; g < FA_MAXG; ++g) s[g] = -INFINITY;
            if (key < kend) {
                float acc[FA_MAXG];
#pragma unroll
                for (int g = 0; g < FA_MAXG; ++g) acc[g] = 0.f;
                const TK * kr = (const TK *) (kb + key * p.k1);
                for (int d = 0; d < D; d += 8) {
                    float kv[8];
                    if (sizeof(TK) == 2 && p.k_aligned) {
                        const uint4 raw = *(const uint4 *) (kr + d);
                        const uint16_t * hh = (const uint16_t *) &raw;
#pragma unroll
                        for (int i = 0; i < 8; ++i) kv[i] = h2f(hh[i]);
                    } else {
#pragma unroll
                        for (int i = 0; i < 8; ++i) kv[i] = ldkv<TK>(kr + d + i);
                    }
#pragma unroll
                    for (int g = 0; g < FA_MAXG; ++g) {
                        if (g < G) {
#pragma unroll
                            for (int i = 0; i < 8; ++i) acc[g] += qs[g][d + i] * kv[i];
                        }
                    }
                }
#pragma unroll
                for (int g = 0; g < FA_MAXG; ++g) {
                    if (g >= G) continue;
                    float mv = 0.f;
                    if (mrow) {
                        const char * mr = mask_per_head ? p.mask + iq1 * p.m1 + ((hk * G + g) % p.mne2) * p.m2 + (iq3 % p.mne3) * p.m3 : mrow;
                        mv = slope[g] * h2f(((const uint16_t *) mr)[key]);
                    }
                    if (mv == -INFINITY) continue;
                    float x = acc[g] * p.scale;
                    if (p.softcap != 0.0f) x = p.softcap * tanhf(x);
                    s[g] = x + mv;
                }
            }
#pragma unroll
            for (int g = 0; g < FA_MAXG; ++g) if (g < G) sc[g][tid] = s[g];
        }
        __syncthreads();
        // ---- softmax update per head: wave w handles heads w, w+4
        for (int g = wave; g < G; g += 4) {
            float mx = -INFINITY;
            for (int i = lane; i < FA_TILE; i += 64) mx = fmaxf(mx, sc[g][i]);
            mx = wave_max(mx);
            const float mold = mrun[g];
            const float mnew = fmaxf(mold, mx);
            float sum = 0.f;
            for (int i = lane; i < FA_TILE; i += 64) {
                const float e = mnew == -INFINITY ? 0.f : expf(sc[g][i] - mnew);
                sc[g][i] = e;
                sum += e;
            }
            sum = wave_sum(sum);
            if (lane == 0) {
                const float a = mold == -INFINITY ? 0.f : expf(mold - mnew);
                alpha[g] = a;
                lrun[g] = lrun[g] * a + sum;
                mrun[g] = mnew;
            }
        }
        __syncthreads();
        // ---- P·V: thread owns outputs o = tid + 256*j → (g, d)
        const int64_t nk = min((int64_t) FA_TILE, kend - t0);
#pragma unroll
        for (int j = 0; j < NO; ++j) {
            const int o = tid + 256 * j;
            const int g = o / D, d = o % D;
            if (g < G) {
                float a = oacc[j] * alpha[g];
                const TV * vp = (const TV *) (vb + t0 * p.v1) + d;
                for (int64_t i = 0; i < nk; ++i) {
                    const float pw = sc[g][i];
                    a += pw * ldkv<TV>((const TV *) ((const char *) vp + i * p.v1));
                }
                oacc[j] = a;
            }
        }
        __syncthreads();
    }
    // ---- write partials
    const int64_t row = (iq3 * p.n_q + iq1) * p.H;   // (seq, query) major, head minor
#pragma unroll
    for (int j = 0; j < NO; ++j) {
        const int o = tid + 256 * j;
        const int g = o / D, d = o % D;
        if (g < G) p.opart[((split * p.ns * p.n_q * p.H) + row + hk * G + g) * D + d] = oacc[j];
    }
    if (tid < G) {
        p.mpart[split * p.ns * p.n_q * p.H + row + hk * G + tid] = mrun[tid];
        p.lpart[split * p.ns * p.n_q * p.H + row + hk * G + tid] = lrun[tid];
    }
}

template <int D>
__global__ void k_fattn_combine(const float * __restrict__ op, const float * __restrict__ mp, const float * __restrict__ lp,
                                const float * __restrict__ sinks, char * __restrict__ dst, size_t nb1, size_t nb2, size_t nb3,
                                int64_t nrows, int64_t nsplit, int64_t H, int64_t n_q) {
    const int64_t r = blockIdx.x;          // (iq3, iq1, h)
    const int64_t h = r % H, iq1 = (r / H) % n_q, iq3 = r / (H * n_q);
    float m = -INFINITY;
    for (int64_t s = 0; s < nsplit; ++s) m = fmaxf(m, mp[s * nrows + r]);
    float sk = 0.f;
    const bool has_sink = sinks != nullptr;
    if (has_sink) { sk = sinks[h]; m = fmaxf(m, sk); }
    float l = 0.f;
    for (int64_t s = 0; s < nsplit; ++s) {
        const float ms = mp[s * nrows + r];
        if (ms != -INFINITY) l += lp[s * nrows + r] * expf(ms - m);
    }
    if (has_sink) l += expf(sk - m);
    const float inv = l == 0.f ? 0.f : 1.0f / l;
    float * out = (float *) (dst + h * nb1 + iq1 * nb2 + iq3 * nb3);
    for (int d = threadIdx.x; d < D; d += blockDim.x) {
        float o = 0.f;
        for (int64_t s = 0; s < nsplit; ++s) {
            const float ms = mp[s * nrows + r];
            if (ms != -INFINITY) o += op[(s * nrows + r) * D + d] * expf(ms - m);
        }
        out[d] = o * inv;
    }
}

static int64_t fa_chunk(const ggml_tensor * dst, int64_t * nsplit_out) {
    const ggml_tensor * q = dst->src[0];
    const ggml_tensor * k = dst->src[1];
    const int64_t n_kv = k->ne[1];
    const int64_t blocks = q->ne[1] * k->ne[2] * q->ne[3];
    // enough blocks to cover the chip: split KV when there are few query rows
    int64_t nsplit = std::max<int64_t>(1, std::min<int64_t>(mx_ceil_div(n_kv, FA_TILE), mx_ceil_div(512, blocks)));
    int64_t chunk = mx_ceil_div(mx_ceil_div(n_kv, nsplit), FA_TILE) * FA_TILE;
    nsplit = mx_ceil_div(n_kv, chunk);
    *nsplit_out = nsplit;
    return chunk;
}

size_t flash_attn_scratch(const ggml_tensor * dst) {
    const ggml_tensor * q = dst->src[0];
    const ggml_tensor * v = dst->src[2];
    int64_t nsplit;
    fa_chunk(dst, &nsplit);
    const int64_t rows = q->ne[1] * q->ne[2] * q->ne[3];
    return nsplit * rows * (v->ne[0] + 2) * sizeof(float) + 4 * 256;
}

bool flash_attn_supported(const ggml_tensor * dst) {
    const ggml_tensor * q = dst->src[0];
    const ggml_tensor * k = dst->src[1];
    const ggml_tensor * v = dst->src[2];
    const ggml_tensor * m = dst->src[3];
    if (q->type != GGML_TYPE_F32 || dst->type != GGML_TYPE_F32) return false;
    if (!((k->type == GGML_TYPE_F16 && v->type == GGML_TYPE_F16) || (k->type == GGML_TYPE_F32 && v->type == GGML_TYPE_F32))) return false;
    if (k->ne[0] != v->ne[0]) return false;
    const int64_t D = k->ne[0];
    if (D != 32 && D != 40 && D != 48 && D != 64 && D != 80 && D != 96 && D != 112 && D != 128 && D != 256) return false;
    if (q->ne[2] % k->ne[2] != 0 || q->ne[2] / k->ne[2] > FA_MAXG) return false;
    if (k->ne[2] != v->ne[2]) return false;
    if (m && m->type != GGML_TYPE_F16) return false;
    if (q->nb[0] != 4 || k->nb[0] != (size_t) mx_type(k->type).size || v->nb[0] != (size_t) mx_type(v->type).size) return false;
    if (q->ne[3] != k->ne[3] && k->ne[3] != 1) return false;
    if (dst->src[4] && dst->src[4]->type != GGML_TYPE_F32) return false;
    return true;
}

template <typename TK, typename TV>
static void fa_launch(OpCtx & c, int D, dim3 grid, const FaArgs & a) {
    switch (D) {
        case 32:  k_fattn<TK, TV, 32><<<grid, 256, 0, c.st>>>(a); break;
        case 40:  k_fattn<TK, TV, 40><<<grid, 256, 0, c.st>>>(a); break;
        case 48:  k_fattn<TK, TV, 48><<<grid, 256, 0, c.st>>>(a); break;
        case 64:  k_fattn<TK, TV, 64><<<grid, 256, 0, c.st>>>(a); break;
        case 80:  k_fattn<TK, TV, 80><<<grid, 256, 0, c.st>>>(a); break;
        case 96:  k_fattn<TK, TV, 96><<<grid, 256, 0, c.st>>>(a); break;
        case 112: k_fattn<TK, TV, 112><<<grid, 256, 0, c.st>>>(a); break;
        case 128: k_fattn<TK, TV, 128><<<grid, 256, 0, c.st>>>(a); break;
        case 256: k_fattn<TK, TV, 256><<<grid, 256, 0, c.st>>>(a); break;
        default: MX_ABORT("fattn D=%d", D);
    }
}

void op_flash_attn_ext(OpCtx & c, ggml_tensor * dst) {
    const ggml_tensor * q = dst->src[0];
    const ggml_tensor * k = dst->src[1];
    const ggml_tensor * v = dst->src[2];
    const ggml_tensor * m = dst->src[3];
    const ggml_tensor * sk = dst->src[4];
    FaArgs a{};
    a.q = (const char *) q->data; a.q1 = q->nb[1]; a.q2 = q->nb[2]; a.q3 = q->nb[3];
    a.k = (const char *) k->data; a.k1 = k->nb[1]; a.k2 = k->nb[2]; a.k3 = k->nb[3];
    a.v = (const char *) v->data; a.v1 = v->nb[1]; a.v2 = v->nb[2]; a.v3 = v->nb[3];
    if (m) { a.mask = (const char *) m->data; a.m1 = m->nb[1]; a.m2 = m->nb[2]; a.m3 = m->nb[3]; a.mne2 = m->ne[2]; a.mne3 = m->ne[3]; }
    a.n_q = q->ne[1]; a.n_kv = k->ne[1]; a.H = q->ne[2]; a.Hkv = k->ne[2]; a.ns = k->ne[3];
    a.scale = mx_op_param<float>(dst, 0);
    a.max_bias = mx_op_param<float>(dst, 1);
    a.softcap = mx_op_param<float>(dst, 2);
    if (a.softcap != 0.0f) a.scale /= a.softcap;
    const uint32_t n_head = (uint32_t) q->ne[2];
    a.n_head_log2 = 1u << (uint32_t) floor(log2((double) n_head));
    a.m0 = powf(2.0f, -(a.max_bias) / a.n_head_log2);
    a.m1f = powf(2.0f, -(a.max_bias / 2.0f) / a.n_head_log2);
    int64_t nsplit;
    a.chunk = fa_chunk(dst, &nsplit);
    a.nsplit = nsplit;
    const int64_t rows = q->ne[1] * q->ne[2] * q->ne[3];
    const int D = (int) v->ne[0];
    a.opart = (float *) c.scratch->take(nsplit * rows * D * sizeof(float));
    a.mpart = (float *) c.scratch->take(nsplit * rows * sizeof(float));
    a.lpart = (float *) c.scratch->take(nsplit * rows * sizeof(float));
    // fold the sequence dim of q into the grid; K/V streams broadcast when ns == 1
    a.ns = k->ne[3];
    dim3 grid((unsigned) (q->ne[1] * k->ne[2] * q->ne[3]), (unsigned) nsplit);
    // FaArgs::ns is used both as kv-stream count (k3 index = iq3 % ns) and in partial indexing below
    FaArgs b = a;
    b.ns = q->ne[3];
    // kernel indexes K/V by (iq3 % ns): pass kv stream count through k3 stride when ns==1
    if (k->ne[3] == 1) { b.k3 = 0; b.v3 = 0; }
    b.k_aligned = ((uintptr_t) k->data % 16 == 0) && k->nb[1] % 16 == 0 && k->nb[2] % 16 == 0 && k->nb[3] % 16 == 0;
    if (k->type == GGML_TYPE_F16) fa_launch<uint16_t, uint16_t>(c, D, grid, b);
    else fa_launch<float, float>(c, D, grid, b);
    const float * psk = sk ? (const float *) sk->data : nullptr;
    switch (D) {
#define CMB(DD) case DD: k_fattn_combine<DD><<<(unsigned) rows, 64, 0, c.st>>>(a.opart, a.mpart, a.lpart, psk, (char *) dst->data, \
                                                       dst->nb[1], dst->nb[2], dst->nb[3], rows, nsplit, q->ne[2], q->ne[1]); break;
        CMB(32) CMB(40) CMB(48) CMB(64) CMB(80) CMB(96) CMB(112) CMB(128) CMB(256)
#undef CMB
    }
}

}  // namespace mx
