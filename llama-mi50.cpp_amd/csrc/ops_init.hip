// ops_init.hip — synthetic weight generation on the device (bench / tests only).
// Fills ggml super-blocks with hashed random quants and scale fields chosen so the
// dequantised weights have roughly zero mean and std ≈ 0.02, i.e. the numerical
// regime of a real checkpoint (there are no real weights offline).
#include "backend.h"

namespace mx {

__device__ __forceinline__ uint32_t hash32(uint64_t x) {
    x ^= x >> 33; x *= 0xff51afd7ed558ccdULL; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ULL; x ^= x >> 33;
    return (uint32_t) x;
}
__device__ __forceinline__ float u01(uint64_t s) { return (hash32(s) >> 8) * (1.0f / 16777216.0f); }

// one thread per 16-bit word of the tensor; scale fields are rewritten by block
__global__ void k_fill_words(uint16_t * p, int64_t nwords, uint64_t seed) {
    for (int64_t i = blockIdx.x * (int64_t) blockDim.x + threadIdx.x; i < nwords; i += (int64_t) gridDim.x * blockDim.x)
        p[i] = (uint16_t) hash32(seed * 0x9E3779B97F4A7C15ULL + (uint64_t) i);
}

template <int T>
__global__ void k_fix_blocks(char * base, int64_t nrows, int64_t nblk_row, size_t row_bytes, uint64_t seed) {
    const int64_t n = nrows * nblk_row;
    for (int64_t i = blockIdx.x * (int64_t) blockDim.x + threadIdx.x; i < n; i += (int64_t) gridDim.x * blockDim.x) {
        const int64_t r = i / nblk_row, b = i % nblk_row;
        const float u = 0.75f + 0.5f * u01(seed + 7 * (uint64_t) i);
        if constexpr (T == GGML_TYPE_Q4_K) {
            char * blk = base + r * row_bytes + b * 144;
            const float d = 9.3e-5f * u;
            *(uint16_t *) blk = f2h(d);
            *(uint16_t *) (blk + 2) = f2h(d * 7.5f);
        } else if constexpr (T == GGML_TYPE_Q5_K) {
            char * blk = base + r * row_bytes + b * 176;
            const float d = 4.6e-5f * u;
            *(uint16_t *) blk = f2h(d);
            *(uint16_t *) (blk + 2) = f2h(d * 15.5f);
        } else if constexpr (T == GGML_TYPE_Q6_K) {
            char * blk = base + r * row_bytes + b * 210;
            for (int j = 0; j < 16; ++j) blk[192 + j] = (char) ((int) (blk[192 + j] & 0x1F) - 16);
            *(uint16_t *) (blk + 208) = f2h(1.2e-4f * u);
        } else if constexpr (T == GGML_TYPE_Q4_0) {
            char * blk = base + r * row_bytes + b * 18;
            *(uint16_t *) blk = f2h(4.3e-3f * u);
        } else if constexpr (T == GGML_TYPE_Q8_0) {
            char * blk = base + r * row_bytes + b * 34;
            *(uint16_t *) blk = f2h(2.7e-4f * u);
        } else if constexpr (T == GGML_TYPE_F16) {
            uint16_t * e = (uint16_t *) (base + r * row_bytes) + b;
            *e = f2h(0.02f * 1.7320508f * (2.0f * u01(seed + 13 * (uint64_t) i) - 1.0f));
        } else if constexpr (T == GGML_TYPE_F32) {
            float * e = (float *) (base + r * row_bytes) + b;
            *e = 0.02f * 1.7320508f * (2.0f * u01(seed + 13 * (uint64_t) i) - 1.0f);
        }
    }
}

__global__ void k_fill_const(float * p, int64_t n, float v) {
    for (int64_t i = blockIdx.x * (int64_t) blockDim.x + threadIdx.x; i < n; i += (int64_t) gridDim.x * blockDim.x) p[i] = v;
}

void fill_random_tensor(const ggml_tensor * t, uint64_t seed, hipStream_t st) {
    const size_t bytes = mx_nbytes(t);
    const int64_t nrows = mx_nrows(t);
    const mx_type_info ti = mx_type(t->type);
    const int64_t nblk = t->ne[0] / ti.blck;
    const unsigned grid = 4096;
    if (t->type != GGML_TYPE_F32 && t->type != GGML_TYPE_F16)
        k_fill_words<<<grid, 256, 0, st>>>((uint16_t *) t->data, (int64_t) (bytes / 2), seed);
    switch (t->type) {
        case GGML_TYPE_Q4_K: k_fix_blocks<GGML_TYPE_Q4_K><<<grid, 256, 0, st>>>((char *) t->data, nrows, nblk, t->nb[1], seed); break;
        case GGML_TYPE_Q5_K: k_fix_blocks<GGML_TYPE_Q5_K><<<grid, 256, 0, st>>>((char *) t->data, nrows, nblk, t->nb[1], seed); break;
        case GGML_TYPE_Q6_K: k_fix_blocks<GGML_TYPE_Q6_K><<<grid, 256, 0, st>>>((char *) t->data, nrows, nblk, t->nb[1], seed); break;
        case GGML_TYPE_Q4_0: k_fix_blocks<GGML_TYPE_Q4_0><<<grid, 256, 0, st>>>((char *) t->data, nrows, nblk, t->nb[1], seed); break;
        case GGML_TYPE_Q8_0: k_fix_blocks<GGML_TYPE_Q8_0><<<grid, 256, 0, st>>>((char *) t->data, nrows, nblk, t->nb[1], seed); break;
        case GGML_TYPE_F16:  k_fix_blocks<GGML_TYPE_F16><<<grid, 256, 0, st>>>((char *) t->data, nrows, nblk, t->nb[1], seed); break;
        case GGML_TYPE_F32:  k_fix_blocks<GGML_TYPE_F32><<<grid, 256, 0, st>>>((char *) t->data, nrows, nblk, t->nb[1], seed); break;
        default: MX_ABORT("fill_random: type %d", (int) t->type);
    }
}

void fill_const_f32(const ggml_tensor * t, float v, hipStream_t st) {
    k_fill_const<<<1024, 256, 0, st>>>((float *) t->data, mx_nelements(t), v);
}

void fill_const_f32_ptr(float * p, int64_t n, float v, hipStream_t st) {
    k_fill_const<<<1024, 256, 0, st>>>(p, n, v);
}

}  // namespace mx
