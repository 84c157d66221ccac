// quants.cuh — ggml block formats on the device (byte layouts of
// ggml/src/ggml-common.h:170-336) and their exact dequantisation.
//
// dequant_one<T>(block, j) reproduces dequantize_row_<T> (ggml-quants.c:307-420,
// 1352-1374, 1554-1584, 1762-1790) bit-for-bit: multiplications and the final
// subtraction are written with _rn intrinsics so hipcc cannot contract them into
// an FMA that the reference's scalar C does not perform.
#pragma once

#include "common.h"
#include <type_traits>

namespace mx {

template <int T> __host__ __device__ constexpr int qk_of() {
    return (T == GGML_TYPE_Q4_K || T == GGML_TYPE_Q5_K || T == GGML_TYPE_Q6_K) ? 256 : 32;
}
template <int T> __host__ __device__ constexpr int qsize_of() {
    return T == GGML_TYPE_Q4_0 ? 18 : T == GGML_TYPE_Q4_1 ? 20 : T == GGML_TYPE_Q5_0 ? 22 : T == GGML_TYPE_Q5_1 ? 24 :
           T == GGML_TYPE_Q8_0 ? 34 : T == GGML_TYPE_Q4_K ? 144 : T == GGML_TYPE_Q5_K ? 176 : T == GGML_TYPE_Q6_K ? 210 : 0;
}

__device__ __forceinline__ uint16_t ld_u16(const char * p) { return *(const uint16_t *) p; }
__device__ __forceinline__ float ld_h(const char * p) { return h2f(ld_u16(p)); }

// get_scale_min_k4 (ggml-quants.c:703-710)
__device__ __forceinline__ void scale_min_k4(int j, const uint8_t * q, int & d, int & m) {
    if (j < 4) {
        d = q[j] & 63;
        m = q[j + 4] & 63;
    } else {
        d = (q[j + 4] & 0xF) | ((q[j - 4] >> 6) << 4);
        m = (q[j + 4] >> 4) | ((q[j - 0] >> 6) << 4);
    }
}

template <int T>
__device__ __forceinline__ float dequant_one(const char * b, int j) {
    if constexpr (T == GGML_TYPE_Q4_0) {
        const uint8_t q = (uint8_t) b[2 + (j & 15)];
        const int x = (j < 16 ? (q & 0xF) : (q >> 4)) - 8;
        return __fmul_rn((float) x, ld_h(b));
    } else if constexpr (T == GGML_TYPE_Q4_1) {
        const uint8_t q = (uint8_t) b[4 + (j & 15)];
        const int x = j < 16 ? (q & 0xF) : (q >> 4);
        return __fadd_rn(__fmul_rn((float) x, ld_h(b)), ld_h(b + 2));
    } else if constexpr (T == GGML_TYPE_Q5_0) {
        uint32_t qh;
        memcpy(&qh, b + 2, 4);
        const int jj = j & 15;
        const uint8_t q = (uint8_t) b[6 + jj];
        int x;
        if (j < 16) x = ((q & 0x0F) | (((qh >> (jj + 0)) << 4) & 0x10)) - 16;
        else        x = ((q >> 4) | ((qh >> (jj + 12)) & 0x10)) - 16;
        return __fmul_rn((float) x, ld_h(b));
    } else if constexpr (T == GGML_TYPE_Q5_1) {
        uint32_t qh;
        memcpy(&qh, b + 4, 4);
        const int jj = j & 15;
        const uint8_t q = (uint8_t) b[8 + jj];
        int x;
        if (j < 16) x = (q & 0x0F) | (((qh >> (jj + 0)) << 4) & 0x10);
        else        x = (q >> 4) | ((qh >> (jj + 12)) & 0x10);
        return __fadd_rn(__fmul_rn((float) x, ld_h(b)), ld_h(b + 2));
    } else if constexpr (T == GGML_TYPE_Q8_0) {
        return __fmul_rn((float) (int8_t) b[2 + j], ld_h(b));
    } else if constexpr (T == GGML_TYPE_Q4_K) {
        const int g = j >> 6, l = j & 63;
        const uint8_t q = (uint8_t) b[16 + 32 * g + (l & 31)];
        int sc, m;
        scale_min_k4(2 * g + (l >> 5), (const uint8_t *) b + 4, sc, m);
        const float d1 = __fmul_rn(ld_h(b), (float) sc);
        const float m1 = __fmul_rn(ld_h(b + 2), (float) m);
        const int x = l < 32 ? (q & 0xF) : (q >> 4);
        return __fsub_rn(__fmul_rn(d1, (float) x), m1);
    } else if constexpr (T == GGML_TYPE_Q5_K) {
        const int g = j >> 6, l = j & 63;
        const uint8_t q = (uint8_t) b[48 + 32 * g + (l & 31)];
        const uint8_t h = (uint8_t) b[16 + (l & 31)];
        int sc, m;
        scale_min_k4(2 * g + (l >> 5), (const uint8_t *) b + 4, sc, m);
        const float d1 = __fmul_rn(ld_h(b), (float) sc);
        const float m1 = __fmul_rn(ld_h(b + 2), (float) m);
        const uint8_t u = (uint8_t) ((l < 32 ? 1 : 2) << (2 * g));
        const int x = (l < 32 ? (q & 0xF) : (q >> 4)) + ((h & u) ? 16 : 0);
        return __fsub_rn(__fmul_rn(d1, (float) x), m1);
    } else if constexpr (T == GGML_TYPE_Q6_K) {
        const int n = j >> 7, r = j & 127, l = r & 31, qq = r >> 5;
        const uint8_t lo = (uint8_t) b[64 * n + l + ((qq & 1) ? 32 : 0)];
        const uint8_t hi = (uint8_t) b[128 + 32 * n + l];
        const int q = (((qq >> 1) ? (lo >> 4) : (lo & 0xF)) | (((hi >> (2 * qq)) & 3) << 4)) - 32;
        const int8_t sc = (int8_t) b[192 + 8 * n + (l >> 4) + 2 * qq];
        return __fmul_rn(__fmul_rn(ld_h(b + 208), (float) sc), (float) q);
    } else {
        return 0.0f;
    }
}

// quantize_row_q8_0_ref (ggml-quants.c:199-226): d = amax/127 (stored f16), q = roundf(x/d)
__device__ __forceinline__ void quantize_block_q8_0(const float * x, char * out) {
    float amax = 0.0f;
    for (int j = 0; j < 32; ++j) amax = fmaxf(amax, fabsf(x[j]));
    const float d = amax / 127.0f;
    const float id = d != 0.0f ? 1.0f / d : 0.0f;
    const uint16_t dh = f2h(d);
    memcpy(out, &dh, 2);
    for (int j = 0; j < 32; ++j) out[2 + j] = (int8_t) roundf(__fmul_rn(x[j], id));
}

// quantize_row_q4_0_ref (ggml-quants.c:36-71), one 32-element block -> block_q4_0 (18 B):
// d = (the value of largest magnitude, first one on ties) / -8 as f16,
// nibble = min(15, (int8) (x/d + 8.5)), elements 0-15 low nibbles, 16-31 high
__device__ __forceinline__ void quantize_block_q4_0(const float * x, char * out) {
    float amax = 0.0f, mx = 0.0f;
    for (int j = 0; j < 32; ++j) {
        const float v = x[j];
        if (amax < fabsf(v)) { amax = fabsf(v); mx = v; }
    }
    // d = mx / -8 exactly (a power of two); an all-zero block gives -0.0 (mx = +0), which
    // the compiler's zero handling lost here when written as a division: the sign is explicit
    const float d = __builtin_copysignf(fabsf(mx) * 0.125f, mx > 0.0f || mx == 0.0f ? -1.0f : 1.0f);
    const float id = d != 0.0f ? 1.0f / d : 0.0f;
    const uint16_t dh = f2h(d);
    memcpy(out, &dh, 2);
    for (int j = 0; j < 16; ++j) {
        const int8_t a0 = (int8_t) (__fmul_rn(x[j], id) + 8.5f), a1 = (int8_t) (__fmul_rn(x[16 + j], id) + 8.5f);
        out[2 + j] = (char) ((uint8_t) min((int) a0, 15) | ((uint8_t) min((int) a1, 15) << 4));
    }
}

}  // namespace mx
