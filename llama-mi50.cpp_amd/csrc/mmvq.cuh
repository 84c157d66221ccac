// mmvq.cuh — decode GEMV (y = W·x, 1..8 activation columns) over ggml quantised
// super-blocks, the replacement for the reference's mul_mat_vec_q
// (ggml-cuda/mmvq.cu:142-356, vecdotq.cuh:461-600,631-723,775-867).
//
// MI355X design
//  * activations are quantised once per column to int8 with one f32 scale d and
//    one f32 d·Σq per 32 values (the information content of block_q8_1,
//    ggml-common.h:226-237, stored as separate SoA arrays so every load is aligned);
//  * a "unit" is the slice of one weight row a lane decodes at once (32 weights).
//    Q4_K/Q5_K units are 16-byte aligned qs chunks read with one dwordx4, the
//    super-block header is a 16-byte load shared by the 8 lanes of a super-block.
//    Q6_K (210-byte blocks, only 2-byte aligned) reads its 8-byte runs as 16-bit pairs;
//  * every lane first issues the weight loads of ALL its units (Regs[UNR]) and only
//    then computes: at decode sizes a GEMV is a few µs long, so memory-level
//    parallelism, not arithmetic, sets its time;
//  * integer dot products use v_dot4_i32_i8 (sdot4), scales are applied in f32;
//  * lanes of a row group reduce with wave64 shuffles.
#pragma once

#include "quants.cuh"
#include "backend.h"

namespace mx {

__device__ __forceinline__ uint32_t ld_u32_a2(const char * p) {  // 2-byte aligned 32-bit load
    const uint16_t * q = (const uint16_t *) p;
    return (uint32_t) q[0] | ((uint32_t) q[1] << 16);
}
__device__ __forceinline__ int4 ld_i4(const void * p) { return *(const int4 *) p; }
__device__ __forceinline__ int2 ld_i2(const void * p) { return *(const int2 *) p; }

// raw weight registers of one unit
template <int QT> struct URegs;
template <> struct URegs<GGML_TYPE_Q4_K> { int4 hd, w; };
template <> struct URegs<GGML_TYPE_Q5_K> { int4 hd, w, qh; };
template <> struct URegs<GGML_TYPE_Q6_K> { uint32_t la0, la1, lb0, lb1, qh0, qh1; uint32_t sc; uint16_t d; };
template <> struct URegs<GGML_TYPE_Q4_0> { uint32_t w[4]; uint16_t d; };
template <> struct URegs<GGML_TYPE_Q8_0> { uint32_t w[8]; uint16_t d; };

template <int QT>
__device__ __forceinline__ void unit_load(const char * __restrict__ row, int u, URegs<QT> & r) {
    if constexpr (QT == GGML_TYPE_Q4_K || QT == GGML_TYPE_Q5_K) {
        const int sb = u >> 3, c = u & 7;
        const char * b = row + (int64_t) sb * qsize_of<QT>();
        r.hd = ld_i4(b);
        r.w = ld_i4(b + (QT == GGML_TYPE_Q4_K ? 16 : 48) + 16 * c);
        if constexpr (QT == GGML_TYPE_Q5_K) r.qh = ld_i4(b + 16 + 16 * (c & 1));
    } else if constexpr (QT == GGML_TYPE_Q6_K) {
        // unit u: super-block sb, half n, 8-wide l-run t: weights 128n + 32qq + 8t + i, qq=0..3
        const int sb = u >> 3, n = (u >> 2) & 1, t = u & 3;
        const char * b = row + (int64_t) sb * 210;
        const char * qlp = b + 64 * n + 8 * t;
        r.la0 = ld_u32_a2(qlp); r.la1 = ld_u32_a2(qlp + 4);
        r.lb0 = ld_u32_a2(qlp + 32); r.lb1 = ld_u32_a2(qlp + 36);
        const char * qhp = b + 128 + 32 * n + 8 * t;
        r.qh0 = ld_u32_a2(qhp); r.qh1 = ld_u32_a2(qhp + 4);
        // scales sc[8n + t/2 + 2qq], qq = 0..3: bytes at stride 2
        const uint8_t * scp = (const uint8_t *) (b + 192 + 8 * n + (t >> 1));
        r.sc = (uint32_t) scp[0] | ((uint32_t) scp[2] << 8) | ((uint32_t) scp[4] << 16) | ((uint32_t) scp[6] << 24);
        r.d = ld_u16(b + 208);
    } else if constexpr (QT == GGML_TYPE_Q4_0) {
        const char * b = row + (int64_t) u * 18;
        r.d = ld_u16(b);
#pragma unroll
        for (int k = 0; k < 4; ++k) r.w[k] = ld_u32_a2(b + 2 + 4 * k);
    } else if constexpr (QT == GGML_TYPE_Q8_0) {
        const char * b = row + (int64_t) u * 34;
        r.d = ld_u16(b);
#pragma unroll
        for (int k = 0; k < 8; ++k) r.w[k] = ld_u32_a2(b + 2 + 4 * k);
    }
}

template <int QT, int NC>
__device__ __forceinline__ void unit_compute(const URegs<QT> & r, int u, const ActQ & a, float (&acc)[NC]) {
    if constexpr (QT == GGML_TYPE_Q4_K || QT == GGML_TYPE_Q5_K) {
        const int sb = u >> 3, c = u & 7, g = c >> 1, h = c & 1;
        const uint32_t s0 = (uint32_t) r.hd.y, s1 = (uint32_t) r.hd.z, s2 = (uint32_t) r.hd.w;
        auto byte = [&](int j) -> int {
            const uint32_t v = j < 4 ? s0 : (j < 8 ? s1 : s2);
            return (v >> (8 * (j & 3))) & 0xFF;
        };
        int sc[2], mn[2];
#pragma unroll
        for (int t = 0; t < 2; ++t) {   // get_scale_min_k4 for sub-blocks 2g, 2g+1
            const int j = 2 * g + t;
            if (j < 4) { sc[t] = byte(j) & 63; mn[t] = byte(j + 4) & 63; }
            else { sc[t] = (byte(j + 4) & 0xF) | ((byte(j - 4) >> 6) << 4); mn[t] = (byte(j + 4) >> 4) | ((byte(j) >> 6) << 4); }
        }
        const float d = h2f((uint16_t) (r.hd.x & 0xFFFF)), dmin = h2f((uint16_t) ((uint32_t) r.hd.x >> 16));
        int lo[4], hi[4];
        const int wv[4] = {r.w.x, r.w.y, r.w.z, r.w.w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            lo[k] = wv[k] & 0x0F0F0F0F;
            hi[k] = (wv[k] >> 4) & 0x0F0F0F0F;
        }
        if constexpr (QT == GGML_TYPE_Q5_K) {
            const int hv[4] = {r.qh.x, r.qh.y, r.qh.z, r.qh.w};
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                lo[k] |= ((hv[k] >> (2 * g)) & 0x01010101) << 4;
                hi[k] |= ((hv[k] >> (2 * g + 1)) & 0x01010101) << 4;
            }
        }
        const int64_t e0 = (int64_t) sb * 256 + 64 * g + 16 * h;  // first activation of the low run
        const int blk0 = (int) (e0 >> 5), blk1 = blk0 + 1;
#pragma unroll
        for (int col = 0; col < NC; ++col) {
            const int8_t * qa = a.q + col * a.kp;
            const int4 a0 = ld_i4(qa + e0);
            const int4 a1 = ld_i4(qa + e0 + 32);
            int d0 = 0, d1 = 0;
            d0 = dot4_i8(lo[0], a0.x, d0); d0 = dot4_i8(lo[1], a0.y, d0);
            d0 = dot4_i8(lo[2], a0.z, d0); d0 = dot4_i8(lo[3], a0.w, d0);
            d1 = dot4_i8(hi[0], a1.x, d1); d1 = dot4_i8(hi[1], a1.y, d1);
            d1 = dot4_i8(hi[2], a1.z, d1); d1 = dot4_i8(hi[3], a1.w, d1);
            const float * ad = a.d + col * (a.kp / 32);
            float v = d * ((float) sc[0] * ad[blk0] * (float) d0 + (float) sc[1] * ad[blk1] * (float) d1);
            if (h == 0) {   // the min term once per 32-block
                const float * as = a.s + col * (a.kp / 32);
                v -= dmin * ((float) mn[0] * as[blk0] + (float) mn[1] * as[blk1]);
            }
            acc[col] += v;
        }
    } else if constexpr (QT == GGML_TYPE_Q6_K) {
        const int sb = u >> 3, n = (u >> 2) & 1, t = u & 3;
        int q[4][2];
        q[0][0] = (r.la0 & 0x0F0F0F0F) | (((r.qh0 >> 0) & 0x03030303) << 4);
        q[0][1] = (r.la1 & 0x0F0F0F0F) | (((r.qh1 >> 0) & 0x03030303) << 4);
        q[1][0] = (r.lb0 & 0x0F0F0F0F) | (((r.qh0 >> 2) & 0x03030303) << 4);
        q[1][1] = (r.lb1 & 0x0F0F0F0F) | (((r.qh1 >> 2) & 0x03030303) << 4);
        q[2][0] = ((r.la0 >> 4) & 0x0F0F0F0F) | (((r.qh0 >> 4) & 0x03030303) << 4);
        q[2][1] = ((r.la1 >> 4) & 0x0F0F0F0F) | (((r.qh1 >> 4) & 0x03030303) << 4);
        q[3][0] = ((r.lb0 >> 4) & 0x0F0F0F0F) | (((r.qh0 >> 6) & 0x03030303) << 4);
        q[3][1] = ((r.lb1 >> 4) & 0x0F0F0F0F) | (((r.qh1 >> 6) & 0x03030303) << 4);
        const float d = h2f(r.d);
        const int64_t e0 = (int64_t) sb * 256 + 128 * n + 8 * t;
#pragma unroll
        for (int col = 0; col < NC; ++col) {
            const int8_t * qa = a.q + col * a.kp;
            const float * ad = a.d + col * (a.kp / 32);
            float v = 0.f;
#pragma unroll
            for (int qq = 0; qq < 4; ++qq) {
                const int2 av = ld_i2(qa + e0 + 32 * qq);
                int dt = 0, sm = 0;
                dt = dot4_i8(q[qq][0], av.x, dt); dt = dot4_i8(q[qq][1], av.y, dt);
                sm = dot4_i8(0x20202020, av.x, sm); sm = dot4_i8(0x20202020, av.y, sm);
                const int scv = (int) (int8_t) ((r.sc >> (8 * qq)) & 0xFF);
                v += (float) scv * ad[(e0 >> 5) + qq] * (float) (dt - sm);
            }
            acc[col] += d * v;
        }
    } else if constexpr (QT == GGML_TYPE_Q4_0) {
        const float d = h2f(r.d);
#pragma unroll
        for (int col = 0; col < NC; ++col) {
            const int8_t * qa = a.q + col * a.kp + (int64_t) u * 32;
            const int4 a0 = ld_i4(qa), a1 = ld_i4(qa + 16);
            int dt = 0;
            dt = dot4_i8(r.w[0] & 0x0F0F0F0F, a0.x, dt); dt = dot4_i8(r.w[1] & 0x0F0F0F0F, a0.y, dt);
            dt = dot4_i8(r.w[2] & 0x0F0F0F0F, a0.z, dt); dt = dot4_i8(r.w[3] & 0x0F0F0F0F, a0.w, dt);
            dt = dot4_i8((r.w[0] >> 4) & 0x0F0F0F0F, a1.x, dt); dt = dot4_i8((r.w[1] >> 4) & 0x0F0F0F0F, a1.y, dt);
            dt = dot4_i8((r.w[2] >> 4) & 0x0F0F0F0F, a1.z, dt); dt = dot4_i8((r.w[3] >> 4) & 0x0F0F0F0F, a1.w, dt);
            const float ad = a.d[col * (a.kp / 32) + u], as = a.s[col * (a.kp / 32) + u];
            acc[col] += d * (ad * (float) dt - 8.0f * as);
        }
    } else if constexpr (QT == GGML_TYPE_Q8_0) {
        const float d = h2f(r.d);
#pragma unroll
        for (int col = 0; col < NC; ++col) {
            const int8_t * qa = a.q + col * a.kp + (int64_t) u * 32;
            const int4 a0 = ld_i4(qa), a1 = ld_i4(qa + 16);
            int dt = 0;
            dt = dot4_i8(r.w[0], a0.x, dt); dt = dot4_i8(r.w[1], a0.y, dt); dt = dot4_i8(r.w[2], a0.z, dt); dt = dot4_i8(r.w[3], a0.w, dt);
            dt = dot4_i8(r.w[4], a1.x, dt); dt = dot4_i8(r.w[5], a1.y, dt); dt = dot4_i8(r.w[6], a1.z, dt); dt = dot4_i8(r.w[7], a1.w, dt);
            acc[col] += d * a.d[col * (a.kp / 32) + u] * (float) dt;
        }
    }
}

// back-compat single-shot form (MoE kernel)
template <int QT, int NC>
__device__ __forceinline__ void unit_dot(const char * __restrict__ row, int u, const ActQ & a, float (&acc)[NC]) {
    URegs<QT> r;
    unit_load<QT>(row, u, r);
    unit_compute<QT, NC>(r, u, a, acc);
}

template <int QT> __host__ __device__ constexpr bool mmvq_has_unit() {
    return QT == GGML_TYPE_Q4_K || QT == GGML_TYPE_Q5_K || QT == GGML_TYPE_Q6_K || QT == GGML_TYPE_Q4_0 || QT == GGML_TYPE_Q8_0;
}

}  // namespace mx
