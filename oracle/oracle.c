/*
 * oracle.c — TEST INFRASTRUCTURE (see oracle.h). A plain-C restatement of the
 * reference CPU algorithms on the MI355X backend's hot path, written from the
 * reference sources cited per function. Scalar, single-threaded, no SIMD.
 */
#include "oracle.h"

#include <math.h>
#include <string.h>
#include <stdlib.h>

/* ggml_type ids (ggml.h:389-431) */
enum { T_F32 = 0, T_F16 = 1, T_Q4_0 = 2, T_Q4_1 = 3, T_Q5_0 = 6, T_Q5_1 = 7, T_Q8_0 = 8, T_Q8_1 = 9,
       T_Q4_K = 12, T_Q5_K = 13, T_Q6_K = 14, T_Q8_K = 15, T_BF16 = 30 };

static uint32_t f2u(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static float u2f(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }

/* IEEE binary16 decode (ggml_compute_fp16_to_fp32 semantics) */
float orc_fp16_to_fp32(uint16_t h) {
    const uint32_t sign = (uint32_t) (h & 0x8000) << 16;
    uint32_t e = (h >> 10) & 0x1F, m = h & 0x3FF;
    if (e == 0) {
        if (m == 0) return u2f(sign);
        /* subnormal: value = m * 2^-24 */
        float v = (float) m * 5.9604644775390625e-8f;
        return sign ? -v : v;
    }
    if (e == 31) return u2f(sign | 0x7F800000 | (m << 13));
    return u2f(sign | ((e + 112) << 23) | (m << 13));
}

/* binary32 → binary16, round to nearest even (ggml_compute_fp32_to_fp16 semantics) */
uint16_t orc_fp32_to_fp16(float f) {
    const uint32_t u = f2u(f);
    const uint16_t sign = (uint16_t) ((u >> 16) & 0x8000);
    const uint32_t a = u & 0x7FFFFFFF;
    if (a > 0x7F800000) return sign | 0x7E00;            /* NaN */
    if (a >= 0x477FF000) return sign | 0x7C00;           /* rounds to inf */
    if (a < 0x38800000) {                                /* subnormal / zero in f16 */
        /* value / 2^-24, rounded to nearest even */
        const float v = u2f(a) * 16777216.0f;            /* exact scaling by 2^24 */
        float r = nearbyintf(v);                         /* default rounding mode: RNE */
        return sign | (uint16_t) r;
    }
    /* normal: keep 10 mantissa bits, RNE on the dropped 13 */
    uint32_t mant = a & 0x7FFFFF, exp = (a >> 23) - 112;
    uint32_t h = (exp << 10) | (mant >> 13);
    const uint32_t rem = mant & 0x1FFF;
    if (rem > 0x1000 || (rem == 0x1000 && (h & 1))) h += 1;
    return sign | (uint16_t) h;
}

#define FP16(p) orc_fp16_to_fp32(*(const uint16_t *) (p))

static int64_t blck(int type) {
    switch (type) {
        case T_Q4_0: case T_Q4_1: case T_Q5_0: case T_Q5_1: case T_Q8_0: return 32;
        case T_Q4_K: case T_Q5_K: case T_Q6_K: return 256;
        default: return 1;
    }
}
static int64_t bsize(int type) {
    switch (type) {
        case T_Q4_0: return 18; case T_Q4_1: return 20; case T_Q5_0: return 22; case T_Q5_1: return 24;
        case T_Q8_0: return 34; case T_Q4_K: return 144; case T_Q5_K: return 176; case T_Q6_K: return 210;
        case T_F32: return 4; case T_F16: return 2; case T_BF16: return 2;
        default: return 0;
    }
}

/* get_scale_min_k4 (ggml-quants.c:703-710) */
static void scale_min_k4(int j, const uint8_t * q, uint8_t * d, uint8_t * m) {
    if (j < 4) { *d = q[j] & 63; *m = q[j + 4] & 63; }
    else { *d = (q[j + 4] & 0xF) | ((q[j - 4] >> 6) << 4); *m = (q[j + 4] >> 4) | ((q[j - 0] >> 6) << 4); }
}

int orc_dequantize_row(int type, const void * vx, float * y, int64_t k) {
    const uint8_t * x = (const uint8_t *) vx;
    const int64_t nb = k / blck(type);
    switch (type) {
    case T_F32: memcpy(y, x, k * 4); return 0;
    case T_F16: for (int64_t i = 0; i < k; ++i) y[i] = FP16(x + 2 * i); return 0;
    case T_BF16: for (int64_t i = 0; i < k; ++i) { uint16_t h; memcpy(&h, x + 2 * i, 2); y[i] = u2f((uint32_t) h << 16); } return 0;
    case T_Q4_0:  /* ggml-quants.c:307-327 */
        for (int64_t i = 0; i < nb; ++i) {
            const uint8_t * b = x + 18 * i; const float d = FP16(b);
            for (int j = 0; j < 16; ++j) {
                y[32 * i + j] = ((b[2 + j] & 0x0F) - 8) * d;
                y[32 * i + j + 16] = ((b[2 + j] >> 4) - 8) * d;
            }
        }
        return 0;
    case T_Q4_1:
        for (int64_t i = 0; i < nb; ++i) {
            const uint8_t * b = x + 20 * i; const float d = FP16(b), m = FP16(b + 2);
            for (int j = 0; j < 16; ++j) {
                y[32 * i + j] = (b[4 + j] & 0x0F) * d + m;
                y[32 * i + j + 16] = (b[4 + j] >> 4) * d + m;
            }
        }
        return 0;
    case T_Q5_0:
        for (int64_t i = 0; i < nb; ++i) {
            const uint8_t * b = x + 22 * i; const float d = FP16(b); uint32_t qh; memcpy(&qh, b + 2, 4);
            for (int j = 0; j < 16; ++j) {
                const uint8_t h0 = ((qh >> (j + 0)) << 4) & 0x10, h1 = ((qh >> (j + 12))) & 0x10;
                y[32 * i + j] = (((b[6 + j] & 0x0F) | h0) - 16) * d;
                y[32 * i + j + 16] = (((b[6 + j] >> 4) | h1) - 16) * d;
            }
        }
        return 0;
    case T_Q5_1:
        for (int64_t i = 0; i < nb; ++i) {
            const uint8_t * b = x + 24 * i; const float d = FP16(b), m = FP16(b + 2); uint32_t qh; memcpy(&qh, b + 4, 4);
            for (int j = 0; j < 16; ++j) {
                const uint8_t h0 = ((qh >> (j + 0)) << 4) & 0x10, h1 = ((qh >> (j + 12))) & 0x10;
                y[32 * i + j] = ((b[8 + j] & 0x0F) | h0) * d + m;
                y[32 * i + j + 16] = ((b[8 + j] >> 4) | h1) * d + m;
            }
        }
        return 0;
    case T_Q8_0:  /* ggml-quants.c:401-416 */
        for (int64_t i = 0; i < nb; ++i) {
            const uint8_t * b = x + 34 * i; const float d = FP16(b);
            for (int j = 0; j < 32; ++j) y[32 * i + j] = ((int8_t) b[2 + j]) * d;
        }
        return 0;
    case T_Q4_K:  /* ggml-quants.c:1352-1374 */
        for (int64_t i = 0; i < nb; ++i) {
            const uint8_t * b = x + 144 * i; const float d = FP16(b), mn = FP16(b + 2);
            const uint8_t * q = b + 16; float * o = y + 256 * i; int is = 0;
            for (int j = 0; j < 256; j += 64) {
                uint8_t sc, m;
                scale_min_k4(is + 0, b + 4, &sc, &m); const float d1 = d * sc, m1 = mn * m;
                scale_min_k4(is + 1, b + 4, &sc, &m); const float d2 = d * sc, m2 = mn * m;
                for (int l = 0; l < 32; ++l) *o++ = d1 * (q[l] & 0xF) - m1;
                for (int l = 0; l < 32; ++l) *o++ = d2 * (q[l] >> 4) - m2;
                q += 32; is += 2;
            }
        }
        return 0;
    case T_Q5_K:  /* ggml-quants.c:1554-1584 */
        for (int64_t i = 0; i < nb; ++i) {
            const uint8_t * b = x + 176 * i; const float d = FP16(b), mn = FP16(b + 2);
            const uint8_t * qh = b + 16, * ql = b + 48; float * o = y + 256 * i; int is = 0;
            uint8_t u1 = 1, u2 = 2;
            for (int j = 0; j < 256; j += 64) {
                uint8_t sc, m;
                scale_min_k4(is + 0, b + 4, &sc, &m); const float d1 = d * sc, m1 = mn * m;
                scale_min_k4(is + 1, b + 4, &sc, &m); const float d2 = d * sc, m2 = mn * m;
                for (int l = 0; l < 32; ++l) *o++ = d1 * ((ql[l] & 0xF) + (qh[l] & u1 ? 16 : 0)) - m1;
                for (int l = 0; l < 32; ++l) *o++ = d2 * ((ql[l] >> 4) + (qh[l] & u2 ? 16 : 0)) - m2;
                ql += 32; is += 2; u1 <<= 2; u2 <<= 2;
            }
        }
        return 0;
    case T_Q6_K:  /* ggml-quants.c:1762-1790 */
        for (int64_t i = 0; i < nb; ++i) {
            const uint8_t * b = x + 210 * i; const float d = FP16(b + 208);
            const uint8_t * ql = b, * qh = b + 128; const int8_t * sc = (const int8_t *) (b + 192);
            float * o = y + 256 * i;
            for (int n = 0; n < 256; n += 128) {
                for (int l = 0; l < 32; ++l) {
                    const int is = l / 16;
                    const int8_t q1 = (int8_t) ((ql[l + 0] & 0xF) | (((qh[l] >> 0) & 3) << 4)) - 32;
                    const int8_t q2 = (int8_t) ((ql[l + 32] & 0xF) | (((qh[l] >> 2) & 3) << 4)) - 32;
                    const int8_t q3 = (int8_t) ((ql[l + 0] >> 4) | (((qh[l] >> 4) & 3) << 4)) - 32;
                    const int8_t q4 = (int8_t) ((ql[l + 32] >> 4) | (((qh[l] >> 6) & 3) << 4)) - 32;
                    o[l + 0] = d * sc[is + 0] * q1;
                    o[l + 32] = d * sc[is + 2] * q2;
                    o[l + 64] = d * sc[is + 4] * q3;
                    o[l + 96] = d * sc[is + 6] * q4;
                }
                o += 128; ql += 64; qh += 32; sc += 8;
            }
        }
        return 0;
    default:
        return -1;
    }
}

/* quantize_row_q8_0_ref (ggml-quants.c:199-226) */
void orc_quantize_row_q8_0(const float * x, void * vy, int64_t k) {
    uint8_t * y = (uint8_t *) vy;
    for (int64_t i = 0; i < k / 32; ++i) {
        float amax = 0.0f;
        for (int j = 0; j < 32; ++j) amax = fmaxf(amax, fabsf(x[32 * i + j]));
        const float d = amax / 127.0f, id = d ? 1.0f / d : 0.0f;
        const uint16_t dh = orc_fp32_to_fp16(d);
        memcpy(y + 34 * i, &dh, 2);
        for (int j = 0; j < 32; ++j) y[34 * i + 2 + j] = (uint8_t) (int8_t) roundf(x[32 * i + j] * id);
    }
}

/* quantize_row_q4_0_ref (ggml-quants.c:36-71): d = (the signed value of largest magnitude)
 * / -8 as f16, nibble = min(15, (int8) (x/d + 8.5)); low nibbles hold elements 0-15, high
 * nibbles 16-31 (a q4_0 V / K cache row: SET_ROWS's from_float) */
void orc_quantize_row_q4_0(const float * x, void * vy, int64_t k) {
    uint8_t * y = (uint8_t *) vy;
    for (int64_t i = 0; i < k / 32; ++i) {
        float amax = 0.0f, max = 0.0f;
        for (int j = 0; j < 32; ++j) {
            const float v = x[32 * i + j];
            if (amax < fabsf(v)) { amax = fabsf(v); max = v; }
        }
        const float d = max / -8, id = d ? 1.0f / d : 0.0f;
        const uint16_t dh = orc_fp32_to_fp16(d);
        memcpy(y + 18 * i, &dh, 2);
        for (int j = 0; j < 16; ++j) {
            const float x0 = x[32 * i + j] * id, x1 = x[32 * i + 16 + j] * id;
            const int8_t a0 = (int8_t) (x0 + 8.5f), a1 = (int8_t) (x1 + 8.5f);
            const uint8_t q0 = (uint8_t) (a0 < 15 ? a0 : 15), q1 = (uint8_t) (a1 < 15 ? a1 : 15);
            y[18 * i + 2 + j] = (uint8_t) (q0 | (q1 << 4));
        }
    }
}

/* quantize_row_q8_1_ref (ggml-quants.c:229-258): 36-byte blocks {d, s=d·Σq, qs[32]} */
void orc_quantize_row_q8_1(const float * x, void * vy, int64_t k) {
    uint8_t * y = (uint8_t *) vy;
    for (int64_t i = 0; i < k / 32; ++i) {
        float amax = 0.0f;
        for (int j = 0; j < 32; ++j) amax = fmaxf(amax, fabsf(x[32 * i + j]));
        const float d = amax / 127.0f, id = d ? 1.0f / d : 0.0f;
        int sum = 0;
        for (int j = 0; j < 32; ++j) {
            const int8_t q = (int8_t) roundf(x[32 * i + j] * id);
            y[36 * i + 4 + j] = (uint8_t) q;
            sum += q;
        }
        const uint16_t dh = orc_fp32_to_fp16(d), sh = orc_fp32_to_fp16(sum * d);
        memcpy(y + 36 * i, &dh, 2);
        memcpy(y + 36 * i + 2, &sh, 2);
    }
}

/* quantize_row_q8_K_ref (ggml-quants.c:2555-2592): block {float d; int8 qs[256]; int16 bsums[16]} = 292 B */
void orc_quantize_row_q8_K(const float * x, void * vy, int64_t k) {
    uint8_t * y = (uint8_t *) vy;
    for (int64_t i = 0; i < k / 256; ++i) {
        const float * xb = x + 256 * i;
        uint8_t * yb = y + 292 * i;
        float max = 0, amax = 0;
        for (int j = 0; j < 256; ++j) { const float ax = fabsf(xb[j]); if (ax > amax) { amax = ax; max = xb[j]; } }
        if (!amax) { memset(yb, 0, 292); continue; }
        const float iscale = -127.f / max;
        int8_t qs[256];
        for (int j = 0; j < 256; ++j) {
            const float v = iscale * xb[j];
            int q = (int) lrintf(v);   /* nearest_int: round half to even under the default mode */
            qs[j] = (int8_t) (q < 127 ? q : 127);
        }
        int16_t bsums[16];
        for (int j = 0; j < 16; ++j) { int s = 0; for (int t = 0; t < 16; ++t) s += qs[16 * j + t]; bsums[j] = (int16_t) s; }
        const float d = 1 / iscale;
        memcpy(yb, &d, 4);
        memcpy(yb + 4, qs, 256);
        memcpy(yb + 260, bsums, 32);
    }
}

/* ---- vec dots (ggml-cpu/quants.c generic paths) ---------------------------------- */
/* q4_0·q8_0 (quants.c:115-146) and q8_0·q8_0 (quants.c:305-330) */
static float dot_q4_0_q8_0(const uint8_t * x, const uint8_t * y, int64_t n) {
    float s = 0;
    for (int64_t i = 0; i < n / 32; ++i) {
        const uint8_t * a = x + 18 * i, * b = y + 34 * i;
        int si = 0;
        for (int j = 0; j < 16; ++j) {
            si += ((a[2 + j] & 0x0F) - 8) * (int8_t) b[2 + j];
            si += ((a[2 + j] >> 4) - 8) * (int8_t) b[2 + 16 + j];
        }
        s += si * (FP16(a) * FP16(b));
    }
    return s;
}
static float dot_q8_0_q8_0(const uint8_t * x, const uint8_t * y, int64_t n) {
    float s = 0;
    for (int64_t i = 0; i < n / 32; ++i) {
        const uint8_t * a = x + 34 * i, * b = y + 34 * i;
        int si = 0;
        for (int j = 0; j < 32; ++j) si += (int8_t) a[2 + j] * (int8_t) b[2 + j];
        s += si * (FP16(a) * FP16(b));
    }
    return s;
}
/* K-quants · q8_K (quants.c:550-705): Σ_sb [ d·dy·Σ_j sc_j Σ q·a  −  dmin·dy·Σ_j m_j Σa ] */
static float dot_k_q8_K(int type, const uint8_t * x, const uint8_t * y, int64_t n) {
    double s = 0;
    for (int64_t i = 0; i < n / 256; ++i) {
        const uint8_t * yb = y + 292 * i;
        float dy; memcpy(&dy, yb, 4);
        const int8_t * q8 = (const int8_t *) (yb + 4);
        int qv[256];
        if (type == T_Q6_K) {
            const uint8_t * b = x + 210 * i;
            const uint8_t * ql = b, * qh = b + 128; const int8_t * sc = (const int8_t *) (b + 192);
            int64_t sumi = 0;
            for (int half = 0; half < 2; ++half) {
                for (int l = 0; l < 32; ++l) {
                    qv[128 * half + l + 0] = ((ql[64 * half + l] & 0xF) | (((qh[32 * half + l] >> 0) & 3) << 4)) - 32;
                    qv[128 * half + l + 32] = ((ql[64 * half + l + 32] & 0xF) | (((qh[32 * half + l] >> 2) & 3) << 4)) - 32;
                    qv[128 * half + l + 64] = ((ql[64 * half + l] >> 4) | (((qh[32 * half + l] >> 4) & 3) << 4)) - 32;
                    qv[128 * half + l + 96] = ((ql[64 * half + l + 32] >> 4) | (((qh[32 * half + l] >> 6) & 3) << 4)) - 32;
                }
            }
            for (int j = 0; j < 16; ++j) {
                int si = 0;
                for (int t = 0; t < 16; ++t) si += qv[16 * j + t] * q8[16 * j + t];
                sumi += (int64_t) sc[j] * si;
            }
            s += (double) FP16(b + 208) * dy * (double) sumi;
        } else {
            const uint8_t * b = x + (type == T_Q4_K ? 144 : 176) * i;
            const uint8_t * qs = b + (type == T_Q4_K ? 16 : 48), * qh = b + 16;
            for (int g = 0; g < 4; ++g)
                for (int l = 0; l < 32; ++l) {
                    qv[64 * g + l] = qs[32 * g + l] & 0xF;
                    qv[64 * g + 32 + l] = qs[32 * g + l] >> 4;
                    if (type == T_Q5_K) {
                        qv[64 * g + l] += (qh[l] >> (2 * g)) & 1 ? 16 : 0;
                        qv[64 * g + 32 + l] += (qh[l] >> (2 * g + 1)) & 1 ? 16 : 0;
                    }
                }
            int64_t sumi = 0, summ = 0;
            for (int j = 0; j < 8; ++j) {
                uint8_t sc, m; scale_min_k4(j, b + 4, &sc, &m);
                int si = 0, sa = 0;
                for (int t = 0; t < 32; ++t) { si += qv[32 * j + t] * q8[32 * j + t]; sa += q8[32 * j + t]; }
                sumi += (int64_t) sc * si;
                summ += (int64_t) m * sa;
            }
            s += (double) FP16(b) * dy * (double) sumi - (double) FP16(b + 2) * dy * (double) summ;
        }
    }
    return (float) s;
}

int orc_mul_mat(int type, const void * w, size_t w_row, const float * x, float * y, int64_t K, int64_t M, int64_t N) {
    const uint8_t * wb = (const uint8_t *) w;
    if (type == T_Q4_0 || type == T_Q8_0) {
        uint8_t * xq = (uint8_t *) malloc((size_t) (K / 32) * 34);
        for (int64_t n = 0; n < N; ++n) {
            orc_quantize_row_q8_0(x + n * K, xq, K);
            for (int64_t m = 0; m < M; ++m)
                y[n * M + m] = type == T_Q4_0 ? dot_q4_0_q8_0(wb + m * w_row, xq, K) : dot_q8_0_q8_0(wb + m * w_row, xq, K);
        }
        free(xq);
        return 0;
    }
    if (type == T_Q4_K || type == T_Q5_K || type == T_Q6_K) {
        uint8_t * xq = (uint8_t *) malloc((size_t) (K / 256) * 292);
        for (int64_t n = 0; n < N; ++n) {
            orc_quantize_row_q8_K(x + n * K, xq, K);
            for (int64_t m = 0; m < M; ++m) y[n * M + m] = dot_k_q8_K(type, wb + m * w_row, xq, K);
        }
        free(xq);
        return 0;
    }
    return orc_mul_mat_exact(type, w, w_row, x, y, K, M, N);
}

int orc_mul_mat_exact(int type, const void * w, size_t w_row, const float * x, float * y, int64_t K, int64_t M, int64_t N) {
    const uint8_t * wb = (const uint8_t *) w;
    float * wr = (float *) malloc((size_t) K * sizeof(float));
    for (int64_t m = 0; m < M; ++m) {
        if (orc_dequantize_row(type, wb + m * w_row, wr, K) != 0) { free(wr); return -1; }
        for (int64_t n = 0; n < N; ++n) {
            double s = 0;
            for (int64_t k = 0; k < K; ++k) s += (double) wr[k] * x[n * K + k];
            y[n * M + m] = (float) s;
        }
    }
    free(wr);
    return 0;
}

void orc_rms_norm(const float * x, float * y, int64_t ne0, int64_t nrows, float eps) {
    for (int64_t r = 0; r < nrows; ++r) {
        const float * px = x + r * ne0;
        double sum = 0.0;
        for (int64_t i = 0; i < ne0; ++i) sum += (double) (px[i] * px[i]);
        const float mean = (float) (sum / ne0);
        const float scale = 1.0f / sqrtf(mean + eps);
        for (int64_t i = 0; i < ne0; ++i) y[r * ne0 + i] = px[i] * scale;
    }
}

/* ggml_rope_yarn_corr_dims (ggml.c:4257-4269) */
static float corr_dim(int n_dims, int n_ctx_orig, float n_rot, float base) {
    return n_dims * logf(n_ctx_orig / (n_rot * 2 * (float) M_PI)) / (2 * logf(base));
}

void orc_rope(const float * x, float * y, int64_t ne0, int64_t ne1, int64_t ne2, const int32_t * pos,
              int n_dims, int mode, int n_ctx_orig, float freq_base, float freq_scale, float ext_factor,
              float attn_factor, float beta_fast, float beta_slow, const float * ff) {
    const float theta_scale = powf(freq_base, -2.0f / n_dims);
    float corr[2];
    corr[0] = fmaxf(0, floorf(corr_dim(n_dims, n_ctx_orig, beta_fast, freq_base)));
    corr[1] = fminf(n_dims - 1, ceilf(corr_dim(n_dims, n_ctx_orig, beta_slow, freq_base)));
    float * cache = (float *) malloc((size_t) ne0 * sizeof(float));
    for (int64_t i2 = 0; i2 < ne2; ++i2) {
        /* ggml_rope_cache_init (ops.cpp:5548-5563) */
        float theta = (float) pos[i2];
        for (int64_t i0 = 0; i0 < ne0; i0 += 2) {
            const float f = ff ? ff[i0 / 2] : 1.0f;
            const float te = theta / f;
            float ti = freq_scale * te, th = ti, ms = attn_factor;
            if (ext_factor != 0.0f) {
                const float yv = (i0 / 2 - corr[0]) / fmaxf(0.001f, corr[1] - corr[0]);
                const float mix = (1 - fminf(1, fmaxf(0, yv))) * ext_factor;
                th = ti * (1 - mix) + te * mix;
                ms *= 1.0f + 0.1f * logf(1.0f / freq_scale);
            }
            cache[i0] = cosf(th) * ms;
            cache[i0 + 1] = sinf(th) * ms;
            theta *= theta_scale;
        }
        for (int64_t i1 = 0; i1 < ne1; ++i1) {
            const float * src = x + (i2 * ne1 + i1) * ne0;
            float * dst = y + (i2 * ne1 + i1) * ne0;
            for (int64_t i0 = 0; i0 < n_dims; i0 += 2) {
                const int64_t a = mode == 2 ? i0 / 2 : i0, b = mode == 2 ? a + n_dims / 2 : a + 1;
                const float c = cache[i0], s = cache[i0 + 1];
                const float x0 = src[a], x1 = src[b];
                dst[a] = x0 * c - x1 * s;
                dst[b] = x0 * s + x1 * c;
            }
            for (int64_t i0 = n_dims; i0 < ne0; ++i0) dst[i0] = src[i0];
        }
    }
    free(cache);
}

void orc_soft_max(const float * x, float * y, int64_t ne00, int64_t ne01, int64_t ne02,
                  const uint16_t * mask, float scale, float max_bias, const float * sinks) {
    const uint32_t n_head = (uint32_t) ne02;
    const uint32_t n_head_log2 = 1u << (uint32_t) floor(log2(n_head));
    const float m0 = powf(2.0f, -(max_bias) / n_head_log2);
    const float m1 = powf(2.0f, -(max_bias / 2.0f) / n_head_log2);
    float * wp = (float *) malloc((size_t) ne00 * sizeof(float));
    for (int64_t i02 = 0; i02 < ne02; ++i02) {
        const uint32_t h = (uint32_t) i02;
        const float slope = max_bias > 0.0f ? (h < n_head_log2 ? powf(m0, h + 1) : powf(m1, 2 * (h - n_head_log2) + 1)) : 1.0f;
        for (int64_t i01 = 0; i01 < ne01; ++i01) {
            const float * sp = x + (i02 * ne01 + i01) * ne00;
            float * dp = y + (i02 * ne01 + i01) * ne00;
            for (int64_t i = 0; i < ne00; ++i) wp[i] = sp[i] * scale + (mask ? slope * orc_fp16_to_fp32(mask[i01 * ne00 + i]) : 0.0f);
            float max = -INFINITY;
            for (int64_t i = 0; i < ne00; ++i) max = fmaxf(max, wp[i]);
            if (sinks) max = fmaxf(max, sinks[i02]);
            double sum = 0.0;
            for (int64_t i = 0; i < ne00; ++i) { const float e = expf(wp[i] - max); dp[i] = e; sum += e; }
            if (sinks) sum += expf(sinks[i02] - max);
            const float inv = (float) (1.0 / sum);
            for (int64_t i = 0; i < ne00; ++i) dp[i] *= inv;
        }
    }
    free(wp);
}

void orc_swiglu(const float * a, const float * b, float * y, int64_t n) {
    for (int64_t i = 0; i < n; ++i) y[i] = (a[i] / (1.0f + expf(-a[i]))) * b[i];
}

void orc_f32_to_f16(const float * x, uint16_t * y, int64_t n) {
    for (int64_t i = 0; i < n; ++i) y[i] = orc_fp32_to_fp16(x[i]);
}

void orc_flash_attn(const float * q, const uint16_t * k, const uint16_t * v, const uint16_t * mask,
                    float * out, int64_t D, int64_t n_q, int64_t n_kv, int64_t H, int64_t Hkv,
                    float scale, float max_bias, float softcap) {
    if (softcap != 0) scale /= softcap;
    const uint32_t n_head_log2 = 1u << (uint32_t) floor(log2((double) H));
    const float m0 = powf(2.0f, -(max_bias) / n_head_log2);
    const float m1 = powf(2.0f, -(max_bias / 2.0f) / n_head_log2);
    float * qh = (float *) malloc((size_t) D * sizeof(float));
    double * acc = (double *) malloc((size_t) D * sizeof(double));
    for (int64_t iq = 0; iq < n_q; ++iq) {
        for (int64_t h = 0; h < H; ++h) {
            const uint32_t hh = (uint32_t) h;
            const float slope = max_bias > 0.0f ? (hh < n_head_log2 ? powf(m0, hh + 1) : powf(m1, 2 * (hh - n_head_log2) + 1)) : 1.0f;
            const int64_t hk = h / (H / Hkv);
            for (int64_t d = 0; d < D; ++d) qh[d] = orc_fp16_to_fp32(orc_fp32_to_fp16(q[(h * n_q + iq) * D + d]));
            double M = -INFINITY, S = 0;
            for (int64_t d = 0; d < D; ++d) acc[d] = 0;
            for (int64_t ic = 0; ic < n_kv; ++ic) {
                const float mv = mask ? slope * orc_fp16_to_fp32(mask[iq * n_kv + ic]) : 0.0f;
                if (mv == -INFINITY) continue;
                double s = 0;
                for (int64_t d = 0; d < D; ++d) s += (double) qh[d] * orc_fp16_to_fp32(k[(hk * n_kv + ic) * D + d]);
                float sf = (float) s * scale;
                if (softcap != 0.0f) sf = softcap * tanhf(sf);
                sf += mv;
                double ms = 1, vs = 1;
                if (sf > M) { const double Mold = M; M = sf; ms = isinf(Mold) ? 0 : exp(Mold - M); for (int64_t d = 0; d < D; ++d) acc[d] *= ms; }
                else vs = exp(sf - M);
                for (int64_t d = 0; d < D; ++d) acc[d] += vs * orc_fp16_to_fp32(v[(hk * n_kv + ic) * D + d]);
                S = S * ms + vs;
            }
            const double inv = S == 0 ? 0 : 1.0 / S;
            for (int64_t d = 0; d < D; ++d) out[(iq * H + h) * D + d] = (float) (acc[d] * inv);
        }
    }
    free(qh);
    free(acc);
}

/* FLASH_ATTN_EXT with K/V of any cache type (f32, f16, bf16, q8_0, q4_0): the one_chunk
 * loop of ggml_compute_forward_flash_attn_ext_f16 (ops.cpp:8045-8260). q is converted to
 * the K type's vec_dot_type (type_traits_cpu: f16 -> f16, bf16 -> bf16, q8_0 / q4_0 ->
 * q8_0 blocks, f32 -> f32), q·k is the vec_dot of the two rows (computed here exactly on
 * the dequantised values, double accumulation), V rows are converted to f32 (v_to_float).
 * k, v: [Hkv][n_kv] rows of ggml_row_size(kv_type, D) bytes. */
static float orc_round_bf16(float f) {
    uint32_t u = f2u(f);
    if ((u & 0x7fffffff) > 0x7f800000) return u2f((u | 0x00400000u) & 0xffff0000u);
    u += 0x7fff + ((u >> 16) & 1);
    return u2f(u & 0xffff0000u);
}

int orc_flash_attn_t(const float * q, const void * k, const void * v, const uint16_t * mask,
                     float * out, int64_t D, int64_t n_q, int64_t n_kv, int64_t H, int64_t Hkv,
                     float scale, float max_bias, float softcap, int kv_type) {
    return orc_flash_attn_kv(q, k, v, mask, out, D, n_q, n_kv, H, Hkv, scale, max_bias, softcap, kv_type, kv_type);
}

/* K and V of different types (ops.cpp:8045-8260 takes q_to_vec_dot from K's type and
 * v_to_float from V's: -ctk q8_0 -ctv f16 and the like) */
int orc_flash_attn_kv(const float * q, const void * k, const void * v, const uint16_t * mask,
                      float * out, int64_t D, int64_t n_q, int64_t n_kv, int64_t H, int64_t Hkv,
                      float scale, float max_bias, float softcap, int kv_type, int v_type) {
    if (kv_type != T_F32 && kv_type != T_F16 && kv_type != T_BF16 && kv_type != T_Q8_0 && kv_type != T_Q4_0) return -1;
    if (v_type != T_F32 && v_type != T_F16 && v_type != T_BF16 && v_type != T_Q8_0 && v_type != T_Q4_0) return -1;
    if (D % blck(kv_type) || D % blck(v_type)) return -1;
    const size_t rb = (size_t) (D / blck(kv_type)) * bsize(kv_type);
    const size_t rbv = (size_t) (D / blck(v_type)) * bsize(v_type);
    if (softcap != 0) scale /= softcap;
    const uint32_t n_head_log2 = 1u << (uint32_t) floor(log2((double) H));
    const float m0 = powf(2.0f, -(max_bias) / n_head_log2);
    const float m1 = powf(2.0f, -(max_bias / 2.0f) / n_head_log2);
    float * qh = (float *) malloc((size_t) D * sizeof(float));
    float * kr = (float *) malloc((size_t) D * sizeof(float));
    float * vr = (float *) malloc((size_t) D * sizeof(float));
    uint8_t * q8 = (uint8_t *) malloc((size_t) (D / 32 + 1) * 34);
    double * acc = (double *) malloc((size_t) D * sizeof(double));
    for (int64_t iq = 0; iq < n_q; ++iq) {
        for (int64_t h = 0; h < H; ++h) {
            const uint32_t hh = (uint32_t) h;
            const float slope = max_bias > 0.0f ? (hh < n_head_log2 ? powf(m0, hh + 1) : powf(m1, 2 * (hh - n_head_log2) + 1)) : 1.0f;
            const int64_t hk = h / (H / Hkv);
            const float * qr = q + (h * n_q + iq) * D;
            if (kv_type == T_Q8_0 || kv_type == T_Q4_0) {
                orc_quantize_row_q8_0(qr, q8, D);
                orc_dequantize_row(T_Q8_0, q8, qh, D);
            } else {
                for (int64_t d = 0; d < D; ++d)
                    qh[d] = kv_type == T_F16 ? orc_fp16_to_fp32(orc_fp32_to_fp16(qr[d])) : kv_type == T_BF16 ? orc_round_bf16(qr[d]) : qr[d];
            }
            double M = -INFINITY, S = 0;
            for (int64_t d = 0; d < D; ++d) acc[d] = 0;
            for (int64_t ic = 0; ic < n_kv; ++ic) {
                const float mv = mask ? slope * orc_fp16_to_fp32(mask[iq * n_kv + ic]) : 0.0f;
                if (mv == -INFINITY) continue;
                orc_dequantize_row(kv_type, (const uint8_t *) k + (size_t) (hk * n_kv + ic) * rb, kr, D);
                double s = 0;
                for (int64_t d = 0; d < D; ++d) s += (double) qh[d] * kr[d];
                float sf = (float) s * scale;
                if (softcap != 0.0f) sf = softcap * tanhf(sf);
                sf += mv;
                double ms = 1, vs = 1;
                if (sf > M) { const double Mold = M; M = sf; ms = isinf(Mold) ? 0 : exp(Mold - M); for (int64_t d = 0; d < D; ++d) acc[d] *= ms; }
                else vs = exp(sf - M);
                orc_dequantize_row(v_type, (const uint8_t *) v + (size_t) (hk * n_kv + ic) * rbv, vr, D);
                for (int64_t d = 0; d < D; ++d) acc[d] += vs * vr[d];
                S = S * ms + vs;
            }
            const double inv = S == 0 ? 0 : 1.0 / S;
            for (int64_t d = 0; d < D; ++d) out[(iq * H + h) * D + d] = (float) (acc[d] * inv);
        }
    }
    free(qh); free(kr); free(vr); free(q8); free(acc);
    return 0;
}
