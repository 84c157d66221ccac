// ops_mmvq.hip — decode path of MUL_MAT (≤ 8 activation columns): activation
// quantisation + quantised GEMV, plus the fused gate/up GLU variant.
// Reference dispatch: ggml_cuda_mul_mat (ggml-cuda.cu:2183-2266) routes src1->ne[1]
// <= MMVQ_MAX_BATCH_SIZE (8, mmvq.cuh:3) to mul_mat_vec_q; fused GLU at
// ggml-cuda.cu:2145-2181 / mmvq.cu:195-351.
#include "backend.h"
#include "mmvq.cuh"
#include "mm.h"
#include "gemv.h"

namespace mx {

void fill_const_f32_ptr(float * p, int64_t n, float v, hipStream_t st);

// ---------------------------------------------------------------------------
// activation quantisation: column c (flattened i11,i12,i13) → int8 + per-32 d, d·Σq
// (quantize_q8_1, ggml-cuda/quantize.cu:5-48: d = amax/127, q = round(x/d))
// ---------------------------------------------------------------------------
__global__ void k_quantize_act(const char * __restrict__ x, int64_t K, int64_t ne11, int64_t ne12,
                               size_t nb11, size_t nb12, size_t nb13, int64_t kp,
                               int8_t * __restrict__ q, float * __restrict__ d, float * __restrict__ s) {
    const int64_t col = blockIdx.y;
    const int64_t i11 = col % ne11, i12 = (col / ne11) % ne12, i13 = col / (ne11 * ne12);
    const float * px = (const float *) (x + i11 * nb11 + i12 * nb12 + i13 * nb13);
    const int64_t blk = blockIdx.x * (int64_t) blockDim.x + threadIdx.x;
    if (blk * 32 >= kp) return;
    float v[32];
    const int64_t e0 = blk * 32;
    if (e0 + 32 <= K && ((uintptr_t) (px + e0) % 16) == 0) {
#pragma unroll
        for (int j = 0; j < 32; j += 4) {
            const float4 f = *(const float4 *) (px + e0 + j);
            v[j] = f.x; v[j + 1] = f.y; v[j + 2] = f.z; v[j + 3] = f.w;
        }
    } else {
#pragma unroll
        for (int j = 0; j < 32; ++j) v[j] = e0 + j < K ? px[e0 + j] : 0.0f;
    }
    float amax = 0.f;
#pragma unroll
    for (int j = 0; j < 32; ++j) amax = fmaxf(amax, fabsf(v[j]));
    const Q8Scale qsc = q8_scale(amax);
    const float dd = qsc.d, id = qsc.id;
    int sum = 0;
    int packed[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        int w = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int qi = q8_round(v[4 * j + k], id);
            sum += qi;
            w |= (qi & 0xFF) << (8 * k);
        }
        packed[j] = w;
    }
    int4 * out = (int4 *) (q + col * kp + e0);
    out[0] = make_int4(packed[0], packed[1], packed[2], packed[3]);
    out[1] = make_int4(packed[4], packed[5], packed[6], packed[7]);
    d[col * (kp / 32) + blk] = dd;
    s[col * (kp / 32) + blk] = dd * (float) sum;
}

static ActQ quantize_into(OpCtx & c, const ggml_tensor * src1, int8_t * q, float * d, float * s) {
    const int64_t K = src1->ne[0];
    const int64_t ncols = src1->ne[1] * src1->ne[2] * src1->ne[3];
    const int64_t kp = (K + 31) / 32 * 32;
    const int64_t nblk = kp / 32;
    dim3 grid((unsigned) mx_ceil_div(nblk, 64), (unsigned) ncols);
    k_quantize_act<<<grid, 64, 0, c.st>>>((const char *) src1->data, K, src1->ne[1], src1->ne[2],
                                           src1->nb[1], src1->nb[2], src1->nb[3], kp, q, d, s);
    return ActQ{q, d, s, kp};
}

// bytes of one quantised activation set (+8 padding columns: the GEMV reads
// NC-padded column groups, NC in {1,2,4,8})
size_t act_slot_bytes(const ggml_tensor * src1) {
    const int64_t ncols = src1->ne[1] * src1->ne[2] * src1->ne[3];
    const int64_t kp = (src1->ne[0] + 31) / 32 * 32;
    return (ncols + 8) * kp + 2 * (ncols + 8) * (kp / 32) * sizeof(float) + 3 * 256;
}

size_t quantize_scratch(const ggml_tensor * src1) { return act_slot_bytes(src1); }

static ActQ carve_raw(char * base, int64_t ne0, int64_t ncols) {
    const int64_t kp = (ne0 + 31) / 32 * 32;
    auto al = [](size_t x) { return (x + 255) & ~(size_t) 255; };
    char * p = base;
    int8_t * q = (int8_t *) p; p += al((ncols + 8) * kp);
    float * d = (float *) p; p += al((ncols + 8) * (kp / 32) * sizeof(float));
    float * s = (float *) p;
    return ActQ{q, d, s, kp};
}
static ActQ carve(char * base, const ggml_tensor * src1) {
    return carve_raw(base, src1->ne[0], src1->ne[1] * src1->ne[2] * src1->ne[3]);
}
static size_t slot_bytes_raw(int64_t ne0, int64_t ncols) {
    const int64_t kp = (ne0 + 31) / 32 * 32;
    return (ncols + 8) * kp + 2 * (ncols + 8) * (kp / 32) * sizeof(float) + 3 * 256;
}

void act_cache_reset(Stream * s) {
    for (auto & e : s->act_cache) e = ActCacheEntry{};
    s->act_next = 0;
    s->f16_src[0] = s->f16_src[1] = nullptr;
}

void act_cache_invalidate(Stream * s, const ggml_tensor * w) {
    const char * lo = (const char *) w->data;
    const char * hi = lo + mx_nbytes(w);
    for (int k = 0; k < 2; ++k) {
        if (!s->f16_src[k]) continue;
        const char * a = (const char *) s->f16_src[k];
        const char * b = a + (size_t) s->f16_key[k][1] * (size_t) s->f16_key[k][2];
        if (a < hi && lo < b) s->f16_src[k] = nullptr;
    }
    for (auto & e : s->act_cache) {
        if (!e.data) continue;
        const char * a = (const char *) e.data, * b = a + e.bytes;
        if (a < hi && lo < b) e = ActCacheEntry{};
    }
}

static ActCacheEntry * act_lookup(Stream * s, const ggml_tensor * t) {
    if (!mx_is_contiguous(t)) return nullptr;
    const int64_t ncols = t->ne[1] * t->ne[2] * t->ne[3];
    for (auto & e : s->act_cache)
        if (e.data && e.data == t->data && e.ne0 == t->ne[0] && e.ncols == ncols) return &e;
    return nullptr;
}

const ActQ * act_cache_find(Stream * s, const ggml_tensor * t) {
    ActCacheEntry * e = act_lookup(s, t);
    return e ? &e->a : nullptr;
}

ActQ * act_cache_alloc_raw(Stream * s, const void * data, int64_t ne0, int64_t ncols, size_t bytes) {
    if (!s->act.base || slot_bytes_raw(ne0, ncols) > s->act_slot) return nullptr;
    const int slot = s->act_next;
    s->act_next = (s->act_next + 1) % 4;
    ActCacheEntry & e = s->act_cache[slot];
    e.data = data; e.ne0 = ne0; e.ncols = ncols; e.bytes = bytes;
    e.a = carve_raw(s->act.base + slot * s->act_slot, ne0, ncols);
    return &e.a;
}

ActQ * act_cache_alloc(Stream * s, const ggml_tensor * t) {
    if (!mx_is_contiguous(t)) return nullptr;
    return act_cache_alloc_raw(s, t->data, t->ne[0], t->ne[1] * t->ne[2] * t->ne[3], mx_nbytes(t));
}

// quantised activations of src1, shared across the GEMVs of one graph pass
ActQ quantize_activations(OpCtx & c, const ggml_tensor * src1) {
    if (ActCacheEntry * e = act_lookup(c.s, src1)) return e->a;
    if (ActQ * a = act_cache_alloc(c.s, src1)) {
        return *a = quantize_into(c, src1, (int8_t *) a->q, (float *) a->d, (float *) a->s);
    }
    ActQ a = carve((char *) c.scratch->take(act_slot_bytes(src1)), src1);
    return quantize_into(c, src1, (int8_t *) a.q, (float *) a.d, (float *) a.s);
}

// ---------------------------------------------------------------------------
// quantised GEMV. LPR lanes cooperate on one weight row (64/LPR rows per wave,
// 4 waves per block); each lane loads UNR units before computing any.
// Channel c = blockIdx.y spans (i12, i13); src0 broadcast by r2 = ne12/ne02.
// ---------------------------------------------------------------------------
struct MmvArgs {
    const char * w;   size_t w_row, w_c2, w_c3;     // weight base and strides (rows, dim2, dim3)
    const char * w2;                                // second weight (fused GLU up), same geometry
    float * dst;      size_t d_col, d_c2, d_c3;     // dst strides in floats
    const float * res; size_t r_col;                // fused residual (ADD), same shape as dst
    int64_t nrows, units;
    int64_t ncols;                                  // activation columns per channel (ne11)
    int64_t ne12, r2, r3;
};

template <int QT, int NC, int LPR, int UNR, int EPI>   // EPI: 0 plain, 1 GLU (silu(W·x)*(W2·x)), 2 +residual
__global__ __launch_bounds__(256) void k_mmvq(MmvArgs p, ActQ a) {
    constexpr bool GLU = EPI == 1;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    constexpr int RPW = 64 / LPR;
    const int64_t row = ((int64_t) blockIdx.x * 4 + wave) * RPW + lane / LPR;
    const int sub = lane % LPR;
    const int64_t ch = blockIdx.y;
    const int64_t i12 = ch % p.ne12, i13 = ch / p.ne12;
    ActQ ac = a;
    const int64_t col0 = ch * p.ncols;
    ac.q += col0 * a.kp; ac.d += col0 * (a.kp / 32); ac.s += col0 * (a.kp / 32);
    float acc[NC], acc2[NC];
#pragma unroll
    for (int c = 0; c < NC; ++c) { acc[c] = 0.f; acc2[c] = 0.f; }
    if (row < p.nrows) {
        const size_t off = (size_t) row * p.w_row + (i12 / p.r2) * p.w_c2 + (i13 / p.r3) * p.w_c3;
        const char * r = p.w + off;
        const char * r2 = GLU ? p.w2 + off : nullptr;
        for (int u0 = sub; u0 < p.units; u0 += LPR * UNR) {
            URegs<QT> rg[UNR];
            URegs<QT> rg2[GLU ? UNR : 1];
            // branch-free issue of every weight load (out-of-range units re-read the
            // last unit and are skipped in the compute loop)
#pragma unroll
            for (int j = 0; j < UNR; ++j) {
                const int u = min(u0 + j * LPR, (int) p.units - 1);
                unit_load<QT>(r, u, rg[j]);
                if constexpr (GLU) unit_load<QT>(r2, u, rg2[j]);
            }
#pragma unroll
            for (int j = 0; j < UNR; ++j) {
                const int u = u0 + j * LPR;
                if (u < p.units) {
                    unit_compute<QT, NC>(rg[j], u, ac, acc);
                    if constexpr (GLU) unit_compute<QT, NC>(rg2[j], u, ac, acc2);
                }
            }
        }
    }
#pragma unroll
    for (int c = 0; c < NC; ++c) {
#pragma unroll
        for (int o = LPR / 2; o > 0; o >>= 1) {
            acc[c] += __shfl_xor(acc[c], o, 64);
            if constexpr (GLU) acc2[c] += __shfl_xor(acc2[c], o, 64);
        }
    }
    if (sub == 0 && row < p.nrows) {
        float * out = p.dst + i12 * p.d_c2 + i13 * p.d_c3 + row;
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            if (c < p.ncols) {
                float v = acc[c];
                if constexpr (GLU) v = (v / (1.0f + expf(-v))) * acc2[c];
                if constexpr (EPI == 2) v += p.res[row + c * p.r_col];
                out[c * p.d_col] = v;
            }
        }
    }
}

// launch geometry: enough blocks to cover 256 CUs, every lane's units in flight at once
template <int QT, int NC, int EPI, int LPR>
static void launch_lpr(OpCtx & c, const MmvArgs & p, const ActQ & a, int64_t nch) {
    constexpr int RPB = 4 * (64 / LPR);
    dim3 grid((unsigned) mx_ceil_div(p.nrows, RPB), (unsigned) nch);
    const int64_t per_lane = mx_ceil_div(p.units, LPR);
    MX_KLOG("mmvq1 qt=%d nc=%d lpr=%d epi=%d M=%d", QT, NC, LPR, EPI, (int) p.nrows);
    // round 6: two columns keep up to 4 units of a lane in flight (g_tune[43] = 2: the round-1
    // depth of 2; the wider groups stay at 2 — their activation registers grow with NC)
    if constexpr (NC == 1) {
        if (per_lane >= 5) k_mmvq<QT, NC, LPR, 8, EPI><<<grid, 256, 0, c.st>>>(p, a);
        else if (per_lane >= 3) k_mmvq<QT, NC, LPR, 4, EPI><<<grid, 256, 0, c.st>>>(p, a);
        else k_mmvq<QT, NC, LPR, 2, EPI><<<grid, 256, 0, c.st>>>(p, a);
    } else if constexpr (NC == 2) {
        if (per_lane >= 3 && g_tune[43] != 2) k_mmvq<QT, NC, LPR, 4, EPI><<<grid, 256, 0, c.st>>>(p, a);
        else k_mmvq<QT, NC, LPR, 2, EPI><<<grid, 256, 0, c.st>>>(p, a);
    } else {
        k_mmvq<QT, NC, LPR, 2, EPI><<<grid, 256, 0, c.st>>>(p, a);
    }
}

template <int QT, int NC, int EPI>
static void launch_mmvq_nc(OpCtx & c, const MmvArgs & p, const ActQ & a, int64_t nch) {
    // GLU streams two matrices: one LPR step wider keeps its register tile (and
    // occupancy) equal to the single-matrix kernels
    const int64_t small_units = EPI == 1 ? 64 : 128;
    if (p.nrows <= 2048 || p.units > 256) launch_lpr<QT, NC, EPI, 64>(c, p, a, nch);
    else if (p.units <= small_units) launch_lpr<QT, NC, EPI, 16>(c, p, a, nch);
    else launch_lpr<QT, NC, EPI, 32>(c, p, a, nch);
}

template <int QT, int EPI>
static void launch_mmvq(OpCtx & c, const MmvArgs & p, const ActQ & a, int64_t nch) {
    switch (p.ncols) {
        case 1: launch_mmvq_nc<QT, 1, EPI>(c, p, a, nch); break;
        case 2: launch_mmvq_nc<QT, 2, EPI>(c, p, a, nch); break;
        case 3: case 4: launch_mmvq_nc<QT, 4, EPI>(c, p, a, nch); break;
        default: launch_mmvq_nc<QT, 8, EPI>(c, p, a, nch); break;
    }
}

bool mmvq_type_ok(int t) {
    return t == GGML_TYPE_Q4_K || t == GGML_TYPE_Q5_K || t == GGML_TYPE_Q6_K || t == GGML_TYPE_Q4_0 || t == GGML_TYPE_Q8_0;
}

static MmvArgs mmv_args(const ggml_tensor * w, const ggml_tensor * src1, ggml_tensor * dst) {
    MmvArgs p{};
    p.w = (const char *) w->data;
    p.w_row = w->nb[1]; p.w_c2 = w->nb[2]; p.w_c3 = w->nb[3];
    p.dst = (float *) dst->data;
    p.d_col = dst->nb[1] / 4; p.d_c2 = dst->nb[2] / 4; p.d_c3 = dst->nb[3] / 4;
    p.nrows = w->ne[1];
    p.units = w->ne[0] / 32;
    p.ncols = src1->ne[1];
    p.ne12 = src1->ne[2];
    p.r2 = src1->ne[2] / w->ne[2];
    p.r3 = src1->ne[3] / w->ne[3];
    return p;
}

template <int EPI>
static void mmvq_dispatch(OpCtx & c, int type, const MmvArgs & p, const ActQ & a, int64_t nch) {
    switch (type) {
        case GGML_TYPE_Q4_K: launch_mmvq<GGML_TYPE_Q4_K, EPI>(c, p, a, nch); break;
        case GGML_TYPE_Q5_K: launch_mmvq<GGML_TYPE_Q5_K, EPI>(c, p, a, nch); break;
        case GGML_TYPE_Q6_K: launch_mmvq<GGML_TYPE_Q6_K, EPI>(c, p, a, nch); break;
        case GGML_TYPE_Q4_0: launch_mmvq<GGML_TYPE_Q4_0, EPI>(c, p, a, nch); break;
        case GGML_TYPE_Q8_0: launch_mmvq<GGML_TYPE_Q8_0, EPI>(c, p, a, nch); break;
        default: MX_ABORT("mmvq type %d", type);
    }
}

// dst = src0 · src1 for quantised src0 with ne11 <= 8 (src1 f32, dst f32, contiguous dst rows)
void mmvq_run(OpCtx & c, ggml_tensor * dst) {
    const ggml_tensor * w = dst->src[0];
    const ggml_tensor * x = dst->src[1];
    ActQ a = quantize_activations(c, x);
    MmvArgs p = mmv_args(w, x, dst);
    mmvq_dispatch<0>(c, w->type, p, a, x->ne[2] * x->ne[3]);
}

bool mmvq_small_batch_ok(const ggml_tensor * mm) {
    const ggml_tensor * w = mm->src[0];
    const ggml_tensor * x = mm->src[1];
    return mm->op == GGML_OP_MUL_MAT && mmvq_type_ok(w->type) && x->type == GGML_TYPE_F32 && x->ne[1] <= 8 &&
           x->nb[0] == 4 && mm->nb[0] == 4 && w->nb[0] == (size_t) mx_type(w->type).size && w->ne[0] % qk_of_type(w->type) == 0;
}

bool mmvq_fused_glu(OpCtx & c, const ggml_tensor * gate, const ggml_tensor * up, ggml_tensor * glu) {
    const ggml_tensor * wg = gate->src[0], * wu = up->src[0];
    const ggml_tensor * x = gate->src[1];
    if (up->src[1] != x || wg->type != wu->type || !mmvq_small_batch_ok(gate) || !mmvq_small_batch_ok(up)) return false;
    if (mx_op_param<int32_t>(glu, 0) != GGML_GLU_OP_SWIGLU) return false;
    if (x->ne[2] != 1 || x->ne[3] != 1) return false;
    for (int i = 0; i < 4; ++i) if (wg->ne[i] != wu->ne[i] || wg->nb[i] != wu->nb[i]) return false;
    if (wg->ne[2] != 1 || wg->ne[3] != 1) return false;
    if (glu->type != GGML_TYPE_F32 || glu->nb[0] != 4 || !mx_are_same_shape(glu, gate)) return false;
    XStage xs;
    if (tensor_is_split(wg) || tensor_is_split(wu)) {
        // row-split gate and up (the same row ranges): one SwiGLU GEMV per slice, each writing
        // its rows of the GLU and of its q8 copy (the down projection's input) — as the
        // unsplit decode does. Round 4 ran them only when every slice was this GPU's; round 5
        // launches each on its own device's stream (split_fork / split_join), reading x and
        // writing the rows on the main device through peer access
        void * dg[MX_MAX_DEVICES], * du[MX_MAX_DEVICES];
        int64_t lg[MX_MAX_DEVICES], hg[MX_MAX_DEVICES], lu[MX_MAX_DEVICES], hu[MX_MAX_DEVICES];
        int vg[MX_MAX_DEVICES], vu[MX_MAX_DEVICES];
        const int ns = split_slices(c.s, wg, dg, lg, hg, vg);
        if (!ns || ns != split_slices(c.s, wu, du, lu, hu, vu) || !g_gemv2 || !mx_is_contiguous(glu)) return false;
        ggml_tensor ws[2][MX_MAX_DEVICES], gv[MX_MAX_DEVICES];
        int remote = 0;
        for (int k = 0; k < ns; ++k) {
            if (lg[k] != lu[k] || hg[k] != hu[k] || vg[k] != vu[k] || lg[k] % 32) return false;
            remote += !split_on_main(c.s, wg, vg[k]);
            const int64_t rows = hg[k] - lg[k];
            for (int t = 0; t < 2; ++t) {
                ggml_tensor & w = ws[t][k];
                w = t ? *wu : *wg; w.ne[1] = rows; w.nb[2] = w.nb[3] = w.nb[1] * rows; w.data = t ? du[k] : dg[k];
                w.buffer = nullptr; w.extra = nullptr; w.view_src = nullptr;
            }
            gv[k] = *glu; gv[k].ne[0] = rows; gv[k].data = (char *) glu->data + lg[k] * 4; gv[k].buffer = nullptr; gv[k].view_src = nullptr;
            gv[k].nb[1] = gv[k].nb[2] = gv[k].nb[3] = (size_t) rows * 4;
            if (!gemv2_ok(&ws[0][k], x, &gv[k])) return false;
        }
        if (!gemv2_stage(c, x, {glu}, {}, &xs, 2)) return false;
        ActQ * q8 = wg->ne[1] % 32 == 0 ? act_cache_alloc(c.s, glu) : nullptr;
        if (q8 && xs.q8 == q8->q) q8 = nullptr;
        MX_KLOG("glu_split M=%lld K=%lld slices=%d remote=%d q8o=%d", (long long) wg->ne[1], (long long) wg->ne[0], ns, remote, q8 != nullptr);
        for (int k = 0; k < ns; ++k) {
            ActQ qs{};
            if (q8) { qs = *q8; qs.q += lg[k]; qs.d += lg[k] / 32; qs.s += lg[k] / 32; }
            if (split_on_main(c.s, wg, vg[k])) { gemv2_launch(c, &ws[0][k], &ws[1][k], xs, (float *) glu->data + lg[k], nullptr, q8 ? &qs : nullptr); continue; }
            OpCtx dc = split_fork(c, vg[k]);
            size_t moved = 0;   // (round 6) x and the norm weight copied to the slice device once
            const XStage lx = split_local_xs(dc, c.s, vg[k], xs, wg->ne[0], &moved);
            gemv2_launch(dc, &ws[0][k], &ws[1][k], lx, (float *) glu->data + lg[k], nullptr, q8 ? &qs : nullptr);
        }
        for (int k = 0; k < ns; ++k) if (!split_on_main(c.s, wg, vg[k])) split_join(c, vg[k]);
        HIP_CHECK(hipSetDevice(c.s->device));
        return true;
    }
    if (g_gemv2 && gemv2_ok(wg, x, glu) && gemv2_stage(c, x, {glu}, {}, &xs, 2)) {
        // the q8 form of the output feeds the down projection's prologue (act cache)
        ActQ * q8 = (wg->ne[1] % 32 == 0 && mx_is_contiguous(glu)) ? act_cache_alloc(c.s, glu) : nullptr;
        if (q8 && xs.q8 == q8->q) q8 = nullptr;
        gemv2_launch(c, wg, wu, xs, (float *) glu->data, nullptr, q8);
        return true;
    }
    ActQ a = quantize_activations(c, x);
    MmvArgs p = mmv_args(wg, x, glu);
    p.w2 = (const char *) wu->data;
    mmvq_dispatch<1>(c, wg->type, p, a, 1);
    return true;
}

bool mmvq_fused_add(OpCtx & c, const ggml_tensor * mm, const ggml_tensor * res, ggml_tensor * add) {
    const ggml_tensor * w = mm->src[0];
    const ggml_tensor * x = mm->src[1];
    if (!mmvq_small_batch_ok(mm) || x->ne[2] != 1 || x->ne[3] != 1) return false;
    if (res->type != GGML_TYPE_F32 || add->type != GGML_TYPE_F32 || !mx_are_same_shape(res, mm) || !mx_are_same_shape(add, mm)) return false;
    if (res->nb[0] != 4 || add->nb[0] != 4 || w->ne[2] != 1 || w->ne[3] != 1) return false;
    XStage xs;
    if (tensor_is_split(w)) {
        // row-split weights: one residual GEMV per slice, each writing its rows of the sum —
        // the unsplit decode's fused launch instead of per-slice GEMVs + an ADD pass; on the
        // slice's own device's stream when it is not this GPU's (as mmvq_fused_glu)
        void * sd[MX_MAX_DEVICES];
        int64_t lo[MX_MAX_DEVICES], hi[MX_MAX_DEVICES];
        int dv[MX_MAX_DEVICES];
        const int ns = split_slices(c.s, w, sd, lo, hi, dv);
        if (!ns || !g_gemv2 || !mx_is_contiguous(res) || !mx_is_contiguous(add)) return false;
        ggml_tensor ws[MX_MAX_DEVICES], av[MX_MAX_DEVICES];
        int remote = 0;
        for (int k = 0; k < ns; ++k) {
            const int64_t rows = hi[k] - lo[k];
            remote += !split_on_main(c.s, w, dv[k]);
            ws[k] = *w; ws[k].ne[1] = rows; ws[k].nb[2] = ws[k].nb[3] = ws[k].nb[1] * rows; ws[k].data = sd[k];
            ws[k].buffer = nullptr; ws[k].extra = nullptr; ws[k].view_src = nullptr;
            av[k] = *add; av[k].ne[0] = rows; av[k].data = (char *) add->data + lo[k] * 4; av[k].buffer = nullptr; av[k].view_src = nullptr;
            av[k].nb[1] = av[k].nb[2] = av[k].nb[3] = (size_t) rows * 4;
            if (!gemv2_ok(&ws[k], x, &av[k])) return false;
        }
        if (!gemv2_stage(c, x, {add}, {res}, &xs)) return false;
        MX_KLOG("mm_split_add M=%lld K=%lld slices=%d remote=%d", (long long) w->ne[1], (long long) w->ne[0], ns, remote);
        for (int k = 0; k < ns; ++k) {
            if (split_on_main(c.s, w, dv[k])) { gemv2_launch(c, &ws[k], nullptr, xs, (float *) add->data + lo[k], (const float *) res->data + lo[k]); continue; }
            OpCtx dc = split_fork(c, dv[k]);
            size_t moved = 0;   // (round 6) x (or its q8 image) copied to the slice device once
            const XStage lx = split_local_xs(dc, c.s, dv[k], xs, w->ne[0], &moved);
            gemv2_launch(dc, &ws[k], nullptr, lx, (float *) add->data + lo[k], (const float *) res->data + lo[k]);
        }
        for (int k = 0; k < ns; ++k) if (!split_on_main(c.s, w, dv[k])) split_join(c, dv[k]);
        HIP_CHECK(hipSetDevice(c.s->device));
        return true;
    }
    if (g_gemv2 && gemv2_ok(w, x, add) && mx_is_contiguous(res)) {
        if (gemv2_stage(c, x, {add}, {res}, &xs)) {
            gemv2_launch(c, w, nullptr, xs, (float *) add->data, (const float *) res->data);
            return true;
        }
        // the output lies over x (libllama's allocator hands the dead input's memory to the
        // ADD: the last layer's MUL_MAT -> GET_ROWS -> ADD chain): quantise x into the
        // activation cache first, then stream the GEMV from that q8 copy — no workgroup reads
        // x while another writes the output (gemv2_stage refused exactly that)
        if (!xs.norm) {
            quantize_activations(c, x);
            xs = xstage_of(c.s, x);
            if (xs.q8 && !xs.norm) {
                gemv2_launch(c, w, nullptr, xs, (float *) add->data, (const float *) res->data);
                act_cache_invalidate(c.s, add);
                return true;
            }
        }
    }
    ActQ a = quantize_activations(c, x);
    MmvArgs p = mmv_args(w, x, add);
    p.res = (const float *) res->data;
    p.r_col = res->nb[1] / 4;
    mmvq_dispatch<2>(c, w->type, p, a, 1);
    return true;
}

// ---------------------------------------------------------------------------
// kernel timing hook for the bench's roofline: quantise x once, then time `iters`
// back-to-back launches of exactly the GEMV kernel the executor would launch for
// MUL_MAT(w, x) (or the fused gate/up GLU when w2 != NULL) with HIP events on the
// backend's own stream. Returns the average µs per launch.
// ---------------------------------------------------------------------------
double time_mmvq(Stream * s, const ggml_tensor * const * w, const ggml_tensor * const * w2, int nw_n,
                 const ggml_tensor * x, ggml_tensor * dst, int iters) {
    OpCtx c{s, s->stream, &s->scratch};
    MX_ASSERT(nw_n >= 1);
    hipEvent_t e0, e1;
    HIP_CHECK(hipEventCreate(&e0));
    HIP_CHECK(hipEventCreate(&e1));
    if (g_gemv2 && gemv2_ok(w[0], x, dst)) {
        // exactly the launch the executor makes in decode: for the SwiGLU pair, the
        // ffn_norm absorbed into the prologue and the q8 form of the output emitted for
        // the down projection; cycling over nw weight sets (e.g. all layers of a model) so
        // the stream comes from HBM, not the 256 MiB MALL
        const int64_t K = w[0]->ne[0], M = w[0]->ne[1];
        float * nw = nullptr;
        ActQ q8{};
        char * q8buf = nullptr;
        if (w2) {
            HIP_CHECK(hipMalloc((void **) &nw, K * sizeof(float)));
            fill_const_f32_ptr(nw, K, 1.0f, s->stream);
            HIP_CHECK(hipMalloc((void **) &q8buf, M + 2 * (M / 32) * sizeof(float) + 512));
            q8.q = (const int8_t *) q8buf;
            q8.d = (const float *) (q8buf + ((M + 255) & ~255));
            q8.s = q8.d + M / 32;
            q8.kp = M;
        }
        const XStage xs = w2 ? XStage{(const float *) x->data, nw, 1e-5f, 1} : XStage{(const float *) x->data, nullptr, 0.0f, 0};
        const bool use_q8 = w2 && M % 32 == 0;
        auto launch = [&](int i) {
            gemv2_launch(c, w[i % nw_n], w2 ? w2[i % nw_n] : nullptr, xs, (float *) dst->data, nullptr, use_q8 ? &q8 : nullptr);
        };
        for (int i = 0; i < 3; ++i) launch(i);
        HIP_CHECK(hipEventRecord(e0, s->stream));
        for (int i = 0; i < iters; ++i) launch(i);
        HIP_CHECK(hipEventRecord(e1, s->stream));
        HIP_CHECK(hipEventSynchronize(e1));
        if (nw) HIP_CHECK(hipFree(nw));
        if (q8buf) HIP_CHECK(hipFree(q8buf));
    } else {
        const size_t need = quantize_scratch(x);
        if (need > s->scratch.cap) {
            HIP_CHECK(hipStreamSynchronize(s->stream));
            if (s->scratch.base) HIP_CHECK(hipFree(s->scratch.base));
            HIP_CHECK(hipMalloc((void **) &s->scratch.base, need));
            s->scratch.cap = need;
            graph_cache_forget(s);
        }
        s->scratch.reset();
        ActQ a = carve((char *) s->scratch.take(act_slot_bytes(x)), x);
        a = quantize_into(c, x, (int8_t *) a.q, (float *) a.d, (float *) a.s);
        auto launch = [&](int i) {
            MmvArgs p = mmv_args(w[i % nw_n], x, dst);
            if (w2) { p.w2 = (const char *) w2[i % nw_n]->data; mmvq_dispatch<1>(c, w[0]->type, p, a, 1); }
            else mmvq_dispatch<0>(c, w[0]->type, p, a, 1);
        };
        for (int i = 0; i < 3; ++i) launch(i);
        HIP_CHECK(hipEventRecord(e0, s->stream));
        for (int i = 0; i < iters; ++i) launch(i);
        HIP_CHECK(hipEventRecord(e1, s->stream));
    }
    HIP_CHECK(hipEventSynchronize(e1));
    float ms = 0.f;
    HIP_CHECK(hipEventElapsedTime(&ms, e0, e1));
    HIP_CHECK(hipEventDestroy(e0));
    HIP_CHECK(hipEventDestroy(e1));
    return 1000.0 * ms / iters;
}

// ---------------------------------------------------------------------------
// generic GEMV: any dequantisable / float weight type, f32 activations, exact
// dequant (used for types without an sdot4 unit, and as the oracle-shaped path)
// ---------------------------------------------------------------------------
template <int QT>
__device__ __forceinline__ float w_elem(const char * row, int64_t k, size_t nb0) {
    if constexpr (QT == GGML_TYPE_F32) return *(const float *) (row + k * nb0);
    else if constexpr (QT == GGML_TYPE_F16) return h2f(*(const uint16_t *) (row + k * nb0));
    else if constexpr (QT == GGML_TYPE_BF16) return bf2f(*(const uint16_t *) (row + k * nb0));
    else return dequant_one<QT>(row + (k / qk_of<QT>()) * qsize_of<QT>(), (int) (k % qk_of<QT>()));
}

struct MmvGen {
    const char * w; size_t w_nb0, w_row, w_c2, w_c3;
    const char * x; size_t x_nb0, x_col, x_c2, x_c3;
    char * dst; size_t d_row, d_col, d_c2, d_c3;
    int64_t K, M, N, ne12, r2, r3;
};

// one wave per (row, column); K-loop strided over 64 lanes
template <int QT>
__global__ __launch_bounds__(256) void k_mmv_generic(MmvGen p) {
    const int lane = threadIdx.x & 63;
    const int64_t gw = (int64_t) blockIdx.x * 4 + (threadIdx.x >> 6);
    const int64_t row = gw % p.M, col = gw / p.M;
    if (col >= p.N) return;
    const int64_t ch = blockIdx.y;
    const int64_t i12 = ch % p.ne12, i13 = ch / p.ne12;
    const char * wr = p.w + row * p.w_row + (i12 / p.r2) * p.w_c2 + (i13 / p.r3) * p.w_c3;
    const char * xr = p.x + col * p.x_col + i12 * p.x_c2 + i13 * p.x_c3;
    float acc = 0.f;
    for (int64_t k = lane; k < p.K; k += 64) acc += w_elem<QT>(wr, k, p.w_nb0) * *(const float *) (xr + k * p.x_nb0);
    acc = wave_sum(acc);
    if (lane == 0) *(float *) (p.dst + row * p.d_row + col * p.d_col + i12 * p.d_c2 + i13 * p.d_c3) = acc;
}

// f32 / f16 weight rows (the MoE router ffn_gate_inp [n_embd, n_expert] f32, small
// unquantised projections) against f32 columns: one workgroup per (row, column), every
// thread's 16-byte loads issued at once, block reduction. The per-wave strided loop above
// took 28.5 us for Mixtral's 8-row router (profiles/r02/prof_mixtral_decode*).
template <typename TW>
__global__ __launch_bounds__(256) void k_mmv_dense(MmvGen p) {
    __shared__ float red[16];
    const int64_t row = blockIdx.x, col = blockIdx.y % p.N, ch = blockIdx.y / p.N;
    const int64_t i12 = ch % p.ne12, i13 = ch / p.ne12;
    const char * wr = p.w + row * p.w_row + (i12 / p.r2) * p.w_c2 + (i13 / p.r3) * p.w_c3;
    const float * xr = (const float *) (p.x + col * p.x_col + i12 * p.x_c2 + i13 * p.x_c3);
    float acc = 0.f;
    constexpr int V = 16 / sizeof(TW);      // weights per 16-byte load
    for (int64_t k = (int64_t) threadIdx.x * V; k < p.K; k += 256 * V) {
        TW wv[V];
        __builtin_memcpy(wv, wr + k * sizeof(TW), 16);
#pragma unroll
        for (int j = 0; j < V; j += 4) {
            const float4 xv = *(const float4 *) (xr + k + j);
            float w0, w1, w2, w3;
            if constexpr (sizeof(TW) == 4) { w0 = wv[j]; w1 = wv[j + 1]; w2 = wv[j + 2]; w3 = wv[j + 3]; }
            else { w0 = h2f(wv[j]); w1 = h2f(wv[j + 1]); w2 = h2f(wv[j + 2]); w3 = h2f(wv[j + 3]); }
            acc += w0 * xv.x + w1 * xv.y + w2 * xv.z + w3 * xv.w;
        }
    }
    acc = block_sum(acc, red);
    if (threadIdx.x == 0) *(float *) (p.dst + row * p.d_row + col * p.d_col + i12 * p.d_c2 + i13 * p.d_c3) = acc;
}

// Round 5: few f32 / f16 weight rows (M <= 64: the MoE router [n_embd, n_expert]) against
// many columns (a prefill ubatch): one wave per column holding all (up to 16 per pass)
// row sums, 16-byte loads, the weight rows re-read from L2 by every wave. The generic
// prefill GEMM took 184 us for Mixtral's 8 x 4096 router at 512 tokens (profiles/r05/).
template <typename TW>
__global__ __launch_bounds__(256) void k_mm_skinny(MmvGen p) {
    const int lane = threadIdx.x & 63;
    const int64_t col = (int64_t) blockIdx.x * 4 + (threadIdx.x >> 6);
    if (col >= p.N) return;                                 // wave-uniform, no barrier below
    const int64_t m0 = (int64_t) blockIdx.y * 16;
    const float * xr = (const float *) (p.x + col * p.x_col);
    float acc[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;
    for (int64_t k = 4 * lane; k < p.K; k += 256) {
        const float4 xv = *(const float4 *) (xr + k);
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            if (m0 + r >= p.M) break;
            const char * wr = p.w + (m0 + r) * p.w_row + k * sizeof(TW);
            float4 w4;
            if constexpr (sizeof(TW) == 4) w4 = *(const float4 *) wr;
            else {
                const uint2 h = *(const uint2 *) wr;
                w4 = make_float4(h2f((uint16_t) (h.x & 0xFFFF)), h2f((uint16_t) (h.x >> 16)), h2f((uint16_t) (h.y & 0xFFFF)),
                                 h2f((uint16_t) (h.y >> 16)));
            }
            acc[r] += w4.x * xv.x + w4.y * xv.y + w4.z * xv.z + w4.w * xv.w;
        }
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        if (m0 + r >= p.M) break;
        const float v = wave_sum(acc[r]);
        if (lane == 0) *(float *) (p.dst + (m0 + r) * p.d_row + col * p.d_col) = v;
    }
}

bool mm_skinny_run(OpCtx & c, ggml_tensor * dst) {
    const ggml_tensor * w = dst->src[0];
    const ggml_tensor * x = dst->src[1];
    if ((w->type != GGML_TYPE_F32 && w->type != GGML_TYPE_F16) || w->ne[1] > 64 || x->ne[1] <= 8) return false;
    if (w->ne[2] != 1 || w->ne[3] != 1 || x->ne[2] != 1 || x->ne[3] != 1 || x->type != GGML_TYPE_F32 || dst->type != GGML_TYPE_F32) return false;
    const size_t ws = w->type == GGML_TYPE_F32 ? 4 : 2;
    if (w->nb[0] != ws || x->nb[0] != 4 || dst->nb[0] != 4 || w->ne[0] % 4 || ((uintptr_t) w->data | w->nb[1]) % (4 * ws) ||
        ((uintptr_t) x->data | x->nb[1]) % 16) return false;
    MmvGen p{};
    p.w = (const char *) w->data; p.w_row = w->nb[1];
    p.x = (const char *) x->data; p.x_col = x->nb[1];
    p.dst = (char *) dst->data; p.d_row = dst->nb[0]; p.d_col = dst->nb[1];
    p.K = w->ne[0]; p.M = w->ne[1]; p.N = x->ne[1];
    const dim3 gd((unsigned) mx_ceil_div(p.N, 4), (unsigned) mx_ceil_div(p.M, 16));
    MX_KLOG("mm_skinny type=%d K=%lld M=%lld N=%lld", (int) w->type, (long long) p.K, (long long) p.M, (long long) p.N);
    if (w->type == GGML_TYPE_F32) k_mm_skinny<float><<<gd, 256, 0, c.st>>>(p);
    else k_mm_skinny<uint16_t><<<gd, 256, 0, c.st>>>(p);
    return true;
}

void mmv_generic_run(OpCtx & c, ggml_tensor * dst) {
    const ggml_tensor * w = dst->src[0];
    const ggml_tensor * x = dst->src[1];
    MmvGen p{};
    p.w = (const char *) w->data; p.w_nb0 = w->nb[0]; p.w_row = w->nb[1]; p.w_c2 = w->nb[2]; p.w_c3 = w->nb[3];
    p.x = (const char *) x->data; p.x_nb0 = x->nb[0]; p.x_col = x->nb[1]; p.x_c2 = x->nb[2]; p.x_c3 = x->nb[3];
    p.dst = (char *) dst->data; p.d_row = dst->nb[0]; p.d_col = dst->nb[1]; p.d_c2 = dst->nb[2]; p.d_c3 = dst->nb[3];
    p.K = w->ne[0]; p.M = w->ne[1]; p.N = x->ne[1]; p.ne12 = x->ne[2];
    p.r2 = x->ne[2] / w->ne[2]; p.r3 = x->ne[3] / w->ne[3];
    const size_t ws = w->type == GGML_TYPE_F32 ? 4 : 2;
    if ((w->type == GGML_TYPE_F32 || w->type == GGML_TYPE_F16) && p.w_nb0 == ws && p.x_nb0 == 4 && p.K % (16 / ws) == 0 &&
        p.M * p.N <= 65536 && (((uintptr_t) p.w | p.w_row | p.w_c2 | p.w_c3) % 16) == 0 &&
        (((uintptr_t) p.x | p.x_col | p.x_c2 | p.x_c3) % 16) == 0) {
        const dim3 gd((unsigned) p.M, (unsigned) (p.N * x->ne[2] * x->ne[3]));
        MX_KLOG("mmv_dense type=%d K=%lld M=%lld N=%lld", (int) w->type, (long long) p.K, (long long) p.M, (long long) p.N);
        if (w->type == GGML_TYPE_F32) k_mmv_dense<float><<<gd, 256, 0, c.st>>>(p);
        else k_mmv_dense<uint16_t><<<gd, 256, 0, c.st>>>(p);
        return;
    }
    dim3 grid((unsigned) mx_ceil_div(p.M * p.N, 4), (unsigned) (x->ne[2] * x->ne[3]));
    switch (w->type) {
#define GEN(T) case T: k_mmv_generic<T><<<grid, 256, 0, c.st>>>(p); break;
        GEN(GGML_TYPE_F32) GEN(GGML_TYPE_F16) GEN(GGML_TYPE_BF16)
        GEN(GGML_TYPE_Q4_0) GEN(GGML_TYPE_Q4_1) GEN(GGML_TYPE_Q5_0) GEN(GGML_TYPE_Q5_1) GEN(GGML_TYPE_Q8_0)
        GEN(GGML_TYPE_Q4_K) GEN(GGML_TYPE_Q5_K) GEN(GGML_TYPE_Q6_K)
#undef GEN
        default: MX_ABORT("mmv_generic type %d", (int) w->type);
    }
}

}  // namespace mx
