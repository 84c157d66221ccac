// ops_gemv.hip — single-token decode GEMV v2 (gemv.cuh): activation quantised (and
// optionally RMS-normalised) in each workgroup's prologue, weights streamed with all
// of a lane's loads in flight. Epilogues: plain store, SwiGLU of two weight streams
// (ggml-cuda.cu:2145-2181 fusion), residual add (the MUL_MAT→ADD pair of every layer).
#include "backend.h"
#include "gemv.cuh"

namespace mx {

int g_tune[48] = {0};
// GGML_MI355X_TUNE="i=v,i=v": the same knobs for processes that load the backend without
// calling ggml_backend_mi355x_set_tune (the reference libllama in drop-in A/B runs)
static const bool g_tune_env = [] {
    if (const char * e = getenv("GGML_MI355X_TUNE")) {
        for (const char * p = e; *p;) {
            int i = 0, v = 0, n = 0;
            if (sscanf(p, "%d=%d%n", &i, &v, &n) != 2) break;
            if (i >= 0 && i < 48) g_tune[i] = v;
            p += n;
            while (*p == ',' || *p == ' ') ++p;
        }
    }
    return true;
}();
bool g_gemv2 = getenv("GGML_MI355X_GEMV_V1") == nullptr;

struct G2Args {
    const char * w; const char * w2;
    size_t w_row;
    float * dst; const float * res;
    int nrows, units, K;
    XStage xs;
    int8_t * q8o; float * q8od; float * q8os;   // EPI 1 with 8 waves: q8 form of the output
    unsigned long long * trace;                 // debug (MX_TRACE), workgroup 0
    unsigned long long * trace_blk;             // debug (MX_TRACE_BLK), every workgroup
    // MUL_MAT_ID (MoE decode): grid.y = item = (slot sl, token t) = (item % n_used,
    // item / n_used); the expert id is read on the device (graph-replay safe)
    const char * ids; size_t id0, id1;           // ids [n_used, n_tok] i32, byte strides
    int n_used, n_expert, ne11, n_items;
    size_t w_exp;                                // weight expert stride (bytes)
    int64_t x_col;                               // f32 source: floats per activation column
    size_t d_slot, d_tok;                        // dst strides (floats)
    // weight prefetch rows (grid.y > 0, dense only; exec.cpp fa_prefetch_plan's second
    // stage): lines [off, off + lines) of the XCD's eighth of each range
    const char * pf[4]; size_t pf_eighth[4], pf_off; unsigned pf_lines; int pf_n;
};

// per-item bases of a MUL_MAT_ID GEMV workgroup; false: no valid expert (block-uniform)
__device__ __forceinline__ bool g2_item(const G2Args & p, const char *& w, const char *& w2, XStage & xs,
                                        float *& dst, int8_t *& q8o, float *& q8od, float *& q8os) {
    const int item = blockIdx.y, sl = item % p.n_used, t = item / p.n_used;
    const int ex = *(const int32_t *) (p.ids + (size_t) sl * p.id0 + (size_t) t * p.id1);
    if (ex < 0 || ex >= p.n_expert) return false;
    w += (size_t) ex * p.w_exp;
    if (w2) w2 += (size_t) ex * p.w_exp;
    const int64_t col = (int64_t) t * p.ne11 + sl % p.ne11;
    if (xs.q8) { xs.q8 += col * p.K; xs.q8d += col * (p.K / 32); xs.q8s += col * (p.K / 32); }
    else xs.x += col * p.x_col;
    dst += sl * p.d_slot + t * p.d_tok;
    if (q8o) { q8o += (int64_t) item * p.nrows; q8od += (int64_t) item * (p.nrows / 32); q8os += (int64_t) item * (p.nrows / 32); }
    return true;
}

// EXT: the MUL_MAT_ID item (p.ids) and prefetch-row (grid.y > 0) branches. Compiled only
// into the launches that use them: as runtime branches in every dense decode GEMV they
// cost tg128 594 -> 602-615 tok/s (same box, profiles/r03/ab_gemv_variants.txt).
// EPI 0 store, 1 SwiGLU(w, w2), 2 + residual. W waves per block; with W = 8 and
// LPR = 16 a block owns 32 consecutive rows and (q8o != null) also emits the q8
// activation of its 32 outputs for the next GEMV (the FFN down projection).
template <int QT, int LPR, int UPL, int EPI, int W, int MODE, bool EXT>
__global__ __launch_bounds__(64 * W) void k_gemv2(G2Args p) {
    extern __shared__ __align__(16) char smem[];
    constexpr int NM = EPI == 1 ? 2 : 1;
    constexpr int RPW = 64 / LPR;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (EXT && !p.ids && blockIdx.y > 0) {   // prefetch rows: workgroup-uniform, before any barrier
        const unsigned L = blockIdx.x + gridDim.x * blockIdx.y, xcd = L & 7;
        const unsigned T = (gridDim.x * (gridDim.y - 1) >> 3) * (64 * W), t0 = ((L - gridDim.x) >> 3) * (64 * W) + threadIdx.x;
        unsigned acc = 0;
        for (int r = 0; r < p.pf_n; ++r) {
            const unsigned * w = (const unsigned *) (p.pf[r] + (size_t) xcd * p.pf_eighth[r] + p.pf_off);
#pragma unroll 4
            for (unsigned l = t0; l < p.pf_lines; l += T) acc ^= w[(size_t) l * 32];
        }
        if (acc == 0x9E3779B9u && p.nrows < 0) p.dst[0] = 0.f;   // never (nrows > 0): keeps the loads
        return;
    }
    const int sub = lane % LPR;
    const int blk = xcd_block((int) blockIdx.x, (int) gridDim.x, p.xs.xcd);
    const int row = (blk * W + wave) * RPW + lane / LPR;
    const bool valid = row < p.nrows;
    const int64_t rr = valid ? row : p.nrows - 1;
    const char * wb = p.w, * wb2 = p.w2;
    XStage xs = p.xs;
    float * dst = p.dst;
    int8_t * q8o = p.q8o; float * q8od = p.q8od, * q8os = p.q8os;
    if (EXT && p.ids && !g2_item(p, wb, wb2, xs, dst, q8o, q8od, q8os)) return;
    const char * rows[NM];
    rows[0] = wb + rr * p.w_row;
    if constexpr (NM == 2) rows[1] = wb2 + rr * p.w_row;
    const LdsAct a = lds_act(smem, p.K);
    float * red = gemv_lds_red(smem, p.K);
    float acc[NM];
    unsigned long long * tr = blockIdx.x == 0 ? p.trace : nullptr;
    MX_TRACE(tr, 0);
    MX_TRACE_BLK(p.trace_blk, 0);
    // residual prefetched with the activation: a load issued after the dot products
    // would add a memory round trip to every workgroup's tail
    float res = 0.f;
    if constexpr (EPI == 2) res = p.res[rr];
    gemv_rows<QT, LPR, UPL, NM, 64 * W, MODE>(rows, p.units, sub, a, xs, p.K, red, acc,
                                              [&] { if constexpr (EPI == 2) asm volatile("" : "+v"(res)); });
    MX_TRACE(tr, 3);
    float v = acc[0];
    // silu by v_exp_f32 / v_rcp_f32: libm expf and the IEEE division sat on every
    // workgroup's tail
    if constexpr (EPI == 1) v = v * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(-v * 1.4426950408889634f)) * acc[1];
    if constexpr (EPI == 2) v += res;
    if (sub == LPR - 1 && valid) dst[row] = v;
    MX_TRACE(tr, 4);
    MX_TRACE_BLK(p.trace_blk, 1);
    constexpr int RPB = W * RPW;
    if constexpr (RPB % 32 == 0 && RPB / 32 <= W) {
        if (q8o) {       // block-uniform: the q8 form of this block's RPB outputs, one wave per 32
            __shared__ float orow[RPB];
            if (sub == LPR - 1) orow[row - blk * RPB] = v;
            __syncthreads();
            if (wave < RPB / 32 && lane < 32) {
                const float x = orow[32 * wave + lane];
                const float amax = lane_bcast(dpp_max_group<32>(fabsf(x)), 31);
                const Q8Scale qs = q8_scale(amax);
                const float dd = qs.d;
                const int qi = q8_round(x, qs.id);
                const int sum = __builtin_amdgcn_readlane(dpp_sum_group_i<32>(qi), 31);
                const int qb = blk * (RPB / 32) + wave;
                q8o[qb * 32 + lane] = (int8_t) qi;
                if (lane == 0) { q8od[qb] = dd; q8os[qb] = dd * (float) sum; }
            }
        }
    }
}

// The geometries compiled with the attention-partials source (XS_FAP*: the output
// projection after fa_dec2_partials): residual epilogue, 4 waves, no EXT items, UPL 4 or
// LPR 64 x UPL 2. ONE predicate for what launch_mode instantiates and what gemv2_fap_ok
// admits (round 5's abort came from two hand-kept lists disagreeing): a geometry outside it
// is declined before the attention runs, never launched.
__host__ __device__ constexpr bool fap_geom(int LPR, int UPL, int EPI, int W, bool EXT) {
    return EPI == 2 && !EXT && W == 4 && (UPL == 4 || (LPR == 64 && UPL == 2));
}

template <int QT, int LPR, int UPL, int EPI, int W, bool EXT>
static void launch_mode(hipStream_t st, const G2Args & p, int mode, dim3 grid, size_t lds) {
    if (xs_fap(mode)) {
        if constexpr (fap_geom(LPR, UPL, EPI, W, EXT)) {
            if (mode == XS_FAP8) k_gemv2<QT, LPR, UPL, EPI, W, XS_FAP8, EXT><<<grid, 64 * W, lds, st>>>(p);
            else k_gemv2<QT, LPR, UPL, EPI, W, XS_FAP4, EXT><<<grid, 64 * W, lds, st>>>(p);
            return;
        }
        MX_ABORT("gemv2: gemv2_fap_ok admitted geometry lpr=%d upl=%d epi=%d w=%d ext=%d", LPR, UPL, EPI, W, (int) EXT);   // (unreachable)
    }
    switch (mode) {
        case XS_Q8: k_gemv2<QT, LPR, UPL, EPI, W, XS_Q8, EXT><<<grid, 64 * W, lds, st>>>(p); break;
        case XS_NORM_LDS: k_gemv2<QT, LPR, UPL, EPI, W, XS_NORM_LDS, EXT><<<grid, 64 * W, lds, st>>>(p); break;
        case XS_F32_LDS: k_gemv2<QT, LPR, UPL, EPI, W, XS_F32_LDS, EXT><<<grid, 64 * W, lds, st>>>(p); break;
        case XS_NORM: k_gemv2<QT, LPR, UPL, EPI, W, XS_NORM, EXT><<<grid, 64 * W, lds, st>>>(p); break;
        case XS_NORM_H2: k_gemv2<QT, LPR, UPL, EPI, W, XS_NORM_H2, EXT><<<grid, 64 * W, lds, st>>>(p); break;
        case XS_F32_H2: k_gemv2<QT, LPR, UPL, EPI, W, XS_F32_H2, EXT><<<grid, 64 * W, lds, st>>>(p); break;
        default: k_gemv2<QT, LPR, UPL, EPI, W, XS_F32, EXT><<<grid, 64 * W, lds, st>>>(p); break;
    }
}

template <int QT, int LPR, int UPL, int EPI, int W = 4>
static void launch_cfg(hipStream_t st, const G2Args & p0, bool regs = false) {
    G2Args p = p0;
    constexpr int RPB = W * (64 / LPR);
    const dim3 grid0((unsigned) ((p.nrows + RPB - 1) / RPB), p.ids ? (unsigned) p.n_items : 1u);
    // regs: register staging of x even on a large grid (the q8-emitting SwiGLU)
    const int mode = gemv_mode(p.xs, p.K, regs && g_tune[9] == 0 ? 0 : (int64_t) grid0.x * grid0.y * W, 64 * W);
    if (p.pf_n && grid0.x % 8) p.pf_n = 0;          // prefetch ids must start on XCD 0
    const size_t lds = gemv_lds_bytes(p.K, mode);
    MX_KLOG("gemv2 qt=%d lpr=%d upl=%d epi=%d w=%d mode=%d K=%d M=%d q8o=%d pf=%d", QT, LPR, UPL, EPI, W, mode, p.K, p.nrows, p.q8o != nullptr, p.pf_n);
    dim3 grid = grid0;
    if (p.pf_n && !p.ids) grid.y = 2;           // one row of prefetch workgroups (grid0.x % 8 == 0)
    if (p.ids || p.pf_n) launch_mode<QT, LPR, UPL, EPI, W, true>(st, p, mode, grid, lds);
    else launch_mode<QT, LPR, UPL, EPI, W, false>(st, p, mode, grid, lds);
}

// the weight types with the full (LPR, UPL) tuning grid in launch_type; the others run
// (LPR in {16, 32, 64}, UPL 2 for the SwiGLU else 4)
__host__ __device__ constexpr bool gemv2_full_grid(int qt) { return qt == GGML_TYPE_Q4_K || qt == GGML_TYPE_Q6_K; }

// the (LPR, UPL) launch_type actually instantiates for a request (epi != 1 or no q8
// emission; waves 4 unless g_tune[16] widens a plain EPI 0 launch)
static void resolve_geom(int type, int epi, int lpr, int upl, int & L, int & U) {
    const bool listed = (lpr == 16 || lpr == 32 || lpr == 64) && (upl == 2 || upl == 4);
    if (gemv2_full_grid(type) && listed) { L = lpr; U = upl; return; }
    U = epi == 1 ? 2 : 4;
    L = lpr == 16 ? 16 : (lpr == 32 ? 32 : 64);
}

template <int QT, int EPI>
static void launch_type(hipStream_t st, const G2Args & p, int lpr, int upl) {
    if constexpr (EPI == 1) {
        if (p.q8o) {   // 32 rows per block; g_tune[4] picks the geometry (sweeps)
            // tools/opbench.py ffn_block --sweep-glu8: W8 LPR16 UPL2 with LDS-staged norm best
            // default 8 waves x 16 lanes x 2 units, x staged by LDS-DMA. The 16-wave form with
            // x in registers timed 0.5 us faster alone (profiles/r01/opbench_glu8_sweep.txt)
            // but 2 % slower in the decode (589 vs 600 tok/s, scripts/ab_bench.sh 4=3 vs 4=0)
            if (g_tune[4] == 1) return launch_cfg<QT, 32, 1, 1, 16>(st, p);
            if (g_tune[4] == 3 && p.nrows % 64 == 0) return launch_cfg<QT, 16, 2, 1, 16>(st, p, true);
            return launch_cfg<QT, 16, 2, 1, 8>(st, p);
        }
    }
    constexpr bool FULL = gemv2_full_grid(QT);   // full tuning grid
    if constexpr (FULL && EPI == 0) {
        // g_tune[16]: waves per workgroup of the plain 16 x 4 geometry (lm_head): 8 or 16
        // halve / quarter the workgroups that each stage (and normalise) the activation —
        // measured slower (lm_head 82.6 / 92.9 / 123.3 us for 4 / 8 / 16 waves), kept for sweeps
        if (g_tune[16] == 8 && lpr == 16 && upl == 4) return launch_cfg<QT, 16, 4, EPI, 8>(st, p);
        if (g_tune[16] == 16 && lpr == 16 && upl == 4) return launch_cfg<QT, 16, 4, EPI, 16>(st, p);
    }
    if constexpr (FULL) {
#define CFG(L, U) if (lpr == L && upl == U) return launch_cfg<QT, L, U, EPI>(st, p);
        CFG(16, 2) CFG(16, 4) CFG(32, 2) CFG(32, 4) CFG(64, 2) CFG(64, 4)
#undef CFG
    }

    constexpr int U = EPI == 1 ? 2 : 4;
    (void) upl;
    if (lpr == 16) return launch_cfg<QT, 16, U, EPI>(st, p);
    if (lpr == 32) return launch_cfg<QT, 32, U, EPI>(st, p);
    return launch_cfg<QT, 64, U, EPI>(st, p);
}

static int units_of(int type, int64_t K) {
    return (int) (K / ((type == GGML_TYPE_Q4_0 || type == GGML_TYPE_Q8_0) ? 32 : 64));
}


// launch geometry: defaults from the tools/opbench.py sweep on MI355X (profiles/r01/
// opbench_sweep.txt); g_tune overrides for sweeps
static void pick_cfg(int type, int units, int nrows, bool glu, int & lpr, int & upl) {
    if (glu) { lpr = 32; upl = 2; }
    else if (units >= 128) { lpr = 32; upl = type == GGML_TYPE_Q6_K ? 2 : 4; }
    else if (nrows <= 2048) { lpr = 64; upl = 2; }
    else { lpr = 16; upl = 4; }
    const int base = glu ? 2 : 0;
    if (g_tune[base]) lpr = g_tune[base];
    if (g_tune[base + 1]) upl = g_tune[base + 1];
    // round 6: the FFN down projections alone (sweeps). tg128, one box (profiles/r06/
    // down_geometry_sweep.txt): default (Q6_K 32x2, Q4_K 32x4) 635.6, 32x4 637.0, 64x4 634.1,
    // 64x2 633.1, 16x4 603.6; every unit of a lane in one batch (32x8, built for the sweep)
    // 632.9 tok/s — the down projection's geometry is not what its time is made of
    if (!glu && units >= 128) {
        if (g_tune[44]) lpr = g_tune[44];
        if (g_tune[45]) upl = g_tune[45];
    }
}

// the residual GEMV can take its x as attention split partials (XS_FAP*: fa_dec2_partials):
// a geometry instantiated for it (launch_mode), one 16-value half per thread
bool gemv2_fap_ok(int type, int64_t K, int64_t M) {
    if (!gemv2_type_ok(type) || K > 16 * 256 || K % 32) return false;
    int lpr, upl, L, U;
    pick_cfg(type, units_of(type, K), (int) M, false, lpr, upl);
    resolve_geom(type, 2, lpr, upl, L, U);
    return fap_geom(L, U, 2, 4, false);   // (gemv2_launch never arms the EXT prefetch with a fap source)
}

bool gemv2_type_ok(int t) {
    return t == GGML_TYPE_Q4_K || t == GGML_TYPE_Q5_K || t == GGML_TYPE_Q6_K || t == GGML_TYPE_Q4_0 || t == GGML_TYPE_Q8_0;
}

bool gemv2_ok(const ggml_tensor * w, const ggml_tensor * x, const ggml_tensor * dst) {
    if (!gemv2_type_ok(w->type) || x->type != GGML_TYPE_F32 || dst->type != GGML_TYPE_F32) return false;
    const int64_t K = w->ne[0];
    const int64_t qk = (w->type == GGML_TYPE_Q4_0 || w->type == GGML_TYPE_Q8_0) ? 32 : 256;
    if (K % qk || K > GEMV2_MAX_K || x->ne[0] != K) return false;
    if (x->ne[1] * x->ne[2] * x->ne[3] != 1 || w->ne[2] != 1 || w->ne[3] != 1) return false;
    if (w->nb[0] != (size_t) mx_type(w->type).size || w->ne[1] > INT32_MAX) return false;
    if (x->nb[0] != 4 || ((uintptr_t) x->data & 15) || dst->nb[0] != 4 || dst->ne[0] != w->ne[1]) return false;
    return true;
}

static void gemv2_launch_p(OpCtx & c, G2Args & p, int type, bool glu, bool res);

void gemv2_launch(OpCtx & c, const ggml_tensor * w, const ggml_tensor * w2, const XStage & xs, float * dst,
                  const float * res, ActQ * q8out) {
    G2Args p{};
    p.w = (const char *) w->data;
    p.w2 = w2 ? (const char *) w2->data : nullptr;
    p.w_row = w->nb[1];
    p.dst = dst;
    p.res = res;
    p.nrows = (int) w->ne[1];
    p.K = (int) w->ne[0];
    p.units = units_of(w->type, w->ne[0]);
    p.xs = xs;
    p.trace = mx_trace_slot(1);
    p.trace_blk = mx_trace_blocks();
    const bool glu = w2 != nullptr;
    if (q8out) {
        MX_ASSERT(glu && p.nrows % 32 == 0);
        p.q8o = (int8_t *) q8out->q; p.q8od = (float *) q8out->d; p.q8os = (float *) q8out->s;
    }
    MX_ASSERT(!(glu && res));
    if (c.s->gpf_armed && !glu && !xs.fap) {    // the executor's second prefetch stage (not with
                                                // partials: fap_geom has no EXT instantiations)
        c.s->gpf_armed = false;
        p.pf_n = c.s->pf_n;
        for (int r = 0; r < p.pf_n; ++r) { p.pf[r] = c.s->pf_ptr[r]; p.pf_eighth[r] = c.s->pf_len[r] / 8; }
        p.pf_off = c.s->gpf_off & ~(size_t) 127;
        p.pf_lines = (unsigned) (c.s->gpf_take / 128);
    }
    gemv2_launch_p(c, p, w->type, glu, res != nullptr);
}

static void gemv2_launch_p(OpCtx & c, G2Args & p, int type, bool glu, bool res) {
    int lpr, upl;
    pick_cfg(type, p.units, p.nrows, glu, lpr, upl);
    const int epi = glu ? 1 : (res ? 2 : 0);
#define TY(T) case T: \
        if (epi == 0) launch_type<T, 0>(c.st, p, lpr, upl); \
        else if (epi == 1) launch_type<T, 1>(c.st, p, lpr, upl); \
        else launch_type<T, 2>(c.st, p, lpr, upl); \
        break;
    switch (type) {
        TY(GGML_TYPE_Q4_K) TY(GGML_TYPE_Q5_K) TY(GGML_TYPE_Q6_K) TY(GGML_TYPE_Q4_0) TY(GGML_TYPE_Q8_0)
        default: MX_ABORT("gemv2 type %d", type);
    }
#undef TY
}

// The output projection that merges the decode attention's split partials (xs.fap) in its
// prologue, + residual: one launch, or (round 5, -sm row) one per row-split slice of wo, each
// on its device's own stream (split_fork / split_join, as mmvq_fused_add), every slice merging
// the partials itself and writing its rows of `add` on the main device
bool gemv2_fap_o_ok(const Stream * s, const ggml_tensor * wo, const ggml_tensor * x, const ggml_tensor * mm) {
    if (!gemv2_ok(wo, x, mm)) return false;
    if (!tensor_is_split(wo)) return gemv2_fap_ok(wo->type, wo->ne[0], wo->ne[1]);
    void * sd[MX_MAX_DEVICES];
    int64_t lo[MX_MAX_DEVICES], hi[MX_MAX_DEVICES];
    int dv[MX_MAX_DEVICES];
    const int ns = split_slices(s, wo, sd, lo, hi, dv);
    // round 6: slices on other GPUs take the merged attention output instead (16 KB per
    // slice device at Llama-3-8B, against 66 KB of split partials); GGML_MI355X_SPLIT_FAP=1
    // keeps the partials for them too (A/B)
    static const bool fap_remote = getenv("GGML_MI355X_SPLIT_FAP") != nullptr;
    for (int k = 0; k < ns; ++k) {
        if (!gemv2_fap_ok(wo->type, wo->ne[0], hi[k] - lo[k])) return false;
        if (!fap_remote && !split_on_main(s, wo, dv[k])) return false;
    }
    return ns > 0;
}

void gemv2_fap_o_launch(OpCtx & c, const ggml_tensor * wo, const XStage & xs, float * add, const float * res) {
    if (!tensor_is_split(wo)) { gemv2_launch(c, wo, nullptr, xs, add, res); return; }
    void * sd[MX_MAX_DEVICES];
    int64_t lo[MX_MAX_DEVICES], hi[MX_MAX_DEVICES];
    int dv[MX_MAX_DEVICES];
    const int ns = split_slices(c.s, wo, sd, lo, hi, dv);
    MX_ASSERT(ns > 0);
    ggml_tensor ws[MX_MAX_DEVICES];
    int remote = 0;
    for (int k = 0; k < ns; ++k) {
        const int64_t rows = hi[k] - lo[k];
        ws[k] = *wo; ws[k].ne[1] = rows; ws[k].nb[2] = ws[k].nb[3] = ws[k].nb[1] * rows; ws[k].data = sd[k];
        ws[k].buffer = nullptr; ws[k].extra = nullptr; ws[k].view_src = nullptr;
        remote += !split_on_main(c.s, wo, dv[k]);
    }
    MX_KLOG("fap_split M=%lld slices=%d remote=%d", (long long) wo->ne[1], ns, remote);
    for (int k = 0; k < ns; ++k) {
        if (split_on_main(c.s, wo, dv[k])) { gemv2_launch(c, &ws[k], nullptr, xs, add + lo[k], res + lo[k]); continue; }
        OpCtx dc = split_fork(c, dv[k]);
        size_t moved = 0;   // (round 6) the attention partials copied to the slice device once
        const XStage lx = split_local_xs(dc, c.s, dv[k], xs, wo->ne[0], &moved);
        gemv2_launch(dc, &ws[k], nullptr, lx, add + lo[k], res + lo[k]);
    }
    for (int k = 0; k < ns; ++k) if (!split_on_main(c.s, wo, dv[k])) split_join(c, dv[k]);
    HIP_CHECK(hipSetDevice(c.s->device));
}

// MUL_MAT_ID of a decode step (n_tok <= 8): one v2 GEMV launch, grid.y = (slot, token)
// items, the expert of each read on the device. gate/up (w2 != null): silu(Wg x) * (Wu x)
// of the two MUL_MAT_IDs in one pass (and the q8 of the result for the down projection's
// prologue when q8out is given: [item][M] int8 + per-32 d, d*sum).
bool gemv2_moe(OpCtx & c, const ggml_tensor * mm, const ggml_tensor * w2, ggml_tensor * dst, ActQ * q8out) {
    const ggml_tensor * as = mm->src[0], * b = mm->src[1], * ids = mm->src[2];
    if (!g_gemv2 || !gemv2_type_ok(as->type) || b->type != GGML_TYPE_F32 || dst->type != GGML_TYPE_F32) return false;
    const int64_t K = as->ne[0];
    const int64_t qk = (as->type == GGML_TYPE_Q4_0 || as->type == GGML_TYPE_Q8_0) ? 32 : 256;
    if (K % qk || K > GEMV2_MAX_K || b->ne[0] != K || b->nb[0] != 4 || b->ne[3] != 1 || as->ne[3] != 1) return false;
    if (as->nb[0] != (size_t) mx_type(as->type).size || as->ne[1] > INT32_MAX) return false;
    if (ids->type != GGML_TYPE_I32 || ids->ne[1] > 8 || ids->ne[0] * ids->ne[1] > 65535 || ids->ne[1] != b->ne[2]) return false;
    if (dst->nb[0] != 4 || dst->ne[0] != as->ne[1] || dst->ne[1] != ids->ne[0]) return false;
    if (b->nb[2] != b->nb[1] * b->ne[1] || b->nb[1] != (size_t) K * 4 || ((uintptr_t) b->data & 15)) return false;
    if (w2 && (w2->type != as->type || w2->nb[1] != as->nb[1] || w2->nb[2] != as->nb[2] || w2->ne[1] != as->ne[1])) return false;
    G2Args p{};
    p.w = (const char *) as->data;
    p.w2 = w2 ? (const char *) w2->data : nullptr;
    p.w_row = as->nb[1];
    p.dst = (float *) dst->data;
    p.nrows = (int) as->ne[1];
    p.K = (int) K;
    p.units = units_of(as->type, K);
    // a q8 copy of b in the act cache (the gate/up SwiGLU's emission) is staged as is
    p.xs = XStage{(const float *) b->data, nullptr, 0.0f, 0};
    p.xs.xcd = g_tune[15] != 1;
    if (const ActQ * a = act_cache_find(c.s, b)) if (a->kp == K) { p.xs.q8 = a->q; p.xs.q8d = a->d; p.xs.q8s = a->s; }
    p.trace = mx_trace_slot(1);
    p.ids = (const char *) ids->data; p.id0 = ids->nb[0]; p.id1 = ids->nb[1];
    p.n_used = (int) ids->ne[0]; p.n_expert = (int) as->ne[2]; p.ne11 = (int) b->ne[1];
    p.n_items = (int) (ids->ne[0] * ids->ne[1]);
    p.w_exp = as->nb[2];
    p.x_col = K;
    p.d_slot = dst->nb[1] / 4; p.d_tok = dst->nb[2] / 4;
    if (q8out) {
        MX_ASSERT(w2 && p.nrows % 32 == 0);
        p.q8o = (int8_t *) q8out->q; p.q8od = (float *) q8out->d; p.q8os = (float *) q8out->s;
    }
    MX_KLOG("gemv2 moe qt=%d K=%d M=%d items=%d glu=%d q8in=%d", (int) as->type, p.K, p.nrows, p.n_items, w2 != nullptr,
            p.xs.q8 != nullptr);
    gemv2_launch_p(c, p, as->type, w2 != nullptr, false);
    return true;
}

}  // namespace mx
