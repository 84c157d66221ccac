// gemv.h — host interface of the single-token decode GEMV v2 (ops_gemv.hip) and of
// the executor's deferred RMS norm that the GEMV prologue absorbs.
#pragma once
#include "backend.h"
#include <initializer_list>

namespace mx {

constexpr int64_t GEMV2_MAX_K = 32768;      // LDS: K + K/4 bytes per workgroup
constexpr int64_t GEMV2_MAX_NORM_K = 8192;  // fused RMS norm keeps 32 values per thread (256 threads)

// f32 activation source of a GEMV; norm != 0: x -> (x * rsqrt(mean(x^2) + eps)) * nw
struct XStage {
    const float * x;
    const float * nw;
    float eps;
    int norm;
    const int8_t * q8 = nullptr;    // q8 activation already in memory (act cache):
    const float * q8d = nullptr;    //   copied, not recomputed
    const float * q8s = nullptr;
    int dbg = 0;                    // timing experiments only (g_tune[11]): 1 skip the
                                    // prologue, 2 skip the dot products, 4 skip epilogue math,
                                    // 8 skip the QKV kernel's KV-cache stores
    int xcd = 1;                    // XCD-contiguous block order (g_tune[15] = 1 turns it off)
    int drain = 0;                  // f32 LDS-staged sources: wait for every weight load
                                    // before the prologue (g_tune[14] = 1; A/B)
    // round 5: x = the decode attention's split partials merged in the prologue (the output
    // projection after fa_dec2_partials): per query head hh and split s, fap + (hh * fap_ns +
    // s) * (fap_d + 2) floats hold the unnormalised O (fap_d values), the max (log2 domain)
    // and the sum
    const float * fap = nullptr;
    int fap_ns = 0, fap_d = 0;
    // round 5: register-staged norm sources (XS_NORM / XS_NORM_H2: the QKV block) quantise x * nw without the
    // RMS scale s and multiply the row sums by s after the dot products: the q8 values of
    // (x s) nw and of x nw are the same (amax scales with them), only the block scales carry
    // s, and the dot is linear in them — so the prologue needs no barrier for the sum of
    // squares before quantising. 0: scale first (g_tune[42] = 1, A/B). The LDS-DMA-staged
    // form (XS_NORM_LDS, the SwiGLU) keeps the scale first: post-scaled it ran 2 % slower
    // (tg128 625-628 vs 641-642, profiles/r05/norm_postscale_ab.txt)
    int postscale = 1;
};

extern int g_tune[48];      // launch-geometry overrides (ggml_backend_mi355x_set_tune)
extern bool g_gemv2;        // v2 GEMV enabled (GGML_MI355X_GEMV_V1 turns it off)

bool gemv2_type_ok(int t);
bool gemv2_fap_ok(int type, int64_t K, int64_t M);   // XStage::fap source instantiated for this GEMV
bool gemv2_ok(const ggml_tensor * w, const ggml_tensor * x, const ggml_tensor * dst);
// dst[r] = epi(W[r]·x): w2 != null → silu(W·x)*(W2·x); res != null → + res[r].
// q8out (SwiGLU only, rows % 32 == 0): also write the q8 form of dst there.
// MUL_MAT_ID `mm` of a decode step (<= 8 tokens) into dst; w2 = the up experts of a fused
// gate/up SwiGLU (dst = the GLU output), q8out its q8 copy. false: not eligible, nothing run
bool gemv2_moe(OpCtx & c, const ggml_tensor * mm, const ggml_tensor * w2, ggml_tensor * dst, ActQ * q8out = nullptr);
void gemv2_launch(OpCtx & c, const ggml_tensor * w, const ggml_tensor * w2, const XStage & xs, float * dst,
                  const float * res, ActQ * q8out = nullptr);
// the output projection over attention split partials (xs.fap) + residual, wo plain or
// row-split (one launch per slice on its device's stream)
bool gemv2_fap_o_ok(const Stream * s, const ggml_tensor * wo, const ggml_tensor * x, const ggml_tensor * mm);
void gemv2_fap_o_launch(OpCtx & c, const ggml_tensor * wo, const XStage & xs, float * add, const float * res);

// MoE decode (ops_gemv_nc.hip): the down projection's MUL_MAT_ID and the expert combine
// (MUL by the router weights, the per-slot ADDs, optionally + residual) in one launch
struct MoeDownComb {
    const ggml_tensor * as;                              // experts [K, M, n_expert]
    const char * ids; size_t id0, id1;                   // [n_used, n_tok] i32, byte strides
    const int8_t * q; const float * qd; const float * qs; int64_t kp;   // q8 of b: column t * n_used + slot
    const float * wt; size_t wt1, wt2;                   // router weights, float strides (slot, token)
    const float * res; size_t r1;                        // residual (nullable), floats per token
    float * out; size_t o1;                              // combined output, floats per token
    int n_used, n_tok;
};
bool moe_down_combine_ok(int type, int64_t K, int64_t M, int n_used, int n_tok);
void moe_down_combine_launch(OpCtx & c, const MoeDownComb & a);

// The activation a GEMV should stage for src1: the deferred RMS_NORM→MUL pair that
// produces src1 when there is one (exec.cpp), else src1 itself.
XStage xstage_of(Stream * s, const ggml_tensor * src1);
// materialise every deferred norm whose input/weight/output memory `t` overlaps
void deferred_guard_write(OpCtx & c, const ggml_tensor * t);
// materialise every deferred norm whose output `t` reads
void deferred_guard_read(OpCtx & c, const ggml_tensor * t);
// Activation staging for a fused GEMV that writes `outs` (and reads `reads`): guards the
// deferred norms, then fails when an output overlaps what the prologue reads (the
// workgroups would race) — the caller then takes the quantise-first path. `absorbs`: the
// consumers of x this launch stands for (2: a gate/up pair, 3: q/k/v).
bool gemv2_stage(OpCtx & c, const ggml_tensor * x, std::initializer_list<const ggml_tensor *> outs,
                 std::initializer_list<const ggml_tensor *> reads, XStage * xs, int absorbs = 1);

}  // namespace mx
