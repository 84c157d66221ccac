// common.h — shared host/device helpers for the MI355X ggml backend.
//
// Host side: ggml type traits and tensor-geometry helpers re-stated from the
// semantics of ggml/src/ggml.c (ggml_nbytes, ggml_row_size, ggml_is_contiguous*,
// type_traits table) so the backend needs nothing from libggml-base at run time.
// Device side: wave64 reductions, fp16 helpers, HIP error handling.
#pragma once

#include <hip/hip_runtime.h>
#include <hip/hip_fp16.h>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <atomic>

#include "ggml_abi.h"

#define MX_WAVE 64

[[noreturn]] void mx_abort(const char * file, int line, const char * fmt, ...);
#define MX_ABORT(...) mx_abort(__FILE__, __LINE__, __VA_ARGS__)
#define MX_ASSERT(x) do { if (!(x)) MX_ABORT("assert failed: %s", #x); } while (0)
// dynamic-LDS opt-in of kernel f once per device (a static at the call site): the attribute
// applies to the current device, and one process may drive several GPUs (layer / row split)
#define MX_LDS_OPTIN(f, bytes) do { static std::atomic<unsigned> done_{0u}; int dev_ = 0; \
    HIP_CHECK(hipGetDevice(&dev_)); const unsigned bit_ = 1u << (dev_ & 31); \
    if (!(done_.load(std::memory_order_relaxed) & bit_)) { \
        HIP_CHECK(hipFuncSetAttribute((const void *) (f), hipFuncAttributeMaxDynamicSharedMemorySize, (int) (bytes))); \
        done_.fetch_or(bit_); } } while (0)

#define HIP_CHECK(call) do { hipError_t err_ = (call); if (err_ != hipSuccess) \
    MX_ABORT("HIP error %d (%s) in %s", (int) err_, hipGetErrorString(err_), #call); } while (0)

// ---------------------------------------------------------------------------
// ggml type traits (ggml.c type_traits[]: blck_size, type_size)
// ---------------------------------------------------------------------------
struct mx_type_info { int blck; int size; bool quant; const char * name; };

static inline mx_type_info mx_type(int t) {
    switch (t) {
        case GGML_TYPE_F32:  return {1, 4, false, "f32"};
        case GGML_TYPE_F16:  return {1, 2, false, "f16"};
        case GGML_TYPE_BF16: return {1, 2, false, "bf16"};
        case GGML_TYPE_F64:  return {1, 8, false, "f64"};
        case GGML_TYPE_I8:   return {1, 1, false, "i8"};
        case GGML_TYPE_I16:  return {1, 2, false, "i16"};
        case GGML_TYPE_I32:  return {1, 4, false, "i32"};
        case GGML_TYPE_I64:  return {1, 8, false, "i64"};
        case GGML_TYPE_Q4_0: return {32, 18, true, "q4_0"};
        case GGML_TYPE_Q4_1: return {32, 20, true, "q4_1"};
        case GGML_TYPE_Q5_0: return {32, 22, true, "q5_0"};
        case GGML_TYPE_Q5_1: return {32, 24, true, "q5_1"};
        case GGML_TYPE_Q8_0: return {32, 34, true, "q8_0"};
        case GGML_TYPE_Q8_1: return {32, 36, true, "q8_1"};
        case GGML_TYPE_Q2_K: return {256, 84, true, "q2_K"};
        case GGML_TYPE_Q3_K: return {256, 110, true, "q3_K"};
        case GGML_TYPE_Q4_K: return {256, 144, true, "q4_K"};
        case GGML_TYPE_Q5_K: return {256, 176, true, "q5_K"};
        case GGML_TYPE_Q6_K: return {256, 210, true, "q6_K"};
        case GGML_TYPE_Q8_K: return {256, 292, true, "q8_K"};
        default:             return {0, 0, false, "?"};
    }
}

static inline size_t mx_row_size(int type, int64_t ne) {
    mx_type_info ti = mx_type(type);
    return (size_t) (ti.size * (ne / ti.blck));
}

// ggml_nbytes (ggml.c): extent of the tensor in memory, honouring strides.
static inline size_t mx_nbytes(const ggml_tensor * t) {
    for (int i = 0; i < GGML_MAX_DIMS; ++i) if (t->ne[i] <= 0) return 0;
    mx_type_info ti = mx_type(t->type);
    size_t n;
    if (ti.blck == 1) {
        n = ti.size;
        for (int i = 0; i < GGML_MAX_DIMS; ++i) n += (t->ne[i] - 1) * t->nb[i];
    } else {
        n = t->ne[0] * t->nb[0] / ti.blck;
        for (int i = 1; i < GGML_MAX_DIMS; ++i) n += (t->ne[i] - 1) * t->nb[i];
    }
    return n;
}

static inline int64_t mx_nelements(const ggml_tensor * t) { return t->ne[0] * t->ne[1] * t->ne[2] * t->ne[3]; }
static inline int64_t mx_nrows(const ggml_tensor * t)     { return t->ne[1] * t->ne[2] * t->ne[3]; }

// ggml_is_contiguous_n: dims >= n may be non-contiguous
static inline bool mx_is_contiguous_n(const ggml_tensor * t, int n) {
    size_t next = mx_type(t->type).size;
    if (t->ne[0] != mx_type(t->type).blck && t->nb[0] != next) return false;
    next *= t->ne[0] / mx_type(t->type).blck;
    for (int i = 1; i < GGML_MAX_DIMS; i++) {
        if (t->ne[i] != 1) {
            if (i > n) {
                if (t->nb[i] != next) return false;
                next *= t->ne[i];
            } else {
                next = t->ne[i] * t->nb[i];
            }
        }
    }
    return true;
}
static inline bool mx_is_contiguous(const ggml_tensor * t)       { return mx_is_contiguous_n(t, 0); }
static inline bool mx_is_contiguous_rows(const ggml_tensor * t)  { return t->ne[0] == mx_type(t->type).blck || t->nb[0] == (size_t) mx_type(t->type).size; }
static inline bool mx_are_same_shape(const ggml_tensor * a, const ggml_tensor * b) {
    return a->ne[0] == b->ne[0] && a->ne[1] == b->ne[1] && a->ne[2] == b->ne[2] && a->ne[3] == b->ne[3];
}
static inline bool mx_is_empty(const ggml_tensor * t) {
    for (int i = 0; i < GGML_MAX_DIMS; ++i) if (t->ne[i] == 0) return true;
    return false;
}
static inline bool mx_is_permuted(const ggml_tensor * t) {
    return t->nb[0] > t->nb[1] || t->nb[1] > t->nb[2] || t->nb[2] > t->nb[3];
}
static inline bool mx_is_transposed(const ggml_tensor * t) { return t->nb[0] > t->nb[1]; }

template <typename T> static inline T mx_op_param(const ggml_tensor * t, int i) {
    T v; memcpy(&v, (const char *) t->op_params + 4 * i, sizeof(T)); return v;
}

static inline int64_t mx_ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

// ---------------------------------------------------------------------------
// device helpers
// ---------------------------------------------------------------------------
namespace mx {
// host: trace buffer of kernel slot (0 flash-attn decode, 1 GEMV, 2 QKV), null unless
// tracing is on (tune index 6)
unsigned long long * mx_trace_slot(int slot);
// host: per-workgroup {start, end} s_memrealtime pairs of the last traced launch (tune 6 == 2)
unsigned long long * mx_trace_blocks();
// host: kernel-choice log (ggml_backend_mi355x_klog / _klog_read). Launch sites record
// the kernel and geometry they picked, so tests can assert which instantiation ran at a
// given shape. Off unless enabled; appended only while launching (eager or capture).
extern int g_klog;
void klog_add(const char * fmt, ...) __attribute__((format(printf, 1, 2)));
}
#define MX_KLOG(...) do { if (mx::g_klog) mx::klog_add(__VA_ARGS__); } while (0)
// A/B-experiment code (timing variants whose results are wrong by construction, debug
// masks, opt-in alternatives measured slower: the balanced QKV layout) is
// compiled only into variant builds (scripts/build_variants.sh: EXTRA=-DMX_AB_VARIANTS=1);
// in the product library those knobs are dead code.
#ifndef MX_AB_VARIANTS
#define MX_AB_VARIANTS 0
#endif
#define MX_DBG(x) (MX_AB_VARIANTS && (x))
#if defined(__HIPCC__)

// Cross-lane reductions on DPP (gfx9 data-parallel primitives: quad_perm, half/row
// mirror, row_bcast15/31) instead of ds_bpermute: no LDS round trip per step.
// dpp_*_group<N>: reduction over aligned groups of N lanes; the result is in every
// lane for N <= 16 and in the LAST lane of each group for N = 32, 64.
template <int CTRL, int ROWM = 0xF>
__device__ __forceinline__ float dpp_f(float old, float v) {
    return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(old), __float_as_int(v), CTRL, ROWM, 0xF, false));
}
template <int CTRL, int ROWM = 0xF>
__device__ __forceinline__ int dpp_i(int old, int v) {
    return __builtin_amdgcn_update_dpp(old, v, CTRL, ROWM, 0xF, false);
}
template <int N>
__device__ __forceinline__ float dpp_sum_group(float v) {
    if constexpr (N >= 2) v += dpp_f<0xB1>(0.f, v);          // quad_perm [1,0,3,2]
    if constexpr (N >= 4) v += dpp_f<0x4E>(0.f, v);          // quad_perm [2,3,0,1]
    if constexpr (N >= 8) v += dpp_f<0x141>(0.f, v);         // row_half_mirror
    if constexpr (N >= 16) v += dpp_f<0x140>(0.f, v);        // row_mirror
    if constexpr (N >= 32) v += dpp_f<0x142, 0xA>(0.f, v);   // row_bcast15 -> rows 1, 3
    if constexpr (N >= 64) v += dpp_f<0x143, 0xC>(0.f, v);   // row_bcast31 -> rows 2, 3
    return v;
}
template <int N>
__device__ __forceinline__ float dpp_max_group(float v) {
    if constexpr (N >= 2) v = fmaxf(v, dpp_f<0xB1>(-INFINITY, v));
    if constexpr (N >= 4) v = fmaxf(v, dpp_f<0x4E>(-INFINITY, v));
    if constexpr (N >= 8) v = fmaxf(v, dpp_f<0x141>(-INFINITY, v));
    if constexpr (N >= 16) v = fmaxf(v, dpp_f<0x140>(-INFINITY, v));
    if constexpr (N >= 32) v = fmaxf(v, dpp_f<0x142, 0xA>(-INFINITY, v));
    if constexpr (N >= 64) v = fmaxf(v, dpp_f<0x143, 0xC>(-INFINITY, v));
    return v;
}
template <int N>
__device__ __forceinline__ int dpp_sum_group_i(int v) {
    if constexpr (N >= 2) v += dpp_i<0xB1>(0, v);
    if constexpr (N >= 4) v += dpp_i<0x4E>(0, v);
    if constexpr (N >= 8) v += dpp_i<0x141>(0, v);
    if constexpr (N >= 16) v += dpp_i<0x140>(0, v);
    if constexpr (N >= 32) v += dpp_i<0x142, 0xA>(0, v);
    if constexpr (N >= 64) v += dpp_i<0x143, 0xC>(0, v);
    return v;
}
__device__ __forceinline__ float lane_bcast(float v, int lane) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), lane));
}

// Debug phase tracing (tools/opbench.py --trace): an instrumented kernel gets a device
// pointer (null unless tracing) for its first workgroup and records s_memtime per wave at
// phase boundaries: ptr[wave * 8 + phase].

#define MX_TRACE(ptr, ph) do { if ((ptr) && (threadIdx.x & 63) == 0) \
    (ptr)[(threadIdx.x >> 6) * 8 + (ph)] = __builtin_amdgcn_s_memtime(); } while (0)

// per-workgroup start/end (100 MHz s_memrealtime, comparable across XCDs)
#define MX_TRACE_BLK(ptr, which) do { if ((ptr) && threadIdx.x == 0) \
    (ptr)[2 * (blockIdx.x + blockIdx.y * gridDim.x) + (which)] = __builtin_amdgcn_s_memrealtime(); } while (0)

// reductions over W lanes with the result in every lane
template <int W = MX_WAVE>
__device__ __forceinline__ float wave_sum(float v) {
    if constexpr (W == 64) return lane_bcast(dpp_sum_group<64>(v), 63);
    else if constexpr (W <= 16) return dpp_sum_group<W>(v);
    else {
#pragma unroll
        for (int o = W / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, W);
        return v;
    }
}
template <int W = MX_WAVE>
__device__ __forceinline__ float wave_max(float v) {
    if constexpr (W == 64) return lane_bcast(dpp_max_group<64>(v), 63);
    else if constexpr (W <= 16) return dpp_max_group<W>(v);
    else {
#pragma unroll
        for (int o = W / 2; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, W));
        return v;
    }
}
template <int W = MX_WAVE>
__device__ __forceinline__ int wave_sum_i(int v) {
    if constexpr (W == 64) return __builtin_amdgcn_readlane(dpp_sum_group_i<64>(v), 63);
    else if constexpr (W <= 16) return dpp_sum_group_i<W>(v);
    else {
#pragma unroll
        for (int o = W / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, W);
        return v;
    }
}

// block-wide sum for blockDim.x multiple of 64, <= 1024; lds >= 16 floats
__device__ __forceinline__ float block_sum(float v, float * lds) {
    v = wave_sum(v);
    const int nw = blockDim.x / MX_WAVE;
    if (nw == 1) return v;
    const int w = threadIdx.x / MX_WAVE, l = threadIdx.x % MX_WAVE;
    __syncthreads();
    if (l == 0) lds[w] = v;
    __syncthreads();
    v = (l & 15) < nw ? lds[l & 15] : 0.0f;  // every 16-lane segment holds all partials
    return wave_sum<16>(v);
}
__device__ __forceinline__ float block_max(float v, float * lds) {
    v = wave_max(v);
    const int nw = blockDim.x / MX_WAVE;
    if (nw == 1) return v;
    const int w = threadIdx.x / MX_WAVE, l = threadIdx.x % MX_WAVE;
    __syncthreads();
    if (l == 0) lds[w] = v;
    __syncthreads();
    v = (l & 15) < nw ? lds[l & 15] : -INFINITY;
    return wave_max<16>(v);
}

__device__ __forceinline__ float h2f(uint16_t h) { return __half2float(__ushort_as_half(h)); }
__device__ __forceinline__ uint16_t f2h(float f) { return __half_as_ushort(__float2half_rn(f)); }
__device__ __forceinline__ float bf2f(uint16_t h) { return __uint_as_float(((uint32_t) h) << 16); }
__device__ __forceinline__ uint16_t f2bf(float f) {  // round-to-nearest-even, NaN kept (ggml_compute_fp32_to_bf16)
    uint32_t u = __float_as_uint(f);
    if ((u & 0x7fffffff) > 0x7f800000) return (uint16_t) ((u >> 16) | 64);
    return (uint16_t) ((u + (0x7fff + ((u >> 16) & 1))) >> 16);
}

__device__ __forceinline__ int dot4_i8(int a, int b, int c) { return __builtin_amdgcn_sdot4(a, b, c, false); }

// The one q8 activation quantiser of the backend (every producer of a q8 activation uses
// it: GEMV prologues, the SwiGLU q8 emission, the fused RMS-norm q8 copy, the standalone
// quantiser, the decode-attention combine), so an activation quantises identically whatever
// path produced it. Semantics of quantize_q8_1 (ggml-cuda/quantize.cu:5-48): per 32 values
// d = amax/127, q = round(x/d). The reciprocal is 127 * v_rcp_f32(amax) and the rounding
// v_rndne_f32 (half to even): one instruction each instead of an IEEE division and roundf's
// half-away sequence; results differ from roundf(x * (1/d)) only at exact .5 ties and in
// the last ulp of 1/d.
struct Q8Scale { float d, id; };
__device__ __forceinline__ Q8Scale q8_scale(float amax) {
    return Q8Scale{amax / 127.0f, amax == 0.0f ? 0.0f : 127.0f * __builtin_amdgcn_rcpf(amax)};
}
__device__ __forceinline__ int q8_round(float x, float id) { return (int) __builtin_rintf(x * id); }

#endif  // __HIPCC__
