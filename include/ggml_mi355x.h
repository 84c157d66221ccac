/*
 * ggml_mi355x.h — exported entry points of libggml-mi355x.so, the MI355X-native
 * ggml backend. The reference loads it unmodified through its dynamic-backend
 * loader; each symbol names the reference interface it stands in for.
 */
#pragma once

#include "ggml_abi.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Dynamic-backend entry point looked up with dlsym by load_backend()
 * (ggml/src/ggml-backend-reg.cpp:194-238; typedef ggml_backend_init_t,
 * ggml/src/ggml-backend-impl.h:222). Returns the registry; api_version == 2. */
ggml_backend_reg_t ggml_backend_init(void);

/* Optional score (ggml_backend_score_t, ggml-backend-impl.h:225): 0 when no
 * HIP device is visible, so the loader skips the library (reg.cpp:207-213). */
int ggml_backend_score(void);

/* Static registration form of the above, the counterpart of
 * ggml_backend_cuda_reg() (ggml/include/ggml-cuda.h, ggml-cuda.cu:5043). */
ggml_backend_reg_t ggml_backend_mi355x_reg(void);

/* Direct stream creation, counterpart of ggml_backend_cuda_init(int device)
 * (ggml-cuda.cu:5100). */
ggml_backend_t ggml_backend_mi355x_init(int device);

/* ggml_backend_cuda_get_device_count() counterpart. */
int ggml_backend_mi355x_get_device_count(void);

/* ggml_backend_is_cuda() counterpart. */
bool ggml_backend_is_mi355x(ggml_backend_t backend);

/* ggml_backend_cuda_buffer_type(int device) counterpart. */
ggml_backend_buffer_type_t ggml_backend_mi355x_buffer_type(int device);

/* Executor counters: [graph_compute calls, HIP-graph replays, nodes run, nodes fused]. */
void ggml_backend_mi355x_stats(ggml_backend_t backend, uint64_t out[4]);

/* Staged small writes of one device: [writes staged, flush launches, queued writes dropped
   because their buffer was freed before a flush]. */
void ggml_backend_mi355x_stage_stats(int device, uint64_t out[3]);

#ifdef __cplusplus
}
#endif

#ifdef __cplusplus
extern "C" {
#endif
/* Profiling hook (bench roofline): average µs of one launch of the decode GEMV that
 * MUL_MAT(w[i], x) (w2 == NULL) or the fused gate/up SWIGLU (w2[i] = up weight) runs,
 * timed with HIP events on `backend`'s stream over `iters` back-to-back launches that
 * cycle over the n_w weight sets (pass every layer's weights to stream from HBM). */
double ggml_backend_mi355x_time_mmvq(ggml_backend_t backend, const struct ggml_tensor * const * w,
                                     const struct ggml_tensor * const * w2, int n_w,
                                     const struct ggml_tensor * x, struct ggml_tensor * dst, int iters);
/* Tuning knobs for A/B runs and sweeps (0 = the built-in choice; every knob is documented
 * at its g_tune[idx] use in the sources, e.g. 17 prefill GEMM choice, 20 forced split-K,
 * 23 FA weight-prefetch MB). The same knobs can be set for a whole process through
 * GGML_MI355X_TUNE="idx=val,idx=val". Timing variants and debug masks only act in an A/B
 * variant build (ggml_backend_mi355x_ab_variants). */
void ggml_backend_mi355x_set_tune(int idx, int value);
/* 1 when this library is an A/B variant build (MX_AB_VARIANTS: the experiment-only code
 * paths the tuning knobs reach), 0 for the product library */
int ggml_backend_mi355x_ab_variants(void);
/* Debug: phase timestamps (s_memtime) of the first workgroup of the instrumented kernels,
 * recorded while tune index 6 is set: slot s (0 decode flash-attn, 1 GEMV, 2 QKV) at
 * out[s*128 + wave*8 + phase]. Read-and-clear; returns n or -1. */
int ggml_backend_mi355x_trace_read(unsigned long long * out, int n);
/* Debug: {start, end} s_memrealtime (100 MHz) of every workgroup of the last GEMV launch
 * recorded while tune index 6 == 2, at out[2*block]. Read-and-clear; returns n or -1. */
int ggml_backend_mi355x_trace_blocks_read(unsigned long long * out, int n);
/* Kernel-choice log: while on, every launch site of the hot-path kernels appends one line
 * naming the kernel and the geometry it picked (e.g. "gemv2 qt=12 lpr=16 upl=2 epi=1 w=8
 * mode=4 ..."), so tests can assert which instantiation ran at a shape. on != 0 clears and
 * starts it, 0 stops it. */
void ggml_backend_mi355x_klog(int on);
/* Copies the log (NUL-terminated, at most n - 1 bytes); returns its full length. */
size_t ggml_backend_mi355x_klog_read(char * out, size_t n);
#ifdef __cplusplus
}
#endif
