/*
 * mx_llama.h — decode/prefill driver for Llama-family GGUF models over the
 * MI355X backend. Host-side counterpart of the reference's libllama path that
 * feeds the backend (src/llama-context.cpp:1117-1700 process_ubatch/decode;
 * graph src/models/llama.cpp:4-165; KV cache src/llama-kv-cache.cpp:1000-1170):
 * it builds the same ggml node graph and hands it to backend_i.graph_compute.
 * Used by bench.py and the end-to-end tests; not a replacement for libllama.
 */
#pragma once

#include "ggml_abi.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct mxr_hparams {
    int32_t n_vocab, n_embd, n_layer, n_head, n_head_kv, n_ff, n_ctx_train;
    int32_t n_expert, n_expert_used;   /* 0 = dense FFN */
    float   rope_freq_base, norm_eps;
} mxr_hparams;

typedef struct mxr_model mxr_model;
typedef struct mxr_context mxr_context;

/* Synthetic weights of the given shape generated on the device.
 * recipe: "q4_k_m" (Q4_K + Q6_K for attn_v/ffn_down on use_more_bits layers and
 * output, src/llama-quant.cpp:185-187,302-303,358-365), "q4_0", "q5_k_m", "q8_0", "f16". */
mxr_model * mxr_model_random(ggml_backend_t backend, const mxr_hparams * hp, const char * recipe, uint64_t seed);
/* Pipeline stage of the same model: layers [layer_begin, layer_end) only (token_embd with
 * the first stage, output_norm/output with the last). Weights are seeded per (layer,
 * tensor), so the stages of a split hold exactly the layers of mxr_model_random's model
 * (the layer split of src/llama-model.cpp:2599-2609 across processes/GPUs). */
mxr_model * mxr_model_random_stage(ggml_backend_t backend, const mxr_hparams * hp, const char * recipe, uint64_t seed,
                                   int32_t layer_begin, int32_t layer_end);
void        mxr_model_stage(const mxr_model * m, int32_t * layer_begin, int32_t * layer_end);
/* Weights from a GGUF file (llama architecture) */
mxr_model * mxr_model_load_gguf(ggml_backend_t backend, const char * path);
void        mxr_model_free(mxr_model * m);
void        mxr_model_hparams(const mxr_model * m, mxr_hparams * out);
/* bytes of all weights a decode step reads (every tensor except token_embd) */
int64_t     mxr_model_decode_bytes(const mxr_model * m);
/* weight of layer il by GGUF role ("attn_q", "attn_k", "attn_v", "attn_output",
 * "ffn_gate", "ffn_up", "ffn_down", "attn_norm", "ffn_norm"); NULL if absent */
struct ggml_tensor * mxr_model_layer_tensor(const mxr_model * m, int32_t il, const char * which);
/* bytes per weight type id (index = ggml_type), for reporting */
void        mxr_model_type_bytes(const mxr_model * m, int64_t out[GGML_TYPE_COUNT]);

mxr_context * mxr_context_new(mxr_model * m, int32_t n_ctx, int32_t n_ubatch, int32_t flash_attn);
void          mxr_context_free(mxr_context * c);
void          mxr_context_reset(mxr_context * c);   /* clear the KV cache (position 0) */
int32_t       mxr_context_pos(const mxr_context * c);

/* Evaluate n_tokens at the current position (split into ubatches). If logits is not
 * NULL the logits of the last token are copied there (n_vocab floats).
 * Returns 0 on success. Blocks until the device finished (llama_decode + synchronize). */
int32_t mxr_decode(mxr_context * c, const int32_t * tokens, int32_t n_tokens, float * logits);
/* all-token logits variant (n_tokens x n_vocab), for parity tests */
/* One ubatch through this stage: the first stage reads `tokens`, later ones the previous
 * stage's hidden state `h_in` (f32 [n_tokens][n_embd], device or host pointer); a
 * non-last stage writes its hidden state to `h_out`, the last one the last token's
 * logits. Synchronous. */
int32_t mxr_decode_stage(mxr_context * c, const int32_t * tokens, const void * h_in, int32_t n_tokens, void * h_out,
                         float * logits);
int32_t mxr_decode_all_logits(mxr_context * c, const int32_t * tokens, int32_t n_tokens, float * logits);

#ifdef __cplusplus
}
#endif
