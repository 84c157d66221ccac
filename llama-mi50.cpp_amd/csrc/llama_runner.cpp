// llama_runner.cpp — drives Llama-family decode/prefill through the backend C-ABI.
//
// Mirrors the reference host path that produces the hot-path graph:
//   graph        src/models/llama.cpp:4-165 (llm_build_llama), build_attn
//                src/llama-graph.cpp:1918-1960, build_attn_mha :1675-1804,
//                build_ffn :960-1100, build_moe_ffn :1159-1380
//   KV cache     src/llama-kv-cache.cpp:1003-1161 (n_kv padded to 256, get_k/get_v
//                views, cpy_k/cpy_v via SET_ROWS; V transposed without flash-attn)
//   decode loop  src/llama-context.cpp:1117-1700 (ubatch split, inputs, logits D2H)
// Inputs of a ubatch live in one device buffer and are uploaded with one async copy
// from pinned memory; graphs are cached per (n_tokens, n_kv, n_outputs) so the
// backend sees an identical cgraph every decode step and replays its HIP graph.
#include "mx_llama.h"
#include "mx_graph.h"
#include "ggml_mi355x.h"
#include "backend.h"

#include <cmath>
#include <map>
#include <memory>
#include <string>
#include <vector>
#include <tuple>

namespace mx {
void fill_random_tensor(const ggml_tensor * t, uint64_t seed, hipStream_t st);
void fill_const_f32(const ggml_tensor * t, float v, hipStream_t st);
}

namespace {

struct Layer {
    ggml_tensor * attn_norm = nullptr, * wq = nullptr, * wk = nullptr, * wv = nullptr, * wo = nullptr;
    ggml_tensor * ffn_norm = nullptr, * gate = nullptr, * up = nullptr, * down = nullptr;
    ggml_tensor * gate_inp = nullptr, * gate_exps = nullptr, * up_exps = nullptr, * down_exps = nullptr;
};

// ---------------------------------------------------------------------------
// GGUF reader (format: gguf.cpp / gguf.h of the reference, v2/v3)
// ---------------------------------------------------------------------------
struct GgufTensor { std::string name; int type; int64_t ne[4]; uint64_t offset; };
struct Gguf {
    std::map<std::string, double> num;
    std::map<std::string, std::string> str;
    std::vector<GgufTensor> tensors;
    uint64_t data_off = 0;
    uint32_t alignment = 32;
};

bool rd(FILE * f, void * p, size_t n) { return fread(p, 1, n, f) == n; }
bool rd_str(FILE * f, std::string & s) {
    uint64_t n;
    if (!rd(f, &n, 8)) return false;
    s.resize(n);
    return n == 0 || rd(f, &s[0], n);
}
bool skip_val(FILE * f, uint32_t t, double * num, std::string * str);
bool read_scalar(FILE * f, uint32_t t, double * num) {
    switch (t) {
        case 0: { uint8_t v; if (!rd(f, &v, 1)) return false; *num = v; return true; }
        case 1: { int8_t v; if (!rd(f, &v, 1)) return false; *num = v; return true; }
        case 2: { uint16_t v; if (!rd(f, &v, 2)) return false; *num = v; return true; }
        case 3: { int16_t v; if (!rd(f, &v, 2)) return false; *num = v; return true; }
        case 4: { uint32_t v; if (!rd(f, &v, 4)) return false; *num = v; return true; }
        case 5: { int32_t v; if (!rd(f, &v, 4)) return false; *num = v; return true; }
        case 6: { float v; if (!rd(f, &v, 4)) return false; *num = v; return true; }
        case 7: { uint8_t v; if (!rd(f, &v, 1)) return false; *num = v; return true; }
        case 10: { uint64_t v; if (!rd(f, &v, 8)) return false; *num = (double) v; return true; }
        case 11: { int64_t v; if (!rd(f, &v, 8)) return false; *num = (double) v; return true; }
        case 12: { double v; if (!rd(f, &v, 8)) return false; *num = v; return true; }
        default: return false;
    }
}
bool skip_val(FILE * f, uint32_t t, double * num, std::string * str) {
    if (t == 8) return rd_str(f, *str);
    if (t == 9) {
        uint32_t it; uint64_t n;
        if (!rd(f, &it, 4) || !rd(f, &n, 8)) return false;
        *num = (double) n;  // arrays: remember the length (e.g. tokenizer.ggml.tokens)
        for (uint64_t i = 0; i < n; ++i) {
            double d; std::string s;
            if (it == 8) { if (!rd_str(f, s)) return false; }
            else if (it == 9) { if (!skip_val(f, 9, &d, &s)) return false; }
            else if (!read_scalar(f, it, &d)) return false;
        }
        return true;
    }
    return read_scalar(f, t, num);
}

bool gguf_read(const char * path, Gguf & g) {
    FILE * f = fopen(path, "rb");
    if (!f) return false;
    char magic[4];
    uint32_t ver; uint64_t nt, nkv;
    bool ok = rd(f, magic, 4) && memcmp(magic, "GGUF", 4) == 0 && rd(f, &ver, 4) && rd(f, &nt, 8) && rd(f, &nkv, 8);
    for (uint64_t i = 0; ok && i < nkv; ++i) {
        std::string key; uint32_t t; double num = 0; std::string s;
        ok = rd_str(f, key) && rd(f, &t, 4) && skip_val(f, t, &num, &s);
        if (ok) { if (t == 8) g.str[key] = s; else g.num[key] = num; }
    }
    for (uint64_t i = 0; ok && i < nt; ++i) {
        GgufTensor tt; uint32_t nd;
        ok = rd_str(f, tt.name) && rd(f, &nd, 4) && nd <= 4;
        for (int d = 0; d < 4; ++d) tt.ne[d] = 1;
        for (uint32_t d = 0; ok && d < nd; ++d) { uint64_t v; ok = rd(f, &v, 8); tt.ne[d] = (int64_t) v; }
        uint32_t ty = 0;
        ok = ok && rd(f, &ty, 4) && rd(f, &tt.offset, 8);
        tt.type = (int) ty;
        g.tensors.push_back(tt);
    }
    if (g.num.count("general.alignment")) g.alignment = (uint32_t) g.num["general.alignment"];
    const uint64_t pos = (uint64_t) ftell(f);
    g.data_off = (pos + g.alignment - 1) / g.alignment * g.alignment;
    fclose(f);
    return ok;
}

hipStream_t stream_of_backend(ggml_backend_t b) { return mx::stream_of(b)->stream; }

}  // namespace

struct mxr_model {
    ggml_backend_t be = nullptr;
    mxr_hparams hp{};
    int l0 = 0, l1 = 0;               // pipeline stage: layers [l0, l1) of hp.n_layer
    mxg_context * wctx = nullptr;
    ggml_tensor * tok_embd = nullptr, * out_norm = nullptr, * output = nullptr;
    std::vector<Layer> layers;
};

struct GraphInst {
    mxg_context * ctx = nullptr;     // intermediates
    mxg_context * ictx = nullptr;    // inputs (one buffer)
    ggml_cgraph * g = nullptr;
    ggml_tensor * tokens = nullptr, * pos = nullptr, * kidx = nullptr, * vidx = nullptr, * mask = nullptr, * out_ids = nullptr;
    ggml_tensor * logits = nullptr;
    ggml_tensor * hin = nullptr, * hout = nullptr;   // stage hand-off (pipeline layer split)
    char * in_base = nullptr; size_t in_bytes = 0;
    int n_tokens = 0, n_kv = 0, n_out = 0;
    uint64_t last_use = 0;
};

struct mxr_context {
    mxr_model * m = nullptr;
    int n_ctx = 0, n_ubatch = 512, fa = 1, pos = 0;
    mxg_context * kvctx = nullptr;
    std::vector<ggml_tensor *> kc, vc;
    std::vector<std::unique_ptr<GraphInst>> graphs;
    uint64_t tick = 0;
    // input staging: two pinned buffers in turn, each guarded by the event recorded after
    // its upload, so the host fills ubatch i+1's inputs while the GPU runs ubatch i (a
    // prompt's ubatches without logits are not synchronised one by one)
    char * h_in_buf[2] = {nullptr, nullptr}; size_t h_in_cap[2] = {0, 0};
    hipEvent_t h_in_ev[2] = {nullptr, nullptr};
    int h_in_k = 0;
    float * h_logits = nullptr; size_t h_logits_cap = 0;
};

// ---------------------------------------------------------------------------
// model construction
// ---------------------------------------------------------------------------
static bool use_more_bits(int i, int n) { return i < n / 8 || i >= 7 * n / 8 || (i - n / 8) % 3 == 2; }

static ggml_tensor * wt(mxr_model * m, const char * name, ggml_type t, int64_t ne0, int64_t ne1, int64_t ne2 = 1) {
    const int64_t ne[3] = {ne0, ne1, ne2};
    ggml_tensor * x = mxg_new_tensor(m->wctx, t, ne2 > 1 ? 3 : (ne1 > 1 ? 2 : 1), ne);
    mxg_set_name(x, name);
    return x;
}

static void create_weights(mxr_model * m, const char * recipe) {
    const mxr_hparams & h = m->hp;
    const std::string r = recipe ? recipe : "q4_k_m";
    ggml_type tmain = GGML_TYPE_Q4_K, tk = GGML_TYPE_Q4_K, tv = GGML_TYPE_Q4_K, tdown = GGML_TYPE_Q4_K, tout = GGML_TYPE_Q6_K,
              temb = GGML_TYPE_Q4_K;
    // llama_tensor_get_type's per-model rules (src/llama-quant.cpp:305-321): the 70B model
    // (LLM_TYPE_70B: 80 layers) takes attn_v Q4_K -> Q5_K; 8-expert models attn_k and
    // attn_v Q8_0
    const bool is70b = h.n_layer == 80 && h.n_expert == 0;
    const bool exp8 = h.n_expert == 8;
    const int hd = h.n_embd / h.n_head;
    const int nkv = hd * h.n_head_kv;
    m->tok_embd = nullptr;
    for (int i = m->l0; i < m->l1; ++i) {
        Layer L;
        char nm[96];
        const bool more = use_more_bits(i, h.n_layer);
        if (r == "q4_k_m") { tmain = GGML_TYPE_Q4_K; tv = tdown = more ? GGML_TYPE_Q6_K : GGML_TYPE_Q4_K; }
        else if (r == "q5_k_m") { tmain = GGML_TYPE_Q5_K; tv = tdown = more ? GGML_TYPE_Q6_K : GGML_TYPE_Q5_K; }
        else if (r == "q4_0") { tmain = tv = tdown = GGML_TYPE_Q4_0; tout = GGML_TYPE_Q6_K; temb = GGML_TYPE_Q4_0; }
        else if (r == "q8_0") { tmain = tv = tdown = tout = temb = GGML_TYPE_Q8_0; }
        else if (r == "f16") { tmain = tv = tdown = tout = temb = GGML_TYPE_F16; }
        else MX_ABORT("unknown recipe %s", r.c_str());
        tk = tmain;
        if (r == "q4_k_m" && is70b && tv == GGML_TYPE_Q4_K) tv = GGML_TYPE_Q5_K;
        if ((r == "q4_k_m" || r == "q5_k_m") && exp8) tk = tv = GGML_TYPE_Q8_0;
        snprintf(nm, sizeof nm, "blk.%d.attn_norm.weight", i); L.attn_norm = wt(m, nm, GGML_TYPE_F32, h.n_embd, 1);
        snprintf(nm, sizeof nm, "blk.%d.attn_q.weight", i); L.wq = wt(m, nm, tmain, h.n_embd, h.n_embd);
        snprintf(nm, sizeof nm, "blk.%d.attn_k.weight", i); L.wk = wt(m, nm, tk, h.n_embd, nkv);
        snprintf(nm, sizeof nm, "blk.%d.attn_v.weight", i); L.wv = wt(m, nm, tv, h.n_embd, nkv);
        snprintf(nm, sizeof nm, "blk.%d.attn_output.weight", i); L.wo = wt(m, nm, tmain, h.n_embd, h.n_embd);
        snprintf(nm, sizeof nm, "blk.%d.ffn_norm.weight", i); L.ffn_norm = wt(m, nm, GGML_TYPE_F32, h.n_embd, 1);
        if (h.n_expert > 0) {
            snprintf(nm, sizeof nm, "blk.%d.ffn_gate_inp.weight", i); L.gate_inp = wt(m, nm, GGML_TYPE_F32, h.n_embd, h.n_expert);
            snprintf(nm, sizeof nm, "blk.%d.ffn_gate_exps.weight", i); L.gate_exps = wt(m, nm, tmain, h.n_embd, h.n_ff, h.n_expert);
            snprintf(nm, sizeof nm, "blk.%d.ffn_up_exps.weight", i); L.up_exps = wt(m, nm, tmain, h.n_embd, h.n_ff, h.n_expert);
            snprintf(nm, sizeof nm, "blk.%d.ffn_down_exps.weight", i); L.down_exps = wt(m, nm, tdown, h.n_ff, h.n_embd, h.n_expert);
        } else {
            snprintf(nm, sizeof nm, "blk.%d.ffn_gate.weight", i); L.gate = wt(m, nm, tmain, h.n_embd, h.n_ff);
            snprintf(nm, sizeof nm, "blk.%d.ffn_up.weight", i); L.up = wt(m, nm, tmain, h.n_embd, h.n_ff);
            snprintf(nm, sizeof nm, "blk.%d.ffn_down.weight", i); L.down = wt(m, nm, tdown, h.n_ff, h.n_embd);
        }
        m->layers.push_back(L);
    }
    if (m->l0 == 0) m->tok_embd = wt(m, "token_embd.weight", temb, h.n_embd, h.n_vocab);
    if (m->l1 == h.n_layer) {
        m->out_norm = wt(m, "output_norm.weight", GGML_TYPE_F32, h.n_embd, 1);
        m->output = wt(m, "output.weight", tout, h.n_embd, h.n_vocab);
    }
}

extern "C" {

mxr_model * mxr_model_random_stage(ggml_backend_t be, const mxr_hparams * hp, const char * recipe, uint64_t seed,
                                   int32_t layer_begin, int32_t layer_end) {
    if (layer_begin < 0 || layer_end > hp->n_layer || layer_begin >= layer_end) return nullptr;
    auto * m = new mxr_model();
    m->be = be;
    m->hp = *hp;
    m->l0 = layer_begin;
    m->l1 = layer_end;
    if (m->hp.n_ctx_train <= 0) m->hp.n_ctx_train = 8192;
    m->wctx = mxg_init();
    create_weights(m, recipe);
    ggml_backend_buffer_type_t buft = be->device->iface.get_buffer_type(be->device);
    if (mxg_alloc(m->wctx, buft) != 0) { mxg_free(m->wctx); delete m; return nullptr; }
    hipStream_t st = stream_of_backend(be);
    // one seed per (layer, tensor): a stage holds exactly the weights of the same
    // layers of the whole model
    const uint64_t base = seed * 1000003ULL;
    auto fill = [&](ggml_tensor * t, bool norm, uint64_t slot) {
        if (!t) return;
        if (norm) mx::fill_const_f32(t, 1.0f, st);
        else mx::fill_random_tensor(t, base + slot, st);
    };
    fill(m->tok_embd, false, 1); fill(m->out_norm, true, 0); fill(m->output, false, 2);
    for (size_t k = 0; k < m->layers.size(); ++k) {
        const Layer & L = m->layers[k];
        const uint64_t b = 64 + 16 * (uint64_t) (m->l0 + k);
        fill(L.attn_norm, true, 0); fill(L.ffn_norm, true, 0);
        fill(L.wq, false, b + 0); fill(L.wk, false, b + 1); fill(L.wv, false, b + 2); fill(L.wo, false, b + 3);
        fill(L.gate, false, b + 4); fill(L.up, false, b + 5); fill(L.down, false, b + 6);
        fill(L.gate_inp, false, b + 7); fill(L.gate_exps, false, b + 8); fill(L.up_exps, false, b + 9); fill(L.down_exps, false, b + 10);
    }
    HIP_CHECK(hipStreamSynchronize(st));
    return m;
}

mxr_model * mxr_model_random(ggml_backend_t be, const mxr_hparams * hp, const char * recipe, uint64_t seed) {
    return mxr_model_random_stage(be, hp, recipe, seed, 0, hp->n_layer);
}

void mxr_model_stage(const mxr_model * m, int32_t * layer_begin, int32_t * layer_end) {
    *layer_begin = m->l0;
    *layer_end = m->l1;
}

mxr_model * mxr_model_load_gguf(ggml_backend_t be, const char * path) {
    Gguf g;
    if (!gguf_read(path, g)) { fprintf(stderr, "mxr: cannot parse %s\n", path); return nullptr; }
    const std::string arch = g.str.count("general.architecture") ? g.str["general.architecture"] : "llama";
    auto kv = [&](const std::string & k, double def) { auto it = g.num.find(arch + "." + k); return it == g.num.end() ? def : it->second; };
    auto * m = new mxr_model();
    m->be = be;
    mxr_hparams & h = m->hp;
    h.n_embd = (int) kv("embedding_length", 0);
    h.n_layer = (int) kv("block_count", 0);
    h.n_head = (int) kv("attention.head_count", 0);
    h.n_head_kv = (int) kv("attention.head_count_kv", h.n_head);
    h.n_ff = (int) kv("feed_forward_length", 0);
    h.n_ctx_train = (int) kv("context_length", 8192);
    h.rope_freq_base = (float) kv("rope.freq_base", 10000.0);
    h.norm_eps = (float) kv("attention.layer_norm_rms_epsilon", 1e-5);
    h.n_expert = (int) kv("expert_count", 0);
    h.n_expert_used = (int) kv("expert_used_count", 0);
    m->l0 = 0;
    m->l1 = h.n_layer;
    m->wctx = mxg_init();
    std::map<std::string, ggml_tensor *> byname;
    for (auto & t : g.tensors) {
        int nd = 1;
        for (int d = 1; d < 4; ++d) if (t.ne[d] > 1) nd = d + 1;
        ggml_tensor * x = mxg_new_tensor(m->wctx, (ggml_type) t.type, nd, t.ne);
        mxg_set_name(x, t.name.c_str());
        byname[t.name] = x;
    }
    auto get = [&](const std::string & n) -> ggml_tensor * { auto it = byname.find(n); return it == byname.end() ? nullptr : it->second; };
    m->tok_embd = get("token_embd.weight");
    m->out_norm = get("output_norm.weight");
    m->output = get("output.weight");
    if (!m->output) m->output = m->tok_embd;  // tied embeddings
    if (!m->tok_embd || !m->out_norm) { fprintf(stderr, "mxr: missing core tensors\n"); mxg_free(m->wctx); delete m; return nullptr; }
    h.n_vocab = (int) m->tok_embd->ne[1];
    for (int i = 0; i < h.n_layer; ++i) {
        Layer L;
        const std::string p = "blk." + std::to_string(i) + ".";
        L.attn_norm = get(p + "attn_norm.weight"); L.wq = get(p + "attn_q.weight"); L.wk = get(p + "attn_k.weight");
        L.wv = get(p + "attn_v.weight"); L.wo = get(p + "attn_output.weight"); L.ffn_norm = get(p + "ffn_norm.weight");
        L.gate = get(p + "ffn_gate.weight"); L.up = get(p + "ffn_up.weight"); L.down = get(p + "ffn_down.weight");
        L.gate_inp = get(p + "ffn_gate_inp.weight"); L.gate_exps = get(p + "ffn_gate_exps.weight");
        L.up_exps = get(p + "ffn_up_exps.weight"); L.down_exps = get(p + "ffn_down_exps.weight");
        if (!L.attn_norm || !L.wq || !L.wk || !L.wv || !L.wo || !L.ffn_norm) { fprintf(stderr, "mxr: layer %d incomplete\n", i); mxg_free(m->wctx); delete m; return nullptr; }
        m->layers.push_back(L);
    }
    ggml_backend_buffer_type_t buft = be->device->iface.get_buffer_type(be->device);
    if (mxg_alloc(m->wctx, buft) != 0) { mxg_free(m->wctx); delete m; return nullptr; }
    // stream the tensor data through a pinned staging buffer
    FILE * f = fopen(path, "rb");
    const size_t chunk = 64u << 20;
    void * stage = nullptr;
    HIP_CHECK(hipHostMalloc(&stage, chunk, hipHostMallocDefault));
    for (auto & t : g.tensors) {
        ggml_tensor * x = byname[t.name];
        const size_t n = mx_nbytes(x);
        fseeko(f, (off_t) (g.data_off + t.offset), SEEK_SET);
        for (size_t done = 0; done < n; done += chunk) {
            const size_t k = std::min(chunk, n - done);
            if (fread(stage, 1, k, f) != k) { fprintf(stderr, "mxr: short read %s\n", t.name.c_str()); fclose(f); return nullptr; }
            mxg_tensor_set(x, stage, done, k);
        }
    }
    fclose(f);
    HIP_CHECK(hipHostFree(stage));
    return m;
}

void mxr_model_free(mxr_model * m) {
    if (!m) return;
    mxg_free(m->wctx);
    delete m;
}

void mxr_model_hparams(const mxr_model * m, mxr_hparams * out) { *out = m->hp; }

static void add_bytes(const ggml_tensor * t, int64_t * acc, int64_t * by_type) {
    if (!t) return;
    const int64_t b = (int64_t) mx_nbytes(t);
    *acc += b;
    if (by_type) by_type[t->type] += b;
}

ggml_tensor * mxr_model_layer_tensor(const mxr_model * m, int32_t il, const char * which) {
    if (!m || il < m->l0 || il >= m->l1 || !which) return nullptr;
    const Layer & L = m->layers[il - m->l0];
    const std::string w = which;
    if (w == "attn_norm") return L.attn_norm;
    if (w == "attn_q") return L.wq;
    if (w == "attn_k") return L.wk;
    if (w == "attn_v") return L.wv;
    if (w == "attn_output") return L.wo;
    if (w == "ffn_norm") return L.ffn_norm;
    if (w == "ffn_gate") return L.gate;
    if (w == "ffn_up") return L.up;
    if (w == "ffn_down") return L.down;
    return nullptr;
}

int64_t mxr_model_decode_bytes(const mxr_model * m) {
    int64_t acc = 0;
    add_bytes(m->out_norm, &acc, nullptr);
    if (m->output) acc += (int64_t) mx_nbytes(m->output);   // (tied embeddings: read as the lm_head)
    for (auto & L : m->layers) {
        for (auto t : {L.attn_norm, L.wq, L.wk, L.wv, L.wo, L.ffn_norm, L.gate, L.up, L.down, L.gate_inp}) add_bytes(t, &acc, nullptr);
        if (L.gate_exps) {  // MoE: only n_expert_used of n_expert expert matrices are read per token
            for (auto t : {L.gate_exps, L.up_exps, L.down_exps})
                acc += (int64_t) mx_nbytes(t) / m->hp.n_expert * m->hp.n_expert_used;
        }
    }
    return acc;
}

void mxr_model_type_bytes(const mxr_model * m, int64_t out[GGML_TYPE_COUNT]) {
    for (int i = 0; i < GGML_TYPE_COUNT; ++i) out[i] = 0;
    int64_t acc = 0;
    add_bytes(m->output, &acc, out);
    add_bytes(m->out_norm, &acc, out);
    for (auto & L : m->layers)
        for (auto t : {L.attn_norm, L.wq, L.wk, L.wv, L.wo, L.ffn_norm, L.gate, L.up, L.down, L.gate_inp, L.gate_exps, L.up_exps, L.down_exps})
            add_bytes(t, &acc, out);
}

// ---------------------------------------------------------------------------
// context: KV cache + graphs
// ---------------------------------------------------------------------------
mxr_context * mxr_context_new(mxr_model * m, int32_t n_ctx, int32_t n_ubatch, int32_t flash_attn) {
    auto * c = new mxr_context();
    c->m = m;
    c->n_ctx = (n_ctx + 255) / 256 * 256;
    c->n_ubatch = n_ubatch > 0 ? n_ubatch : 512;
    c->fa = flash_attn;
    c->kvctx = mxg_init();
    const mxr_hparams & h = m->hp;
    const int nkv = h.n_embd / h.n_head * h.n_head_kv;
    for (int i = m->l0; i < m->l1; ++i) {
        char nm[64];
        snprintf(nm, sizeof nm, "cache_k_l%d", i);
        ggml_tensor * k = mxg_new_tensor_4d(c->kvctx, GGML_TYPE_F16, nkv, c->n_ctx, 1, 1);
        mxg_set_name(k, nm);
        snprintf(nm, sizeof nm, "cache_v_l%d", i);
        ggml_tensor * v = mxg_new_tensor_4d(c->kvctx, GGML_TYPE_F16, nkv, c->n_ctx, 1, 1);
        mxg_set_name(v, nm);
        c->kc.push_back(k);
        c->vc.push_back(v);
    }
    ggml_backend_buffer_type_t buft = m->be->device->iface.get_buffer_type(m->be->device);
    if (mxg_alloc(c->kvctx, buft) != 0) { mxg_free(c->kvctx); delete c; return nullptr; }
    c->kc[0]->buffer->iface.clear(c->kc[0]->buffer, 0);  // one buffer holds the whole cache
    return c;
}

void mxr_context_free(mxr_context * c) {
    if (!c) return;
    mxg_synchronize(c->m->be);   // a prompt's last ubatches may still run (decode_ubatch syncs only for outputs)
    for (auto & g : c->graphs) { mxg_free(g->ctx); mxg_free(g->ictx); }
    mxg_free(c->kvctx);
    for (int k = 0; k < 2; ++k) {
        if (c->h_in_ev[k]) (void) hipEventSynchronize(c->h_in_ev[k]);
        if (c->h_in_buf[k]) hipHostFree(c->h_in_buf[k]);
        if (c->h_in_ev[k]) hipEventDestroy(c->h_in_ev[k]);
    }
    if (c->h_logits) hipHostFree(c->h_logits);
    delete c;
}

void mxr_context_reset(mxr_context * c) { c->pos = 0; }
int32_t mxr_context_pos(const mxr_context * c) { return c->pos; }

}  // extern "C"

// llm_build_llama (+ build_attn / build_attn_mha / build_ffn / build_moe_ffn)
static GraphInst * build_graph(mxr_context * c, int n_tokens, int n_kv, int n_out) {
    mxr_model * m = c->m;
    const mxr_hparams & h = m->hp;
    const int hd = h.n_embd / h.n_head;
    const int nkv_embd = hd * h.n_head_kv;
    auto gi = std::make_unique<GraphInst>();
    gi->n_tokens = n_tokens; gi->n_kv = n_kv; gi->n_out = n_out;
    gi->ictx = mxg_init();
    gi->ctx = mxg_init();
    mxg_context * ictx = gi->ictx;
    mxg_context * ctx = gi->ctx;

    // inputs (llm_graph_input_*)
    gi->tokens = mxg_new_tensor_4d(ictx, GGML_TYPE_I32, n_tokens, 1, 1, 1); mxg_set_input(gi->tokens); mxg_set_name(gi->tokens, "inp_tokens");
    gi->pos = mxg_new_tensor_4d(ictx, GGML_TYPE_I32, n_tokens, 1, 1, 1); mxg_set_input(gi->pos); mxg_set_name(gi->pos, "inp_pos");
    gi->kidx = mxg_new_tensor_4d(ictx, GGML_TYPE_I64, n_tokens, 1, 1, 1); mxg_set_input(gi->kidx); mxg_set_name(gi->kidx, "inp_k_idxs");
    gi->vidx = mxg_new_tensor_4d(ictx, GGML_TYPE_I64, c->fa ? n_tokens : (int64_t) n_tokens * nkv_embd, 1, 1, 1);
    mxg_set_input(gi->vidx); mxg_set_name(gi->vidx, "inp_v_idxs");
    gi->mask = mxg_new_tensor_4d(ictx, GGML_TYPE_F32, n_kv, n_tokens, 1, 1); mxg_set_input(gi->mask); mxg_set_name(gi->mask, "inp_kq_mask");
    if (n_out < n_tokens) {
        gi->out_ids = mxg_new_tensor_4d(ictx, GGML_TYPE_I32, n_out, 1, 1, 1); mxg_set_input(gi->out_ids); mxg_set_name(gi->out_ids, "inp_out_ids");
    }

    const bool first = m->l0 == 0, last = m->l1 == h.n_layer;
    if (!first) {   // pipeline stage > 0: the previous stage's hidden state comes in
        gi->hin = mxg_new_tensor_4d(ictx, GGML_TYPE_F32, h.n_embd, n_tokens, 1, 1);
        mxg_set_input(gi->hin); mxg_set_name(gi->hin, "inp_embd");
    }
    ggml_tensor * inpL = first ? mxg_get_rows(ctx, m->tok_embd, gi->tokens) : gi->hin;
    ggml_tensor * kq_mask = c->fa ? mxg_cast(ctx, gi->mask, GGML_TYPE_F16) : gi->mask;
    const float kq_scale = 1.0f / sqrtf((float) hd);
    std::vector<ggml_tensor *> order;  // explicit expansion order (ggml_build_forward_expand calls)
    ggml_cgraph * g = nullptr;
    auto expand = [&](ggml_tensor * t) { if (!g) g = mxg_build(ctx, t); else mxg_expand(ctx, g, t); };

    for (int il = 0; il < (int) m->layers.size(); ++il) {
        const Layer & L = m->layers[il];
        const int il_global = m->l0 + il;
        ggml_tensor * inpSA = inpL;
        ggml_tensor * cur = mxg_binary(ctx, GGML_OP_MUL, mxg_rms_norm(ctx, inpL, h.norm_eps), L.attn_norm);
        ggml_tensor * Q = mxg_mul_mat(ctx, L.wq, cur);
        ggml_tensor * K = mxg_mul_mat(ctx, L.wk, cur);
        ggml_tensor * V = mxg_mul_mat(ctx, L.wv, cur);
        Q = mxg_reshape_4d(ctx, Q, hd, h.n_head, n_tokens, 1);
        K = mxg_reshape_4d(ctx, K, hd, h.n_head_kv, n_tokens, 1);
        V = mxg_reshape_4d(ctx, V, hd, h.n_head_kv, n_tokens, 1);
        Q = mxg_rope_ext(ctx, Q, gi->pos, nullptr, hd, GGML_ROPE_TYPE_NORMAL, h.n_ctx_train, h.rope_freq_base, 1.0f, 0.0f, 1.0f, 32.0f, 1.0f);
        K = mxg_rope_ext(ctx, K, gi->pos, nullptr, hd, GGML_ROPE_TYPE_NORMAL, h.n_ctx_train, h.rope_freq_base, 1.0f, 0.0f, 1.0f, 32.0f, 1.0f);
        // build_attn: q, v, k expanded first, then the cache stores
        expand(Q); expand(V); expand(K);
        ggml_tensor * kcache = c->kc[il], * vcache = c->vc[il];
        {
            ggml_tensor * k2 = mxg_view_4d(ctx, K, nkv_embd, n_tokens, 1, 1, K->nb[2], K->nb[2] * n_tokens, K->nb[2] * n_tokens, 0);
            expand(mxg_set_rows(ctx, kcache, k2, gi->kidx));
            if (c->fa) {
                ggml_tensor * v2 = mxg_view_4d(ctx, V, nkv_embd, n_tokens, 1, 1, V->nb[2], V->nb[2] * n_tokens, V->nb[2] * n_tokens, 0);
                expand(mxg_set_rows(ctx, vcache, v2, gi->vidx));
            } else {
                ggml_tensor * v2 = mxg_reshape_4d(ctx, V, nkv_embd, n_tokens, 1, 1);
                ggml_tensor * vview = mxg_reshape_4d(ctx, vcache, 1, mx_nelements(vcache), 1, 1);
                v2 = mxg_reshape_4d(ctx, v2, 1, mx_nelements(v2), 1, 1);
                expand(mxg_set_rows(ctx, vview, v2, gi->vidx));
            }
        }
        const size_t es = 2;  // f16 cache
        ggml_tensor * k = mxg_view_4d(ctx, kcache, hd, h.n_head_kv, n_kv, 1, es * hd, es * nkv_embd, es * nkv_embd * c->n_ctx, 0);
        ggml_tensor * v;
        if (c->fa) v = mxg_view_4d(ctx, vcache, hd, h.n_head_kv, n_kv, 1, es * hd, es * nkv_embd, es * nkv_embd * c->n_ctx, 0);
        else v = mxg_view_4d(ctx, vcache, n_kv, h.n_head_kv, hd, 1, es * c->n_ctx * hd, es * c->n_ctx, es * c->n_ctx * nkv_embd, 0);
        // build_attn_mha
        ggml_tensor * q = mxg_view_4d(ctx, Q, Q->ne[0], Q->ne[1], Q->ne[2], 1, Q->nb[1], Q->nb[2], Q->nb[3], 0);
        q = mxg_permute(ctx, q, 0, 2, 1, 3);
        k = mxg_permute(ctx, k, 0, 2, 1, 3);
        v = mxg_permute(ctx, v, 0, 2, 1, 3);
        if (c->fa) {
            cur = mxg_flash_attn_ext(ctx, q, k, v, kq_mask, kq_scale, 0.0f, 0.0f);
            cur = mxg_reshape_4d(ctx, cur, cur->ne[0] * cur->ne[1], cur->ne[2] * cur->ne[3], 1, 1);
        } else {
            ggml_tensor * kq = mxg_mul_mat(ctx, k, q);
            kq->op_params[0] = GGML_PREC_F32;  // ggml_mul_mat_set_prec
            kq = mxg_soft_max_ext(ctx, kq, kq_mask, kq_scale, 0.0f);
            ggml_tensor * kqv = mxg_mul_mat(ctx, v, kq);
            cur = mxg_permute(ctx, kqv, 0, 2, 1, 3);
            cur = mxg_cont_4d(ctx, cur, cur->ne[0] * cur->ne[1], cur->ne[2] * cur->ne[3], 1, 1);
        }
        expand(cur);
        cur = mxg_mul_mat(ctx, L.wo, cur);
        if (il_global == h.n_layer - 1 && gi->out_ids) {
            cur = mxg_get_rows(ctx, cur, gi->out_ids);
            inpSA = mxg_get_rows(ctx, inpSA, gi->out_ids);
        }
        ggml_tensor * ffn_inp = mxg_binary(ctx, GGML_OP_ADD, cur, inpSA);
        cur = mxg_binary(ctx, GGML_OP_MUL, mxg_rms_norm(ctx, ffn_inp, h.norm_eps), L.ffn_norm);
        if (!L.gate_exps) {
            ggml_tensor * up = mxg_mul_mat(ctx, L.up, cur);
            ggml_tensor * gate = mxg_mul_mat(ctx, L.gate, cur);
            cur = mxg_glu_split(ctx, gate, up, GGML_GLU_OP_SWIGLU);
            cur = mxg_mul_mat(ctx, L.down, cur);
        } else {
            // build_moe_ffn, softmax gating, weights normalised (Mixtral)
            const int64_t nt = cur->ne[1];
            ggml_tensor * logits = mxg_mul_mat(ctx, L.gate_inp, cur);                       // [n_expert, nt]
            ggml_tensor * probs = mxg_soft_max_ext(ctx, logits, nullptr, 1.0f, 0.0f);
            ggml_tensor * sorted = mxg_argsort(ctx, probs, GGML_SORT_ORDER_DESC);
            ggml_tensor * sel = mxg_view_4d(ctx, sorted, h.n_expert_used, nt, 1, 1, sorted->nb[1], sorted->nb[1] * nt, sorted->nb[1] * nt, 0);
            ggml_tensor * w = mxg_get_rows(ctx, mxg_reshape_4d(ctx, probs, 1, h.n_expert, nt, 1), sel);  // [1, n_used, nt]
            ggml_tensor * wsum = mxg_sum_rows(ctx, mxg_reshape_4d(ctx, w, h.n_expert_used, nt, 1, 1));
            wsum = mxg_clamp(ctx, wsum, 6.103515625e-5f, INFINITY);
            w = mxg_binary(ctx, GGML_OP_DIV, mxg_reshape_4d(ctx, w, h.n_expert_used, nt, 1, 1), wsum);
            w = mxg_reshape_4d(ctx, w, 1, h.n_expert_used, nt, 1);
            ggml_tensor * x3 = mxg_reshape_4d(ctx, cur, h.n_embd, 1, nt, 1);
            ggml_tensor * up = mxg_mul_mat_id(ctx, L.up_exps, x3, sel);
            ggml_tensor * gate = mxg_mul_mat_id(ctx, L.gate_exps, x3, sel);
            ggml_tensor * par = mxg_glu_split(ctx, gate, up, GGML_GLU_OP_SWIGLU);
            ggml_tensor * experts = mxg_mul_mat_id(ctx, L.down_exps, par, sel);        // [n_embd, n_used, nt]
            experts = mxg_binary(ctx, GGML_OP_MUL, experts, w);
            ggml_tensor * moe = nullptr;
            for (int e = 0; e < h.n_expert_used; ++e) {
                ggml_tensor * ev = mxg_view_4d(ctx, experts, h.n_embd, nt, 1, 1, experts->nb[2], experts->nb[2] * nt, experts->nb[2] * nt, e * experts->nb[1]);
                moe = moe ? mxg_binary(ctx, GGML_OP_ADD, moe, ev) : ev;
            }
            cur = moe;
        }
        cur = mxg_binary(ctx, GGML_OP_ADD, cur, ffn_inp);
        inpL = cur;
    }
    if (last) {
        ggml_tensor * cur = mxg_binary(ctx, GGML_OP_MUL, mxg_rms_norm(ctx, inpL, h.norm_eps), m->out_norm);
        cur = mxg_mul_mat(ctx, m->output, cur);
        mxg_set_output(cur);
        gi->logits = cur;
        expand(cur);
    } else {        // hand the hidden state to the next stage
        mxg_set_output(inpL);
        gi->hout = inpL;
        expand(inpL);
    }
    gi->g = g;
    // no CPU fallback in this driver: every node must be supported by the device
    for (int i = 0; i < g->n_nodes; ++i) {
        if (!m->be->device->iface.supports_op(m->be->device, g->nodes[i])) {
            fprintf(stderr, "mxr: node %d (%s, op %d, type %d) is not supported by the MI355X backend\n",
                    i, g->nodes[i]->name, (int) g->nodes[i]->op, (int) g->nodes[i]->type);
            mxg_free(gi->ctx); mxg_free(gi->ictx);
            return nullptr;
        }
    }

    ggml_backend_buffer_type_t buft = m->be->device->iface.get_buffer_type(m->be->device);
    if (mxg_alloc(ictx, buft) != 0 || mxg_alloc(ctx, buft) != 0) return nullptr;
    // inputs are contiguous in one buffer: remember base + extent
    gi->in_base = (char *) gi->tokens->data;
    char * end = gi->in_base;
    for (ggml_tensor * t : {gi->tokens, gi->pos, gi->kidx, gi->vidx, gi->mask, gi->out_ids}) {   // hin: device hand-off, not staged
        if (!t) continue;
        MX_ASSERT((char *) t->data >= gi->in_base);
        end = std::max(end, (char *) t->data + mx_nbytes(t));
    }
    gi->in_bytes = (size_t) (end - gi->in_base);
    GraphInst * raw = gi.get();
    c->graphs.push_back(std::move(gi));
    return raw;
}

// Graph instances are cached by shape (n_tokens, n_kv, n_out); each holds its own
// intermediates and inputs (no buffer sharing between instances: one graph per shape can be
// replayed without re-planning). Bounded by count AND bytes: GGML_MI355X_RUNNER_GRAPHS (default
// 6 — a pp2048 prompt alone has 4 shapes, n_kv 512 .. 2048) and GGML_MI355X_RUNNER_GRAPH_MB
// (default 32768). Llama-3-8B pp512 ubatch ≈ 4.4 GB per instance, 70B ≈ 22 GB: at 70B the
// byte bound keeps one or two.
static size_t runner_env(const char * name, size_t dflt) {
    const char * v = getenv(name);
    return v && *v ? (size_t) strtoull(v, nullptr, 10) : dflt;
}

static GraphInst * get_graph(mxr_context * c, int n_tokens, int n_kv, int n_out) {
    for (auto & g : c->graphs)
        if (g->n_tokens == n_tokens && g->n_kv == n_kv && g->n_out == n_out) { g->last_use = ++c->tick; return g.get(); }
    static const size_t max_n = std::max<size_t>(1, runner_env("GGML_MI355X_RUNNER_GRAPHS", 6));
    static const size_t max_b = runner_env("GGML_MI355X_RUNNER_GRAPH_MB", 32768) << 20;
    auto evict_lru = [&](const GraphInst * keep) {
        size_t victim = SIZE_MAX;
        for (size_t i = 0; i < c->graphs.size(); ++i)
            if (c->graphs[i].get() != keep && (victim == SIZE_MAX || c->graphs[i]->last_use < c->graphs[victim]->last_use)) victim = i;
        if (victim == SIZE_MAX) return false;
        mxg_synchronize(c->m->be);
        mxg_free(c->graphs[victim]->ctx);
        mxg_free(c->graphs[victim]->ictx);
        c->graphs.erase(c->graphs.begin() + victim);
        return true;
    };
    while (c->graphs.size() >= max_n && evict_lru(nullptr)) {}
    GraphInst * g = build_graph(c, n_tokens, n_kv, n_out);
    if (!g) return g;
    g->last_use = ++c->tick;
    auto bytes = [&] {
        size_t b = 0;
        for (auto & x : c->graphs) b += mxg_alloc_bytes(x->ctx) + mxg_alloc_bytes(x->ictx);
        return b;
    };
    while (c->graphs.size() > 1 && bytes() > max_b && evict_lru(g)) {}
    return g;
}

static int32_t decode_ubatch(mxr_context * c, const int32_t * tokens, int n_tokens, bool all_logits, float * out,
                             const void * h_in = nullptr, void * h_out = nullptr) {
    const mxr_hparams & h = c->m->hp;
    if (c->pos + n_tokens > c->n_ctx) return -1;
    const int used = c->pos + n_tokens;
    const int n_kv = std::min(c->n_ctx, std::max(256, (used + 255) / 256 * 256));
    const int n_out = all_logits ? n_tokens : 1;
    GraphInst * g = get_graph(c, n_tokens, n_kv, n_out);
    if (!g) return -2;
    // host staging (pinned) laid out exactly like the device input buffer; this buffer's
    // previous upload (two ubatches ago) must have completed before it is rewritten
    const int hk = c->h_in_k;
    c->h_in_k ^= 1;
    if (c->h_in_ev[hk]) HIP_CHECK(hipEventSynchronize(c->h_in_ev[hk]));
    else HIP_CHECK(hipEventCreateWithFlags(&c->h_in_ev[hk], hipEventDisableTiming));
    if (c->h_in_cap[hk] < g->in_bytes) {
        if (c->h_in_buf[hk]) HIP_CHECK(hipHostFree(c->h_in_buf[hk]));
        HIP_CHECK(hipHostMalloc((void **) &c->h_in_buf[hk], g->in_bytes, hipHostMallocDefault));
        c->h_in_cap[hk] = g->in_bytes;
    }
    char * h_stage = c->h_in_buf[hk];
    auto at = [&](ggml_tensor * t) { return h_stage + ((char *) t->data - g->in_base); };
    if (tokens) memcpy(at(g->tokens), tokens, n_tokens * sizeof(int32_t));
    else memset(at(g->tokens), 0, n_tokens * sizeof(int32_t));   // later pipeline stages: unused
    int32_t * pos = (int32_t *) at(g->pos);
    int64_t * kidx = (int64_t *) at(g->kidx);
    for (int i = 0; i < n_tokens; ++i) { pos[i] = c->pos + i; kidx[i] = c->pos + i; }
    int64_t * vidx = (int64_t *) at(g->vidx);
    if (c->fa) {
        for (int i = 0; i < n_tokens; ++i) vidx[i] = c->pos + i;
    } else {
        // transposed V: element (token i, dim j) goes to cell j*n_ctx + pos (llama-kv-cache.cpp set_input_v_idxs)
        const int nkv_embd = h.n_embd / h.n_head * h.n_head_kv;
        for (int i = 0; i < n_tokens; ++i)
            for (int j = 0; j < nkv_embd; ++j) vidx[(int64_t) i * nkv_embd + j] = (int64_t) j * c->n_ctx + c->pos + i;
    }
    float * mask = (float *) at(g->mask);
    for (int i = 0; i < n_tokens; ++i)
        for (int j = 0; j < n_kv; ++j) mask[(int64_t) i * n_kv + j] = (j <= c->pos + i) ? 0.0f : -INFINITY;
    if (g->out_ids) ((int32_t *) at(g->out_ids))[0] = n_tokens - 1;
    ggml_backend_t be = c->m->be;
    be->iface.set_tensor_async(be, g->tokens, h_stage, 0, g->in_bytes);
    hipStream_t st_be = stream_of_backend(be);
    HIP_CHECK(hipEventRecord(c->h_in_ev[hk], st_be));
    if (g->hin) {   // previous stage's hidden state (device or host pointer)
        if (!h_in) return -4;
        HIP_CHECK(hipMemcpyAsync(g->hin->data, h_in, mx_nbytes(g->hin), hipMemcpyDefault, st_be));
    }
    ggml_status st = be->iface.graph_compute(be, g->g);
    if (st != GGML_STATUS_SUCCESS) return -3;
    if (g->hout && h_out) HIP_CHECK(hipMemcpyAsync(h_out, g->hout->data, mx_nbytes(g->hout), hipMemcpyDefault, st_be));
    const size_t lbytes = (size_t) n_out * h.n_vocab * sizeof(float);
    if (out && g->logits) {
        if (c->h_logits_cap < lbytes) {
            if (c->h_logits) HIP_CHECK(hipHostFree(c->h_logits));
            HIP_CHECK(hipHostMalloc((void **) &c->h_logits, lbytes, hipHostMallocDefault));
            c->h_logits_cap = lbytes;
        }
        be->iface.get_tensor_async(be, g->logits, c->h_logits, 0, lbytes);
    }
    // results the caller reads (logits, the hand-off hidden state) need the stream done;
    // a prompt ubatch without outputs returns at once
    if ((out && g->logits) || (g->hout && h_out)) mxg_synchronize(be);
    if (out && g->logits) memcpy(out, c->h_logits, lbytes);
    c->pos += n_tokens;
    return 0;
}

extern "C" {

int32_t mxr_decode(mxr_context * c, const int32_t * tokens, int32_t n_tokens, float * logits) {
    for (int i = 0; i < n_tokens; i += c->n_ubatch) {
        const int n = std::min(c->n_ubatch, n_tokens - i);
        const bool last = i + n >= n_tokens;
        int32_t r = decode_ubatch(c, tokens + i, n, false, last ? logits : nullptr);
        if (r != 0) return r;
    }
    return 0;
}

int32_t mxr_decode_stage(mxr_context * c, const int32_t * tokens, const void * h_in, int32_t n_tokens, void * h_out,
                         float * logits) {
    if (n_tokens > c->n_ubatch) return -5;
    return decode_ubatch(c, tokens, n_tokens, false, logits, h_in, h_out);
}

int32_t mxr_decode_all_logits(mxr_context * c, const int32_t * tokens, int32_t n_tokens, float * logits) {
    const int nv = c->m->hp.n_vocab;
    for (int i = 0; i < n_tokens; i += c->n_ubatch) {
        const int n = std::min(c->n_ubatch, n_tokens - i);
        int32_t r = decode_ubatch(c, tokens + i, n, true, logits ? logits + (int64_t) i * nv : nullptr);
        if (r != 0) return r;
    }
    return 0;
}

}  // extern "C"
