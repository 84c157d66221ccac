// state_probe.cpp — KV-cache state save / restore through a backend (TEST INFRASTRUCTURE,
// not part of the product). Built against the reference's own libllama + ggml
// (oracle/_ref, oracle/Makefile); the process loads libggml-mi355x.so through
// GGML_BACKEND_PATH like any reference tool.
//
// llama_state_seq_get_data / llama_state_seq_set_data (src/llama-context.cpp:3416-3431,
// the kv cache's state_write / state_read, src/llama-kv-cache.cpp:1648-1867) move raw KV
// bytes through the backend's get_tensor / set_tensor; llama_state_save_file /
// llama_state_load_file the whole context state. The probe:
//   A  GPU context: prompt, blob_a = seq 0 state, state file, then the generation tokens
//      one by one -> logits_a (the uninterrupted run)
//   B  fresh GPU context: set_data(blob_a), blob_b = get_data (round trip), generation
//      -> logits_b (must equal logits_a bit for bit)
//   F  fresh GPU context: load the state file, generation -> logits_f (bit-equal again)
//   C  CPU context (n_gpu_layers 0, KV on the host, no op offload): prompt, blob_c, then
//      generation -> logits_c (the reference's own uninterrupted run)
//   D  CPU context: set_data(blob_a) (GPU state into the CPU), generation -> logits_d
//   E  GPU context: set_data(blob_c) (CPU state into the GPU), generation -> logits_e
// Everything is written to --out; tests/test_dropin_gpu.py compares.
//
//   state-probe -m model.gguf -fa 1 [-ctk type] [-ctv type] --prompt p.i32 --gen g.i32 --out dir
#include "llama.h"
#include "ggml-backend.h"

#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

static std::vector<int32_t> read_i32(const std::string & p) {
    std::vector<int32_t> v;
    FILE * f = fopen(p.c_str(), "rb");
    if (!f) return v;
    int32_t t;
    while (fread(&t, 4, 1, f) == 1) v.push_back(t);
    fclose(f);
    return v;
}

static void write_bytes(const std::string & p, const void * d, size_t n) {
    FILE * f = fopen(p.c_str(), "wb");
    fwrite(d, 1, n, f);
    fclose(f);
}

int main(int argc, char ** argv) {
    std::string model, prompt_f, gen_f, out;
    int fa = 1, ctk = -1, ctv = -1;
    for (int i = 1; i < argc; ++i) {
        std::string a = argv[i];
        auto next = [&]() { return std::string(argv[++i]); };
        if (a == "-m") model = next();
        else if (a == "-fa") fa = std::stoi(next());
        else if (a == "-ctk") ctk = std::stoi(next());
        else if (a == "-ctv") ctv = std::stoi(next());   // V cache type alone (K q8_0 + V f16)
        else if (a == "--prompt") prompt_f = next();
        else if (a == "--gen") gen_f = next();
        else if (a == "--out") out = next();
    }
    const std::vector<int32_t> prompt = read_i32(prompt_f), gen = read_i32(gen_f);
    if (prompt.empty() || gen.empty() || out.empty()) { fprintf(stderr, "usage\n"); return 2; }
    llama_log_set([](ggml_log_level, const char *, void *) {}, nullptr);
    llama_backend_init();
    ggml_backend_load_all();

    llama_model_params mpg = llama_model_default_params();
    mpg.n_gpu_layers = 99;
    llama_model * mg = llama_model_load_from_file(model.c_str(), mpg);
    llama_model_params mpc = llama_model_default_params();
    mpc.n_gpu_layers = 0;
    static ggml_backend_dev_t no_gpu[1] = {nullptr};   // the CPU model offloads to no device
    mpc.devices = no_gpu;
    llama_model * mc = llama_model_load_from_file(model.c_str(), mpc);
    if (!mg || !mc) { fprintf(stderr, "load failed\n"); return 1; }
    const int n_vocab = llama_vocab_n_tokens(llama_model_get_vocab(mg));

    auto mkctx = [&](llama_model * m, bool gpu) {
        llama_context_params cp = llama_context_default_params();
        cp.n_ctx = 256;
        cp.n_batch = cp.n_ubatch = 256;
        cp.n_threads = cp.n_threads_batch = 8;
        cp.flash_attn_type = fa ? LLAMA_FLASH_ATTN_TYPE_ENABLED : LLAMA_FLASH_ATTN_TYPE_DISABLED;
        if (ctk >= 0) { cp.type_k = (ggml_type) ctk; cp.type_v = (ggml_type) ctk; }
        if (ctv >= 0) cp.type_v = (ggml_type) ctv;
        cp.offload_kqv = gpu;
        cp.op_offload = gpu;
        cp.no_perf = true;
        return llama_init_from_model(m, cp);
    };
    auto run_prompt = [&](llama_context * c) {
        llama_batch b = llama_batch_init((int) prompt.size(), 0, 1);
        for (size_t i = 0; i < prompt.size(); ++i) {
            b.token[i] = prompt[i]; b.pos[i] = (llama_pos) i; b.n_seq_id[i] = 1; b.seq_id[i][0] = 0;
            b.logits[i] = i + 1 == prompt.size();
        }
        b.n_tokens = (int) prompt.size();
        const int rc = llama_decode(c, b);
        llama_synchronize(c);
        llama_batch_free(b);
        return rc;
    };
    auto run_gen = [&](llama_context * c, const std::string & tag) {
        std::vector<float> lg;
        for (size_t i = 0; i < gen.size(); ++i) {
            llama_batch b = llama_batch_init(1, 0, 1);
            b.token[0] = gen[i]; b.pos[0] = (llama_pos) (prompt.size() + i); b.n_seq_id[0] = 1; b.seq_id[0][0] = 0;
            b.logits[0] = 1; b.n_tokens = 1;
            if (llama_decode(c, b) != 0) { fprintf(stderr, "decode %s failed\n", tag.c_str()); exit(1); }
            llama_synchronize(c);
            const float * l = llama_get_logits_ith(c, -1);
            lg.insert(lg.end(), l, l + n_vocab);
            llama_batch_free(b);
        }
        write_bytes(out + "/logits_" + tag + ".f32", lg.data(), lg.size() * 4);
    };
    auto get_blob = [&](llama_context * c, const std::string & tag) {
        std::vector<uint8_t> blob(llama_state_seq_get_size(c, 0));
        const size_t n = llama_state_seq_get_data(c, blob.data(), blob.size(), 0);
        blob.resize(n);
        write_bytes(out + "/blob_" + tag + ".bin", blob.data(), blob.size());
        return blob;
    };

    // A: the uninterrupted GPU run, its state after the prompt
    llama_context * a = mkctx(mg, true);
    if (run_prompt(a) != 0) { fprintf(stderr, "prompt A failed\n"); return 1; }
    std::vector<uint8_t> blob_a = get_blob(a, "a");
    const std::string sf = out + "/state_a.bin";
    std::vector<llama_token> ptoks(prompt.begin(), prompt.end());
    const bool saved = llama_state_save_file(a, sf.c_str(), ptoks.data(), ptoks.size());
    run_gen(a, "a");
    llama_free(a);
    // B: restore into a fresh GPU context
    llama_context * b = mkctx(mg, true);
    const size_t nb = llama_state_seq_set_data(b, blob_a.data(), blob_a.size(), 0);
    get_blob(b, "b");
    run_gen(b, "b");
    llama_free(b);
    // F: the state file into a fresh GPU context
    llama_context * f = mkctx(mg, true);
    std::vector<llama_token> ftoks(prompt.size() + 8);
    size_t nf_tok = 0;
    const bool loaded = llama_state_load_file(f, sf.c_str(), ftoks.data(), ftoks.size(), &nf_tok);
    run_gen(f, "f");
    llama_free(f);
    // C: the reference CPU backend's own run
    llama_context * c = mkctx(mc, false);
    if (run_prompt(c) != 0) { fprintf(stderr, "prompt C failed\n"); return 1; }
    std::vector<uint8_t> blob_c = get_blob(c, "c");
    run_gen(c, "c");
    llama_free(c);
    // D: GPU state into the CPU; E: CPU state into the GPU
    llama_context * d = mkctx(mc, false);
    const size_t nd = llama_state_seq_set_data(d, blob_a.data(), blob_a.size(), 0);
    run_gen(d, "d");
    llama_free(d);
    llama_context * e = mkctx(mg, true);
    const size_t ne = llama_state_seq_set_data(e, blob_c.data(), blob_c.size(), 0);
    run_gen(e, "e");
    llama_free(e);
    printf("{\"n_vocab\": %d, \"n_gen\": %zu, \"blob_bytes\": %zu, \"set_b\": %zu, \"set_d\": %zu, \"set_e\": %zu, "
           "\"saved\": %d, \"loaded\": %d, \"file_tokens\": %zu}\n",
           n_vocab, gen.size(), blob_a.size(), nb, nd, ne, (int) saved, (int) loaded, nf_tok);
    llama_model_free(mg);
    llama_model_free(mc);
    return 0;
}
