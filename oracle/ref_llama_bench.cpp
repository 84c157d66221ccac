// ref_llama_bench.cpp — TEST INFRASTRUCTURE. A minimal llama-bench-style driver over
// the reference's own libllama (built from /root/reference/src by oracle/Makefile).
// Used only by bench.py's cpu_baseline leg and by tests (never by the product):
//   bench mode : pp<P> then tg<N> timings, the measurement loop of
//                tools/llama-bench/llama-bench.cpp:1962-2010 (random tokens, decode,
//                synchronise per token), printed as one JSON line;
//   logits mode: --logits <tokens.i32> <out.f32> writes the logits of every position
//                (end-to-end parity of the MI355X runner vs the reference CPU backend).
// -ngl > 0 with GGML_BACKEND_PATH=libggml-mi355x.so runs the reference libllama on the
// MI355X backend unmodified (the drop-in check).
#include "llama.h"
#include "ggml-backend.h"

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

static double now_s() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char ** argv) {
    std::string model, tok_in, logits_out;
    int threads = 8, pp = 32, tg = 16, ngl = 0, fa = 1, n_ctx = 0, incremental = 0;
    for (int i = 1; i < argc; ++i) {
        std::string a = argv[i];
        auto next = [&]() { return std::string(argv[++i]); };
        if (a == "-m") model = next();
        else if (a == "-t") threads = std::stoi(next());
        else if (a == "-p") pp = std::stoi(next());
        else if (a == "-n") tg = std::stoi(next());
        else if (a == "-ngl") ngl = std::stoi(next());
        else if (a == "-fa") fa = std::stoi(next());
        else if (a == "-c") n_ctx = std::stoi(next());
        else if (a == "--logits") { tok_in = next(); logits_out = next(); }
        else if (a == "--incremental") incremental = 1;   // logits mode: one token per llama_decode
    }
    llama_log_set([](ggml_log_level, const char *, void *) {}, nullptr);
    llama_backend_init();
    ggml_backend_load_all();
    for (size_t i = 0; i < ggml_backend_dev_count(); ++i)
        fprintf(stderr, "device %zu: %s (%s)\n", i, ggml_backend_dev_name(ggml_backend_dev_get(i)),
                ggml_backend_dev_description(ggml_backend_dev_get(i)));
    llama_model_params mp = llama_model_default_params();
    mp.n_gpu_layers = ngl;
    llama_model * m = llama_model_load_from_file(model.c_str(), mp);
    if (!m) { fprintf(stderr, "load failed\n"); return 1; }
    const int n_vocab = llama_vocab_n_tokens(llama_model_get_vocab(m));

    std::vector<llama_token> toks;
    if (!tok_in.empty()) {
        FILE * f = fopen(tok_in.c_str(), "rb");
        int32_t t;
        while (fread(&t, 4, 1, f) == 1) toks.push_back(t);
        fclose(f);
    }
    llama_context_params cp = llama_context_default_params();
    cp.n_ctx = n_ctx > 0 ? n_ctx : std::max(512, (int) (pp + tg + toks.size() + 64));
    cp.n_batch = std::max<int>({pp, (int) toks.size(), 1});
    cp.n_ubatch = std::min<int>(512, cp.n_batch);
    cp.n_threads = threads;
    cp.n_threads_batch = threads;
    cp.flash_attn_type = fa ? LLAMA_FLASH_ATTN_TYPE_ENABLED : LLAMA_FLASH_ATTN_TYPE_DISABLED;
    cp.no_perf = true;
    llama_context * ctx = llama_init_from_model(m, cp);
    if (!ctx) { fprintf(stderr, "context failed\n"); return 1; }

    if (!toks.empty() && incremental) {
        FILE * f = fopen(logits_out.c_str(), "wb");
        for (size_t i = 0; i < toks.size(); ++i) {
            llama_token t = toks[i];
            if (llama_decode(ctx, llama_batch_get_one(&t, 1)) != 0) { fprintf(stderr, "decode failed\n"); return 1; }
            llama_synchronize(ctx);
            fwrite(llama_get_logits_ith(ctx, -1), sizeof(float), n_vocab, f);
        }
        fclose(f);
        printf("{\"n_tokens\": %zu, \"n_vocab\": %d, \"incremental\": 1}\n", toks.size(), n_vocab);
    } else if (!toks.empty()) {
        llama_batch b = llama_batch_init((int) toks.size(), 0, 1);
        for (size_t i = 0; i < toks.size(); ++i) {
            b.token[i] = toks[i]; b.pos[i] = (llama_pos) i; b.n_seq_id[i] = 1; b.seq_id[i][0] = 0; b.logits[i] = 1;
        }
        b.n_tokens = (int) toks.size();
        if (llama_decode(ctx, b) != 0) { fprintf(stderr, "decode failed\n"); return 1; }
        llama_synchronize(ctx);
        FILE * f = fopen(logits_out.c_str(), "wb");
        for (size_t i = 0; i < toks.size(); ++i) fwrite(llama_get_logits_ith(ctx, (int) i), sizeof(float), n_vocab, f);
        fclose(f);
        llama_batch_free(b);
        printf("{\"n_tokens\": %zu, \"n_vocab\": %d}\n", toks.size(), n_vocab);
    } else {
        std::srand(0);
        std::vector<llama_token> p(pp);
        for (auto & t : p) t = std::rand() % n_vocab;
        double pp_s = 0;
        if (pp > 0) {
            const double t0 = now_s();
            llama_decode(ctx, llama_batch_get_one(p.data(), pp));
            llama_synchronize(ctx);
            pp_s = now_s() - t0;
        }
        llama_memory_clear(llama_get_memory(ctx), false);
        const double t1 = now_s();
        llama_token t = std::rand() % n_vocab;
        for (int i = 0; i < tg; ++i) {
            llama_decode(ctx, llama_batch_get_one(&t, 1));
            llama_synchronize(ctx);
            t = std::rand() % n_vocab;
        }
        const double tg_s = now_s() - t1;
        printf("{\"pp\": %d, \"tg\": %d, \"threads\": %d, \"pp_tok_s\": %.3f, \"tg_tok_s\": %.3f}\n",
               pp, tg, threads, pp > 0 ? pp / pp_s : 0.0, tg > 0 ? tg / tg_s : 0.0);
    }
    llama_free(ctx);
    llama_model_free(m);
    return 0;
}
