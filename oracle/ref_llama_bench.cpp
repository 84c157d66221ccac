// ref_llama_bench.cpp — TEST INFRASTRUCTURE. A minimal llama-bench-style driver over
// the reference's own libllama (built from /root/reference/src by oracle/Makefile).
// Used only by bench.py's cpu_baseline leg and by tests (never by the product):
//   bench mode : pp<P> then tg<N> timings, the measurement loop of
//                tools/llama-bench/llama-bench.cpp:1962-2010 (random tokens, decode,
//                synchronise per token), printed as one JSON line;
//   logits mode: --logits <tokens.i32> <out.f32> writes the logits of every position
//                (end-to-end parity of the MI355X runner vs the reference CPU backend);
//                --last N writes only the last N positions' logits (long prompts, e.g.
//                pp2048 as 4 ubatches with -b 2048 -ub 512);
//   -r R       : bench mode repeats pp / tg R times and reports the mean and the
//                per-repetition rates, llama-bench's avg_ts / samples_ts.
//   -ctk T / -ctv T : K and V cache types (ggml_type ids; -ctk alone sets both, as the
//                tests have always used it; -ctk 8 -ctv 1 = K q8_0 + V f16, AGENTS.md:166-176).
//   -d D       : llama-bench's depth (tools/llama-bench/llama-bench.cpp:2191-2226): before
//                every timed pp / tg repetition the cleared cache is filled with a
//                D-token prompt (untimed), so tg runs against D + i keys.
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

// --dump <file>: the scheduler's eval callback (llama_context_params::cb_eval, as
// tools/eval-callback uses it) records every f32 node of the graph: name, op, shape, sum,
// sum of squares and the first values — diffing a -ngl 0 and a -ngl 99 dump finds the
// first node where the MI355X backend departs from the reference CPU backend.
static FILE * g_dump = nullptr;
static std::string g_dump_dir;   // --dump-dir: also the raw f32 values, one file per node
static int g_dump_idx = 0;
static std::string g_dump_filter;   // --dump-filter <substring>: observe only nodes whose name contains it
                                    // (keeps the rest of the graph in one piece, so backend fusions still run)
static bool dump_cb(ggml_tensor * t, bool ask, void *) {
    const bool want = (t->type == GGML_TYPE_F32 || t->type == GGML_TYPE_I32) &&
                      (g_dump_filter.empty() || strstr(t->name, g_dump_filter.c_str()) != nullptr);
    if (ask) return want;
    if (!g_dump || !want || !ggml_is_contiguous(t)) return true;
    std::vector<float> v(ggml_nelements(t));
    if (t->type == GGML_TYPE_F32) ggml_backend_tensor_get(t, v.data(), 0, ggml_nbytes(t));
    else {
        std::vector<int32_t> iv(ggml_nelements(t));
        ggml_backend_tensor_get(t, iv.data(), 0, ggml_nbytes(t));
        for (size_t i = 0; i < iv.size(); ++i) v[i] = (float) iv[i];
    }
    double s = 0, s2 = 0;
    for (float x : v) { s += x; s2 += (double) x * x; }
    fprintf(g_dump, "%s %s %lld %lld %lld %lld %.9g %.9g", t->name, ggml_op_desc(t), (long long) t->ne[0],
            (long long) t->ne[1], (long long) t->ne[2], (long long) t->ne[3], s, s2);
    for (size_t i = 0; i < v.size() && i < 4; ++i) fprintf(g_dump, " %.7g", v[i]);
    fprintf(g_dump, "\n");
    if (!g_dump_dir.empty()) {
        char fn[512];
        snprintf(fn, sizeof(fn), "%s/%03d.f32", g_dump_dir.c_str(), g_dump_idx++);
        if (FILE * f = fopen(fn, "wb")) { fwrite(v.data(), 4, v.size(), f); fclose(f); }
    }
    return true;
}

static double now_s() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char ** argv) {
    std::string model, tok_in, logits_out;
    int threads = 8, pp = 32, tg = 16, ngl = 0, fa = 1, n_ctx = 0, incremental = 0, last = 0, n_batch = 0, n_ubatch = 0, reps = 1;
    int ctk = -1;   // K/V cache type (ggml_type id), -1: default f16
    int ctv = -1;   // -ctv: the V cache type alone (default: as -ctk) — K q8_0 + V f16 is the fork's line
    int depth = 0;
    int prefix = 0;                    // logits mode, incremental: the first N tokens as one batch (no logits)
    std::string sm = "layer";          // -sm none|layer|row
    std::vector<float> ts;             // -ts a,b,...
    int mg = 0;
    int use_mmap = 1;                  // -mmp 0: libllama's async upload through pinned host buffers
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
        else if (a == "--last") last = std::stoi(next());
        else if (a == "--prefix") prefix = std::stoi(next());
        else if (a == "-b") n_batch = std::stoi(next());
        else if (a == "-ub") n_ubatch = std::stoi(next());
        else if (a == "-r") reps = std::max(1, std::stoi(next()));
        else if (a == "-d") depth = std::stoi(next());
        else if (a == "-ctk") ctk = std::stoi(next());
        else if (a == "-ctv") ctv = std::stoi(next());
        else if (a == "-sm") sm = next();
        else if (a == "-mg") mg = std::stoi(next());
        else if (a == "-mmp") use_mmap = std::stoi(next());
        else if (a == "-ts") {
            std::string v = next();
            for (size_t p = 0; p <= v.size();) {
                size_t q = v.find_first_of(",/", p);
                if (q == std::string::npos) q = v.size();
                ts.push_back(std::stof(v.substr(p, q - p)));
                p = q + 1;
            }
        }
        else if (a == "--dump") g_dump = fopen(next().c_str(), "w");
        else if (a == "--dump-dir") g_dump_dir = next();
        else if (a == "--dump-filter") g_dump_filter = next();
    }
    // libllama's log is silenced except its scheduler summary (src/llama-context.cpp:523-533,
    // "graph splits = N"): the drop-in tests assert the split count, which shows any node
    // the MI355X backend refused (it runs on the CPU backend as an extra split)
    llama_log_set([](ggml_log_level, const char * text, void *) {
        if (strstr(text, "graph splits") || strstr(text, "graph nodes")) fprintf(stderr, "[llama] %s", text);
    }, nullptr);
    llama_backend_init();
    ggml_backend_load_all();
    for (size_t i = 0; i < ggml_backend_dev_count(); ++i)
        fprintf(stderr, "device %zu: %s (%s)\n", i, ggml_backend_dev_name(ggml_backend_dev_get(i)),
                ggml_backend_dev_description(ggml_backend_dev_get(i)));
    llama_model_params mp = llama_model_default_params();
    mp.n_gpu_layers = ngl;
    mp.split_mode = sm == "row" ? LLAMA_SPLIT_MODE_ROW : sm == "none" ? LLAMA_SPLIT_MODE_NONE : LLAMA_SPLIT_MODE_LAYER;
    mp.main_gpu = mg;
    mp.use_mmap = use_mmap != 0;
    static float tsplit[128] = {};
    if (!ts.empty()) { for (size_t i = 0; i < ts.size() && i < 128; ++i) tsplit[i] = ts[i]; mp.tensor_split = tsplit; }
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
    cp.n_ctx = n_ctx > 0 ? n_ctx : std::max(512, (int) (pp + tg + depth + toks.size() + 64));
    cp.n_batch = n_batch > 0 ? n_batch : std::max<int>({pp, (int) toks.size(), 1, std::min(depth, 2048)});
    cp.n_ubatch = n_ubatch > 0 ? n_ubatch : std::min<int>(512, cp.n_batch);
    if (ctk >= 0) { cp.type_k = (ggml_type) ctk; cp.type_v = (ggml_type) ctk; }
    if (ctv >= 0) cp.type_v = (ggml_type) ctv;
    cp.n_threads = threads;
    cp.n_threads_batch = threads;
    cp.flash_attn_type = fa ? LLAMA_FLASH_ATTN_TYPE_ENABLED : LLAMA_FLASH_ATTN_TYPE_DISABLED;
    cp.no_perf = true;
    if (g_dump) { cp.cb_eval = dump_cb; cp.cb_eval_user_data = nullptr; }
    llama_context * ctx = llama_init_from_model(m, cp);
    if (!ctx) { fprintf(stderr, "context failed\n"); return 1; }

    if (!toks.empty() && incremental) {
        FILE * f = fopen(logits_out.c_str(), "wb");
        size_t i0 = 0;
        if (prefix > 0 && (size_t) prefix < toks.size()) {   // a cache of `prefix` positions, then one token at a time
            if (llama_decode(ctx, llama_batch_get_one(toks.data(), prefix)) != 0) { fprintf(stderr, "decode failed\n"); return 1; }
            i0 = (size_t) prefix;
        }
        for (size_t i = i0; i < toks.size(); ++i) {
            llama_token t = toks[i];
            if (llama_decode(ctx, llama_batch_get_one(&t, 1)) != 0) { fprintf(stderr, "decode failed\n"); return 1; }
            llama_synchronize(ctx);
            fwrite(llama_get_logits_ith(ctx, -1), sizeof(float), n_vocab, f);
        }
        fclose(f);
        printf("{\"n_tokens\": %zu, \"n_vocab\": %d, \"incremental\": 1, \"prefix\": %d}\n", toks.size() - i0, n_vocab, (int) i0);
    } else if (!toks.empty()) {
        llama_batch b = llama_batch_init((int) toks.size(), 0, 1);
        const size_t first = last > 0 && (size_t) last < toks.size() ? toks.size() - last : 0;
        for (size_t i = 0; i < toks.size(); ++i) {
            b.token[i] = toks[i]; b.pos[i] = (llama_pos) i; b.n_seq_id[i] = 1; b.seq_id[i][0] = 0; b.logits[i] = i >= first;
        }
        b.n_tokens = (int) toks.size();
        if (llama_decode(ctx, b) != 0) { fprintf(stderr, "decode failed\n"); return 1; }
        llama_synchronize(ctx);
        FILE * f = fopen(logits_out.c_str(), "wb");
        for (size_t i = first; i < toks.size(); ++i) fwrite(llama_get_logits_ith(ctx, (int) i), sizeof(float), n_vocab, f);
        fclose(f);
        llama_batch_free(b);
        printf("{\"n_tokens\": %zu, \"n_out\": %zu, \"n_vocab\": %d}\n", toks.size(), toks.size() - first, n_vocab);
    } else {
        // llama-bench.cpp:1962-2010: a warmup run of each test, then R timed repetitions,
        // each on a cleared KV cache; pp in n_batch-sized llama_decode calls
        std::srand(0);
        auto run_pp = [&](int n) {
            std::vector<llama_token> p(n);
            for (auto & t : p) t = std::rand() % n_vocab;
            for (int i = 0; i < n; i += cp.n_batch) {
                const int nb = std::min<int>(cp.n_batch, n - i);
                llama_decode(ctx, llama_batch_get_one(p.data() + i, nb));
            }
            llama_synchronize(ctx);
        };
        auto run_tg = [&](int n) {
            llama_token t = std::rand() % n_vocab;
            for (int i = 0; i < n; ++i) {
                llama_decode(ctx, llama_batch_get_one(&t, 1));
                llama_synchronize(ctx);
                t = std::rand() % n_vocab;
            }
        };
        std::vector<double> pp_ts, tg_ts;
        for (int r = -1; r < reps; ++r) {   // r = -1: warmup
            if (pp > 0) {
                llama_memory_clear(llama_get_memory(ctx), false);
                if (depth > 0 && r >= 0) run_pp(depth);
                const double t0 = now_s();
                run_pp(pp);
                if (r >= 0) pp_ts.push_back(pp / (now_s() - t0));
            }
            if (tg > 0) {
                llama_memory_clear(llama_get_memory(ctx), false);
                if (depth > 0 && r >= 0) run_pp(depth);
                const double t1 = now_s();
                run_tg(r < 0 ? 1 : tg);
                if (r >= 0) tg_ts.push_back(tg / (now_s() - t1));
            }
        }
        auto mean = [](const std::vector<double> & v) { double s = 0; for (double x : v) s += x; return v.empty() ? 0.0 : s / v.size(); };
        auto list = [](const std::vector<double> & v) {
            std::string s = "[";
            for (size_t i = 0; i < v.size(); ++i) { char b[32]; snprintf(b, sizeof(b), "%s%.3f", i ? ", " : "", v[i]); s += b; }
            return s + "]";
        };
        printf("{\"pp\": %d, \"tg\": %d, \"depth\": %d, \"threads\": %d, \"reps\": %d, \"n_batch\": %d, \"n_ubatch\": %d, \"fa\": %d, "
               "\"pp_tok_s\": %.3f, \"tg_tok_s\": %.3f, \"pp_samples\": %s, \"tg_samples\": %s}\n",
               pp, tg, depth, threads, reps, (int) cp.n_batch, (int) cp.n_ubatch, fa, mean(pp_ts), mean(tg_ts),
               list(pp_ts).c_str(), list(tg_ts).c_str());
    }
    llama_free(ctx);
    llama_model_free(m);
    if (g_dump) fclose(g_dump);
    return 0;
}
