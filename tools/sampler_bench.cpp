// Wall time per batch of one host sampler stream as the runner drives it
// (gs_sample_pack_run_multi_team: draws, sets, union, lists on a helper team,
// pack into a buffer) on the bench workload: R-MAT scale 21, 20M pairs,
// fanouts 25,10, B=512, random roots.  Developer tool, not part of the library:
//   g++ -O3 -march=x86-64-v3 -std=c++17 -pthread -I include -I graphsage-pytorch_amd/csrc/host \
//       tools/sampler_bench.cpp graphsage-pytorch_amd/csrc/host/graph.cpp \
//       graphsage-pytorch_amd/csrc/host/errors.cpp -o /tmp/sampler_bench
//   /tmp/sampler_bench [helpers=1] [batches=300] [streams=1] [shared=0] [pair file B fan0 fan1]
// With streams > 1, that many independent streams run on their own threads
// (each with its own team), as the runner's layout does; shared=1 gives them
// one pool of helpers x streams threads (GS_SHARED_HELPERS=1 in the runner).
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <thread>

using clk = std::chrono::steady_clock;
// phase marks of stream 0's sampler thread (helpers and other streams ignored)
static thread_local bool t_main = false;
static double g_phase[8];
static thread_local clk::time_point t_last;
#define GS_PHASE(i)                                                                              \
    do {                                                                                         \
        if (t_main) {                                                                            \
            const auto now_ = clk::now();                                                        \
            if (i) g_phase[i] += std::chrono::duration<double, std::micro>(now_ - t_last).count(); \
            t_last = now_;                                                                       \
        }                                                                                        \
    } while (0)

#include "../graphsage-pytorch_amd/csrc/host/sampler.cpp"

int main(int argc, char** argv) {
    const int helpers = argc > 1 ? std::atoi(argv[1]) : 1;
    const int batches = argc > 2 ? std::atoi(argv[2]) : 300;
    const int streams = argc > 3 ? std::atoi(argv[3]) : 1;
    const bool shared = argc > 4 && std::atoi(argv[4]) == 1;
    // [graph file B fan0 fan1]: a pair file (int64 n, int64 count, count src ids,
    // count dst ids; e.g. tools/lab/dump_pairs.py pubmed) instead of the R-MAT
    const char* gfile = argc > 5 ? argv[5] : nullptr;
    const int scale = 21;
    int64_t pairs = 20000000, n = int64_t(1) << scale;
    std::vector<int64_t> src, dst;
    int64_t np = 0;
    if (gfile) {
        FILE* f = std::fopen(gfile, "rb");
        if (!f || std::fread(&n, 8, 1, f) != 1 || std::fread(&pairs, 8, 1, f) != 1) return 1;
        src.resize(pairs);
        dst.resize(pairs);
        if (std::fread(src.data(), 8, pairs, f) != size_t(pairs) || std::fread(dst.data(), 8, pairs, f) != size_t(pairs))
            return 1;
        std::fclose(f);
        np = pairs;
    } else {
        src.resize(pairs);
        dst.resize(pairs);
        if (gs_rmat_pairs(scale, pairs, 0.57, 0.19, 0.19, 824, 1, 8, src.data(), dst.data(), &np) != GS_OK) return 1;
    }
    gs_graph* gp = nullptr;
    if (gs_graph_build(src.data(), dst.data(), np, n, 8, &gp) != GS_OK) return 1;
    const auto& g = *reinterpret_cast<const gs::Graph*>(gp);
    std::vector<int64_t> cand;
    for (int64_t v = 0; v < n; ++v)
        if (g.degree(v) > 0) cand.push_back(v);
    const int32_t fan[2] = {gfile && argc > 7 ? std::atoi(argv[7]) : 25, gfile && argc > 8 ? std::atoi(argv[8]) : 10};
    const int64_t B = gfile && argc > 6 ? std::atoll(argv[6]) : 512;
    std::vector<double> per(streams, 0.0);
    std::vector<uint64_t> check(streams, 0);
    gs_team* pool = nullptr;  // shared mode: the handle the streams' teams share threads with
    if (shared && helpers > 0) gs_team_create(helpers * streams, &pool);
    auto body = [&](int w) {
        t_main = w == 0;
        gs_rng* rng = nullptr;
        gs_rng_create(&rng);
        const uint32_t key = 824 + 64 * w;
        gs_rng_seed_words(rng, &key, 1);
        gs_team* team = nullptr;
        if (pool) gs_team_create_shared(pool, &team);
        else if (helpers > 0) gs_team_create(helpers, &team);
        const int64_t cap = gs_sample_pack_bound(gp, B, fan, 2) + B;
        std::vector<int32_t> buf(cap);
        int64_t hs[4 * GS_MAX_HOPS], off[GS_MAX_HOPS * GS_PK_NFIELDS], used = 0;
        uint64_t lcg = 12345 + w;
        std::vector<int64_t> roots(B);
        double tot = 0, win = 0;
        std::vector<double> wins;  // means over windows of 20 batches (noise: report the min and median)
        uint64_t h = 1469598103934665603ull;
        for (int b = -3; b < batches; ++b) {  // 3 warm batches
            for (auto& r : roots) {
                lcg = lcg * 6364136223846793005ull + 1442695040888963407ull;
                r = cand[(lcg >> 33) % cand.size()];
            }
            if (b == 0)
                for (double& x : g_phase) x = 0;
            const auto t0 = clk::now();
            if (gs_sample_pack_run_multi_team(gp, rng, roots.data(), B, B, fan, 2, 0, buf.data(), cap, hs, off, &used,
                                              team) != GS_OK) {
                std::fprintf(stderr, "sample: %s\n", gs_last_error());
                std::exit(1);
            }
            if (b >= 0) {
                const double us = std::chrono::duration<double, std::micro>(clk::now() - t0).count();
                tot += us;
                win += us;
                if ((b + 1) % 20 == 0) {
                    wins.push_back(win / 20);
                    win = 0;
                }
            }
            for (int64_t i = 0; i < used; ++i) h = (h ^ static_cast<uint32_t>(buf[i])) * 1099511628211ull;
        }
        per[w] = tot / batches;
        std::sort(wins.begin(), wins.end());
        if (w == 0 && !wins.empty())
            std::printf("stream 0: 20-batch windows min %.1f median %.1f us\n", wins.front(), wins[wins.size() / 2]);
        check[w] = h;
        gs_team_destroy(team);
        gs_rng_destroy(rng);
    };
    const auto t0 = clk::now();
    std::vector<std::thread> th;
    for (int w = 0; w < streams; ++w) th.emplace_back(body, w);
    for (auto& t : th) t.join();
    const double wall = std::chrono::duration<double>(clk::now() - t0).count();
    double mean = 0;
    for (double p : per) mean += p / streams;
    std::printf("stream 0 phases (us per batch): draws hop 1 %.1f, sets + union %.1f, frontier %.1f, last-hop draws %.1f, "
                "join %.1f\n", g_phase[1] / batches, g_phase[2] / batches, g_phase[3] / batches, g_phase[4] / batches,
                g_phase[5] / batches);
    gs_team_destroy(pool);
    std::printf("helpers %d streams %d%s: %.1f us per batch per stream, %.0f batches/s total; pack hash %016llx\n",
                helpers, streams, shared ? " shared" : "", mean, streams * batches / wall, static_cast<unsigned long long>(check[0]));
    gs_graph_destroy(gp);
    return 0;
}
