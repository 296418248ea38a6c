// Phase timing of the host sampler on the bench workload (R-MAT scale 21,
// 20M pairs, fanouts 25,10, B=512).  Developer tool, not part of the library:
//   g++ -O3 -march=x86-64-v3 -std=c++17 -pthread -I include -I graphsage-pytorch_amd/csrc/host \
//       tools/sampler_prof.cpp graphsage-pytorch_amd/csrc/host/graph.cpp \
//       graphsage-pytorch_amd/csrc/host/errors.cpp -o /tmp/sampler_prof
#include <chrono>
#include <cstdio>
#include <cstdlib>

using clk = std::chrono::steady_clock;
static double g_phase[8];
static clk::time_point g_last;
#define GS_PHASE(i)                                                                       \
    do {                                                                                  \
        const auto now_ = clk::now();                                                     \
        if (i) g_phase[i] += std::chrono::duration<double, std::micro>(now_ - g_last).count(); \
        g_last = now_;                                                                    \
    } while (0)

#include "../graphsage-pytorch_amd/csrc/host/sampler.cpp"

namespace gs {
static void materialise(const Graph& g, Hop& h, bool gcn) {
    HopScratch sc;
    sets_union(g, h, sc, nullptr);
    union_map(h, sc);
    gather_sets(h, sc);
    lists(h, sc, gcn);
}
}  // namespace gs

static double us(clk::time_point a, clk::time_point b) {
    return std::chrono::duration<double, std::micro>(b - a).count();
}

int main(int argc, char** argv) {
    const int scale = argc > 1 ? std::atoi(argv[1]) : 21;
    const int64_t pairs = argc > 2 ? std::atoll(argv[2]) : 20000000;
    const int batches = argc > 3 ? std::atoi(argv[3]) : 200;
    const int64_t n = int64_t(1) << scale;
    std::vector<int64_t> src(pairs), dst(pairs);
    int64_t np = 0;
    if (gs_rmat_pairs(scale, pairs, 0.57, 0.19, 0.19, 824, 1, 8, src.data(), dst.data(), &np) != GS_OK) {
        std::fprintf(stderr, "rmat: %s\n", gs_last_error());
        return 1;
    }
    gs_graph* gp = nullptr;
    if (gs_graph_build(src.data(), dst.data(), np, n, 8, &gp) != GS_OK) {
        std::fprintf(stderr, "build: %s\n", gs_last_error());
        return 1;
    }
    const auto& g = *reinterpret_cast<const gs::Graph*>(gp);
    std::vector<int64_t> cand;
    for (int64_t v = 0; v < n; ++v)
        if (g.degree(v) > 0) cand.push_back(v);
    gs::MT19937 rng;
    rng.init_genrand(824);
    uint64_t lcg = 12345;
    const int32_t fan[2] = {25, 10};
    double t_draw[2] = {0, 0}, t_empty[2] = {0, 0}, t_mat = 0, t_pack = 0;
    int64_t n_pos[2] = {0, 0}, n_dst[2] = {0, 0};
    std::vector<int32_t> buf(1 << 26);
    for (int b = 0; b < batches; ++b) {
        std::vector<int64_t> roots(512);
        for (auto& r : roots) {
            lcg = lcg * 6364136223846793005ull + 1442695040888963407ull;
            r = cand[(lcg >> 33) % cand.size()];
        }
        gs::Sample s;
        s.n_hops = 2;
        std::vector<int64_t> frontier = roots;
        for (int j = 0; j < 2; ++j) {
            gs::Hop& h = s.hops[j];
            h.k = fan[j];
            h.dst_ids = frontier;
            auto t0 = clk::now();
            gs::draw_positions(g, rng, h);
            auto t1 = clk::now();
            h.n_empty = gs::count_empty(g, h, false);
            auto t2 = clk::now();
            t_draw[j] += us(t0, t1);
            t_empty[j] += us(t1, t2);
            n_pos[j] += h.pos.size();
            n_dst[j] += h.dst_ids.size();
            if (j == 0) {
                gs::materialise(g, h, false);
                t_mat += us(t2, clk::now());
                frontier = h.src_ids;
            }
        }
        auto t3 = clk::now();
        gs_sample_pack(reinterpret_cast<const gs_sample*>(&s), buf.data(), buf.size());
        t_pack += us(t3, clk::now());
    }
    // last-hop draw split: degree pass alone vs full, on the final batch's frontier replayed
    {
        gs::Hop h;
        h.k = 10;
        std::vector<int64_t> roots(512);
        for (auto& r : roots) {
            lcg = lcg * 6364136223846793005ull + 1442695040888963407ull;
            r = cand[(lcg >> 33) % cand.size()];
        }
        gs::Sample s;
        gs::Hop& h0 = s.hops[0];
        h0.k = 25;
        h0.dst_ids = roots;
        gs::draw_positions(g, rng, h0);
        gs::materialise(g, h0, false);
        h.dst_ids = h0.src_ids;
        const int reps = 200;
        auto a = clk::now();
        for (int i = 0; i < reps; ++i) gs::draw_positions(g, rng, h);
        auto b = clk::now();
        int64_t acc = 0;
        const int64_t* rp = g.row_ptr.data();
        for (int i = 0; i < reps; ++i)
            for (int64_t v : h.dst_ids) acc += rp[v + 1] - rp[v];
        auto c = clk::now();
        int64_t n_pool = 0, n_sel = 0, n_full = 0;
        for (int64_t v : h.dst_ids) {
            const int64_t d = rp[v + 1] - rp[v];
            if (d < 10) ++n_full; else if (d <= 85) ++n_pool; else ++n_sel;
        }
        std::printf("draw1 replay: full %.1f us, degree pass %.1f us (acc %ld); nodes full %ld pool %ld select %ld\n",
                    us(a, b) / reps, us(b, c) / reps, (long)acc, (long)n_full, (long)n_pool, (long)n_sel);
    }
    const double B = batches;
    std::printf("per batch (us): draw0 %.1f (dst %.0f pos %.0f)  empty0 %.1f  materialise0 %.1f\n", t_draw[0] / B,
                n_dst[0] / B, n_pos[0] / B, t_empty[0] / B, t_mat / B);
    std::printf("                draw1 %.1f (dst %.0f pos %.0f)  empty1 %.1f  pack %.1f  total %.1f\n",
                t_draw[1] / B, n_dst[1] / B, n_pos[1] / B, t_empty[1] / B, t_pack / B,
                (t_draw[0] + t_draw[1] + t_empty[0] + t_empty[1] + t_mat + t_pack) / B);
    std::printf("materialise phases (us): sets %.1f union %.1f map %.1f lists %.1f transpose %.1f\n",
                g_phase[1] / B, g_phase[2] / B, g_phase[3] / B, g_phase[4] / B, g_phase[5] / B);
    gs_graph_destroy(gp);
    return 0;
}
