// Host graph construction: adjacency rows in CPython-set iteration order
// (dataCenter.py:33-41 / :77-86 semantics) and the synthetic R-MAT pair
// generator used for the 2M/16M configs.
#include <algorithm>
#include <atomic>
#include <cstring>
#include <memory>
#include <thread>
#include <vector>

#include "common.hpp"
#include "graph.hpp"
#include "pyset.hpp"

namespace gs {

// Split [0, n) into n_threads equal chunks (chunk t = [t*c, min(n,(t+1)*c)),
// c = ceil(n / n_threads)) and run body(lo, hi, t) on one thread per chunk.
template <class F>
void parallel_chunks(int64_t n, int32_t n_threads, F&& body) {
    const int64_t nt = std::max<int32_t>(1, n_threads);
    const int64_t c = (n + nt - 1) / nt;
    if (nt == 1 || n < 4096) {
        for (int64_t t = 0; t < nt; ++t) {
            const int64_t lo = std::min(n, t * c), hi = std::min(n, lo + c);
            body(lo, hi, static_cast<int32_t>(t));
        }
        return;
    }
    std::vector<std::thread> th;
    for (int64_t t = 0; t < nt; ++t) {
        const int64_t lo = std::min(n, t * c), hi = std::min(n, lo + c);
        th.emplace_back([&, lo, hi, t] { body(lo, hi, static_cast<int32_t>(t)); });
    }
    for (auto& x : th) x.join();
}

template <class F>
void parallel_for(int64_t n, int32_t n_threads, F&& body) {
    parallel_chunks(n, n_threads, std::forward<F>(body));
}

static inline uint64_t splitmix64(uint64_t& s) {
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

Graph* build_graph(const int64_t* src, const int64_t* dst, int64_t n_pairs, int64_t n_nodes,
                   int32_t n_threads) {
    GS_REQUIRE(n_nodes > 0 && n_nodes < (int64_t(1) << 31), GS_EINVAL,
               "n_nodes must be in [1, 2^31)");
    GS_REQUIRE(n_pairs >= 0 && (n_pairs == 0 || (src && dst)), GS_EINVAL, "bad pair arrays");
    for (int64_t p = 0; p < n_pairs; ++p)
        GS_REQUIRE(src[p] >= 0 && src[p] < n_nodes && dst[p] >= 0 && dst[p] < n_nodes,
                   GS_ERANGE, "pair endpoint out of [0, n_nodes)");

    // 1. Insertion lists per node, in pair order: adj[a].add(b); adj[b].add(a).
    std::vector<int64_t> ins_ptr(n_nodes + 1, 0);
    for (int64_t p = 0; p < n_pairs; ++p) {
        ++ins_ptr[src[p] + 1];
        ++ins_ptr[dst[p] + 1];
    }
    for (int64_t v = 0; v < n_nodes; ++v) ins_ptr[v + 1] += ins_ptr[v];
    std::vector<int32_t> ins(ins_ptr[n_nodes]);
    {
        std::vector<int64_t> cur(ins_ptr.begin(), ins_ptr.end() - 1);
        for (int64_t p = 0; p < n_pairs; ++p) {
            ins[cur[src[p]]++] = static_cast<int32_t>(dst[p]);
            ins[cur[dst[p]]++] = static_cast<int32_t>(src[p]);
        }
    }

    // 2. Replay each row's adds through the CPython set; keep its final slot
    //    order (compacted in place of the insertion list) and slot indices.
    std::vector<int32_t> tkey(ins.size());
    std::vector<uint32_t> tslot(ins.size());
    std::vector<int64_t> deg(n_nodes, 0);
    std::vector<uint8_t> lg(n_nodes, 3);
    parallel_for(n_nodes, n_threads, [&](int64_t lo, int64_t hi, int32_t) {
        PySet s;
        for (int64_t v = lo; v < hi; ++v) {
            s.reset();
            for (int64_t t = ins_ptr[v]; t < ins_ptr[v + 1]; ++t) s.add(ins[t]);
            int64_t w = ins_ptr[v];
            for (size_t sl = 0; sl <= s.mask; ++sl) {
                if (s.tab[sl] == PySet::EMPTY) continue;
                tkey[w] = static_cast<int32_t>(s.tab[sl]);
                tslot[w] = static_cast<uint32_t>(sl);
                ++w;
            }
            deg[v] = w - ins_ptr[v];
            lg[v] = static_cast<uint8_t>(__builtin_ctzll(s.mask + 1));
        }
    });

    auto* g = new Graph();
    g->n_nodes = n_nodes;
    g->row_ptr.assign(n_nodes + 1, 0);
    for (int64_t v = 0; v < n_nodes; ++v) g->row_ptr.own[v + 1] = g->row_ptr.own[v] + deg[v];
    g->n_entries = g->row_ptr[n_nodes];
    g->col.resize(g->n_entries);
    g->slot.resize(g->n_entries);
    g->log2size.assign(lg.begin(), lg.end());
    g->max_degree = 0;
    for (int64_t v = 0; v < n_nodes; ++v) g->max_degree = std::max(g->max_degree, deg[v]);
    parallel_for(n_nodes, n_threads, [&](int64_t lo, int64_t hi, int32_t) {
        for (int64_t v = lo; v < hi; ++v) {
            const int64_t d = deg[v];
            if (!d) continue;
            std::memcpy(&g->col.own[g->row_ptr[v]], &tkey[ins_ptr[v]], d * sizeof(int32_t));
            std::memcpy(&g->slot.own[g->row_ptr[v]], &tslot[ins_ptr[v]], d * sizeof(uint32_t));
        }
    });
    return g;
}

Graph* graph_from_tables(int64_t n_nodes, const int64_t* row_ptr, const int32_t* col,
                         const uint32_t* slot, const uint8_t* log2size, const uint8_t* dirty) {
    GS_REQUIRE(n_nodes > 0 && n_nodes < (int64_t(1) << 31), GS_EINVAL, "n_nodes must be in [1, 2^31)");
    GS_REQUIRE(row_ptr && log2size, GS_EINVAL, "NULL row_ptr/log2size");
    GS_REQUIRE(row_ptr[0] == 0, GS_EINVAL, "row_ptr[0] must be 0");
    auto* g = new Graph();
    std::unique_ptr<Graph> guard(g);
    g->n_nodes = n_nodes;
    g->row_ptr.assign(row_ptr, row_ptr + n_nodes + 1);
    g->n_entries = g->row_ptr[n_nodes];
    GS_REQUIRE(g->n_entries == 0 || (col && slot), GS_EINVAL, "NULL col/slot");
    g->col.assign(col, col + g->n_entries);
    g->slot.assign(slot, slot + g->n_entries);
    g->log2size.assign(log2size, log2size + n_nodes);
    if (dirty) g->dirty.assign(dirty, dirty + n_nodes);
    for (int64_t v = 0; v < n_nodes; ++v) {
        const int64_t d = g->row_ptr[v + 1] - g->row_ptr[v];
        GS_REQUIRE(d >= 0, GS_EINVAL, "row_ptr not monotone");
        GS_REQUIRE(g->log2size[v] >= 3 && g->log2size[v] < 40, GS_EINVAL, "bad table size");
        const uint64_t size = uint64_t(1) << g->log2size[v];
        GS_REQUIRE(static_cast<uint64_t>(d) <= size, GS_EINVAL, "row longer than its table");
        uint32_t prev = 0;
        for (int64_t e = g->row_ptr[v]; e < g->row_ptr[v + 1]; ++e) {
            GS_REQUIRE(g->col[e] >= 0 && g->col[e] < n_nodes, GS_ERANGE, "neighbour id out of range");
            GS_REQUIRE(g->slot[e] < size && (e == g->row_ptr[v] || g->slot[e] > prev), GS_EINVAL,
                       "slots must be increasing within the table");
            prev = g->slot[e];
        }
        g->max_degree = std::max(g->max_degree, d);
    }
    return guard.release();
}

// ---- flat image of a graph (one node-wide CSR shared by the rank processes)
//
// [header: 8 x int64 = magic, version, n_nodes, n_entries, max_degree, has_dirty,
//  0, 0] then row_ptr, col, slot, log2size, dirty, each 64-byte aligned.
namespace {
constexpr int64_t kImgMagic = 0x4753435352494d47;  // "GMIRSCSG"
constexpr int64_t kImgVersion = 1;
inline int64_t al64(int64_t b) { return (b + 63) & ~int64_t(63); }
struct ImgLayout {
    int64_t row_ptr, col, slot, log2size, dirty, total;
};
ImgLayout img_layout(int64_t n_nodes, int64_t n_entries, bool has_dirty) {
    ImgLayout L{};
    int64_t at = 64;
    L.row_ptr = at;
    at = al64(at + (n_nodes + 1) * 8);
    L.col = at;
    at = al64(at + n_entries * 4);
    L.slot = at;
    at = al64(at + n_entries * 4);
    L.log2size = at;
    at = al64(at + n_nodes);
    L.dirty = at;
    at = al64(at + (has_dirty ? n_nodes : 0));
    L.total = at;
    return L;
}
}  // namespace

int64_t graph_image_bytes(const Graph& g) { return img_layout(g.n_nodes, g.n_entries, !g.dirty.empty()).total; }

void graph_write_image(const Graph& g, void* dst, int64_t cap) {
    const ImgLayout L = img_layout(g.n_nodes, g.n_entries, !g.dirty.empty());
    GS_REQUIRE(dst && cap >= L.total, GS_EINVAL, "image buffer below gs_graph_image_bytes");
    auto* b = static_cast<uint8_t*>(dst);
    int64_t hdr[8] = {kImgMagic, kImgVersion, g.n_nodes, g.n_entries, g.max_degree, g.dirty.empty() ? 0 : 1, 0, 0};
    std::memcpy(b, hdr, sizeof(hdr));
    std::memcpy(b + L.row_ptr, g.row_ptr.data(), (g.n_nodes + 1) * 8);
    if (g.n_entries) {
        std::memcpy(b + L.col, g.col.data(), g.n_entries * 4);
        std::memcpy(b + L.slot, g.slot.data(), g.n_entries * 4);
    }
    std::memcpy(b + L.log2size, g.log2size.data(), g.n_nodes);
    if (!g.dirty.empty()) std::memcpy(b + L.dirty, g.dirty.data(), g.n_nodes);
}

Graph* graph_from_image(const void* img, int64_t bytes) {
    GS_REQUIRE(img && bytes >= 64, GS_EINVAL, "image too small");
    int64_t hdr[8];
    std::memcpy(hdr, img, sizeof(hdr));
    GS_REQUIRE(hdr[0] == kImgMagic && hdr[1] == kImgVersion, GS_EINVAL, "not a graph image (magic/version)");
    const int64_t n_nodes = hdr[2], n_entries = hdr[3];
    GS_REQUIRE(n_nodes > 0 && n_nodes < (int64_t(1) << 31) && n_entries >= 0, GS_EINVAL, "bad image dims");
    const ImgLayout L = img_layout(n_nodes, n_entries, hdr[5] != 0);
    GS_REQUIRE(bytes >= L.total, GS_EINVAL, "image truncated");
    GS_REQUIRE(reinterpret_cast<uintptr_t>(img) % 64 == 0, GS_EINVAL, "image not 64-byte aligned");
    const auto* b = static_cast<const uint8_t*>(img);
    auto g = std::make_unique<Graph>();
    g->n_nodes = n_nodes;
    g->n_entries = n_entries;
    g->max_degree = hdr[4];
    g->row_ptr.view(reinterpret_cast<const int64_t*>(b + L.row_ptr), n_nodes + 1);
    g->col.view(reinterpret_cast<const int32_t*>(b + L.col), n_entries);
    g->slot.view(reinterpret_cast<const uint32_t*>(b + L.slot), n_entries);
    g->log2size.view(b + L.log2size, n_nodes);
    if (hdr[5]) g->dirty.view(b + L.dirty, n_nodes);
    GS_REQUIRE(g->row_ptr.data()[0] == 0 && g->row_ptr.data()[n_nodes] == n_entries, GS_EINVAL,
               "image row_ptr inconsistent with its entry count");
    // Everything the samplers index memory with, checked once (a truncated or
    // stale /dev/shm image must fail here, not read out of bounds later):
    // row_ptr monotone, every col in [0, n_nodes), each row's table size
    // a power of two above its degree, every slot inside its row's table,
    // and the header's max degree.
    std::atomic<int> bad{0};
    std::atomic<int64_t> maxd{0};
    const int64_t* rp = g->row_ptr.data();
    const int32_t* col = g->col.data();
    const uint32_t* sl = g->slot.data();
    const uint8_t* l2 = g->log2size.data();
    const int32_t nthr = static_cast<int32_t>(std::max(1u, std::min(16u, std::thread::hardware_concurrency())));
    parallel_chunks(n_nodes, nthr, [&](int64_t lo, int64_t hi, int32_t) {
        int local = 0;
        int64_t md = 0;
        for (int64_t v = lo; v < hi && !local; ++v) {
            const int64_t a = rp[v], e = rp[v + 1], d = e - a;
            if (d < 0 || a < 0 || e > n_entries || l2[v] > 31 || (d > 0 && (int64_t(1) << l2[v]) <= d)) {
                local = 1;
                break;
            }
            md = std::max(md, d);
            const uint32_t tsz = uint32_t(1) << l2[v];
            for (int64_t t = a; t < e; ++t)
                if (col[t] < 0 || col[t] >= n_nodes || sl[t] >= tsz) {
                    local = 1;
                    break;
                }
        }
        if (local) bad.store(1);
        int64_t cur = maxd.load();
        while (md > cur && !maxd.compare_exchange_weak(cur, md)) {
        }
    });
    GS_REQUIRE(!bad.load(), GS_EINVAL, "graph image corrupt: row_ptr, col, table sizes or slots out of range");
    GS_REQUIRE(maxd.load() == g->max_degree, GS_EINVAL, "graph image corrupt: max degree differs from its rows");
    return g.release();
}

int64_t rmat_pairs(int32_t scale, int64_t n_pairs, double a, double b, double c, uint64_t seed,
                   int32_t permute, int32_t n_threads, int64_t* src, int64_t* dst) {
    GS_REQUIRE(scale >= 1 && scale <= 30, GS_EINVAL, "scale must be in [1, 30]");
    GS_REQUIRE(a >= 0 && b >= 0 && c >= 0 && a + b + c <= 1.0, GS_EINVAL, "bad R-MAT probabilities");
    const double ab = a + b, abc = a + b + c;
    const int32_t nthr = std::max<int32_t>(1, n_threads);
    std::vector<int64_t> lo_of(nthr, 0), kept(nthr, 0);
    // Each pair p draws from its own splitmix64 stream keyed by (seed, p), so
    // the output is independent of the thread count.
    parallel_chunks(n_pairs, nthr, [&](int64_t lo, int64_t hi, int32_t t) {
        int64_t w = lo;
        for (int64_t p = lo; p < hi; ++p) {
            uint64_t st = seed * 0xD1B54A32D192ED03ull + static_cast<uint64_t>(p) * 0x9E3779B97F4A7C15ull;
            int64_t u = 0, v = 0;
            for (int32_t l = 0; l < scale; ++l) {
                const double r = (splitmix64(st) >> 11) * (1.0 / 9007199254740992.0);
                int bu, bv;
                if (r < a) { bu = 0; bv = 0; }
                else if (r < ab) { bu = 0; bv = 1; }
                else if (r < abc) { bu = 1; bv = 0; }
                else { bu = 1; bv = 1; }
                u = (u << 1) | bu;
                v = (v << 1) | bv;
            }
            if (u == v) continue;  // self pairs dropped
            src[w] = u;
            dst[w] = v;
            ++w;
        }
        lo_of[t] = lo;
        kept[t] = w - lo;
    });
    // Close the per-chunk gaps in order.
    int64_t out = 0;
    for (int32_t t = 0; t < nthr; ++t) {
        if (out != lo_of[t] && kept[t]) {
            std::memmove(src + out, src + lo_of[t], kept[t] * sizeof(int64_t));
            std::memmove(dst + out, dst + lo_of[t], kept[t] * sizeof(int64_t));
        }
        out += kept[t];
    }
    if (permute) {
        const int64_t n = int64_t(1) << scale;
        std::vector<int64_t> perm(n);
        for (int64_t i = 0; i < n; ++i) perm[i] = i;
        uint64_t st = seed ^ 0x5DEECE66Dull;
        for (int64_t i = n - 1; i > 0; --i) {
            const int64_t j = static_cast<int64_t>(splitmix64(st) % static_cast<uint64_t>(i + 1));
            std::swap(perm[i], perm[j]);
        }
        parallel_for(out, n_threads, [&](int64_t lo, int64_t hi, int32_t) {
            for (int64_t p = lo; p < hi; ++p) {
                src[p] = perm[src[p]];
                dst[p] = perm[dst[p]];
            }
        });
    }
    return out;
}

}  // namespace gs

using gs::Graph;

extern "C" {

int gs_graph_build(const int64_t* src, const int64_t* dst, int64_t n_pairs, int64_t n_nodes,
                   int32_t n_threads, gs_graph** out) {
    GS_API_BEGIN
    GS_REQUIRE(out, GS_EINVAL, "out is NULL");
    *out = reinterpret_cast<gs_graph*>(gs::build_graph(src, dst, n_pairs, n_nodes, n_threads));
    GS_API_END
}

int gs_graph_from_tables(int64_t n_nodes, const int64_t* row_ptr, const int32_t* col, const uint32_t* slot,
                         const uint8_t* log2size, const uint8_t* dirty, gs_graph** out) {
    GS_API_BEGIN
    GS_REQUIRE(out, GS_EINVAL, "out is NULL");
    *out = reinterpret_cast<gs_graph*>(gs::graph_from_tables(n_nodes, row_ptr, col, slot, log2size, dirty));
    GS_API_END
}

void gs_graph_destroy(gs_graph* g) { delete reinterpret_cast<Graph*>(g); }

int gs_graph_dims(const gs_graph* gp, int64_t* n_nodes, int64_t* n_entries, int64_t* max_degree) {
    GS_API_BEGIN
    GS_REQUIRE(gp, GS_EINVAL, "graph is NULL");
    auto* g = reinterpret_cast<const Graph*>(gp);
    if (n_nodes) *n_nodes = g->n_nodes;
    if (n_entries) *n_entries = g->n_entries;
    if (max_degree) *max_degree = g->max_degree;
    GS_API_END
}

const int64_t* gs_graph_row_ptr(const gs_graph* g) {
    return g ? reinterpret_cast<const Graph*>(g)->row_ptr.data() : nullptr;
}

const int32_t* gs_graph_col(const gs_graph* g) {
    return g ? reinterpret_cast<const Graph*>(g)->col.data() : nullptr;
}

int64_t gs_graph_image_bytes(const gs_graph* g) {
    return g ? gs::graph_image_bytes(*reinterpret_cast<const Graph*>(g)) : -1;
}

int gs_graph_write_image(const gs_graph* g, void* dst, int64_t cap) {
    GS_API_BEGIN
    GS_REQUIRE(g, GS_EINVAL, "graph is NULL");
    gs::graph_write_image(*reinterpret_cast<const Graph*>(g), dst, cap);
    GS_API_END
}

int gs_graph_from_image(const void* img, int64_t bytes, gs_graph** out) {
    GS_API_BEGIN
    GS_REQUIRE(out, GS_EINVAL, "out is NULL");
    *out = reinterpret_cast<gs_graph*>(gs::graph_from_image(img, bytes));
    GS_API_END
}

int gs_rmat_pairs(int32_t scale, int64_t n_pairs, double a, double b, double c, uint64_t seed,
                  int32_t permute, int32_t n_threads, int64_t* src, int64_t* dst, int64_t* n_kept) {
    GS_API_BEGIN
    GS_REQUIRE(src && dst && n_kept && n_pairs >= 0, GS_EINVAL, "bad output arrays");
    *n_kept = gs::rmat_pairs(scale, n_pairs, a, b, c, seed, permute, n_threads, src, dst);
    GS_API_END
}

}  // extern "C"
