// UnsupervisedLoss.extend_nodes (models.py:135-147) on the host, bit-exact
// with the reference's CPython `random` stream and set iteration orders, and
// the index plan the device loss kernels (kernels/unsup.hip) read.
//
// extend_nodes(nodes, num_neg):
//   positives  models.py:166-186  for each node with a non-empty row: N_WALKS
//              walks of WALK_LEN steps, each step random.choice(list(adj[cur]))
//              = randbelow(deg) over the CSR row (the row IS list(set)); the
//              pair (node, next) is kept when next != node and next is a
//              training node.                                   (sequential rng)
//   negatives  models.py:152-164  the N_WALK_LEN-hop ball of each node, then
//              far = set(train) - ball and random.sample(far, num_neg) unless
//              num_neg >= len(far) (then far itself).  The ball only matters
//              through membership; far's iteration order follows CPython's
//              set_difference:
//                (len(train) >> 2) > len(ball): copy(set(train)), then discard
//                    -> the copy's slot order, ball members skipped;
//                otherwise: a fresh set filled in set(train)'s slot order
//                    with the non-members -> that set's slot order.
//              The balls of a chunk of roots grow together (bit-parallel
//              multi-source BFS, 64 roots per word); far lists are built in
//              parallel (no rng); the draws then run in node order on the
//              one stream.
//   unique     models.py:146  list(set(flat positives) | set(flat negatives)).
#include <algorithm>
#include <atomic>
#include <memory>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "common.hpp"
#include "graph.hpp"
#include "pyset.hpp"
#include "team.hpp"
#include "rng.hpp"
#include "unsup_dev.hpp"

namespace gs {
namespace {

// Bit-parallel multi-source BFS: bit b of word w stands for root 64*w + b.
// The balls of models.py:154-162 are pure membership (set order never
// reaches the result, see far_list), so all roots of a chunk expand together:
// per level, every node with a frontier word pushes it to its neighbours.
// Layout is word-major ([w][node]) so each worker thread owns whole words and
// the level loop needs no synchronisation.
struct BallSet {
    int64_t n_nodes = 0, n_words = 0;
    std::vector<uint64_t> seen, edge, next;  // [n_words][n_nodes]

    void grow(const Graph& g, const int64_t* roots, int64_t n_roots, int hops, int32_t n_threads,
              std::vector<int64_t>& sizes) {
        n_nodes = g.n_nodes;
        n_words = (n_roots + 63) / 64;
        const size_t total = static_cast<size_t>(n_words * n_nodes);
        seen.assign(total, 0);
        edge.assign(total, 0);
        next.resize(total);
        for (int64_t r = 0; r < n_roots; ++r) {
            const uint64_t bit = uint64_t(1) << (r & 63);
            seen[(r >> 6) * n_nodes + roots[r]] |= bit;
            edge[(r >> 6) * n_nodes + roots[r]] |= bit;
        }
        auto body = [&](int64_t w) {
            uint64_t* S = seen.data() + w * n_nodes;
            uint64_t* E = edge.data() + w * n_nodes;
            uint64_t* X = next.data() + w * n_nodes;
            for (int h = 0; h < hops; ++h) {
                std::fill_n(X, n_nodes, 0);
                bool any = false;
                for (int64_t u = 0; u < n_nodes; ++u) {
                    const uint64_t f = E[u];
                    if (!f) continue;
                    const int32_t* c = g.col.data() + g.row_ptr[u];
                    const int64_t d = g.row_ptr[u + 1] - g.row_ptr[u];
                    for (int64_t e = 0; e < d; ++e) X[c[e]] |= f;
                }
                for (int64_t u = 0; u < n_nodes; ++u) {
                    const uint64_t nw = X[u] & ~S[u];
                    E[u] = nw;
                    S[u] |= nw;
                    any |= nw != 0;
                }
                if (!any) break;
            }
            int64_t cnt[64] = {0};  // len(neighbors) of this word's roots
            for (int64_t u = 0; u < n_nodes; ++u)
                for (uint64_t m = S[u]; m; m &= m - 1) ++cnt[__builtin_ctzll(m)];
            for (int b = 0; b < 64 && 64 * w + b < n_roots; ++b) sizes[64 * w + b] = cnt[b];
        };
        sizes.assign(n_roots, 0);
        const int32_t nt = static_cast<int32_t>(std::max<int64_t>(1, std::min<int64_t>(n_threads, n_words)));
        if (nt == 1) {
            for (int64_t w = 0; w < n_words; ++w) body(w);
        } else {
            std::vector<std::thread> th;
            for (int32_t t = 0; t < nt; ++t)
                th.emplace_back([&, t] {
                    for (int64_t w = t; w < n_words; w += nt) body(w);
                });
            for (auto& x : th) x.join();
        }
    }
    bool has(int64_t r, int32_t x) const { return (seen[(r >> 6) * n_nodes + x] >> (r & 63)) & 1; }
};

}  // namespace
}  // namespace gs

struct gs_unsup {
    const gs::Graph* g = nullptr;
    int32_t n_walks = 6, walk_len = 1, n_walk_len = 5;
    std::vector<uint8_t> is_train;      // [n_nodes]
    std::vector<int32_t> train_order;   // list(set(train_nodes))
    std::vector<int32_t> copy_order;    // list(set(train_nodes).copy())
    int64_t n_train_set = 0;
    gs::BallSet balls;                  // the chunk's 5-hop balls
    // last extend_nodes
    std::vector<int64_t> nodes, unique, pos, neg;  // pairs flattened (a, b)
    std::vector<int64_t> pos_cnt, neg_cnt;
    std::vector<uint8_t> has_pos;
    std::vector<uint64_t> seen;         // [n_nodes / 64] scratch bitmap, all clear between calls
    int32_t subset_ok = 0;
    gs::UnsupDev* dev = nullptr;        // gs_unsup_attach_device: balls + far picks on the GPU
    std::unique_ptr<gs::Team> team;     // persistent helpers (fresh-set orders beside the draws)
    ~gs_unsup();
};

#ifndef GS_HOST_ONLY
gs_unsup::~gs_unsup() { gs::unsup_dev_destroy(dev); }
#else
gs_unsup::~gs_unsup() {}
#endif

namespace {

using gs::PySet;

template <class Fn>
void run_workers(int32_t n_threads, int64_t n, Fn&& fn) {
    const int32_t nt = static_cast<int32_t>(std::max<int64_t>(1, std::min<int64_t>(n_threads, n)));
    if (nt <= 1) {
        for (int64_t i = 0; i < n; ++i) fn(i, 0);
        return;
    }
    std::vector<std::thread> th;
    for (int32_t t = 0; t < nt; ++t)
        th.emplace_back([&, t] {
            for (int64_t i = t; i < n; i += nt) fn(i, t);
        });
    for (auto& x : th) x.join();
}

// far = set(train) - ball, in CPython iteration order (see file header), for
// the roots r0 .. r0+nr-1 that live in ball word w: one pass over the train
// order serves all 64 roots of the word (one load of the word per key).
// far[r - r0] receives root r's list.
void fresh_set_order(std::vector<int32_t>& out);

void far_lists_word(const gs_unsup& u, int64_t w, int64_t r0, int64_t nr, const std::vector<int64_t>& ball_size,
                    std::vector<std::vector<int32_t>>& far) {
    const gs::BallSet& b = u.balls;
    uint64_t copy_roots = 0, fresh_roots = 0;
    for (int bit = 0; bit < 64; ++bit) {
        const int64_t r = 64 * w + bit;
        if (r < r0 || r >= r0 + nr) continue;
        far[r - r0].clear();
        if ((u.n_train_set >> 2) > ball_size[r])
            copy_roots |= uint64_t(1) << bit;
        else
            fresh_roots |= uint64_t(1) << bit;
    }
    const uint64_t* S = b.seen.data() + w * b.n_nodes;
    auto pass = [&](const std::vector<int32_t>& order, uint64_t roots) {
        if (!roots) return;
        for (int32_t x : order)
            for (uint64_t m = ~S[x] & roots; m; m &= m - 1)
                far[64 * w + __builtin_ctzll(m) - r0].push_back(x);
    };
    pass(u.copy_order, copy_roots);    // copy(set(train)) then discard the ball
    pass(u.train_order, fresh_roots);  // a fresh set filled in set(train) order
    for (uint64_t m = fresh_roots; m; m &= m - 1) fresh_set_order(far[64 * w + __builtin_ctzll(m) - r0]);
}

// Final table mask of a fresh set after k adds of distinct keys (no deletions:
// fill == used at every growth check, so the size follows from k alone).
size_t fresh_mask(int64_t k) {
    size_t mask = PySet::MINSIZE - 1;
    for (int64_t used = 1; used <= k; ++used) {
        if (static_cast<size_t>(used) * 5 < mask * 3) {
            used = std::max<int64_t>(used, static_cast<int64_t>((mask * 3 + 4) / 5) - 1);  // skip to the next check
            continue;
        }
        size_t ns = PySet::MINSIZE;
        const size_t minused = static_cast<size_t>(used > 50000 ? used * 2 : used * 4);
        while (ns <= minused) ns <<= 1;
        mask = ns - 1;
    }
    return mask;
}

// The iteration order of a fresh set built by adding `out`'s keys in order.
void fresh_set_order(std::vector<int32_t>& out) {
    // A fresh set filled by adds in this order.  When every key owns its home
    // slot key & mask in the final table, each add (and the insert_clean of
    // the last resize) lands at home whatever came before, so the iteration
    // order is the home-slot order: place directly.  Any shared home slot:
    // replay the adds through the emulator.
    const size_t mask = fresh_mask(static_cast<int64_t>(out.size()));
    thread_local std::vector<int32_t> home;
    home.assign(mask + 1, -1);
    bool clash = false;
    for (int32_t x : out) {
        int32_t& h = home[static_cast<size_t>(x) & mask];
        clash |= h != -1;
        h = x;
    }
    if (!clash) {
        out.clear();
        for (int32_t h : home)
            if (h != -1) out.push_back(h);
        return;
    }
    PySet r;
    for (int32_t x : out) r.add(x);
    out.clear();
    r.for_each([&](int32_t x) { out.push_back(x); });
}

void walk_pairs(gs_unsup& u, gs_rng* rng) {
    const gs::Graph& g = *u.g;
    const int64_t n = static_cast<int64_t>(u.nodes.size());
    for (int64_t i = 0; i < n; ++i) {
        const int64_t v = u.nodes[i];
        if (g.degree(v) == 0) continue;  // models.py:168
        u.has_pos[i] = 1;
        for (int32_t w = 0; w < u.n_walks; ++w) {
            int64_t cur = v;
            for (int32_t s = 0; s < u.walk_len; ++s) {
                const int64_t d = g.degree(cur);
                GS_REQUIRE(d > 0, GS_EEMPTY, "Cannot choose from an empty sequence (walk reached an isolated node)");
                const int64_t nxt = g.col[g.row_ptr[cur] + rng->mt.randbelow(static_cast<uint64_t>(d))];
                if (nxt != v && u.is_train[nxt]) {
                    u.pos.push_back(v);
                    u.pos.push_back(nxt);
                    ++u.pos_cnt[i];
                }
                cur = nxt;
            }
        }
    }
}

void negative_pairs(gs_unsup& u, gs_rng* rng, int64_t num_neg, int32_t n_threads) {
    const int64_t n = static_cast<int64_t>(u.nodes.size());
    const int32_t nt = std::max<int32_t>(1, n_threads);
    // roots per ball chunk: whole words, ~96 MiB of ball bitmaps at most
    const int64_t words = std::max<int64_t>(1, std::min<int64_t>(16, (int64_t(96) << 20) / (24 * u.g->n_nodes + 1)));
    const int64_t chunk = 64 * words;
    // far lists held at once: the whole chunk unless that exceeds ~256 MiB
    const int64_t sub = 64 * std::max<int64_t>(1, std::min<int64_t>(words, (int64_t(1) << 20) / (u.n_train_set + 1)));
    std::vector<std::vector<int32_t>> far(static_cast<size_t>(sub));
    std::vector<int64_t> ball_size;
    const int64_t setsize = gs::sample_setsize(num_neg);
    std::vector<int32_t> pool;
    std::vector<int64_t> picks(static_cast<size_t>(std::max<int64_t>(num_neg, 1)));
    static const bool prof = std::getenv("GS_UNSUP_PROF") != nullptr;
    using clk = std::chrono::steady_clock;
    double t_ball = 0, t_far = 0, t_draw = 0;
    for (int64_t c0 = 0; c0 < n; c0 += chunk) {
        const int64_t cn = std::min(chunk, n - c0);
        auto t0 = clk::now();
        u.balls.grow(*u.g, u.nodes.data() + c0, cn, u.n_walk_len, nt, ball_size);
        t_ball += std::chrono::duration<double>(clk::now() - t0).count();
        if (prof) std::fprintf(stderr, "[unsup] balls %.2f ms\n", t_ball * 1e3);
        for (int64_t s0 = 0; s0 < cn; s0 += sub) {
            const int64_t sn = std::min(sub, cn - s0);
            auto t1 = clk::now();
            run_workers(nt, (sn + 63) / 64, [&](int64_t j, int32_t) {
                far_lists_word(u, s0 / 64 + j, s0, sn, ball_size, far);
            });
            auto t2 = clk::now();
            t_far += std::chrono::duration<double>(t2 - t1).count();
            for (int64_t j = 0; j < sn; ++j) {  // the draws, in node order
                const int64_t i = c0 + s0 + j, v = u.nodes[i];
                const std::vector<int32_t>& f = far[j];
                const int64_t len = static_cast<int64_t>(f.size());
                if (num_neg < len) {
                    if (len <= setsize) pool.resize(static_cast<size_t>(len));
                    gs::sample_positions(rng->mt, len, num_neg, setsize, picks.data(), pool.data());
                    for (int64_t t = 0; t < num_neg; ++t) {
                        u.neg.push_back(v);
                        u.neg.push_back(f[picks[t]]);
                    }
                    u.neg_cnt[i] = num_neg;
                } else {
                    for (int32_t x : f) {
                        u.neg.push_back(v);
                        u.neg.push_back(x);
                    }
                    u.neg_cnt[i] = len;
                }
            }
            t_draw += std::chrono::duration<double>(clk::now() - t2).count();
        }
        (void)t0;
    }
    if (prof) std::fprintf(stderr, "[unsup] far %.2f ms draw %.2f ms\n", t_far * 1e3, t_draw * 1e3);
}

#ifndef GS_HOST_ONLY
// negative_pairs with the balls and the far-list picks on the device (the
// draws unchanged, on this thread, in node order).  Far-list order per node
// (see the file header): the copy order when (len(train) >> 2) > len(ball);
// else a fresh set, whose order is ascending ids when its final table has a
// home slot per id (mask + 1 >= n_nodes), and otherwise comes from the host
// emulator on the node's ball bits.
void negative_pairs_dev(gs_unsup& u, gs_rng* rng, int64_t num_neg, int32_t n_threads) {
    static const bool prof = std::getenv("GS_UNSUP_PROF") != nullptr;
    using clk = std::chrono::steady_clock;
    const auto t0 = clk::now();
    const int64_t n = static_cast<int64_t>(u.nodes.size());
    if (n == 0) return;  // no nodes, no negatives (and no device launch)
    std::vector<int64_t> bsize(n), tib(n);
    gs::unsup_dev_balls(u.dev, u.nodes.data(), static_cast<int>(n), u.n_walk_len, bsize.data(), tib.data());
    const auto t1 = clk::now();
    const int64_t setsize = gs::sample_setsize(num_neg);
    // far-list order per node: 0 copy order, 1 ascending ids, 2 a fresh set
    // whose table has fewer slots than ids — its order comes from the host
    // emulator, over the node's whole far list in set(train) order (fetched
    // from the device in one batch of select queries)
    std::vector<int> kind(n);
    std::vector<int32_t> k2;           // fresh-set nodes
    std::vector<int64_t> k2base(1, 0);
    for (int64_t i = 0; i < n; ++i) {
        const int64_t len = u.n_train_set - tib[i];
        kind[i] = (u.n_train_set >> 2) > bsize[i] ? 0 : (fresh_mask(len) + 1 >= static_cast<size_t>(u.g->n_nodes) ? 1 : 2);
        if (kind[i] == 2) {
            k2.push_back(static_cast<int32_t>(i));
            k2base.push_back(k2base.back() + len);
        }
    }
    std::vector<int32_t> host_far;
    gs::unsup_dev_far_lists(u.dev, k2, k2base, host_far);
    const auto t1a = clk::now();
    // the fresh sets' orders are independent per node and the draws need only
    // the lengths: emulate the orders on worker threads (a shared queue, the
    // lists differ in length) while this thread draws and fetches the other
    // nodes' picks, then helps with what is left
    std::vector<std::vector<int32_t>> fars(k2.size());
    const int helpers = std::min<int>(std::max<int32_t>(1, n_threads) - 1, static_cast<int>(k2.size()));
    if (helpers > 0 && (!u.team || u.team->helpers() < helpers)) u.team = std::make_unique<gs::Team>(helpers, 0);
    struct Waited {  // the job reads this frame: it has finished on every exit
        gs::Team* t;
        ~Waited() {
            if (t) t->wait();
        }
    } job{helpers > 0 ? u.team.get() : nullptr};
    auto emulate = [&](int q) {
        fars[static_cast<size_t>(q)].assign(host_far.begin() + k2base[q], host_far.begin() + k2base[q + 1]);
        fresh_set_order(fars[static_cast<size_t>(q)]);
    };
    if (job.t) job.t->start(static_cast<int>(k2.size()), emulate);
    // the draws, in node order on the one stream: positions into each far list
    const int64_t kmax = std::max<int64_t>(num_neg, 1);
    std::vector<int32_t> pick(static_cast<size_t>(n * kmax));
    std::vector<int32_t> pool;
    for (int64_t i = 0; i < n; ++i) {
        const int64_t len = u.n_train_set - tib[i];
        int32_t* out = pick.data() + i * kmax;
        if (num_neg < len) {
            if (len <= setsize) pool.resize(static_cast<size_t>(len));
            gs::sample_positions(rng->mt, len, num_neg, setsize, out, pool.data());
            u.neg_cnt[i] = num_neg;
        } else {
            for (int64_t t = 0; t < len; ++t) out[t] = static_cast<int32_t>(t);
            u.neg_cnt[i] = len;
        }
    }
    const auto t1b = clk::now();
    // copy-order and ascending-order picks: select queries on the device
    std::vector<int32_t> req_r, req_j;
    std::vector<uint8_t> req_kind;
    for (int64_t i = 0; i < n; ++i)
        if (kind[i] != 2)
            for (int64_t t = 0; t < u.neg_cnt[i]; ++t) {
                req_r.push_back(static_cast<int32_t>(i));
                req_j.push_back(pick[static_cast<size_t>(i * kmax + t)]);
                req_kind.push_back(static_cast<uint8_t>(kind[i] == 1));
            }
    const auto t2 = clk::now();
    std::vector<int32_t> ids;
    gs::unsup_dev_select(u.dev, req_r, req_j, req_kind, ids);
    const auto t2a = clk::now();
    if (job.t) {
        job.t->wait();
        job.t = nullptr;
    } else {
        for (int q = 0; q < static_cast<int>(k2.size()); ++q) emulate(q);
    }
    const auto t2b = clk::now();
    int64_t total = 0;
    for (int64_t i = 0; i < n; ++i) total += u.neg_cnt[i];
    u.neg.resize(static_cast<size_t>(2 * total));
    size_t q = 0, k2i = 0, at = 0;
    for (int64_t i = 0; i < n; ++i) {
        const int64_t v = u.nodes[static_cast<size_t>(i)];
        const int32_t* pk = pick.data() + i * kmax;
        const std::vector<int32_t>* farp = kind[i] == 2 ? &fars[k2i++] : nullptr;
        for (int64_t t = 0; t < u.neg_cnt[i]; ++t) {
            u.neg[at++] = v;
            u.neg[at++] = farp ? (*farp)[static_cast<size_t>(pk[t])] : ids[q++];
        }
    }
    if (prof) {
        auto ms = [](clk::time_point a, clk::time_point b) { return std::chrono::duration<double>(b - a).count() * 1e3; };
        std::fprintf(stderr,
                     "[unsup dev] balls %.2f far lists %.2f (%zu fresh sets, %lld ids) draws %.2f requests %.2f "
                     "select %.2f (%zu picks) fresh-order wait %.2f compose %.2f ms\n",
                     ms(t0, t1), ms(t1, t1a), k2.size(), static_cast<long long>(k2base.back()), ms(t1a, t1b),
                     ms(t1b, t2), ms(t2, t2a), req_r.size(), ms(t2a, t2b), ms(t2b, clk::now()));
    }
}
#endif

}  // namespace

extern "C" {

int gs_unsup_attach_device(gs_unsup* u, void* stream) {
    GS_API_BEGIN
    GS_REQUIRE(u, GS_EINVAL, "NULL argument");
#ifdef GS_HOST_ONLY
    (void)stream;
    gs::fail(GS_EINVAL, "host-only build: no device");
#else
    if (!u->dev) u->dev = gs::unsup_dev_create(*u->g, u->copy_order, u->train_order, stream);
#endif
    GS_API_END
}

int gs_unsup_create(const gs_graph* graph, const int64_t* train_nodes, int64_t n_train, int32_t n_walks,
                    int32_t walk_len, int32_t n_walk_len, gs_unsup** out) {
    GS_API_BEGIN
    GS_REQUIRE(graph && out && (train_nodes || n_train == 0) && n_train >= 0, GS_EINVAL, "bad arguments");
    GS_REQUIRE(n_walks >= 0 && walk_len >= 0 && n_walk_len >= 0, GS_EINVAL, "walk parameters must be >= 0");
    const auto* g = reinterpret_cast<const gs::Graph*>(graph);
    auto u = std::make_unique<gs_unsup>();
    u->g = g;
    u->n_walks = n_walks;
    u->walk_len = walk_len;
    u->n_walk_len = n_walk_len;
    u->is_train.assign(g->n_nodes, 0);
    PySet ts;  // set(self.train_nodes), models.py:163
    for (int64_t i = 0; i < n_train; ++i) {
        GS_REQUIRE(train_nodes[i] >= 0 && train_nodes[i] < g->n_nodes, GS_ERANGE, "train node id out of range");
        u->is_train[train_nodes[i]] = 1;
        ts.add(static_cast<int32_t>(train_nodes[i]));
    }
    u->n_train_set = ts.used;
    ts.for_each([&](int32_t x) { u->train_order.push_back(x); });
    gs::copy_of(ts).for_each([&](int32_t x) { u->copy_order.push_back(x); });
    *out = u.release();
    GS_API_END
}

void gs_unsup_destroy(gs_unsup* u) { delete u; }

int gs_unsup_extend(gs_unsup* u, gs_rng* rng, const int64_t* nodes, int64_t n, int64_t num_neg,
                    int32_t parts, int32_t n_threads, int64_t* sizes) {
    GS_API_BEGIN
    GS_REQUIRE(u && rng && sizes && (nodes || n == 0) && n >= 0, GS_EINVAL, "bad arguments");
    GS_REQUIRE(num_neg >= 0, GS_ERANGE, "Sample larger than population or is negative");
    GS_REQUIRE(parts >= 1 && parts <= 3, GS_EINVAL, "parts: 1 walks, 2 negatives, 3 both");
    const gs::Graph& g = *u->g;
    for (int64_t i = 0; i < n; ++i) GS_REQUIRE(nodes[i] >= 0 && nodes[i] < g.n_nodes, GS_ERANGE, "node id out of range");
    u->nodes.assign(nodes, nodes + n);
    u->pos.clear();
    u->neg.clear();
    u->unique.clear();
    u->pos_cnt.assign(n, 0);
    u->neg_cnt.assign(n, 0);
    u->has_pos.assign(n, 0);
    u->subset_ok = 0;
    static const bool prof = std::getenv("GS_UNSUP_PROF") != nullptr;
    using clk = std::chrono::steady_clock;
    const auto tw = clk::now();
    if (parts & 1) walk_pairs(*u, rng);
    const auto tn = clk::now();
#ifndef GS_HOST_ONLY
    if ((parts & 2) && u->dev) negative_pairs_dev(*u, rng, num_neg, n_threads);
    else
#endif
    if (parts & 2) negative_pairs(*u, rng, num_neg, n_threads);

    const auto tu = clk::now();
    PySet a, b;  // models.py:146
    // adding a present key leaves a set unchanged (no fill, no resize), so
    // only first occurrences reach the emulator: a bitmap filters the repeats
    // (a negatives list repeats its node once per pair)
    u->seen.resize(static_cast<size_t>((g.n_nodes + 63) >> 6), 0);
    auto add_distinct = [&](PySet& S, const std::vector<int64_t>& keys) {
        for (int64_t x : keys) {
            uint64_t& w = u->seen[static_cast<size_t>(x >> 6)];
            const uint64_t bit = uint64_t(1) << (x & 63);
            if (w & bit) continue;
            w |= bit;
            S.add(static_cast<int32_t>(x));
        }
        S.for_each([&](int32_t x) { u->seen[static_cast<size_t>(x >> 6)] = 0; });
    };
    add_distinct(a, u->pos);
    add_distinct(b, u->neg);
    const auto tu1 = clk::now();
    PySet r = gs::copy_of(a);
    r.merge(b);
    r.for_each([&](int32_t x) { u->unique.push_back(x); });
    const auto tu2 = clk::now();

    // set(target) < set(unique) (models.py:147): every target present and the
    // union strictly larger than the distinct targets.
    PySet tgt;
    for (int64_t x : u->nodes) tgt.add(static_cast<int32_t>(x));
    bool ok = r.used > tgt.used;
    for (int64_t x : u->nodes) ok = ok && r.find_slot(static_cast<int32_t>(x)) >= 0;
    u->subset_ok = ok ? 1 : 0;

    if (prof) {
        auto ms = [](clk::time_point x, clk::time_point y) { return std::chrono::duration<double>(y - x).count() * 1e3; };
        std::fprintf(stderr, "[unsup] walks %.2f negatives %.2f unique: sets %.2f union %.2f subset %.2f ms (%zu pos, %zu neg, %zu unique)\n",
                     ms(tw, tn), ms(tn, tu), ms(tu, tu1), ms(tu1, tu2), ms(tu2, clk::now()), u->pos.size() / 2,
                     u->neg.size() / 2, u->unique.size());
    }
    sizes[0] = static_cast<int64_t>(u->unique.size());
    sizes[1] = static_cast<int64_t>(u->pos.size() / 2);
    sizes[2] = static_cast<int64_t>(u->neg.size() / 2);
    sizes[3] = u->subset_ok;
    GS_API_END
}

int gs_unsup_fetch(const gs_unsup* u, int64_t* unique, int64_t* pos_pairs, int64_t* neg_pairs, int64_t* pos_cnt,
                   int64_t* neg_cnt, uint8_t* has_pos) {
    GS_API_BEGIN
    GS_REQUIRE(u, GS_EINVAL, "bad arguments");
    auto put = [](auto* dst, const auto& v) {
        if (dst && !v.empty()) std::memcpy(dst, v.data(), v.size() * sizeof(v[0]));
    };
    put(unique, u->unique);
    put(pos_pairs, u->pos);
    put(neg_pairs, u->neg);
    put(pos_cnt, u->pos_cnt);
    put(neg_cnt, u->neg_cnt);
    put(has_pos, u->has_pos);
    GS_API_END
}

// The loss loops of models.py:65-96 / :98-132 as index lists.  Dict semantics
// of node_positive_pairs / node_negtive_pairs: a key's position is its first
// occurrence in `nodes`, its value the last occurrence's pairs.  Scored nodes
// (both lists non-empty) in key order; rows are positions in unique
// (node2index, models.py:69).  Layout (int32):
//   pos_ptr[M+1] | neg_ptr[M+1] | pos_a[P] | pos_b[P] | neg_a[Nn] | neg_b[Nn]
//   | tptr[U+1] | tidx[2(P+Nn)]
// tidx lists, per embedding row, 2*g + side for every pair g it belongs to
// (g < P: positive pair g, else negative pair g-P; side 0 = first element),
// ascending: the fixed summation order of the row gradient.
int gs_unsup_loss_plan(const gs_unsup* u, int32_t* buf, int64_t cap, int64_t* dims, int64_t* used) {
    GS_API_BEGIN
    GS_REQUIRE(u && dims && used, GS_EINVAL, "bad arguments");
    const int64_t n = static_cast<int64_t>(u->nodes.size());
    const int64_t U = static_cast<int64_t>(u->unique.size());
    std::vector<int64_t> pofs(n + 1, 0), nofs(n + 1, 0);
    for (int64_t i = 0; i < n; ++i) {
        pofs[i + 1] = pofs[i] + u->pos_cnt[i];
        nofs[i + 1] = nofs[i] + u->neg_cnt[i];
    }
    // last occurrence per node id, key order = first occurrence
    PySet seen;
    std::vector<int64_t> keys;  // index of first occurrence
    std::vector<int64_t> last_of(n);
    {
        std::vector<int64_t> ids(u->nodes);
        std::vector<int64_t> order(n);
        for (int64_t i = 0; i < n; ++i) order[i] = i;
        std::stable_sort(order.begin(), order.end(), [&](int64_t a, int64_t b) { return ids[a] < ids[b]; });
        for (int64_t s = 0; s < n;) {
            int64_t e = s;
            while (e < n && ids[order[e]] == ids[order[s]]) ++e;
            for (int64_t t = s; t < e; ++t) last_of[order[t]] = order[e - 1];
            s = e;
        }
    }
    int64_t n_pos_keys = 0, n_neg_keys = 0;
    std::vector<int64_t> scored;  // occurrence whose lists are scored
    for (int64_t i = 0; i < n; ++i) {
        if (!seen.add(static_cast<int32_t>(u->nodes[i]))) continue;
        ++n_neg_keys;
        if (!u->has_pos[i]) continue;
        ++n_pos_keys;
        const int64_t li = last_of[i];
        if (u->pos_cnt[li] > 0 && u->neg_cnt[li] > 0) scored.push_back(li);
    }
    const int64_t M = static_cast<int64_t>(scored.size());
    int64_t P = 0, N = 0;
    for (int64_t li : scored) {
        P += u->pos_cnt[li];
        N += u->neg_cnt[li];
    }
    const int64_t need = 2 * (M + 1) + 2 * P + 2 * N + (U + 1) + 2 * (P + N);
    dims[0] = M;
    dims[1] = P;
    dims[2] = N;
    dims[3] = U;
    dims[4] = n_pos_keys;
    dims[5] = n_neg_keys;
    *used = need;
    if (!buf) return GS_OK;
    GS_REQUIRE(cap >= need, GS_EINVAL, "plan buffer too small");
    GS_REQUIRE(U < (int64_t(1) << 31) && P + N < (int64_t(1) << 30), GS_ERANGE, "batch too large for int32 plan");
    std::vector<int32_t> where(u->g->n_nodes, -1);
    for (int64_t r = 0; r < U; ++r) where[u->unique[r]] = static_cast<int32_t>(r);
    int32_t* pos_ptr = buf;
    int32_t* neg_ptr = pos_ptr + (M + 1);
    int32_t* pa = neg_ptr + (M + 1);
    int32_t* pb = pa + P;
    int32_t* na = pb + P;
    int32_t* nb = na + N;
    int32_t* tptr = nb + N;
    int32_t* tidx = tptr + (U + 1);
    int64_t p = 0, q = 0;
    auto row = [&](int64_t id) {
        const int32_t r = where[id];
        GS_REQUIRE(r >= 0, GS_EINVAL, "pair node missing from unique_nodes_batch");
        return r;
    };
    for (int64_t m = 0; m < M; ++m) {
        const int64_t li = scored[m];
        pos_ptr[m] = static_cast<int32_t>(p);
        neg_ptr[m] = static_cast<int32_t>(q);
        for (int64_t t = pofs[li]; t < pofs[li + 1]; ++t, ++p) {
            pa[p] = row(u->pos[2 * t]);
            pb[p] = row(u->pos[2 * t + 1]);
        }
        for (int64_t t = nofs[li]; t < nofs[li + 1]; ++t, ++q) {
            na[q] = row(u->neg[2 * t]);
            nb[q] = row(u->neg[2 * t + 1]);
        }
    }
    pos_ptr[M] = static_cast<int32_t>(P);
    neg_ptr[M] = static_cast<int32_t>(N);
    // transposed contribution lists (counting sort keeps 2g+side ascending)
    std::fill_n(tptr, U + 1, 0);
    auto each = [&](auto&& f) {
        for (int64_t g = 0; g < P; ++g) {
            f(pa[g], 2 * g);
            f(pb[g], 2 * g + 1);
        }
        for (int64_t g = 0; g < N; ++g) {
            f(na[g], 2 * (P + g));
            f(nb[g], 2 * (P + g) + 1);
        }
    };
    each([&](int32_t r, int64_t) { ++tptr[r + 1]; });
    for (int64_t r = 0; r < U; ++r) tptr[r + 1] += tptr[r];
    std::vector<int32_t> fillp(tptr, tptr + U);
    each([&](int32_t r, int64_t code) { tidx[fillp[r]++] = static_cast<int32_t>(code); });
    GS_API_END
}

}  // extern "C"
