// Host neighbour sampler: GraphSage._get_unique_neighs_list (models.py:277-289)
// applied hop by hop as GraphSage.forward does (models.py:246-251), bit-exact
// with the reference's CPython `random` stream and set iteration order.
//
// Per hop j (frontier F(j-1) -> union Fj), for every frontier node v in order:
//   deg(v) >= k : positions = random.sample(range(deg), k)   (consumes rng)
//   otherwise   : the whole row                               (no rng)
// Only the hops whose union feeds a later hop need the CPython-set replay
// (set(sample) | {v}, then set.union over the frontier).  The last hop's union
// only orders the rows of a gather, so by default it is skipped and the
// device expands the sampled positions through the CSR itself.
#include <algorithm>
#include <exception>
#include <mutex>
#include <atomic>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <vector>

#include <immintrin.h>

#include "common.hpp"
#include "graph.hpp"
#include "mt19937.hpp"
#include "pyset.hpp"
#include "rng.hpp"
#include "team.hpp"

#ifndef GS_PHASE  // phase marks of the sampler thread for tools/sampler_bench.cpp; no-ops in the library
#define GS_PHASE(i)  // 1 draws (hops before the last), 2 sets + union, 3 frontier list, 4 last-hop draws, 5 join
#endif

namespace gs {

struct Hop {
    int64_t k = 0;
    bool materialised = false;
    std::vector<int64_t> dst_ids;
    std::vector<int32_t> pos_ptr, pos;
    std::vector<int32_t> ent;  // absolute CSR entries row_ptr[dst] + pos (what the pack carries)
    std::vector<int64_t> src_ids;
    std::vector<int32_t> nbr_ptr, nbr, self_local;
    std::vector<int32_t> set_ptr;
    std::vector<int64_t> set_items;
    std::vector<int32_t> tptr, tidx;  // transposed (src -> dst) incl. self edges as -(r+1)
    int64_t n_empty = 0;              // empty neighbourhoods after the self rule
    int64_t n_pos = 0;                // sampled entries (== pos.size() unless drawn into a pack)
};

// A pack written while sampling (gs_sample_pack_run's path): the last hop's
// pos_ptr / entries / dst_ids go straight into the caller's buffer from the
// draws, and each earlier hop's lists are copied in by whoever built them (a
// helper, beside the next hop's draws), so the sampler thread never copies
// the pack afterwards.  `off` follows layout_of's field order and alignment.
struct PackOut {
    int32_t* buf = nullptr;
    int64_t cap = 0;
    int64_t at = 0;  // next free element
    int64_t off[GS_MAX_HOPS][GS_PK_NFIELDS];
    int64_t put(int32_t hop, int field, int64_t n) {
        off[hop][field] = at;
        at += (n + 3) & ~int64_t(3);  // every array 16-byte aligned
        GS_REQUIRE(at <= cap, GS_EINVAL, "pack exceeds its bound");
        return off[hop][field];
    }
};

struct Sample {
    int32_t n_hops = 0;
    int32_t flags = 0;
    Hop hops[GS_MAX_HOPS];
};

// Draw the sampled row positions of every frontier node, in frontier order.
// With `po` (the last hop of a pack run) the absolute CSR entries, pos_ptr
// and dst_ids go straight into the pack, h.pos / h.ent stay empty, and the
// destinations left empty by the self rule are counted on the way when asked
// (only a lone entry can be self: one col read — a cache miss — for those).
static void draw_positions(const Graph& g, MT19937& rng, Hop& h, PackOut* po = nullptr, int32_t hop = 0,
                           bool gcn = false, bool count_empties = false) {
    const int64_t n = static_cast<int64_t>(h.dst_ids.size());
    int32_t* pptr;
    if (po) {
        pptr = po->buf + po->put(hop, GS_PK_POS_PTR, n + 1);
    } else {
        h.pos_ptr.resize(n + 1);
        pptr = h.pos_ptr.data();
    }
    pptr[0] = 0;
    thread_local std::vector<int64_t> deg;
    deg.resize(n);
    int64_t total = 0;
    const int64_t* rp = g.row_ptr.data();
    constexpr int64_t kAhead = 48;  // frontier ids are known: prefetch their row_ptr (DRAM misses)
    for (int64_t r = 0; r < std::min(n, kAhead); ++r) __builtin_prefetch(rp + h.dst_ids[r]);
    for (int64_t r = 0; r < n; ++r) {
        if (r + kAhead < n) __builtin_prefetch(rp + h.dst_ids[r + kAhead]);
        const int64_t v = h.dst_ids[r];
        const int64_t d = rp[v + 1] - rp[v];
        deg[r] = d;
        total += (h.k > 0 && d >= h.k) ? h.k : d;
        GS_REQUIRE(total < (int64_t(1) << 31), GS_ERANGE, "sampled entries exceed int32");
        pptr[r + 1] = static_cast<int32_t>(total);
    }
    h.n_pos = total;
    int32_t* ent;
    int32_t* posv = nullptr;
    if (po) {
        ent = po->buf + po->put(hop, GS_PK_POS, total);
        int32_t* d = po->buf + po->put(hop, GS_PK_DST_IDS, n);
        for (int64_t r = 0; r < n; ++r) d[r] = static_cast<int32_t>(h.dst_ids[r]);
        h.pos.clear();
        h.ent.clear();
    } else {
        h.pos.resize(total);
        h.ent.resize(total);
        ent = h.ent.data();
        posv = h.pos.data();
    }
    const int64_t setsize = sample_setsize(h.k);
    thread_local std::vector<int32_t> pool, tmp;
    pool.resize(std::max<int64_t>(setsize, 1));
    int64_t empty = 0;
    for (int64_t r = 0; r < n; ++r) {
        const int64_t d = deg[r];
        const int64_t cnt = pptr[r + 1] - pptr[r];
        const int32_t rs = static_cast<int32_t>(rp[h.dst_ids[r]]);  // < 2^31 (checked in run_sample)
        int32_t* ep = ent + pptr[r];
        if (h.k > 0 && d >= h.k) {
            int32_t* dstp = posv ? posv + pptr[r] : ep;  // positions, then entries in place
            sample_positions(rng, d, h.k, setsize, dstp, pool.data());
            for (int64_t t = 0; t < cnt; ++t) ep[t] = rs + dstp[t];
        } else {
            if (posv)
                for (int64_t t = 0; t < d; ++t) posv[pptr[r] + t] = static_cast<int32_t>(t);
            for (int64_t t = 0; t < d; ++t) ep[t] = rs + static_cast<int32_t>(t);
        }
        if (count_empties && !gcn) empty += cnt == 0 || (cnt == 1 && g.col[ep[0]] == h.dst_ids[r]);
    }
    if (po) h.n_empty = empty;  // 0 unless counted
}

// Destinations left without neighbours once self is removed (non-gcn): the
// sampled entries are distinct, so only 0 entries or a lone self qualify.
static int64_t count_empty(const Graph& g, const Hop& h, bool gcn) {
    int64_t e = 0;
    for (size_t r = 0; r < h.dst_ids.size(); ++r) {
        const int64_t c = h.pos_ptr[r + 1] - h.pos_ptr[r];
        if (gcn) continue;  // self is always present
        if (c == 0) ++e;
        else if (c == 1 && g.col[g.row_ptr[h.dst_ids[r]] + h.pos[h.pos_ptr[r]]] == h.dst_ids[r]) ++e;
    }
    return e;
}

// CPython-set replay of :282-288 for one hop, in three phases:
//   sets_range    samp_neighs[r] = S_r | {v} for a range of r: kept only as
//                 each set's iteration order (set_items) — all the union needs
//                 from r >= 1 — plus the full table of r == 0, which the union
//                 copies.  Independent per r (helper threads split it).
//   union_map     list(set.union(*samp_neighs)) (:286): the next frontier in
//                 iteration order, and each union slot's rank in it.
//   lists         per-destination neighbour lists in union-local ids and the
//                 transposed lists the backward pass gathers over.  Needs
//                 nothing the next hop's draws produce, so it overlaps them.
struct HopScratch {
    PySet first, u;                   // samp_neighs[0]; the union
    std::vector<int32_t> slot_local;  // union slot -> rank in iteration order
    std::vector<std::vector<int64_t>> part_items;  // per chunk of sets_union (per part of build_sets)
    std::unique_ptr<std::atomic<int>[]> chunk_done;  // sets_union: chunk c's sets are built
    int64_t n_chunk_cap = 0;
    std::atomic<int64_t> next_chunk{0};  // sets_union: the next chunk to build
    int64_t n_items = 0;              // items of all sets of the hop
    std::vector<int32_t> counts;      // sets_union: items per set
    std::vector<int64_t> chunk_base;  // lists: chunk c's first item
    std::vector<int32_t> cur;         // lists: transpose cursors
};

static void sets_range(const Graph& g, const Hop& h, int64_t a, int64_t b, std::vector<int64_t>& items,
                       int32_t* counts, PySet* first) {
    PySet s, t;
    // the rows read below are known ahead (positions are drawn): prefetch the
    // col / slot lines of the row kAhead destinations on (random row reads
    // dominate this loop on large graphs), and its row_ptr / table-size bytes
    // further ahead still
    constexpr int64_t kAhead = 4, kMeta = 16;
    auto prefetch_row = [&](int64_t q) {
        const int64_t v = h.dst_ids[q];
        const int64_t rs = g.row_ptr[v], d = g.row_ptr[v + 1] - rs;
        if (h.k > 0 && d >= h.k) {
            for (int32_t t = h.pos_ptr[q]; t < h.pos_ptr[q + 1]; ++t) __builtin_prefetch(g.col.data() + rs + h.pos[t]);
        } else {
            for (int64_t t = 0; t < d; t += 16) {
                __builtin_prefetch(g.col.data() + rs + t);
                __builtin_prefetch(g.slot.data() + rs + t);
            }
        }
    };
    auto prefetch_meta = [&](int64_t q) {
        const int64_t v = h.dst_ids[q];
        __builtin_prefetch(g.row_ptr.data() + v);
        __builtin_prefetch(g.log2size.data() + v);
    };
    for (int64_t q = a; q < std::min(b, a + kMeta); ++q) prefetch_meta(q);
    for (int64_t q = a; q < std::min(b, a + kAhead); ++q) prefetch_row(q);
    for (int64_t r = a; r < b; ++r) {
        if (r + kMeta < b) prefetch_meta(r + kMeta);
        if (r + kAhead < b) prefetch_row(r + kAhead);
        const int64_t v = h.dst_ids[r];
        const int64_t rs = g.row_ptr[v], d = g.degree(v);
        const int64_t cnt = h.pos_ptr[r + 1] - h.pos_ptr[r];
        if (h.k > 0 && d >= h.k) {
            // set(random.sample(adj, k)) : adds in result order
            s.reset();  // the sampled entries are distinct positions of one row: distinct keys
            for (int64_t q = 0; q < cnt; ++q) s.add_absent(g.col[rs + h.pos[h.pos_ptr[r] + q]]);
            copy_into(t, s);  // samp_neigh | set([v])  (:285)
        } else {
            // the adjacency set object itself (its own table layout; dummies
            // disable the slot-copy fast path), copied by the `|`
            t.assign_copy_of_layout((size_t(1) << g.log2size[v]) - 1, g.col.data() + rs, g.slot.data() + rs, d,
                                    !g.dirty.empty() && g.dirty[v]);
        }
        t.merge_single(v);
        if (r == 0 && first) *first = t;
        const size_t before = items.size();
        t.for_each([&](int64_t key) { items.push_back(key); });
        counts[r] = static_cast<int32_t>(items.size() - before);
    }
}

// The frontier union list(set.union(*samp_neighs)) (:286) merged in set
// order while the sets are still being built: the sets are cut into chunks
// of kChunk destinations, taken in order from a shared counter by the
// helpers and by this thread; this thread merges chunk c into the union as
// soon as it is complete (set 0's full table first), and builds the next
// unclaimed chunk itself whenever the one it needs is still in progress.
// The union sees exactly the sequential merge order; only the set builds
// overlap it.  Leaves each chunk's items in sc.part_items and per-set counts
// in sc.counts[r] (the lists job makes set_ptr / set_items from them).
static constexpr int64_t kChunk = 32;

static void sets_union(const Graph& g, Hop& h, HopScratch& sc, Team* team) {
    const int64_t n = static_cast<int64_t>(h.dst_ids.size());
    const int64_t nch = (n + kChunk - 1) / kChunk;
    h.set_ptr.resize(n + 1);
    sc.counts.resize(n);
    if (static_cast<int64_t>(sc.part_items.size()) < nch) sc.part_items.resize(nch);
    if (sc.n_chunk_cap < nch) {
        sc.chunk_done.reset(new std::atomic<int>[nch]);
        sc.n_chunk_cap = nch;
    }
    for (int64_t c = 0; c < nch; ++c) sc.chunk_done[c].store(0, std::memory_order_relaxed);
    sc.next_chunk.store(0, std::memory_order_relaxed);
    int32_t* counts = sc.counts.data();
    // A chunk build that throws (bad_alloc in a set or an items vector) marks
    // its chunk failed (2) instead of done (1), so the merge loop stops
    // instead of spinning on it; the first exception is rethrown here once
    // every helper has left the chunk loop (their job refers to this frame).
    std::exception_ptr err;
    std::mutex err_mu;
    auto keep_error = [&] {
        std::lock_guard<std::mutex> lk(err_mu);
        if (!err) err = std::current_exception();
    };
    auto build = [&](int64_t c) {
        try {
            const int64_t a = c * kChunk, b = std::min(n, a + kChunk);
            auto& items = sc.part_items[c];
            items.clear();
            sets_range(g, h, a, b, items, counts, c == 0 ? &sc.first : nullptr);
            sc.chunk_done[c].store(1, std::memory_order_release);
        } catch (...) {
            keep_error();
            sc.chunk_done[c].store(2, std::memory_order_release);
        }
    };
    const bool helped = team && nch > 1;
    if (helped)
        team->start(static_cast<int>(std::min<int64_t>(team->helpers(), nch - 1)), [&](int) {
            for (int64_t c; (c = sc.next_chunk.fetch_add(1, std::memory_order_relaxed)) < nch;) build(c);
        });
    PySet& u = sc.u;
    int64_t n_items = 0;
    try {
        u.reset();
        for (int64_t c = 0; c < nch; ++c) {
            int st;
            while ((st = sc.chunk_done[c].load(std::memory_order_acquire)) == 0) {
                const int64_t m = sc.next_chunk.fetch_add(1, std::memory_order_relaxed);
                if (m < nch) build(m);  // m >= c: everything before c was claimed already
                else _mm_pause();
            }
            if (st != 1) break;  // that chunk's build failed: err holds why
            const int64_t a = c * kChunk, b = std::min(n, a + kChunk);
            const auto& items = sc.part_items[c];
            n_items += static_cast<int64_t>(items.size());
            // this chunk's runs: set_ptr-style offsets into `items`
            int32_t ptr[kChunk + 1];
            ptr[0] = 0;
            for (int64_t r = a; r < b; ++r) ptr[r - a + 1] = ptr[r - a] + counts[r];
            if (c == 0) {
                copy_into(u, sc.first);  // non-empty: merge_runs never sees fill == 0
                u.merge_runs(items.data(), ptr + 1, b - a - 1);
            } else {
                u.merge_runs(items.data(), ptr, b - a);
            }
        }
    } catch (...) {
        keep_error();
    }
    if (err) sc.next_chunk.store(nch, std::memory_order_relaxed);  // no helper claims another chunk
    if (helped) team->wait();  // every helper is out of the chunk loop
    if (err) std::rethrow_exception(err);
    sc.n_items = n_items;
    GS_PHASE(2);
}

static void union_map(Hop& h, HopScratch& sc) {
    PySet& u = sc.u;
    // The next frontier: the union's keys in slot order (a vector compaction
    // of the table).  The slot -> rank map the lists need is built by lists().
    h.src_ids.resize(static_cast<size_t>(u.used));
    int64_t* dst = h.src_ids.data();
    const __m256i empty = _mm256_set1_epi32(PySet::EMPTY);
    size_t sl = 0;
    for (; sl + 8 <= u.mask + 1; sl += 8) {
        const __m256i v = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(u.tab + sl));
        uint32_t m = ~static_cast<uint32_t>(_mm256_movemask_ps(_mm256_castsi256_ps(_mm256_cmpeq_epi32(v, empty)))) & 0xFFu;
        while (m) {
            *dst++ = u.tab[sl + __builtin_ctz(m)];
            m &= m - 1;
        }
    }
    for (; sl <= u.mask; ++sl)
        if (u.tab[sl] != PySet::EMPTY) *dst++ = u.tab[sl];
}

// part 0: the neighbour lists and self ids; part 1: the transposed lists
static void copy_lists(const Hop& h, PackOut& po, int32_t j, int part) {
    auto cpy = [&](int f, const std::vector<int32_t>& v) {
        if (!v.empty()) std::memcpy(po.buf + po.off[j][f], v.data(), v.size() * sizeof(int32_t));
    };
    if (part == 0) {
        cpy(GS_PK_NBR_PTR, h.nbr_ptr);
        cpy(GS_PK_NBR, h.nbr);
        cpy(GS_PK_SELF, h.self_local);
    } else {
        cpy(GS_PK_TPTR, h.tptr);
        cpy(GS_PK_TIDX, h.tidx);
    }
}

// A hop's lists from its sets and the union (lists_task on up to
// `workers` threads at once, each taking units of each stage in turn):
//   stage 0  the union's slot -> rank map (one unit);
//   stage 1  per sets_union chunk: h.set_items / h.set_ptr (the chunks'
//            items concatenated and scanned, for the Sample view), each
//            destination's neighbourhood in union-local ids, ascending (the
//            dense mask's column order, :305-308; non-gcn drops self,
//            :297-298), and its self id;
//   stage 2  the transposed lists over the sources (for source c, the
//            destinations reading it, r >= 0, and those whose self row it is,
//            -(r+1), r ascending) and their pack copy; beside it (a second
//            unit, with a pack) the pack copy of the stage-1 lists.
// A worker claims units until its stage has none left, then waits for the
// units other workers claimed (each is running: no wait depends on a task
// that has not started), so one worker alone runs everything, in order, and
// more workers give the same lists.  Every buffer is sized by lists_prepare
// on the submitting thread: the tasks allocate nothing.
struct ListsJob {
    static constexpr int kStages = 3;
    Hop* h = nullptr;
    HopScratch* sc = nullptr;
    PackOut* po = nullptr;
    int32_t j = 0;
    bool gcn = false;
    int64_t units[kStages] = {1, 0, 1};
    std::atomic<int64_t> claim[kStages], done[kStages];
    std::atomic<bool> failed{false};
};

static void lists_prepare(ListsJob& L, Hop& h, HopScratch& sc, bool gcn, PackOut* po, int32_t j) {
    const int64_t n = static_cast<int64_t>(h.dst_ids.size());
    const int64_t nch = (n + kChunk - 1) / kChunk;
    const int64_t ns = static_cast<int64_t>(h.src_ids.size());
    L.h = &h;
    L.sc = &sc;
    L.po = po;
    L.j = j;
    L.gcn = gcn;
    L.units[1] = nch;
    L.units[2] = po ? 2 : 1;
    for (int s = 0; s < ListsJob::kStages; ++s) {
        L.claim[s].store(0, std::memory_order_relaxed);
        L.done[s].store(0, std::memory_order_relaxed);
    }
    L.failed.store(false, std::memory_order_relaxed);
    // chunk c's first item (sc.chunk_base[c]); the per-set counts are in sc.counts
    // (the lists job writes h.set_ptr itself)
    sc.chunk_base.resize(static_cast<size_t>(nch) + 1);
    sc.chunk_base[0] = 0;
    for (int64_t c = 0; c < nch; ++c)
        sc.chunk_base[c + 1] = sc.chunk_base[c] + static_cast<int64_t>(sc.part_items[c].size());
    h.set_items.resize(static_cast<size_t>(sc.n_items));
    sc.slot_local.resize(sc.u.mask + 1);
    h.nbr_ptr.resize(static_cast<size_t>(n) + 1);
    h.nbr.resize(static_cast<size_t>(sc.n_items - (gcn ? 0 : n)));
    h.self_local.resize(static_cast<size_t>(n));
    h.tptr.assign(static_cast<size_t>(ns) + 1, 0);
    h.tidx.resize(h.nbr.size() + static_cast<size_t>(n));
    sc.cur.resize(static_cast<size_t>(ns));
}

static void lists_unit(ListsJob& L, int stage, int64_t unit) {
    Hop& h = *L.h;
    HopScratch& sc = *L.sc;
    const PySet& u = sc.u;
    const int64_t n = static_cast<int64_t>(h.dst_ids.size());
    if (stage == 0) {
        // union-local position = rank of the key's slot in the union's table
        // (its iteration order): a probe of that cache-resident table instead
        // of a graph-sized node -> position array
        int32_t rank = 0;
        for (size_t sl = 0; sl <= u.mask; ++sl) {
            sc.slot_local[sl] = rank;
            rank += u.tab[sl] != PySet::EMPTY;
        }
        return;
    }
    if (stage == 1) {
        const int64_t c = unit, a = c * kChunk, b = std::min(n, a + kChunk);
        const std::vector<int64_t>& items = sc.part_items[c];
        const int64_t base = sc.chunk_base[c];
        if (!items.empty()) std::memcpy(h.set_items.data() + base, items.data(), items.size() * sizeof(int64_t));
        const int32_t* cnt = sc.counts.data() + a;
        int64_t q = 0;  // item index within the chunk
        const int64_t m = static_cast<int64_t>(items.size());
        for (int64_t r = a; r < b; ++r) {
            const int64_t v = h.dst_ids[r];
            const int64_t beg = base + q;
            h.set_ptr[r] = static_cast<int32_t>(beg);
            int32_t* out = h.nbr.data() + (beg - (L.gcn ? 0 : r));
            h.nbr_ptr[r] = static_cast<int32_t>(beg - (L.gcn ? 0 : r));
            int32_t k = 0;
            for (const int64_t qe = q + cnt[r - a]; q < qe; ++q) {
                if (q + 16 < m) __builtin_prefetch(u.tab + (static_cast<size_t>(items[q + 16]) & u.mask));
                const int64_t key = items[q];
                if (!L.gcn && key == v) continue;
                const int32_t x = sc.slot_local[static_cast<size_t>(u.find_slot(static_cast<int32_t>(key)))];
                int32_t p = k++;  // insertion sort: lists are <= k+1 long
                for (; p > 0 && out[p - 1] > x; --p) out[p] = out[p - 1];
                out[p] = x;
            }
            h.self_local[r] = sc.slot_local[static_cast<size_t>(u.find_slot(static_cast<int32_t>(v)))];
        }
        if (b == n) {
            h.set_ptr[n] = static_cast<int32_t>(base + m);
            h.nbr_ptr[n] = static_cast<int32_t>(h.nbr.size());
        }
        return;
    }
    // stage 2
    if (unit == 1) {
        copy_lists(h, *L.po, L.j, 0);
        return;
    }
    const int64_t ns = static_cast<int64_t>(h.src_ids.size());
    for (int32_t c : h.nbr) ++h.tptr[c + 1];
    for (int32_t c : h.self_local) ++h.tptr[c + 1];
    for (int64_t c = 0; c < ns; ++c) h.tptr[c + 1] += h.tptr[c];
    std::vector<int32_t>& cur = sc.cur;
    std::copy(h.tptr.begin(), h.tptr.end() - 1, cur.begin());
    for (int64_t r = 0; r < n; ++r) {
        h.tidx[cur[h.self_local[r]]++] = static_cast<int32_t>(-(r + 1));
        for (int32_t e = h.nbr_ptr[r]; e < h.nbr_ptr[r + 1]; ++e) h.tidx[cur[h.nbr[e]]++] = static_cast<int32_t>(r);
    }
    h.materialised = true;
    if (L.po) copy_lists(h, *L.po, L.j, 1);
}

// A unit that throws marks the job failed (later units are skipped, their
// stages still complete); the worker that caught it rethrows once every stage
// is done, so the team's wait() (or the inline caller) sees it.
static void lists_task(ListsJob& L) {
    std::exception_ptr mine;
    for (int s = 0; s < ListsJob::kStages; ++s) {
        for (int64_t t; (t = L.claim[s].fetch_add(1, std::memory_order_relaxed)) < L.units[s];) {
            if (!L.failed.load(std::memory_order_relaxed)) {
                try {
                    lists_unit(L, s, t);
                } catch (...) {
                    mine = std::current_exception();
                    L.failed.store(true, std::memory_order_relaxed);
                }
            }
            L.done[s].fetch_add(1, std::memory_order_acq_rel);
        }
        while (L.done[s].load(std::memory_order_acquire) < L.units[s]) _mm_pause();
    }
    if (mine) std::rethrow_exception(mine);
}

// Sampling state reused from batch to batch by one thread (the runner's
// sampler streams): every vector keeps its capacity, so a batch allocates
// nothing once the first few have run.
struct SampleCtx {
    Sample s;
    HopScratch scratch[2];  // hop j's lists may still run on a helper while hop j+1 builds its sets
    ListsJob lists[2];      // hop j's lists job (on scratch[j & 1])
    std::vector<int64_t> frontier;
};

// count_empties: fill Hop::n_empty (the Sample view reports it; a pack run
// needs it only to fail MAX batches, GS_SAMPLE_FAIL_EMPTY — its scan re-reads
// a row entry of every single-sample destination, ~2-3 % of a batch).
// po: write the pack while sampling (PackOut; not with GS_SAMPLE_FULL).
static void run_sample_into(SampleCtx& c, const Graph& g, MT19937& rng, const int64_t* roots, int64_t n_roots,
                            const int32_t* fanouts, int32_t n_hops, int32_t flags, Team* team,
                            bool count_empties = true, PackOut* po = nullptr) {
    GS_REQUIRE(n_hops >= 1 && n_hops <= GS_MAX_HOPS, GS_EINVAL, "n_hops out of [1, 8]");
    GS_REQUIRE(n_roots >= 1 && roots, GS_EINVAL, "empty nodes_batch");
    GS_REQUIRE(g.n_entries < (int64_t(1) << 31), GS_ERANGE, "graph has >= 2^31 CSR entries (int32 pack entries)");
    GS_REQUIRE(!po || !(flags & GS_SAMPLE_FULL), GS_EINVAL, "pack output with GS_SAMPLE_FULL");
    for (int64_t i = 0; i < n_roots; ++i)
        GS_REQUIRE(roots[i] >= 0 && roots[i] < g.n_nodes, GS_ERANGE, "node id out of range");
    if (team && team->helpers() == 0) team = nullptr;
    Sample* s = &c.s;
    s->n_hops = n_hops;
    s->flags = flags;
    for (int32_t j = 0; j < GS_MAX_HOPS; ++j) s->hops[j].materialised = false;
    const bool gcn = flags & GS_SAMPLE_GCN;
    std::vector<int64_t>& frontier = c.frontier;
    frontier.assign(roots, roots + n_roots);
    bool pending = false;  // a lists job is outstanding on the team
    struct Join {           // never leave a helper job behind (an exception unwinds through here)
        Team* t;
        bool& p;
        ~Join() {
            if (p) t->wait();
        }
    } join{team, pending};
    GS_PHASE(0);
    for (int32_t j = 0; j < n_hops; ++j) {
        Hop& h = s->hops[j];
        h.k = fanouts ? fanouts[j] : 10;
        h.dst_ids.swap(frontier);
        const bool last = (j == n_hops - 1);
        if (last && po) {
            draw_positions(g, rng, h, po, j, gcn, count_empties);  // pos_ptr, entries, dst_ids into the pack
            GS_PHASE(4);
            continue;
        }
        draw_positions(g, rng, h);
        h.n_empty = count_empties ? count_empty(g, h, gcn) : 0;
        GS_PHASE(last ? 4 : 1);
        if (!last || (flags & GS_SAMPLE_FULL)) {
            HopScratch& sc = c.scratch[j & 1];
            if (pending) {  // the team is needed for the sets below
                team->wait();
                pending = false;
            }
            sets_union(g, h, sc, team);
            union_map(h, sc);
            frontier.assign(h.src_ids.begin(), h.src_ids.end());
            GS_PHASE(3);
            if (po) {  // this hop's list fields: sizes are known from the sets and the union
                const int64_t n = static_cast<int64_t>(h.dst_ids.size());
                const int64_t n_nbr = sc.n_items - (gcn ? 0 : n);
                po->put(j, GS_PK_NBR_PTR, n + 1);
                po->put(j, GS_PK_NBR, n_nbr);
                po->put(j, GS_PK_SELF, n);
                po->put(j, GS_PK_TPTR, static_cast<int64_t>(h.src_ids.size()) + 1);
                po->put(j, GS_PK_TIDX, n_nbr + n);
            }
            ListsJob& L = c.lists[j & 1];
            lists_prepare(L, h, sc, gcn, po, j);
            if (team) {  // lists + transpose (+ their pack copy) on the helpers, under the next hop's draws
                const int64_t nw = std::min<int64_t>(team->helpers(), L.units[1]);
                team->start(static_cast<int>(std::max<int64_t>(nw, 1)), [&L](int) { lists_task(L); });
                pending = true;
            } else {
                lists_task(L);
            }
        }
    }
    if (pending) {
        team->wait();
        pending = false;
    }
    GS_PHASE(5);
}

static Sample* run_sample(const Graph& g, MT19937& rng, const int64_t* roots, int64_t n_roots,
                          const int32_t* fanouts, int32_t n_hops, int32_t flags, Team* team = nullptr) {
    std::unique_ptr<SampleCtx> c(new SampleCtx());
    run_sample_into(*c, g, rng, roots, n_roots, fanouts, n_hops, flags, team);
    return new Sample(std::move(c->s));
}

}  // namespace gs

using gs::Hop;
using gs::Sample;

extern "C" {

int gs_rng_create(gs_rng** out) {
    GS_API_BEGIN
    GS_REQUIRE(out, GS_EINVAL, "out is NULL");
    *out = new gs_rng();
    const uint32_t zero = 0;
    (*out)->mt.init_by_array(&zero, 1);
    GS_API_END
}

void gs_rng_destroy(gs_rng* rng) { delete rng; }

int gs_rng_seed_words(gs_rng* rng, const uint32_t* key, int64_t key_len) {
    GS_API_BEGIN
    GS_REQUIRE(rng && key && key_len >= 1, GS_EINVAL, "bad seed key");
    rng->mt.init_by_array(key, static_cast<size_t>(key_len));
    GS_API_END
}

int gs_rng_set_state(gs_rng* rng, const uint32_t* mt624, int64_t pos) {
    GS_API_BEGIN
    GS_REQUIRE(rng && mt624, GS_EINVAL, "bad state");
    GS_REQUIRE(pos >= 0 && pos <= gs::MT19937::N, GS_EINVAL, "state index out of range");
    std::memcpy(rng->mt.mt, mt624, sizeof(rng->mt.mt));
    rng->mt.index = static_cast<int>(pos);
    rng->mt.refresh();
    GS_API_END
}

int gs_rng_get_state(const gs_rng* rng, uint32_t* mt624, int64_t* pos) {
    GS_API_BEGIN
    GS_REQUIRE(rng && mt624 && pos, GS_EINVAL, "bad state buffers");
    std::memcpy(mt624, rng->mt.mt, sizeof(rng->mt.mt));
    *pos = rng->mt.index;
    GS_API_END
}

int gs_rng_getrandbits(gs_rng* rng, int32_t k, int64_t count, uint32_t* out) {
    GS_API_BEGIN
    GS_REQUIRE(rng && out && count >= 0, GS_EINVAL, "bad arguments");
    GS_REQUIRE(k >= 1 && k <= 32, GS_EINVAL, "k must be in [1, 32]");
    for (int64_t i = 0; i < count; ++i) out[i] = rng->mt.getrandbits(k);
    GS_API_END
}

int gs_rng_randbelow(gs_rng* rng, uint32_t n, int64_t count, uint32_t* out) {
    GS_API_BEGIN
    GS_REQUIRE(rng && out && count >= 0, GS_EINVAL, "bad arguments");
    for (int64_t i = 0; i < count; ++i) out[i] = rng->mt.randbelow(n);
    GS_API_END
}

int gs_rng_sample_positions(gs_rng* rng, int64_t n, int64_t k, int64_t* out) {
    GS_API_BEGIN
    GS_REQUIRE(rng && (out || k == 0), GS_EINVAL, "bad arguments");
    GS_REQUIRE(n >= 0 && n < (int64_t(1) << 32), GS_EINVAL, "population size out of range");
    GS_REQUIRE(k >= 0 && k <= n, GS_ERANGE, "Sample larger than population or is negative");
    const int64_t setsize = gs::sample_setsize(k);
    std::vector<int32_t> pool(static_cast<size_t>(std::max<int64_t>(std::min(setsize, n), 1)));
    gs::sample_positions(rng->mt, n, k, setsize, out, pool.data());
    GS_API_END
}

int gs_rng_choice_position(gs_rng* rng, int64_t n, int64_t* out) {
    GS_API_BEGIN
    GS_REQUIRE(rng && out, GS_EINVAL, "bad arguments");
    GS_REQUIRE(n >= 1 && n < (int64_t(1) << 32), GS_EINVAL, "choice from an empty sequence");
    *out = rng->mt.randbelow(static_cast<uint64_t>(n));
    GS_API_END
}

int gs_pyset_union_of_lists(const int64_t* items, const int64_t* ptr, int64_t n_lists, int64_t* out,
                            int64_t* out_len) {
    GS_API_BEGIN
    GS_REQUIRE(ptr && out && out_len && n_lists >= 1, GS_EINVAL, "bad arguments");
    std::vector<gs::PySet> sets(n_lists);
    for (int64_t l = 0; l < n_lists; ++l)
        for (int64_t t = ptr[l]; t < ptr[l + 1]; ++t) {
            GS_REQUIRE(items[t] >= 0, GS_EINVAL, "keys must be non-negative");
            sets[l].add(items[t]);
        }
    gs::PySet u = gs::copy_of(sets[0]);
    for (int64_t l = 1; l < n_lists; ++l) u.merge(sets[l]);
    int64_t w = 0;
    u.for_each([&](int64_t key) { out[w++] = key; });
    *out_len = w;
    GS_API_END
}

int gs_sample_run(const gs_graph* gp, gs_rng* rng, const int64_t* roots, int64_t n_roots,
                  const int32_t* fanouts, int32_t n_hops, int32_t flags, gs_sample** out) {
    GS_API_BEGIN
    GS_REQUIRE(gp && rng && out, GS_EINVAL, "NULL graph/rng/out");
    const auto& g = *reinterpret_cast<const gs::Graph*>(gp);
    *out = reinterpret_cast<gs_sample*>(
        gs::run_sample(g, rng->mt, roots, n_roots, fanouts, n_hops, flags));
    GS_API_END
}

void gs_sample_destroy(gs_sample* s) { delete reinterpret_cast<Sample*>(s); }

int gs_sample_n_hops(const gs_sample* sp, int32_t* n_hops) {
    GS_API_BEGIN
    GS_REQUIRE(sp && n_hops, GS_EINVAL, "NULL argument");
    *n_hops = reinterpret_cast<const Sample*>(sp)->n_hops;
    GS_API_END
}

int gs_sample_hop(const gs_sample* sp, int32_t hop, gs_hop_view* v) {
    GS_API_BEGIN
    GS_REQUIRE(sp && v, GS_EINVAL, "NULL argument");
    const Sample& s = *reinterpret_cast<const Sample*>(sp);
    GS_REQUIRE(hop >= 1 && hop <= s.n_hops, GS_EINVAL, "hop out of range");
    const Hop& h = s.hops[hop - 1];
    std::memset(v, 0, sizeof(*v));
    v->n_dst = static_cast<int64_t>(h.dst_ids.size());
    v->n_pos = static_cast<int64_t>(h.pos.size());
    v->dst_ids = h.dst_ids.data();
    v->pos_ptr = h.pos_ptr.data();
    v->pos = h.pos.data();
    v->n_empty = h.n_empty;
    if (h.materialised) {
        v->n_src = static_cast<int64_t>(h.src_ids.size());
        v->n_nbr = static_cast<int64_t>(h.nbr.size());
        v->src_ids = h.src_ids.data();
        v->nbr_ptr = h.nbr_ptr.data();
        v->nbr = h.nbr.data();
        v->self_local = h.self_local.data();
        v->set_ptr = h.set_ptr.data();
        v->set_items = h.set_items.data();
    } else {
        v->n_src = -1;
        v->n_nbr = -1;
    }
    GS_API_END
}

static void layout_of(const Sample& s, gs_pack_layout* L) {
    for (auto& row : L->off)
        for (auto& o : row) o = -1;
    int64_t at = 0;
    auto put = [&](int32_t hop, int field, int64_t n) {
        L->off[hop][field] = at;
        at += (n + 3) & ~int64_t(3);  // keep every array 16-byte aligned
    };
    for (int32_t j = 0; j < s.n_hops; ++j) {
        const Hop& h = s.hops[j];
        const int64_t nd = static_cast<int64_t>(h.dst_ids.size());
        if (j == s.n_hops - 1) {
            put(j, GS_PK_POS_PTR, nd + 1);
            put(j, GS_PK_POS, static_cast<int64_t>(h.pos.size()));
            put(j, GS_PK_DST_IDS, nd);
        } else {
            put(j, GS_PK_NBR_PTR, nd + 1);
            put(j, GS_PK_NBR, static_cast<int64_t>(h.nbr.size()));
            put(j, GS_PK_SELF, nd);
            put(j, GS_PK_TPTR, static_cast<int64_t>(h.tptr.size()));
            put(j, GS_PK_TIDX, static_cast<int64_t>(h.tidx.size()));
        }
    }
    L->total = at;
}

int gs_sample_pack_layout(const gs_sample* sp, gs_pack_layout* out) {
    GS_API_BEGIN
    GS_REQUIRE(sp && out, GS_EINVAL, "NULL argument");
    layout_of(*reinterpret_cast<const Sample*>(sp), out);
    GS_API_END
}

int64_t gs_sample_pack_bound(const gs_graph* gp, int64_t n_roots, const int32_t* fanouts, int32_t n_hops) {
    if (!gp || n_roots < 1 || n_hops < 1 || n_hops > GS_MAX_HOPS) return -1;
    const auto& g = *reinterpret_cast<const gs::Graph*>(gp);
    auto al = [](int64_t n) { return (n + 3) & ~int64_t(3); };
    int64_t nd = n_roots, total = 0;
    for (int32_t j = 0; j < n_hops; ++j) {
        const int64_t k = fanouts ? fanouts[j] : 10;
        const int64_t per = (k > 0) ? std::min<int64_t>(k, g.max_degree) : g.max_degree;
        const int64_t npos = nd * per;
        const int64_t nsrc = std::min<int64_t>(g.n_nodes, nd + npos);
        const int64_t nnbr = npos + nd;
        if (j == n_hops - 1) total += al(nd + 1) + al(npos) + al(nd);
        else total += al(nd + 1) + al(nnbr) + al(nd) + al(nsrc + 1) + al(nnbr + nd);
        nd = nsrc;
    }
    return total + al(n_roots);
}

static int pack_run(const gs_graph* gp, gs_rng* rng, const int64_t* roots, int64_t n_roots, const int32_t* fanouts,
                    int32_t n_hops, int32_t flags, int32_t* buf, int64_t cap, int64_t* hop_sizes, int64_t* offsets,
                    int64_t* used, gs::Team* team);

int gs_sample_pack_run(const gs_graph* gp, gs_rng* rng, const int64_t* roots, int64_t n_roots,
                       const int32_t* fanouts, int32_t n_hops, int32_t flags, int32_t* buf, int64_t cap,
                       int64_t* hop_sizes, int64_t* offsets, int64_t* used) {
    return pack_run(gp, rng, roots, n_roots, fanouts, n_hops, flags, buf, cap, hop_sizes, offsets, used, nullptr);
}

static int pack_run(const gs_graph* gp, gs_rng* rng, const int64_t* roots, int64_t n_roots, const int32_t* fanouts,
                    int32_t n_hops, int32_t flags, int32_t* buf, int64_t cap, int64_t* hop_sizes, int64_t* offsets,
                    int64_t* used, gs::Team* team) {
    GS_API_BEGIN
    GS_REQUIRE(gp && rng && buf && hop_sizes && offsets && used, GS_EINVAL, "NULL argument");
    const int64_t bound = gs_sample_pack_bound(gp, n_roots, fanouts, n_hops);
    GS_REQUIRE(bound >= 0 && cap >= bound, GS_EINVAL, "buffer below gs_sample_pack_bound");
    const auto& g = *reinterpret_cast<const gs::Graph*>(gp);
    thread_local std::unique_ptr<gs::SampleCtx> ctx;  // reused batch to batch by this thread
    if (!ctx) ctx.reset(new gs::SampleCtx());
    const bool direct = !(flags & GS_SAMPLE_FULL);  // the pack written while sampling
    gs::PackOut po;
    for (auto& row : po.off)
        for (auto& o : row) o = -1;
    po.buf = buf;
    po.cap = cap - n_roots;
    gs::run_sample_into(*ctx, g, rng->mt, roots, n_roots, fanouts, n_hops, flags, team,
                        (flags & GS_SAMPLE_FAIL_EMPTY) != 0, direct ? &po : nullptr);
    const Sample* s = &ctx->s;
    gs_pack_layout L;
    if (direct) {
        for (int32_t j = 0; j < GS_MAX_HOPS; ++j)
            for (int f = 0; f < GS_PK_NFIELDS; ++f) L.off[j][f] = po.off[j][f];
        L.total = po.at;
    } else {
        layout_of(*s, &L);
        gs_sample_pack(reinterpret_cast<const gs_sample*>(s), buf, cap);
    }
    for (int32_t j = 0; j < n_hops; ++j) {
        const Hop& h = s->hops[j];
        hop_sizes[4 * j] = static_cast<int64_t>(h.dst_ids.size());
        hop_sizes[4 * j + 1] = h.n_pos;
        hop_sizes[4 * j + 2] = h.materialised ? static_cast<int64_t>(h.src_ids.size()) : -1;
        hop_sizes[4 * j + 3] = h.materialised ? static_cast<int64_t>(h.nbr.size()) : -1;
        if (h.n_empty && (flags & GS_SAMPLE_FAIL_EMPTY)) gs::fail(GS_EEMPTY, "empty neighbourhood");
    }
    for (int32_t j = 0; j < GS_MAX_HOPS; ++j)
        for (int f = 0; f < GS_PK_NFIELDS; ++f) offsets[j * GS_PK_NFIELDS + f] = L.off[j][f];
    int32_t* r = buf + L.total;  // roots (int32) right after the pack
    for (int64_t i = 0; i < n_roots; ++i) r[i] = static_cast<int32_t>(roots[i]);
    *used = L.total + n_roots;
    GS_API_END
}

int gs_sample_pack(const gs_sample* sp, int32_t* buf, int64_t cap) {
    GS_API_BEGIN
    GS_REQUIRE(sp && buf, GS_EINVAL, "NULL argument");
    const Sample& s = *reinterpret_cast<const Sample*>(sp);
    gs_pack_layout L;
    layout_of(s, &L);
    GS_REQUIRE(cap >= L.total, GS_EINVAL, "pack buffer too small");
    auto cpy = [&](int32_t j, int f, const int32_t* p, size_t n) {
        if (n) std::memcpy(buf + L.off[j][f], p, n * sizeof(int32_t));
    };
    for (int32_t j = 0; j < s.n_hops; ++j) {
        const Hop& h = s.hops[j];
        if (j == s.n_hops - 1) {
            cpy(j, GS_PK_POS_PTR, h.pos_ptr.data(), h.pos_ptr.size());
            // absolute CSR entries row_ptr[dst] + position: the device gather
            // then reads col[] without first looking up row_ptr[dst]
            cpy(j, GS_PK_POS, h.ent.data(), h.ent.size());
            int32_t* d = buf + L.off[j][GS_PK_DST_IDS];
            for (size_t r = 0; r < h.dst_ids.size(); ++r) d[r] = static_cast<int32_t>(h.dst_ids[r]);
        } else {
            cpy(j, GS_PK_NBR_PTR, h.nbr_ptr.data(), h.nbr_ptr.size());
            cpy(j, GS_PK_NBR, h.nbr.data(), h.nbr.size());
            cpy(j, GS_PK_SELF, h.self_local.data(), h.self_local.size());
            cpy(j, GS_PK_TPTR, h.tptr.data(), h.tptr.size());
            cpy(j, GS_PK_TIDX, h.tidx.data(), h.tidx.size());
        }
    }
    GS_API_END
}


int64_t gs_sample_pack_bound_multi(const gs_graph* gp, int64_t n_roots, int64_t group, const int32_t* fanouts,
                                   int32_t n_hops) {
    if (group < 1 || n_roots < 1) return -1;
    if (n_roots <= group) return gs_sample_pack_bound(gp, n_roots, fanouts, n_hops);
    // every field of the merged image is at most the sum of the groups' (one
    // pointer terminator and one alignment pad instead of one per group)
    const int64_t full = gs_sample_pack_bound(gp, group, fanouts, n_hops);
    const int64_t rest = n_roots % group;
    const int64_t tail = rest ? gs_sample_pack_bound(gp, rest, fanouts, n_hops) : 0;
    if (full < 0 || tail < 0) return -1;
    return (n_roots / group) * full + tail;
}

int gs_team_create(int32_t helpers, gs_team** out) {
    GS_API_BEGIN
    GS_REQUIRE(out && helpers >= 0 && helpers <= 64, GS_EINVAL, "helpers out of [0, 64]");
    constexpr int spin_us = 500;  // how long an idle helper polls before sleeping
    *out = reinterpret_cast<gs_team*>(new gs::Team(helpers, spin_us));
    GS_API_END
}

int gs_team_create_shared(const gs_team* peer, gs_team** out) {
    GS_API_BEGIN
    GS_REQUIRE(out && peer, GS_EINVAL, "null team");
    *out = reinterpret_cast<gs_team*>(new gs::Team(reinterpret_cast<const gs::Team*>(peer)->pool()));
    GS_API_END
}

void gs_team_destroy(gs_team* team) { delete reinterpret_cast<gs::Team*>(team); }

int gs_sample_pack_run_multi(const gs_graph* gp, gs_rng* rng, const int64_t* roots, int64_t n_roots, int64_t group,
                             const int32_t* fanouts, int32_t n_hops, int32_t flags, int32_t* buf, int64_t cap,
                             int64_t* hop_sizes, int64_t* offsets, int64_t* used) {
    return gs_sample_pack_run_multi_team(gp, rng, roots, n_roots, group, fanouts, n_hops, flags, buf, cap, hop_sizes,
                                         offsets, used, nullptr);
}

int gs_sample_pack_run_multi_team(const gs_graph* gp, gs_rng* rng, const int64_t* roots, int64_t n_roots,
                                  int64_t group, const int32_t* fanouts, int32_t n_hops, int32_t flags, int32_t* buf,
                                  int64_t cap, int64_t* hop_sizes, int64_t* offsets, int64_t* used, gs_team* tp) {
    gs::Team* team = reinterpret_cast<gs::Team*>(tp);
    if (group >= 1 && n_roots <= group)
        return pack_run(gp, rng, roots, n_roots, fanouts, n_hops, flags, buf, cap, hop_sizes, offsets, used, team);
    GS_API_BEGIN
    GS_REQUIRE(gp && rng && roots && buf && hop_sizes && offsets && used, GS_EINVAL, "NULL argument");
    GS_REQUIRE(group >= 1 && n_hops >= 1 && n_hops <= GS_MAX_HOPS, GS_EINVAL, "bad group / n_hops");
    const int64_t bound = gs_sample_pack_bound_multi(gp, n_roots, group, fanouts, n_hops);
    GS_REQUIRE(bound >= 0 && cap >= bound, GS_EINVAL, "buffer below gs_sample_pack_bound_multi");
    const auto& g = *reinterpret_cast<const gs::Graph*>(gp);
    // the groups in order on one stream; an empty neighbourhood fails right
    // after its own group, as the reference raises inside that batch
    std::vector<std::unique_ptr<Sample>> parts;
    for (int64_t lo = 0; lo < n_roots; lo += group) {
        parts.emplace_back(gs::run_sample(g, rng->mt, roots + lo, std::min(group, n_roots - lo), fanouts, n_hops,
                                          flags, team));
        if (flags & GS_SAMPLE_FAIL_EMPTY)
            for (int32_t j = 0; j < n_hops; ++j)
                if (parts.back()->hops[j].n_empty) gs::fail(GS_EEMPTY, "empty neighbourhood");
    }
    // merged layout: the field order and alignment of layout_of
    gs_pack_layout L;
    for (auto& row : L.off)
        for (auto& o : row) o = -1;
    int64_t at = 0;
    auto put = [&](int32_t j, int f, int64_t n) {
        L.off[j][f] = at;
        at += (n + 3) & ~int64_t(3);
    };
    for (int32_t j = 0; j < n_hops; ++j) {
        int64_t nd = 0, n1 = 0, ns = 0, nt = 0;
        for (const auto& p : parts) {
            const Hop& h = p->hops[j];
            nd += static_cast<int64_t>(h.dst_ids.size());
            GS_REQUIRE(j < n_hops - 1 || h.ent.size() == h.pos.size(), GS_EINVAL, "pack entries mismatch");
            n1 += static_cast<int64_t>(j == n_hops - 1 ? h.pos.size() : h.nbr.size());
            ns += static_cast<int64_t>(h.src_ids.size());
            nt += static_cast<int64_t>(h.tidx.size());
        }
        hop_sizes[4 * j] = nd;
        if (j == n_hops - 1) {
            put(j, GS_PK_POS_PTR, nd + 1);
            put(j, GS_PK_POS, n1);
            put(j, GS_PK_DST_IDS, nd);
            hop_sizes[4 * j + 1] = n1;
            hop_sizes[4 * j + 2] = hop_sizes[4 * j + 3] = -1;
        } else {
            put(j, GS_PK_NBR_PTR, nd + 1);
            put(j, GS_PK_NBR, n1);
            put(j, GS_PK_SELF, nd);
            put(j, GS_PK_TPTR, ns + 1);
            put(j, GS_PK_TIDX, nt);
            int64_t np = 0;
            for (const auto& p : parts) np += static_cast<int64_t>(p->hops[j].pos.size());
            hop_sizes[4 * j + 1] = np;
            hop_sizes[4 * j + 2] = ns;
            hop_sizes[4 * j + 3] = n1;
        }
    }
    L.total = at;
    GS_REQUIRE(L.total + n_roots <= cap, GS_EINVAL, "merged pack exceeds its bound");
    // fields, group by group, indices rebased on the groups before
    for (int32_t j = 0; j < n_hops; ++j) {
        int32_t* o[GS_PK_NFIELDS];
        for (int f = 0; f < GS_PK_NFIELDS; ++f) o[f] = L.off[j][f] >= 0 ? buf + L.off[j][f] : nullptr;
        int64_t bd = 0, b1 = 0, bs = 0, bt = 0;  // dst, pos / nbr, src, tidx bases
        for (const auto& p : parts) {
            const Hop& h = p->hops[j];
            const int64_t nd = static_cast<int64_t>(h.dst_ids.size());
            if (j == n_hops - 1) {
                for (int64_t r = 0; r < nd; ++r) {
                    o[GS_PK_POS_PTR][bd + r] = static_cast<int32_t>(h.pos_ptr[r] + b1);
                    o[GS_PK_DST_IDS][bd + r] = static_cast<int32_t>(h.dst_ids[r]);
                }
                if (!h.ent.empty()) std::memcpy(o[GS_PK_POS] + b1, h.ent.data(), h.ent.size() * sizeof(int32_t));
                b1 += static_cast<int64_t>(h.ent.size());
            } else {
                const int64_t ns = static_cast<int64_t>(h.src_ids.size());
                GS_REQUIRE(ns == static_cast<int64_t>(p->hops[j + 1].dst_ids.size()), GS_EINVAL,
                           "hop frontier mismatch");
                for (int64_t r = 0; r < nd; ++r) {
                    o[GS_PK_NBR_PTR][bd + r] = static_cast<int32_t>(h.nbr_ptr[r] + b1);
                    o[GS_PK_SELF][bd + r] = static_cast<int32_t>(h.self_local[r] + bs);
                }
                for (size_t e = 0; e < h.nbr.size(); ++e) o[GS_PK_NBR][b1 + e] = static_cast<int32_t>(h.nbr[e] + bs);
                for (int64_t c = 0; c < ns; ++c) o[GS_PK_TPTR][bs + c] = static_cast<int32_t>(h.tptr[c] + bt);
                for (size_t t = 0; t < h.tidx.size(); ++t) {  // r -> r + bd; -(r+1) -> -(r+bd+1)
                    const int32_t v = h.tidx[t];
                    o[GS_PK_TIDX][bt + t] = static_cast<int32_t>(v >= 0 ? v + bd : v - bd);
                }
                b1 += static_cast<int64_t>(h.nbr.size());
                bs += ns;
                bt += static_cast<int64_t>(h.tidx.size());
            }
            bd += nd;
        }
        if (j == n_hops - 1) {
            o[GS_PK_POS_PTR][bd] = static_cast<int32_t>(b1);
        } else {
            o[GS_PK_NBR_PTR][bd] = static_cast<int32_t>(b1);
            o[GS_PK_TPTR][bs] = static_cast<int32_t>(bt);
        }
    }
    for (int32_t j = 0; j < GS_MAX_HOPS; ++j)
        for (int f = 0; f < GS_PK_NFIELDS; ++f) offsets[j * GS_PK_NFIELDS + f] = L.off[j][f];
    int32_t* r = buf + L.total;
    for (int64_t i = 0; i < n_roots; ++i) r[i] = static_cast<int32_t>(roots[i]);
    *used = L.total + n_roots;
    GS_API_END
}

}  // extern "C"
