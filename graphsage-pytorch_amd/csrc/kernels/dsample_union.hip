// Device sampler, hops before the last (see dsample.hip): the CPython-set part
// of _get_unique_neighs_list (models.py:282-288) and the lists the aggregate
// kernels read, written into the pack exactly as host/sampler.cpp writes them.
//
//   sets_kernel   samp_neighs[r] = set(sample) | {node} (:282, :285), one
//                 lane per frontier node on a lane-private 128-slot table in
//                 LDS: Objects/setobject.c's add / resize / copy / merge rules
//                 as host/pyset.hpp restates them.  Out: each set's iteration
//                 order (all the union needs) and samp_neighs[0]'s table.
//   union_kernel  list(set.union(*samp_neighs)) (:286), one block, table in
//                 LDS.  The union is a copy of samp_neighs[0] followed by one
//                 set_merge per other set; a merge can only resize before its
//                 first add (its pre-resize leaves room for all of them), and
//                 no key is ever deleted.  So the final table is a sequence of
//                 stages — resize, re-insert the previous table in slot
//                 order, insert the keys new to the union in merge order —
//                 and each stage is "every key takes the first free slot of
//                 its probe sequence, in priority order".  That assignment is
//                 computed in parallel by priority displacement (a key claims
//                 its current probe slot with an LDS atomicMin of its
//                 priority; a key that loses, or is later displaced, moves to
//                 its next probe slot), which converges to exactly the
//                 sequential result: the highest-priority key always keeps its
//                 first free slot, and by induction so does every key after
//                 it.  Keys new to the union are found with one 64-bit
//                 atomicMax per item on a per-node mark (epoch, first index).
//                 Then: the frontier in slot order, each destination's
//                 neighbourhood in frontier-local ids (ascending), its self id.
//   t*_kernels    the transposed lists (per source, ascending destination;
//                 self entries -(r+1) first), counted (in uout_kernel),
//                 scanned, scattered and sorted per source.
#include "dsample.hpp"

namespace gs {
namespace ds {

namespace {

constexpr int kMaxItems = 33;                       // |samp_neighs[r]| <= k + 1 <= 33

__device__ __forceinline__ uint32_t mask_for(int64_t minused) {
    uint32_t ns = 8;
    while (ns <= minused) ns <<= 1;
    return ns - 1;
}

// ---- union probe state: slot i (14 bits), linear step (4 bits), perturb shifts (4 bits)
__device__ __forceinline__ uint32_t pr_slot(uint32_t ps) { return (ps & 0xFFFFu) + ((ps >> 16) & 15u); }
__device__ __forceinline__ uint32_t pr_init(int32_t key, uint32_t mask) { return static_cast<uint32_t>(key) & mask; }
__device__ __forceinline__ uint32_t pr_next(uint32_t ps, int32_t key, uint32_t mask) {
    uint32_t i = ps & 0xFFFFu, lin = (ps >> 16) & 15u, steps = ps >> 20;
    if (lin < 9 && i + 9 <= mask) return i | ((lin + 1) << 16) | (steps << 20);
    steps = min(steps + 1, 15u);
    const uint32_t perturb = steps * 5 >= 32 ? 0u : static_cast<uint32_t>(key) >> (steps * 5);
    i = (i * 5 + 1 + perturb) & mask;
    return i | (steps << 20);
}

// Keys of one stage, densely indexed in priority order (the previous table's
// keys in slot order, then the stage's new keys in merge order): key t is
// thread t % 1024's q-th key (q = t / 1024), and t is its priority.  A stage's
// table is at most 3/5 full, so kKPT keys per thread cover kUnionMax slots.
constexpr int kKPT = (kUnionMax * 3 / 5) / 1024 + 1;
constexpr int kStageKeys = kKPT * 1024;
constexpr size_t kUnionLds = (kUnionMax + kStageKeys) * sizeof(uint32_t);  // table + a stage's old keys

// Keys per lane of ublock's one-wave stages (stages of at most 64 * KPL keys;
// A/B build switch: -DGS_UNION_KPL=8 takes stages up to 512 keys in one wave).
#ifndef GS_UNION_KPL
#define GS_UNION_KPL 4
#endif
constexpr int kUnionKpl = GS_UNION_KPL;

}  // namespace

// ---- one wave per set: CPython's set operations on a 128-slot LDS table,
// each probe run (slots i .. i+9) read by ten lanes at once

__device__ __forceinline__ int wlane() { return static_cast<int>(threadIdx.x & 63); }

__device__ __forceinline__ void w_clear(volatile int32_t* T, uint32_t nslots) {
    for (uint32_t i = wlane(); i < nslots; i += 64) T[i] = -1;
}

// set_add_entry (no dummies): the first slot of the probe sequence holding
// the key (already present: false) or empty (the key goes there: true).
// More than probe_cap(mask) probe groups (a full table: never expected) set
// `bad` and return false.
__device__ __forceinline__ bool w_add(volatile int32_t* T, uint32_t mask, int32_t key, bool& bad) {
    const int lane = wlane();
    uint32_t i = static_cast<uint32_t>(key) & mask;
    uint32_t perturb = static_cast<uint32_t>(key);
    for (uint32_t step = 0; step < probe_cap(mask); ++step) {
        const uint32_t probes = (i + 9 <= mask) ? 9u : 0u;
        const bool in = static_cast<uint32_t>(lane) <= probes;
        const int32_t x = in ? T[i + lane] : 0;
        const uint64_t hit = __ballot(in && (x == -1 || x == key));
        if (hit) {
            const int l = __ffsll(static_cast<unsigned long long>(hit)) - 1;
            if (__shfl(x, l, 64) == key) return false;
            if (lane == 0) T[i + l] = key;
            return true;
        }
        perturb >>= 5;
        i = (i * 5 + 1 + perturb) & mask;
    }
    bad = true;
    return false;
}

// One table stage of distinct keys: the table is cleared to mask m and lane
// t < nk inserts `key` with priority t — every key takes the first free slot
// of its probe sequence in priority order, exactly as nk sequential
// set_add_entry calls (distinct keys: every add is fresh).  Computed by
// priority displacement inside the wave (the frontier union's method,
// settle_keys): a key claims its probe slot with an LDS atomicMin of its
// priority and moves on when a higher priority holds it or later takes it;
// after the divergent claims reconverge, every lane re-reads its slot, so a
// round needs no barrier.  Then each slot gets its key.
//
// Termination: a slot's value only decreases and a key only moves forward,
// so the stage ends once every key has a slot — provided the table has a
// free slot for each (nk <= 3/5 (m + 1) by the callers' resize rules).  Each
// key's probe steps are bounded by probe_cap(m) anyway: past it the key
// stops (its lane's `bad` is set, its slot left unwritten) and the stage
// ends, so a broken invariant surfaces as a status bit, never as a hang.
__device__ __forceinline__ void w_stage(volatile int32_t* T, uint32_t m, int nk, int32_t key, bool& bad) {
    const int lane = wlane();
    w_clear(T, m + 1);  // -1 = priority 0xFFFFFFFF: empty
    __atomic_signal_fence(__ATOMIC_SEQ_CST);  // the clear before the claims (one wave: LDS keeps its order)
    uint32_t* U = const_cast<uint32_t*>(reinterpret_cast<volatile uint32_t*>(T));
    const bool act = lane < nk;
    const uint32_t t = static_cast<uint32_t>(lane);
    const uint32_t cap = probe_cap(m);
    uint32_t ps = act ? pr_init(key, m) : 0u;
    uint32_t steps = 0;
    bool placed = !act, stop = !act;
    for (;;) {
        if (!placed) {
            while (atomicMin(&U[pr_slot(ps)], t) < t && ++steps < cap) ps = pr_next(ps, key, m);
            placed = true;
            if (steps >= cap) stop = true;
        }
        const uint32_t h = stop ? t : reinterpret_cast<volatile uint32_t*>(T)[pr_slot(ps)];
        if (h != t) {
            ps = pr_next(ps, key, m);
            placed = false;
            if (++steps >= cap) {
                stop = true;
                placed = true;
            }
        }
        if (!__ballot(!placed)) break;
    }
    if (act && stop) bad = true;
    if (act && !stop) T[pr_slot(ps)] = key;
}

// w_stage with up to 64 * KPL keys: lane l's q-th key has priority l + 64 q
// (the frontier union's small stages).  A lane's later key may displace its
// earlier one within a claim pass; the re-read after the pass sees it.  The
// probe bound is per key, as in w_stage.
template <int KPL>
__device__ __forceinline__ void w_stage_n(volatile int32_t* T, uint32_t m, int nk, const int32_t (&key)[KPL],
                                          bool& bad) {
    const int lane = wlane();
    w_clear(T, m + 1);
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    uint32_t* U = const_cast<uint32_t*>(reinterpret_cast<volatile uint32_t*>(T));
    const uint32_t cap = probe_cap(m);
    uint32_t ps[KPL], steps[KPL];
    bool placed[KPL], stop[KPL];
#pragma unroll
    for (int q = 0; q < KPL; ++q) {
        const bool act = lane + 64 * q < nk;
        ps[q] = act ? pr_init(key[q], m) : 0u;
        placed[q] = !act;
        stop[q] = !act;
        steps[q] = 0;
    }
    for (;;) {
#pragma unroll
        for (int q = 0; q < KPL; ++q)
            if (!placed[q]) {
                const uint32_t t = static_cast<uint32_t>(lane + 64 * q);
                while (atomicMin(&U[pr_slot(ps[q])], t) < t && ++steps[q] < cap) ps[q] = pr_next(ps[q], key[q], m);
                placed[q] = true;
                if (steps[q] >= cap) stop[q] = true;
            }
        bool moved = false;
#pragma unroll
        for (int q = 0; q < KPL; ++q) {
            const uint32_t t = static_cast<uint32_t>(lane + 64 * q);
            if (!stop[q] && reinterpret_cast<volatile uint32_t*>(T)[pr_slot(ps[q])] != t) {
                ps[q] = pr_next(ps[q], key[q], m);
                if (++steps[q] >= cap) {
                    stop[q] = true;
                } else {
                    placed[q] = false;
                    moved = true;
                }
            }
        }
        if (!__ballot(moved)) break;
    }
#pragma unroll
    for (int q = 0; q < KPL; ++q)
        if (lane + 64 * q < nk) {
            if (stop[q]) bad = true;
            else T[pr_slot(ps[q])] = key[q];
        }
}

// The keys of T (mask + 1 <= 128 slots) in slot order into K; returns their count.
__device__ __forceinline__ int w_compact(const volatile int32_t* T, uint32_t mask, volatile int32_t* K) {
    const int lane = wlane();
    int n = 0;
    for (uint32_t b = 0; b <= mask; b += 64) {
        const uint32_t sl = b + lane;
        const int32_t x = sl <= mask ? T[sl] : -1;
        const uint64_t bal = __ballot(x != -1);
        if (x != -1) K[n + __popcll(bal & ((1ull << lane) - 1ull))] = x;
        n += __popcll(bal);
    }
    return n;
}

// set_table_resize: smallest power of two > minused, keys re-inserted in slot order.
__device__ __forceinline__ uint32_t w_resize(volatile int32_t* T, uint32_t mask, int minused, volatile int32_t* K,
                                             bool& bad) {
    const int n = w_compact(T, mask, K);
    uint32_t ns = 8;
    while (ns <= static_cast<uint32_t>(minused)) ns <<= 1;
    w_stage(T, ns - 1, n, K[min(wlane(), kSmallSet - 1)], bad);
    return ns - 1;
}

// samp_neighs[r] = set(random.sample(...)) | {node} (models.py:282, :285), or
// the adjacency set itself | {node} when deg < k; then its iteration order,
// each item's first-occurrence mark for the frontier union (item q of run
// r >= 1 has merge-order key t = pos_ptr[r] + r + q, increasing in merge
// order; the largest mark is the earliest occurrence; run 0's keys are in the
// union from the start, never new), and samp_neighs[0]'s table.
constexpr int kSetWaves = 4;
__global__ __launch_bounds__(64 * kSetWaves) void sets_kernel(DevGraph g, Ctl* c, HopBufs hb, UnionBufs ub, int hop,
                                                              int k) {
    GS_DS_BAIL(c);
    __shared__ int32_t tabs[kSetWaves][kSmallSet], keys[kSetWaves][kSmallSet];
    const int wave = static_cast<int>(threadIdx.x >> 6), lane = wlane();
    const int r = blockIdx.x * kSetWaves + wave;
    const int n = c->hop[hop].n_dst;
    if (r >= n) return;
    volatile int32_t* T = tabs[wave];
    volatile int32_t* K = keys[wave];
    const int32_t v = hb.dst[r];
    const int d = hb.deg[r];
    uint32_t mask = 7;
    int used = 0;
    bool bad = false;  // a stage or add past its probe bound (kStSpin)
    w_clear(T, 8);
    if (k > 0 && d >= k) {
        // set(list): set_add_key per item in result order, resizing to used * 4
        const int32_t e = lane < k ? hb.ent[hb.pos_ptr[r] + lane] : 0;
        const int32_t mine = lane < k ? g.col[e] : 0;
        // The k sampled keys are distinct (distinct entries of one adjacency
        // set), so every add is fresh and `used` after key i is i + 1: the
        // resizes (to used * 4 once used * 5 >= mask * 3) fall at known keys.
        // Each stage — the previous table's keys in slot order, then the keys
        // up to the next resize — is one w_stage.
        int i0 = 0, n_old = 0;
        while (i0 < k || n_old > 0) {
            int i1 = i0;
            while (i1 < k) {
                ++i1;
                if (static_cast<uint32_t>(i1) * 5 >= mask * 3) break;
            }
            const int src = min(max(i0 + lane - n_old, 0), 63);
            const int32_t fresh = __shfl(mine, src, 64);
            w_stage(T, mask, n_old + (i1 - i0), lane < n_old ? K[min(lane, kSmallSet - 1)] : fresh, bad);
            used = i1;
            n_old = 0;
            i0 = i1;
            if (static_cast<uint32_t>(used) * 5 >= mask * 3) {  // set_table_resize(used * 4)
                n_old = w_compact(T, mask, K);
                uint32_t ns = 8;
                while (ns <= static_cast<uint32_t>(used * 4)) ns <<= 1;
                mask = ns - 1;
            }
        }
        // the copy `|` makes: resized to 2 * used when used * 5 >= 21, else
        // the same size (then a slot copy)
        uint32_t nm = 7;
        if (used * 5 >= 21) nm = mask_for(2 * used);
        if (nm != mask) {
            const int m = w_compact(T, mask, K);
            w_stage(T, nm, m, K[min(lane, kSmallSet - 1)], bad);
            mask = nm;
        }
    } else {
        // the adjacency set itself, copied by `|`: its own layout when the
        // copy's table has its size and it holds no dummies
        const int64_t rs = g.row_ptr[v];
        const uint32_t m0 = (1u << g.log2size[v]) - 1;
        const bool dirty = g.dirty && g.dirty[v];
        uint32_t ns = 8;
        if (d * 5 >= 21)
            while (ns <= static_cast<uint32_t>(2 * d)) ns <<= 1;
        mask = ns - 1;
        used = d;
        w_clear(T, ns);
        if (mask == m0 && !dirty) {
            if (lane < d) T[g.slot[rs + lane]] = g.col[rs + lane];
        } else {
            // the set's keys in its iteration order, all distinct: one stage
            w_stage(T, mask, d, lane < d ? g.col[rs + lane] : 0, bad);
        }
    }
    // | set([node]): set_merge with a one-element set
    if (static_cast<uint32_t>(used + 1) * 5 >= mask * 3) mask = w_resize(T, mask, (used + 1) * 2, K, bad);
    if (used == 0 && mask == 7) {
        w_clear(T, 8);
        if (lane == 0) T[v & 7] = v;
        used = 1;
    } else if (w_add(T, mask, v, bad)) {
        ++used;
        if (static_cast<uint32_t>(used) * 5 >= mask * 3)
            mask = w_resize(T, mask, used > 50000 ? used * 2 : used * 4, K, bad);
    }
    if (__ballot(bad)) {  // a broken table invariant: report it, never spin
        if (lane == 0) atomicOr(&c->status, kStSpin);
        return;
    }
    // iteration order, marks
    const uint64_t E = static_cast<uint64_t>(static_cast<uint32_t>(c->epoch + 1)) << 32;
    const uint32_t t0 = static_cast<uint32_t>(hb.pos_ptr[r] + r);
    int32_t* out = ub.set_items + hb.pos_ptr[r] + r;
    int q0 = 0;
    for (uint32_t b = 0; b <= mask; b += 64) {
        const uint32_t sl = b + lane;
        const int32_t x = sl <= mask ? T[sl] : -1;
        const uint64_t bal = __ballot(x != -1);
        if (x != -1) {
            const int q = q0 + __popcll(bal & ((1ull << lane) - 1ull));
            out[q] = x;
            atomicMax(reinterpret_cast<unsigned long long*>(&ub.mark[x]),
                      static_cast<unsigned long long>(E | (r == 0 ? 0xFFFFFFFFu : 0xFFFFFFFEu - (t0 + q))));
        }
        q0 += __popcll(bal);
    }
    if (lane == 0) ub.set_cnt[r] = used;
    if (r == 0) {
        for (uint32_t i = lane; i <= mask; i += 64) ub.first_tab[i] = T[i];
        if (lane == 0) {
            ub.first_meta[0] = static_cast<int32_t>(mask);
            ub.first_meta[1] = used;
        }
    }
}

// Per run r >= 1 (one wave, lane q = item q): the items new to the union —
// those whose mark is their own (the union's first occurrence of the key).
__global__ __launch_bounds__(64) void ufresh_kernel(Ctl* c, HopBufs hb, UnionBufs ub, int hop) {
    GS_DS_BAIL(c);
    const int r = blockIdx.x, lane = threadIdx.x;
    if (r >= c->hop[hop].n_dst) return;
    const uint64_t E = static_cast<uint64_t>(static_cast<uint32_t>(c->epoch + 1)) << 32;
    const int cn = ub.set_cnt[r];
    bool fresh = false;
    if (r > 0 && lane < cn) {
        const uint32_t t = static_cast<uint32_t>(hb.pos_ptr[r] + r + lane);
        const int32_t key = ub.set_items[hb.pos_ptr[r] + r + lane];
        fresh = __hip_atomic_load(&ub.mark[key], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
                (E | (0xFFFFFFFEu - t));
    }
    const uint64_t m = __ballot(fresh);
    if (lane == 0) ub.fmask[r] = m;
}

// Priority-displacement insertion of this thread's keys (t = t0 + tid + 1024 q
// < t1, priority t) into the LDS table (every slot EMPTY or holding a
// priority); returns the rounds once every key sits in its final slot.  A key
// walks its probe sequence until it wins a slot — an empty one, or one held by
// a lower priority (whose key notices and moves on).  A slot's value only
// decreases, so no key revisits a slot it left, and the assignment converges
// to the sequential one whatever the timing (the highest priority always
// keeps its first free slot, and by induction every later key).
//
// Each thread runs to its own fixpoint (re-placing its displaced keys until a
// pass finds all of them holding their slots) without waiting for the
// others; a round ends at a barrier, after which a pass with no claims in
// flight confirms every key.  (Displacement chains across waves still take a
// round per link: 2-9 rounds at the headline's stages, as with a barrier per
// step.  A lane-level queue over a thread's keys — one probe step per
// iteration — measured slower at rmat2m and 15 % faster at Pubmed's 60 %-full
// stage.)  claim(slot, t) -> t now holds the slot; held(slot) -> its priority.
__device__ __forceinline__ uint32_t lds_load(const uint32_t* p) { return __atomic_load_n(p, __ATOMIC_RELAXED); }

template <typename Claim, typename Held>
__device__ __forceinline__ int settle_keys(uint32_t mask, int t0, int t1, const int32_t (&key)[kKPT],
                                           uint32_t (&ps)[kKPT], Claim claim, Held held, int64_t* first_round,
                                           bool& bad) {
    const int base = t0 + static_cast<int>(threadIdx.x);
    // probe steps of this thread's keys together: past the bound (a table
    // with fewer free slots than keys — never expected) the thread stops
    // claiming and reports itself settled, so the block leaves the loop and
    // the caller raises kStSpin instead of spinning forever
    const uint32_t cap = kKPT * probe_cap(mask);
    uint32_t steps = 0;
    bool placed[kKPT];
#pragma unroll
    for (int q = 0; q < kKPT; ++q) placed[q] = false;
    int rounds = 0;
    for (;; ++rounds) {
        for (;;) {
            bool moved = false;
#pragma unroll
            for (int q = 0; q < kKPT; ++q) {
                const int t = base + 1024 * q;
                if (t < t1 && !bad) {
                    if (placed[q] && held(pr_slot(ps[q])) != static_cast<uint32_t>(t)) {
                        ps[q] = pr_next(ps[q], key[q], mask);
                        placed[q] = false;
                    }
                    if (!placed[q]) {
                        while (!claim(pr_slot(ps[q]), static_cast<uint32_t>(t)) && ++steps < cap)
                            ps[q] = pr_next(ps[q], key[q], mask);
                        placed[q] = true;
                        moved = true;
                        if (++steps >= cap) bad = true;
                    }
                }
            }
            if (!moved) break;
        }
        __syncthreads();
        int any = 0;
#pragma unroll
        for (int q = 0; q < kKPT; ++q) {
            const int t = base + 1024 * q;
            if (t < t1 && !bad) any |= held(pr_slot(ps[q])) != static_cast<uint32_t>(t);
        }
        if (rounds == 0 && threadIdx.x == 0 && first_round)
            *first_round = static_cast<int64_t>(__builtin_amdgcn_s_memrealtime());
        if (!__syncthreads_or(any)) break;
    }
    return rounds + 1;
}

__device__ __forceinline__ int settle(uint32_t* T, uint32_t mask, int nk, const int32_t (&key)[kKPT],
                                      uint32_t (&ps)[kKPT], int64_t& first_round, bool& bad) {
    return settle_keys(
        mask, 0, nk, key, ps, [&](uint32_t slot, uint32_t t) { return atomicMin(&T[slot], t) > t; },
        [&](uint32_t slot) { return lds_load(&T[slot]); }, &first_round, bad);
}

// The next frontier in the final table's slot order, each key's position in
// it (lid), the pack layout of this hop, the transposed counts zeroed.
// key_at(slot) -> key or -1.
// occupied(slot) -> bool (no global read).  The write pass gathers the keys
// of kGather slots before storing any (the stores could alias the gathered
// array, so a plain loop waits out one gather per slot).
constexpr int kGather = 16;
template <typename KeyAt, typename Occ>
__device__ __forceinline__ void finish_union(Ctl* c, const HopBufs& hb, const UnionBufs& ub, const HopBufs& next,
                                             int hop, int gcn, int32_t* __restrict__ pack, int nd_next_max,
                                             uint32_t mf, int used0, int epoch, KeyAt key_at, Occ occupied, int* shi) {
    HopCtl& h = c->hop[hop];
    const int tid = threadIdx.x;
    const int n = h.n_dst;
    const int sper = static_cast<int>((mf + 1 + 1023) / 1024);
    const uint32_t sa = min<uint32_t>(mf + 1, tid * sper), sb = min<uint32_t>(mf + 1, sa + sper);
    int my_keys = 0;
    for (uint32_t i = sa; i < sb; ++i) my_keys += occupied(i);
    int n_src;
    int rk = block_excl_scan(my_keys, shi, &n_src);
    if (n_src > nd_next_max) {
        if (tid == 0) c->status |= kStSize;
        return;
    }
    for (uint32_t i0 = sa; i0 < sb; i0 += kGather) {
        int32_t kk[kGather];
#pragma unroll
        for (int j = 0; j < kGather; ++j) kk[j] = i0 + j < sb ? key_at(i0 + j) : -1;
#pragma unroll
        for (int j = 0; j < kGather; ++j)
            if (kk[j] != -1) {
                ub.lid[kk[j]] = rk;
                next.dst[rk++] = kk[j];
            }
    }
    const int g1 = gcn ? 0 : 1;
    const int items_tot = ub.tpre[n];
    const int n_nbr = used0 + items_tot - n * g1;
    if (tid == 0) {
        int at = c->total;
        int off[GS_PK_NFIELDS];
        off[GS_PK_NBR_PTR] = at;
        at += al4(n + 1);
        off[GS_PK_NBR] = at;
        at += al4(n_nbr);
        off[GS_PK_SELF] = at;
        at += al4(n);
        off[GS_PK_TPTR] = at;
        at += al4(n_src + 1);
        off[GS_PK_TIDX] = at;
        at += al4(n_nbr + n);
        c->total = at;
        for (int f2 = 0; f2 < GS_PK_NFIELDS; ++f2) h.off[f2] = (f2 >= GS_PK_NBR_PTR) ? off[f2] : -1;
        h.n_src = n_src;
        h.n_nbr = n_nbr;
        pack[off[GS_PK_NBR_PTR] + n] = n_nbr;
        c->dbg[4] = static_cast<int64_t>(__builtin_amdgcn_s_memrealtime());
        c->epoch = epoch;  // every kernel of this hop read epoch + 1 before this launch's end
    }
    for (int i = tid; i <= n_src; i += 1024) ub.tcnt[i] = 0;
}

// ---- a union whose final table exceeds kUnionMax slots (ublock_kernel's
// schedule says so): the same stages on a table of uint16 priorities (up to
// kUnionBig slots in LDS, two slots per 32-bit word, claimed by
// compare-and-swap), the stage's keys by priority in global memory (skeys,
// two stages), keys settled in priority chunks of kStageKeys (a chunk's keys
// only compete among themselves: every earlier chunk holds higher
// priorities, final before the chunk starts).

__device__ __forceinline__ uint32_t t16_get(const uint32_t* T, uint32_t slot) {
    return (T[slot >> 1] >> ((slot & 1) * 16)) & 0xFFFFu;
}

// Claim `slot` for priority t: true when t is now its holder (it was empty
// or held a lower priority), false when a higher priority holds it.
__device__ __forceinline__ bool t16_claim(uint32_t* T, uint32_t slot, uint32_t t) {
    uint32_t* wp = T + (slot >> 1);
    const uint32_t sh = (slot & 1) * 16;
    uint32_t old = *reinterpret_cast<volatile uint32_t*>(wp);
    for (;;) {
        if (((old >> sh) & 0xFFFFu) <= t) return false;
        const uint32_t nw = (old & ~(0xFFFFu << sh)) | (t << sh);
        const uint32_t prev = atomicCAS(wp, old, nw);
        if (prev == old) return true;
        old = prev;
    }
}

__device__ __forceinline__ uint32_t t16_load(const uint32_t* T, uint32_t slot) {
    return (lds_load(T + (slot >> 1)) >> ((slot & 1) * 16)) & 0xFFFFu;
}

// settle() on the uint16 table, keys t0 .. t1-1.
__device__ __forceinline__ void settle16(uint32_t* T, uint32_t mask, int t0, int t1, const int32_t (&key)[kKPT],
                                         uint32_t (&ps)[kKPT], bool& bad) {
    (void)settle_keys(
        mask, t0, t1, key, ps, [&](uint32_t slot, uint32_t t) { return t16_claim(T, slot, t); },
        [&](uint32_t slot) { return t16_load(T, slot); }, nullptr, bad);
}

__global__ __launch_bounds__(1024) void ubig_kernel(Ctl* c, HopBufs hb, UnionBufs ub, HopBufs next, int hop, int gcn,
                                                    int32_t* __restrict__ pack, int nd_next_max) {
    GS_DS_BAIL(c);
    extern __shared__ uint32_t T[];  // kUnionBig uint16 slots
    __shared__ int shi[17];
    __shared__ int32_t oldslot[kSmallSet];
    HopCtl& h = c->hop[hop];
    if (!h.big || (c->status & kStTable)) return;
    const int tid = threadIdx.x;
    const int used0 = ub.set_cnt[0];
    const uint32_t m_first = static_cast<uint32_t>(ub.first_meta[0]);
    const int nst = ub.sched[2 * kMaxStages + 1];
    const int epoch = c->epoch + 1;
    uint32_t prev_mask = m_first;
    int32_t key[kKPT];
    uint32_t ps[kKPT];
    if (tid == 0) {
        c->dbg[2] = static_cast<int64_t>(__builtin_amdgcn_s_memrealtime());
        c->dbg[3] = nst;
    }
    for (int s = 0; s < nst; ++s) {
        const uint32_t m = static_cast<uint32_t>(ub.sched[2 * s + 1]);
        if (tid == 0 && s < 12) c->dbg[8 + 4 * s] = static_cast<int64_t>(__builtin_amdgcn_s_memrealtime());
        int32_t* sk = ub.skeys + (s & 1) * static_cast<int64_t>(kBigKeys);
        const int32_t* sk_prev = ub.skeys + ((s + 1) & 1) * static_cast<int64_t>(kBigKeys);
        // the previous table's keys in slot order, by priority into sk
        int n_old;
        {
            const int sp = static_cast<int>((prev_mask + 1 + 1023) / 1024);
            const uint32_t a0 = min<uint32_t>(prev_mask + 1, tid * sp), a1 = min<uint32_t>(prev_mask + 1, a0 + sp);
            auto key_of = [&](uint32_t i) -> int32_t {
                if (s == 0) return ub.first_tab[i];
                const uint32_t p = t16_get(T, i);
                return p == 0xFFFFu ? -1 : sk_prev[p];
            };
            int mine = 0;
            for (uint32_t i = a0; i < a1; ++i) mine += s == 0 ? ub.first_tab[i] != -1 : t16_get(T, i) != 0xFFFFu;
            int at = block_excl_scan(mine, shi, &n_old);
            // kGather gathers in flight before the stores (sk may alias sk_prev
            // for the compiler: a plain loop waits out one gather per slot)
            for (uint32_t i0 = a0; i0 < a1; i0 += kGather) {
                int32_t kk[kGather];
#pragma unroll
                for (int j = 0; j < kGather; ++j) kk[j] = i0 + j < a1 ? key_of(i0 + j) : -1;
#pragma unroll
                for (int j = 0; j < kGather; ++j)
                    if (kk[j] != -1) {
                        sk[at] = kk[j];
                        if (s == 0) oldslot[at] = static_cast<int32_t>(i0 + j);
                        ++at;
                    }
            }
        }
        const int f0 = ub.ubef[ub.sched[2 * s]] - used0, f1 = ub.ubef[ub.sched[2 * (s + 1)]] - used0;
        const int nk = n_old + (f1 - f0);
        if (nk > kBigKeys) {
            if (tid == 0) c->status |= kStTable;
            return;
        }
        for (int i = tid; i < f1 - f0; i += 1024) sk[n_old + i] = ub.fresh[f0 + i];
        __threadfence_block();
        __syncthreads();  // sk complete (and the previous table read): T may be cleared
        for (uint32_t i = tid; i <= m / 2; i += 1024) T[i] = 0xFFFFFFFFu;
        __syncthreads();
        const bool copy = s == 0 && m == m_first;
        if (tid == 0 && s < 12) {
            c->dbg[9 + 4 * s] = static_cast<int64_t>(__builtin_amdgcn_s_memrealtime());
            c->dbg[11 + 4 * s] = (static_cast<int64_t>(nk) << 32) | m;
        }
        for (int t0 = 0; t0 < nk; t0 += kStageKeys) {
            const int t1 = min(nk, t0 + kStageKeys);
#pragma unroll
            for (int q = 0; q < kKPT; ++q) {
                const int t = t0 + tid + 1024 * q;
                int32_t kk = -1;
                uint32_t p0 = 0;
                if (t < t1) {
                    kk = sk[t];
                    p0 = (copy && t < n_old) ? static_cast<uint32_t>(oldslot[t]) : pr_init(kk, m);
                }
                key[q] = kk;
                ps[q] = p0;
            }
            bool bad = false;
            settle16(T, m, t0, t1, key, ps, bad);
            if (__syncthreads_or(bad)) {
                if (tid == 0) atomicOr(&c->status, kStSpin);
                return;
            }
        }
        if (tid == 0 && s < 12) c->dbg[10 + 4 * s] = static_cast<int64_t>(__builtin_amdgcn_s_memrealtime());
        prev_mask = m;
    }
    const int32_t* sk_last = ub.skeys + ((nst - 1) & 1) * static_cast<int64_t>(kBigKeys);
    finish_union(c, hb, ub, next, hop, gcn, pack, nd_next_max, prev_mask, used0, epoch,
                 [&](uint32_t i) -> int32_t {
                     const uint32_t p = t16_get(T, i);
                     return p == 0xFFFFu ? -1 : sk_last[p];
                 },
                 [&](uint32_t i) { return t16_get(T, i) != 0xFFFFu; }, shi);
}

// The union's table (one block, LDS): the runs' new keys in merge order,
// the resize schedule, the stages, then the next frontier in slot order and
// each key's position in it (lid), the pack layout of this hop.
__global__ __launch_bounds__(1024) void ublock_kernel(Ctl* c, HopBufs hb, UnionBufs ub, HopBufs next, int hop,
                                                      int gcn, int32_t* __restrict__ pack, int nd_next_max) {
    GS_DS_BAIL(c);
    extern __shared__ uint32_t T[];
    __shared__ int shi[17];
    __shared__ int st_run[kMaxStages + 1];
    __shared__ uint32_t st_mask[kMaxStages];
    __shared__ int s_nst, s_bad, s_epoch, s_big;
    HopCtl& h = c->hop[hop];
    const int n = h.n_dst;
    const int tid = threadIdx.x;
    const int used0 = ub.set_cnt[0];
    const uint32_t m_first = static_cast<uint32_t>(ub.first_meta[0]);
    if (tid == 0) {
        s_epoch = c->epoch + 1;
        s_bad = 0;
        c->dbg[0] = static_cast<int64_t>(__builtin_amdgcn_s_memrealtime());
    }
    // runs 1..n-1 in contiguous chunks, one per thread: item and new-key counts
    const int per = (n - 1 + 1023) / 1024;
    const int ra = min(n, 1 + tid * per), rb = min(n, ra + per);
    int my_items = 0, my_fresh = 0;
    for (int r = ra; r < rb; ++r) {
        my_items += ub.set_cnt[r];
        my_fresh += __popcll(ub.fmask[r]);
    }
    int items_tot, fresh_tot;
    int tp = block_excl_scan(my_items, shi, &items_tot);
    int f = block_excl_scan(my_fresh, shi, &fresh_tot);
    for (int r = ra; r < rb; ++r) {
        ub.tpre[r] = tp;
        ub.ubef[r] = used0 + f;
        // this run's new keys at their merge-order place (all loads first)
        const int32_t* it = ub.set_items + hb.pos_ptr[r] + r;
        const int cn = ub.set_cnt[r];
        const uint64_t fm = ub.fmask[r];
        int32_t key[kMaxItems];
#pragma unroll
        for (int q = 0; q < kMaxItems; ++q) key[q] = ((fm >> q) & 1) ? it[q] : 0;
#pragma unroll
        for (int q = 0; q < kMaxItems; ++q)
            if ((fm >> q) & 1) ub.fresh[f++] = key[q];
        tp += cn;
    }
    if (tid == 0) {
        ub.tpre[0] = 0;
        ub.tpre[n] = items_tot;
        ub.ubef[n] = used0 + fresh_tot;
    }
    __threadfence_block();
    __syncthreads();
    if (tid == 0) c->dbg[1] = static_cast<int64_t>(__builtin_amdgcn_s_memrealtime());
    // resize schedule: stage 0 is the copy of samp_neighs[0] (resized to
    // 2 * used when used * 5 >= 21) plus the runs up to the first merge whose
    // pre-resize fires, (used + other.used) * 5 >= mask * 3 (no dummies: fill
    // == used); every such merge starts a stage.  The runs' sizes after their
    // merge are staged in LDS; one wave finds the triggers with ballots.
    int32_t* need = reinterpret_cast<int32_t*>(T + kUnionMax);  // [kStageKeys], free until the stages
    const bool need_lds = n <= kStageKeys;
    if (need_lds)
        for (int r = ra; r < rb; ++r) need[r] = ub.ubef[r] + ub.set_cnt[r];
    __syncthreads();
    if (tid < 64) {
        const int lane = tid;
        int64_t cur_m = used0 * 5 >= 21 ? mask_for(2 * used0) : 7u;
        int cur = 1, nst = 1;
        if (lane == 0) {
            st_run[0] = 1;
            st_mask[0] = static_cast<uint32_t>(cur_m);
        }
        for (int base = 1; base < n; base += 64) {
            const int r = base + lane;
            const int64_t v = r < n ? (need_lds ? need[r] : ub.ubef[r] + ub.set_cnt[r]) : 0;
            uint64_t bits = __ballot(r < n && r >= cur && v * 5 >= cur_m * 3);
            while (bits) {
                const int rr = base + __ffsll(static_cast<unsigned long long>(bits)) - 1;
                const int64_t vr = __shfl(v, rr - base, 64);
                if (nst >= kMaxStages) {
                    if (lane == 0) s_bad = 1;
                    break;
                }
                cur_m = mask_for(2 * vr);
                if (lane == 0) {
                    st_run[nst] = rr;
                    st_mask[nst] = static_cast<uint32_t>(cur_m);
                }
                ++nst;
                cur = rr + 1;
                bits = __ballot(r < n && r >= cur && v * 5 >= cur_m * 3);
            }
        }
        if (lane == 0) {
            s_nst = nst;
            st_run[nst] = n;
            if (cur_m + 1 > kUnionBig) s_bad = 1;
            s_big = cur_m + 1 > kUnionMax;
            h.n_src = -1;
            h.big = s_big;
        }
    }
    __syncthreads();
    if (s_bad) {
        if (tid == 0) c->status |= kStTable;
        return;
    }
    const int nst = s_nst;
    if (tid == 0) c->dbg[5] = static_cast<int64_t>(__builtin_amdgcn_s_memrealtime());
    if (s_big) {  // the table needs uint16 priorities: ubig_kernel takes over from the schedule
        if (tid <= nst) {
            ub.sched[2 * tid] = st_run[tid];
            ub.sched[2 * tid + 1] = tid < nst ? static_cast<int32_t>(st_mask[tid]) : 0;
        }
        if (tid == 0) ub.sched[2 * kMaxStages + 1] = nst;
        return;
    }
    if (tid == 0) {
        c->dbg[2] = static_cast<int64_t>(__builtin_amdgcn_s_memrealtime());
        c->dbg[3] = nst;
    }
    // stages: the previous table's keys in slot order (samp_neighs[0]'s own
    // table for stage 0), then the stage's new keys in merge order
    int32_t* oldk = need;                    // [kStageKeys]
    __shared__ int32_t oldslot[kSmallSet];   // stage 0: the first table's slots
    int32_t key[kKPT];
    uint32_t ps[kKPT];
    uint32_t prev_mask = m_first;
    for (int s = 0; s < nst; ++s) {
        const uint32_t m = st_mask[s];
        // A stage of at most 256 keys (the first three or four) in one wave:
        // the previous table compacted in slot order, then w_stage_n (the
        // per-node sets' wave-level insert, four keys per lane) — no block
        // barrier inside the stage.
        const int nk_w = ub.ubef[st_run[s + 1]];  // the union's size after the stage
        if (nk_w <= 64 * kUnionKpl && !(s == 0 && m == m_first)) {  // uniform
            if (tid < 64) {
                const volatile int32_t* P = s == 0 ? reinterpret_cast<const volatile int32_t*>(ub.first_tab)
                                                   : reinterpret_cast<const volatile int32_t*>(T);
                volatile int32_t* K = need;
                const int n_old = w_compact(P, prev_mask, K);
                const int f0 = ub.ubef[st_run[s]] - used0;
                int32_t kk[kUnionKpl];
#pragma unroll
                for (int q = 0; q < kUnionKpl; ++q) {
                    const int t = tid + 64 * q;
                    kk[q] = t < n_old ? K[t] : (t < nk_w ? ub.fresh[f0 + t - n_old] : 0);
                }
                bool bad = false;
                w_stage_n<kUnionKpl>(reinterpret_cast<volatile int32_t*>(T), m, nk_w, kk, bad);
                if (__ballot(bad) && tid == 0) s_bad = 2;
            }
            __syncthreads();
            if (s_bad) {  // uniform
                if (tid == 0) atomicOr(&c->status, kStSpin);
                return;
            }
            prev_mask = m;
            continue;
        }
        // compaction of the previous table
        int n_old;
        {
            const int sp = static_cast<int>((prev_mask + 1 + 1023) / 1024);
            const uint32_t a0 = min<uint32_t>(prev_mask + 1, tid * sp), a1 = min<uint32_t>(prev_mask + 1, a0 + sp);
            int mine = 0;
            for (uint32_t i = a0; i < a1; ++i) {
                const int32_t kk = s == 0 ? ub.first_tab[i] : static_cast<int32_t>(T[i]);
                mine += kk != -1;
            }
            int at = block_excl_scan(mine, shi, &n_old);
            for (uint32_t i = a0; i < a1; ++i) {
                const int32_t kk = s == 0 ? ub.first_tab[i] : static_cast<int32_t>(T[i]);
                if (kk != -1) {
                    oldk[at] = kk;
                    if (s == 0) oldslot[at] = static_cast<int32_t>(i);
                    ++at;
                }
            }
        }
        const int f0 = ub.ubef[st_run[s]] - used0, f1 = ub.ubef[st_run[s + 1]] - used0;
        const int nk = n_old + (f1 - f0);
        if (nk > kStageKeys) {  // uniform: every thread sees the same counts
            if (tid == 0) c->status |= kStTable;
            return;
        }
        __syncthreads();  // oldk complete; T free to clear
        // stage 0 with the copy's table size equal to the set's: slot copy
        const bool copy = s == 0 && m == m_first;
#pragma unroll
        for (int q = 0; q < kKPT; ++q) {
            const int t = tid + 1024 * q;
            int32_t kk = -1;
            uint32_t p0 = 0;
            if (t < n_old) {
                kk = oldk[t];
                p0 = copy ? static_cast<uint32_t>(oldslot[t]) : pr_init(kk, m);
            } else if (t < nk) {
                kk = ub.fresh[f0 + t - n_old];
                p0 = pr_init(kk, m);
            }
            key[q] = kk;
            ps[q] = p0;
        }
        for (uint32_t i = tid; i <= m; i += 1024) T[i] = 0xFFFFFFFFu;
        __syncthreads();
        int64_t first_round = 0;
        if (tid == 0 && s < 12) c->dbg[8 + 4 * s] = static_cast<int64_t>(__builtin_amdgcn_s_memrealtime());
        bool bad = false;
        const int rounds = settle(T, m, nk, key, ps, first_round, bad);
        if (__syncthreads_or(bad)) {
            if (tid == 0) atomicOr(&c->status, kStSpin);
            return;
        }
        if (tid == 0 && s < 12) {
            c->dbg[9 + 4 * s] = first_round;
            c->dbg[10 + 4 * s] = static_cast<int64_t>(__builtin_amdgcn_s_memrealtime());
            c->dbg[11 + 4 * s] = (static_cast<int64_t>(rounds) << 48) | (static_cast<int64_t>(nk) << 32) | m;
        }
        // priorities -> keys (every slot has one owner)
#pragma unroll
        for (int q = 0; q < kKPT; ++q)
            if (tid + 1024 * q < static_cast<uint32_t>(nk)) T[pr_slot(ps[q])] = static_cast<uint32_t>(key[q]);
        __syncthreads();
        prev_mask = m;
    }
    // the next frontier: keys in slot order, each key's position (lid)
    finish_union(c, hb, ub, next, hop, gcn, pack, nd_next_max, prev_mask, used0, s_epoch,
                 [&](uint32_t i) { return T[i] == 0xFFFFFFFFu ? -1 : static_cast<int32_t>(T[i]); },
                 [&](uint32_t i) { return T[i] != 0xFFFFFFFFu; }, shi);
}

// Per run (one wave, lane q = item q): the destination's neighbourhood in
// frontier-local ids, ascending (the dense mask's column order,
// models.py:305-308; non-gcn drops self, :297-298), and its self id.
__global__ __launch_bounds__(64) void uout_kernel(Ctl* c, HopBufs hb, UnionBufs ub, int hop, int gcn,
                                                  int32_t* __restrict__ pack) {
    GS_DS_BAIL(c);
    const HopCtl& h = c->hop[hop];
    const int r = blockIdx.x, lane = threadIdx.x;
    if (r >= h.n_dst || h.n_src < 0 || (c->status & (kStTable | kStSize))) return;
    const int g1 = gcn ? 0 : 1;
    const int32_t v = hb.dst[r];
    const int cn = ub.set_cnt[r];
    const int32_t key = lane < cn ? ub.set_items[hb.pos_ptr[r] + r + lane] : -1;
    const bool keep = lane < cn && !(g1 && key == v);
    const int loc = keep ? ub.lid[key] : INT_MAX;
    int pos = 0;
#pragma unroll
    for (int p = 0; p < kMaxItems; ++p) pos += __shfl(loc, p, 64) < loc;
    const int used0 = ub.set_cnt[0];
    const int base = r == 0 ? 0 : used0 + ub.tpre[r] - r * g1;
    if (keep) {
        pack[h.off[GS_PK_NBR] + base + pos] = loc;
        atomicAdd(&ub.tcnt[loc], 1);  // the transposed lists' counts (tscan_kernel)
    }
    if (lane == 0) {
        const int sl = ub.lid[v];
        pack[h.off[GS_PK_NBR_PTR] + r] = base;
        pack[h.off[GS_PK_SELF] + r] = sl;
        atomicAdd(&ub.tcnt[sl], 1);
    }
}

// ---- transposed lists (GS_PK_TPTR / GS_PK_TIDX)

__global__ __launch_bounds__(1024) void tscan_kernel(Ctl* c, int hop, int32_t* __restrict__ pack, int32_t* tcnt,
                                                     int32_t* __restrict__ longs) {
    GS_DS_BAIL(c);
    __shared__ int shi[17];
    const HopCtl& h = c->hop[hop];
    if (threadIdx.x == 0) longs[0] = 0;  // tsort_kernel's queue of long lists
    const int ns = h.n_src;
    if (ns <= 0) return;
    const int per = (ns + 1023) / 1024;
    const int a = min(ns, static_cast<int>(threadIdx.x) * per), b = min(ns, a + per);
    int mine = 0;
    for (int i = a; i < b; ++i) mine += tcnt[i];
    int tot;
    int p = block_excl_scan(mine, shi, &tot);
    int32_t* tp = pack + h.off[GS_PK_TPTR];
    for (int i = a; i < b; ++i) {
        const int cc = tcnt[i];
        tp[i] = p;
        tcnt[i] = p;
        p += cc;
    }
    if (threadIdx.x == 0) tp[ns] = tot;
}

// One wave per destination r: its self entry -(r+1) and its neighbour
// entries r at the sources' cursors (order fixed by tsort_kernel).
__global__ __launch_bounds__(64) void tfill_kernel(Ctl* c, int hop, int32_t* __restrict__ pack, int32_t* tcnt) {
    GS_DS_BAIL(c);
    const HopCtl& h = c->hop[hop];
    const int r = blockIdx.x, lane = threadIdx.x;
    if (r >= h.n_dst || h.n_src <= 0) return;
    int32_t* tidx = pack + h.off[GS_PK_TIDX];
    const int32_t* np = pack + h.off[GS_PK_NBR_PTR];
    const int e0 = np[r], e1 = np[r + 1];
    if (lane == 0) tidx[atomicAdd(&tcnt[pack[h.off[GS_PK_SELF] + r]], 1)] = -(r + 1);
    for (int e = e0 + lane; e < e1; e += 64) tidx[atomicAdd(&tcnt[pack[h.off[GS_PK_NBR] + e]], 1)] = r;
}

// per source: ascending destination, a destination's self entry before its
// neighbour entry (host order: -(r+1) then r).  Lists longer than kSortReg
// (the hubs') go to tlong_kernel's queue.
constexpr int kSortReg = 16;
__device__ __forceinline__ int32_t tkey(int32_t v) { return v >= 0 ? 2 * v + 1 : -2 * v - 2; }
__device__ __forceinline__ int32_t tval(int32_t k) { return (k & 1) ? (k - 1) / 2 : -(k + 2) / 2; }
__global__ void tsort_kernel(Ctl* c, int hop, int32_t* __restrict__ pack, int32_t* __restrict__ longs) {
    GS_DS_BAIL(c);
    const HopCtl& h = c->hop[hop];
    const int cidx = blockIdx.x * blockDim.x + threadIdx.x;
    if (cidx >= h.n_src) return;
    const int32_t* tp = pack + h.off[GS_PK_TPTR];
    int32_t* x = pack + h.off[GS_PK_TIDX];
    const int lo = tp[cidx], hi = tp[cidx + 1];
    if (hi - lo <= kSortReg) {
        // short lists (the usual case): every load in flight at once, a
        // bitonic network on the keys in registers, the keys mapped back
        // (tkey is one-to-one: odd keys are neighbour entries, even ones self)
        const int len = hi - lo;
        if (len <= 1) return;
        int32_t k[kSortReg];
#pragma unroll
        for (int j = 0; j < kSortReg; ++j) k[j] = j < len ? tkey(x[lo + j]) : INT_MAX;
#pragma unroll
        for (int kk = 2; kk <= kSortReg; kk <<= 1)
#pragma unroll
            for (int jj = kk >> 1; jj > 0; jj >>= 1)
#pragma unroll
                for (int i = 0; i < kSortReg; ++i) {
                    const int l = i ^ jj;
                    if (l > i) {
                        const int32_t a = k[i], b = k[l];
                        const bool up = (i & kk) == 0;
                        k[i] = up ? min(a, b) : max(a, b);
                        k[l] = up ? max(a, b) : min(a, b);
                    }
                }
#pragma unroll
        for (int j = 0; j < kSortReg; ++j)
            if (j < len) x[lo + j] = tval(k[j]);
        return;
    }
    longs[1 + atomicAdd(&longs[0], 1)] = cidx;
}

// The long lists: a bitonic sort of the keys in LDS per list (a block per
// list, grid-stride over the queue); the keys of a list are distinct.  A list
// beyond kLongLds entries is sorted by one thread (never at the configs'
// sizes: in-degree within one hop's lists).
constexpr int kLongLds = 8192;
constexpr int kLongThreads = 256;
__global__ __launch_bounds__(kLongThreads) void tlong_kernel(Ctl* c, int hop, int32_t* __restrict__ pack,
                                                             const int32_t* __restrict__ longs) {
    GS_DS_BAIL(c);
    __shared__ int32_t sk[kLongLds];
    const HopCtl& h = c->hop[hop];
    if (h.n_src <= 0) return;
    const int n_long = longs[0];
    const int32_t* tp = pack + h.off[GS_PK_TPTR];
    int32_t* x = pack + h.off[GS_PK_TIDX];
    for (int q = blockIdx.x; q < n_long; q += gridDim.x) {
        const int src = longs[1 + q];
        const int lo = tp[src], len = tp[src + 1] - lo;
        if (len > kLongLds) {
            if (threadIdx.x == 0)
                for (int i = lo + 1; i < lo + len; ++i) {
                    const int32_t v = x[i], kv = tkey(v);
                    int j = i;
                    while (j > lo && tkey(x[j - 1]) > kv) {
                        x[j] = x[j - 1];
                        --j;
                    }
                    x[j] = v;
                }
            continue;
        }
        int P = 1;
        while (P < len) P <<= 1;
        for (int i = threadIdx.x; i < P; i += kLongThreads) sk[i] = i < len ? tkey(x[lo + i]) : INT_MAX;
        __syncthreads();
        for (int kk = 2; kk <= P; kk <<= 1)
            for (int jj = kk >> 1; jj > 0; jj >>= 1) {
                for (int i = threadIdx.x; i < P; i += kLongThreads) {
                    const int l = i ^ jj;
                    if (l > i) {
                        const int32_t a = sk[i], b = sk[l];
                        const bool up = (i & kk) == 0;
                        if (up ? a > b : a < b) {
                            sk[i] = b;
                            sk[l] = a;
                        }
                    }
                }
                __syncthreads();
            }
        for (int i = threadIdx.x; i < len; i += kLongThreads) x[lo + i] = tval(sk[i]);
        __syncthreads();  // sk is reused by the next list
    }
}

void launch_hop_union(const DevGraph& g, Ctl* c, const HopBufs& hb, UnionBufs& ub, const HopBufs& next, int hop,
                      int k, int64_t nd_max, int64_t nd_next_max, int flags, int32_t* pack, hipStream_t st,
                      bool with_lists) {
    static const bool attr = [] {
        return hipFuncSetAttribute(reinterpret_cast<const void*>(ublock_kernel),
                                   hipFuncAttributeMaxDynamicSharedMemorySize,
                                   kUnionLds) == hipSuccess;
    }();
    if (!attr) fail(GS_EHIP, "ublock_kernel: cannot raise its LDS limit");
    const int gcn = (flags & GS_SAMPLE_GCN) ? 1 : 0;
    sets_kernel<<<static_cast<unsigned>((nd_max + kSetWaves - 1) / kSetWaves), 64 * kSetWaves, 0, st>>>(g, c, hb, ub,
                                                                                                    hop, k);
    check_launch("sets_kernel");
    ufresh_kernel<<<static_cast<unsigned>(nd_max), 64, 0, st>>>(c, hb, ub, hop);
    check_launch("ufresh_kernel");
    ublock_kernel<<<1, 1024, kUnionLds, st>>>(c, hb, ub, next, hop, gcn, pack,
                                                                   static_cast<int>(nd_next_max));
    check_launch("ublock_kernel");
    static const bool attr_big = [] {
        return hipFuncSetAttribute(reinterpret_cast<const void*>(ubig_kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                                   kUnionBig * sizeof(uint16_t)) == hipSuccess;
    }();
    if (!attr_big) fail(GS_EHIP, "ubig_kernel: cannot raise its LDS limit");
    ubig_kernel<<<1, 1024, kUnionBig * sizeof(uint16_t), st>>>(c, hb, ub, next, hop, gcn, pack,
                                                               static_cast<int>(nd_next_max));
    check_launch("ubig_kernel");
    if (with_lists) launch_hop_lists(c, hb, ub, hop, nd_max, nd_next_max, flags, pack, st);
}

void launch_hop_lists(Ctl* c, const HopBufs& hb, UnionBufs& ub, int hop, int64_t nd_max, int64_t nd_next_max,
                      int flags, int32_t* pack, hipStream_t st) {
    const int gcn = (flags & GS_SAMPLE_GCN) ? 1 : 0;
    uout_kernel<<<static_cast<unsigned>(nd_max), 64, 0, st>>>(c, hb, ub, hop, gcn, pack);
    check_launch("uout_kernel");
    tscan_kernel<<<1, 1024, 0, st>>>(c, hop, pack, ub.tcnt, ub.longs);
    check_launch("tscan_kernel");
    tfill_kernel<<<static_cast<unsigned>(nd_max), 64, 0, st>>>(c, hop, pack, ub.tcnt);
    check_launch("tfill_kernel");
    tsort_kernel<<<static_cast<unsigned>((nd_next_max + 255) / 256), 256, 0, st>>>(c, hop, pack, ub.longs);
    check_launch("tsort_kernel");
    tlong_kernel<<<256, kLongThreads, 0, st>>>(c, hop, pack, ub.longs);
    check_launch("tlong_kernel");
}

}  // namespace ds
}  // namespace gs
