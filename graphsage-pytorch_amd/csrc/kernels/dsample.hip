// Device-resident neighbour sampler: GraphSage.forward's hop
// loop over _get_unique_neighs_list (models.py:246-251, :277-289) run on the
// GPU, bit-exact with the host sampler (host/sampler.cpp) and therefore with
// the reference's CPython `random` stream and set iteration order.  It writes
// the same device pack the host sampler writes (gs_sample_pack_run), straight
// into device memory, so nothing downstream changes.
//
// Pieces (each one documented at its kernel):
//   word stream   MT19937 (CPython's genrand_uint32, Modules/_randommodule.c)
//                 regenerated on the device into a ring of tempered words,
//                 indexed by absolute stream position.  x[A] = x[A-227] ^
//                 twist(x[A-624], x[A-623]) is the whole recurrence, so one
//                 wave produces 227 words per dependent step.
//   draws         random.sample (Lib/random.py 3.10, both branches) for every
//                 frontier node of a hop, in frontier order.  The only
//                 sequential quantity is the stream position, and it is the
//                 hop's draw count plus the rejections so far (j).  Frontier
//                 nodes are cut into blocks; for every block and every entry
//                 j in a window around the expected rejection count the exit
//                 j' is computed in parallel (one lane per entry), the block
//                 maps are composed group by group in LDS, one lane chains the
//                 group maps, and every block then re-walks from its true
//                 entry and emits its positions.  A true entry outside its
//                 window is detected and reported (never silently wrong).
//   sets/union    (hops before the last) samp_neigh | {node} per frontier node
//                 and list(set.union(*samp_neighs)) — see dsample_union.hip.
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "../host/graph.hpp"
#include "../host/mt19937.hpp"
#include "dsample.hpp"

namespace gs {
namespace ds {

// ------------------------------------------------------------ word stream

__device__ __forceinline__ uint32_t temper(uint32_t y) {
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= (y >> 18);
    return y;
}

// One block extends the stream from c->gen_end until it covers `need`
// (absolute word index, exclusive): stages of 227 words, each word
// x[A] = x[A-227] ^ ((y >> 1) ^ (y & 1 ? MATRIX_A : 0)), y = (x[A-624] & UPPER)
// | (x[A-623] & LOWER) — CPython's twist loop written on absolute indices (its
// three index ranges are this one recurrence).  Thread i < 227 owns residue i
// of A - g0 mod 227, so x[A-227] is its own previous value (a register); the
// two older words were written to the LDS ring at least two stages earlier
// (A-623 <= g-397), so one barrier per stage orders every read after its
// write.  Only the tempered words go to global memory (what the draws read);
// the raw words the next launch and getstate need are the last 624, written
// once at the end.
constexpr int kGenThreads = 256;
constexpr int kGenRing = 2048;  // LDS ring: reads reach back 624 words, a step writes 454 ahead
// spec = 1 (the sampler's aux stream, beside the last hop's draws): extend
// the stream to `need_fixed` words past hop need_hop's first draw, into
// gen_spec, never touching gen_end or any word below it (the draws in flight
// read only words below gen_end).  The main stream's next launch, ordered
// after the aux stream by an event, takes gen_spec over as its gen_end.  The
// lead stays bounded by need_fixed, far inside the ring.
constexpr int64_t kGenAhead = int64_t(1) << 18;  // a rmat2m batch reads ~75k words
__global__ __launch_bounds__(kGenThreads) void mt_gen_kernel(uint32_t* __restrict__ xr, uint32_t* __restrict__ wr,
                                                             Ctl* c, int64_t need_fixed, int need_hop, int spec = 0) {
    __shared__ uint32_t L[kGenRing];
    constexpr int64_t M = kGenRing - 1;
    const int i = threadIdx.x;
    const int64_t ge = c->gen_end;
    const int64_t g0 = max(ge, c->gen_spec);
    const int64_t need = spec ? c->hop[need_hop].P0 + need_fixed : need_hop >= 0 ? c->hop[need_hop].need_end : need_fixed;
    if (g0 >= need) {
        if (!spec && i == 0 && g0 != ge) c->gen_end = g0;
        return;
    }
    for (int q = i; q < 624; q += kGenThreads) {
        const int64_t A = g0 - 624 + q;
        L[A & M] = xr[A & kRingMask];
    }
    __syncthreads();
    uint32_t prev = i < 227 ? L[(g0 - 227 + i) & M] : 0u;
    int64_t g = g0;
    // Two stages per barrier: word A = g + 227 + i reads x[A - 624] and
    // x[A - 623] (<= g - 170, written before the barrier) and x[A - 227] =
    // the thread's word of the first stage, a register.
    while (g < need) {
        if (i < 227) {
            const int64_t A = g + i;
            const uint32_t a = L[(A - 624) & M], b = L[(A - 623) & M];
            const uint32_t a2 = L[(A - 397) & M], b2 = L[(A - 396) & M];
            const uint32_t y = (a & 0x80000000u) | (b & 0x7fffffffu);
            const uint32_t x = prev ^ (y >> 1) ^ ((0u - (y & 1u)) & 0x9908b0dfu);
            const uint32_t y2 = (a2 & 0x80000000u) | (b2 & 0x7fffffffu);
            const uint32_t x2 = x ^ (y2 >> 1) ^ ((0u - (y2 & 1u)) & 0x9908b0dfu);
            prev = x2;
            L[A & M] = x;
            L[(A + 227) & M] = x2;
            xr[A & kRingMask] = x;
            xr[(A + 227) & kRingMask] = x2;
            wr[A & kRingMask] = temper(x);
            wr[(A + 227) & kRingMask] = temper(x2);
        }
        __syncthreads();
        g += 454;
    }
    if (i == 0) {
        if (spec) c->gen_spec = g;
        else c->gen_end = g;
    }
}

// Seed the stream from random.setstate's (mt[624], pos): block 0 = mt, the
// next word is at absolute index pos.
__global__ void mt_seed_kernel(const uint32_t* __restrict__ mt, int64_t pos, uint32_t* __restrict__ xr,
                               uint32_t* __restrict__ wr, Ctl* c) {
    for (int i = threadIdx.x; i < 624; i += blockDim.x) {
        xr[i] = mt[i];
        wr[i] = temper(mt[i]);
    }
    if (threadIdx.x == 0) {
        c->gen_end = 624;
        c->gen_spec = 0;
        c->pos_cur = pos;
        c->status = 0;
    }
}

// --------------------------------------------------------------- draws

// Expected rejections (and their variance) before the k accepted draws of
// one frontier node: geometric with acceptance m / 2^bitlen per word (pool
// branch, m = d - i), (d - i) / 2^bitlen(d) in the selected-set branch.
__device__ __forceinline__ void rejection_moments(uint32_t d, int k, int setsize, float& mean, float& var) {
    mean = 0.f;
    var = 0.f;
    if (k <= 0 || d < static_cast<uint32_t>(k)) return;
    const bool pool = d <= static_cast<uint32_t>(setsize);
    // per draw, words until acceptance ~ geometric(p), p = m / 2^bitlen:
    // E[rejections] = 1/p - 1, Var = (1/p)(1/p - 1) (window sizing only, so
    // the fast reciprocal is enough)
    for (int i = 0; i < k; ++i) {
        const uint32_t m = d - i;
        const uint32_t span = pool ? m : d;
        const float full = ldexpf(1.f, 32 - __clz(span));
        const float q = full * __frcp_rn(static_cast<float>(m));
        mean += q - 1.f;
        var += q * (q - 1.f);
    }
}

constexpr int kSetupBatch = 8;

// Per hop, one 1024-thread block: degrees of the frontier, the scans of the
// sampled counts (pos_ptr) and draw counts, the rejection-count windows of
// the blocks, the word need of the hop, and (last hop) the pack offsets.
__global__ __launch_bounds__(1024) void hop_setup_kernel(DevGraph g, Ctl* c, HopBufs hb, int hop, int k, int setsize,
                                                         int R, int last, int n_roots, int gcn) {
    GS_DS_BAIL(c);
    __shared__ int shi[17];
    __shared__ float shf[17];
    __shared__ int s_maxw, s_maxlo;
    HopCtl& h = c->hop[hop];
    const int n = hop == 0 ? n_roots : c->hop[hop - 1].n_src;
    if (threadIdx.x == 0) {
        s_maxw = 0;
        s_maxlo = 0;
    }
    const int per = (n + 1023) / 1024;
    const int r0 = min(n, static_cast<int>(threadIdx.x) * per), r1 = min(n, r0 + per);
    int cnt_sum = 0, draw_sum = 0;
    float mean_sum = 0.f, var_sum = 0.f;
    // Up to kSetupRows rows per thread (n <= 16 Ki) stay in registers between
    // the passes: every id, then every row_ptr pair loaded at once, and no
    // pass re-reads what an earlier one stored (a store-then-load per row
    // costs a memory round each).  Larger frontiers take the global passes.
    constexpr int kSetupRows = 16;
    const bool cached = per <= kSetupRows;
    int32_t dc[kSetupRows];
    float2 mc[kSetupRows];
    auto moments = [&](int r, int32_t d, float2& mv) {
        const bool sampled = k > 0 && d >= k;
        cnt_sum += sampled ? k : d;
        draw_sum += sampled ? k : 0;
        float mu, va;
        rejection_moments(static_cast<uint32_t>(d), k, setsize, mu, va);
        mv = make_float2(mu, va);
        hb.mv[r] = mv;
        mean_sum += mu;
        var_sum += va;
    };
    if (cached) {
        int32_t vv[kSetupRows];
        int64_t lo[kSetupRows], hi[kSetupRows];
#pragma unroll
        for (int q = 0; q < kSetupRows; ++q) vv[q] = r0 + q < r1 ? hb.dst[r0 + q] : 0;
#pragma unroll
        for (int q = 0; q < kSetupRows; ++q) {
            lo[q] = r0 + q < r1 ? g.row_ptr[vv[q]] : 0;
            hi[q] = r0 + q < r1 ? g.row_ptr[vv[q] + 1] : 0;
        }
#pragma unroll
        for (int q = 0; q < kSetupRows; ++q) {
            dc[q] = static_cast<int32_t>(hi[q] - lo[q]);
            if (r0 + q < r1) {
                hb.deg[r0 + q] = dc[q];
                moments(r0 + q, dc[q], mc[q]);
            }
        }
    } else {
        // degrees, kSetupBatch nodes at a time: every id, then every row_ptr
        // pair, loaded before any is used (independent loads in flight together)
        for (int rb = r0; rb < r1; rb += kSetupBatch) {
            int32_t vv[kSetupBatch];
            int64_t lo[kSetupBatch], hi[kSetupBatch];
#pragma unroll
            for (int q = 0; q < kSetupBatch; ++q) vv[q] = rb + q < r1 ? hb.dst[rb + q] : 0;
#pragma unroll
            for (int q = 0; q < kSetupBatch; ++q) {
                lo[q] = rb + q < r1 ? g.row_ptr[vv[q]] : 0;
                hi[q] = rb + q < r1 ? g.row_ptr[vv[q] + 1] : 0;
            }
#pragma unroll
            for (int q = 0; q < kSetupBatch; ++q)
                if (rb + q < r1) hb.deg[rb + q] = static_cast<int32_t>(hi[q] - lo[q]);
        }
        for (int r = r0; r < r1; ++r) {
            float2 mv;
            moments(r, hb.deg[r], mv);
        }
    }
    int cnt_tot, draw_tot;
    float mean_tot, var_tot;
    int cnt_pre = block_excl_scan(cnt_sum, shi, &cnt_tot);
    int draw_pre = block_excl_scan(draw_sum, shi, &draw_tot);
    float mean_pre = block_excl_scan(mean_sum, shf, &mean_tot);
    float var_pre = block_excl_scan(var_sum, shf, &var_tot);
    auto place = [&](int r, int32_t d, float2 mv) {
        const bool sampled = k > 0 && d >= k;
        hb.pos_ptr[r] = cnt_pre;
        if (r % R == 0) {
            const int b = r / R;
            const float sd = sqrtf(var_pre);
            const int lo = max(0, static_cast<int>(floorf(mean_pre - 6.f * sd)) - 16);
            const int hi = static_cast<int>(ceilf(mean_pre + 6.f * sd)) + 16;
            hb.blo[b] = lo;
            hb.bw[b] = (hi - lo + 63) & ~63;  // this block's window (the hop-wide W bounds it)
            hb.dbase[b] = draw_pre;
            atomicMax(&s_maxw, hi - lo);
            atomicMax(&s_maxlo, lo);
        }
        cnt_pre += sampled ? k : d;
        draw_pre += sampled ? k : 0;
        mean_pre += mv.x;
        var_pre += mv.y;
    };
    if (cached) {
#pragma unroll
        for (int q = 0; q < kSetupRows; ++q)
            if (r0 + q < r1) place(r0 + q, dc[q], mc[q]);
    } else {
        for (int r = r0; r < r1; ++r) place(r, hb.deg[r], hb.mv[r]);
    }
    if (threadIdx.x == 0) {
        hb.pos_ptr[n] = cnt_tot;
        const int nb = (n + R - 1) / R;
        hb.dbase[nb] = draw_tot;
        hb.blo[nb] = 0;  // never an entry window (the last group's exit is absolute)
        hb.bw[nb] = 0;
    }
    __syncthreads();
    // The table kernel's work list: the 256-entry parts of every block's
    // window, blocks ascending.  Its grid is launched at the bound, and the
    // items come first, so the workgroups with work are dispatched first and
    // spread over the chip (the parts past a window no longer sit between them).
    {
        const int nb = (n + R - 1) / R;
        const int pb = (nb + 1023) / 1024;
        const int b0 = min(nb, static_cast<int>(threadIdx.x) * pb), b1 = min(nb, b0 + pb);
        int cnt = 0;
        for (int b = b0; b < b1; ++b) cnt += (min(hb.bw[b], kWMax) + kMEntries - 1) / kMEntries;
        int tot;
        int at = block_excl_scan(cnt, shi, &tot);
        for (int b = b0; b < b1; ++b) {
            const int parts = (min(hb.bw[b], kWMax) + kMEntries - 1) / kMEntries;
            for (int y = 0; y < parts; ++y) hb.wg[at++] = b | (y << 16);
        }
        if (threadIdx.x == 0) h.n_wg = tot;
    }
    if (threadIdx.x == 0) {
        int W = 64;
        while (W < s_maxw) W <<= 1;
        if (W > kWMax) c->status |= kStWindow;
        W = min(W, kWMax);
        const int nb = (n + R - 1) / R;
        const int G = max(1, kComposeEntries / W);
        h.n_dst = n;
        h.n_pos = cnt_tot;
        h.n_draws = draw_tot;
        h.n_blocks = nb;
        h.W = W;
        h.G = G;
        h.n_groups = (nb + G - 1) / G;
        h.P0 = c->pos_cur;
        h.n_empty = 0;
        h.need_end = h.P0 + draw_tot + s_maxlo + W + 3 * R * max(k, 1) + 256;
        if (last) {
            int at = c->total;
            h.off[GS_PK_POS_PTR] = at;
            at += al4(n + 1);
            h.off[GS_PK_POS] = at;
            at += al4(cnt_tot);
            h.off[GS_PK_DST_IDS] = at;
            at += al4(n);
            c->total = at;
        }
    }
}

// Words of block b's window into LDS: relative positions dbase + lo .. , as
// many as are generated (the count is returned).
__device__ __forceinline__ int load_words(const uint32_t* __restrict__ wr, const Ctl* c, int64_t A0, int nw,
                                          uint32_t* __restrict__ dst) {
    const int64_t gen = c->gen_end;
    const int nvalid = static_cast<int>(max<int64_t>(0, min<int64_t>(nw, gen - A0)));
    // kLoadBatch loads in flight per thread before their LDS stores (a
    // load-then-store loop waits out one global latency per iteration)
    constexpr int kLoadBatch = 8;
    for (int base = threadIdx.x; base < nvalid; base += kLoadBatch * blockDim.x) {
        uint32_t v[kLoadBatch];
#pragma unroll
        for (int u = 0; u < kLoadBatch; ++u) {
            const int i = base + u * static_cast<int>(blockDim.x);
            v[u] = i < nvalid ? wr[(A0 + i) & kRingMask] : 0u;
        }
#pragma unroll
        for (int u = 0; u < kLoadBatch; ++u) {
            const int i = base + u * static_cast<int>(blockDim.x);
            if (i < nvalid) dst[i] = v[u];
        }
    }
    return nvalid;
}

// ---- block maps by acceptance bitmasks
//
// Block maps: E[b][e] = rejections inside block b when it is entered with
// lo_b + e rejections so far (0xFFFF: ran past the loaded words).  For every sampled node of the block and every one of
// its draws, the words that draw would accept form a bitmask over the node's
// word window: pool branch, draw i accepts word x iff
// (x >> clz(d - i)) < d - i; selected-set branch, every draw accepts
// (x >> clz(d)) < d, minus repeats of the node's earlier picks.  A walk then
// costs one 64-bit window read and a ctz per draw (the first accepted word at
// or after the walk's position), the same instructions for every lane; the
// selected-set branch reads the accepted word's value once for its repeat
// test.  A walk past its node's mask window (more than kRejBudget rejections
// in the block) continues word by word, so the result is exact either way.
//
// One 256-thread workgroup per (block, 256 entries): the work is the block's
// window width times its draws, so wide blocks (late in the hop) are split
// over several CUs, and each workgroup builds masks only over the words its
// 256 entries can reach.
constexpr int kRejBudget = 192;                                   // mask-covered rejections per block
constexpr int kMChunks = (kMEntries + kRejBudget + 63) / 64 + 1;  // mask words per draw (+1 for the 2-word window)

// Walk one node from block word u (relative to the workgroup's first word),
// the node's words starting at a; M: its masks as 32-bit words, kMChunks * 2
// per draw.  The 32-bit window at the walk's position is one alignbit of
// two adjacent mask words; its first set bit is the next accepted word.
// The exact word-by-word walk of one node from block word u (the fallback
// of walk_masked for a walk that leaves its mask window).
template <int KMAX>
__device__ __noinline__ int walk_words(const uint32_t* __restrict__ w, int nvalid, int u, uint32_t d, int k, bool pool) {
    if (pool) {
        for (int i = 0; i < k; ++i) {
            const uint32_t m = d - i;
            const int sh = __clz(m);
            for (;;) {
                if (u >= nvalid) return -1;
                if ((w[u++] >> sh) < m) break;
            }
        }
        return u;
    }
    const int sh = __clz(d);
    uint32_t sel[KMAX];
    int cnt = 0;
    while (cnt < k) {
        if (u >= nvalid) return -1;
        const uint32_t v = w[u++] >> sh;
        bool fresh = v < d;
#pragma unroll
        for (int t = 0; t < KMAX; ++t) fresh &= !(t < cnt && sel[t] == v);
#pragma unroll
        for (int t = 0; t < KMAX; ++t)
            if (t == cnt) sel[t] = v;
        cnt += fresh;
    }
    return u;
}

// Walk one node from block word u (relative to the workgroup's first word),
// the node's words starting at a; M: its masks as 32-bit words, kMChunks * 2
// per draw.  The 32-bit window at the walk's position is one alignbit of
// two adjacent mask words; its first set bit is the next accepted word.  A
// walk that finds no accepted word in its window (more rejections than the
// masks cover) redoes the node word by word; the draw loop itself has a
// fixed trip count and no per-lane exit.
template <int KMAX>
__device__ __forceinline__ int walk_masked(const uint32_t* __restrict__ M, int a, int u, uint32_t d, int k,
                                           bool pool, const uint32_t* __restrict__ w, int nvalid) {
    constexpr int C32 = 2 * kMChunks;
    constexpr int lim = (C32 - 1) * 32;
    if (u < 0) return -1;
    int rel = u - a;
    bool bad = false;
    if (pool) {
        for (int i = 0; i < k; ++i) {
            const uint32_t* Mi = M + i * C32;
            const int j = min(rel >> 5, C32 - 2);
            // both mask words read unconditionally (j is clamped), the window
            // zeroed past the masks: no branch around the LDS read
            const uint32_t win = __builtin_amdgcn_alignbit(Mi[j + 1], Mi[j], rel & 31) & (0u - (rel < lim));
            const int adv = __ffs(win);  // 1 + the accepted word's offset; 0: none in the window
            bad |= adv == 0;
            rel += adv;
        }
    } else {
        // The picks so far as a set: slots start at a sentinel no in-range
        // value equals (values < d < 2^31) and a fresh value enters by a shift
        // (membership is all the repeat test needs), so each word costs KMAX
        // compares and KMAX selects, none of them on the pick count.
        const int sh = __clz(d);
        // Speculative pass: the first k accepted words by their masks alone
        // (one dependent LDS read per draw), then their values all at once.
        // Without a repeat among them they are exactly the k picks; at the
        // first repeat l the exact loop below resumes with picks 0..l-1 and
        // the walk just past word l.
        // (KMAX <= 16 only: at the root hop's KMAX = 25 the pairwise repeat
        // test and its registers cost more than the chain saves, measured)
        constexpr int KS = KMAX <= 16 ? KMAX : 1;
        int rels[KS];
        uint32_t vals[KS];
        if constexpr (KMAX <= 16) {
            int r = rel;
#pragma unroll
            for (int i = 0; i < KMAX; ++i) {
                if (i < k) {
                    const int j = min(r >> 5, C32 - 2);
                    const uint32_t win = __builtin_amdgcn_alignbit(M[j + 1], M[j], r & 31) & (0u - (r < lim));
                    const int adv = __ffs(win);
                    bad |= adv == 0;
                    r += adv;
                }
                rels[i] = r;
            }
#pragma unroll
            for (int i = 0; i < KMAX; ++i) vals[i] = i < k ? w[a + max(rels[i] - 1, 0)] >> sh : 0xFFFFFFFFu - i;
        }
        int keep = 0;  // picks the speculative pass settled
        if constexpr (KMAX <= 16) {
            int first = k;  // the first pick index whose value repeats an earlier one
#pragma unroll
            for (int l = KMAX - 1; l > 0; --l) {
                bool rep = false;
#pragma unroll
                for (int i = 0; i < l; ++i) rep |= vals[i] == vals[l];
                first = (rep && l < k) ? l : first;
            }
            if (!bad && first == k) return a + rels[KMAX - 1];  // rels[i >= k] hold the walk after draw k-1
            // resume just past the repeated word with picks 0..first-1; a
            // speculative walk that left its masks restarts from the node's start
            keep = bad ? 0 : first;
#pragma unroll
            for (int t = 1; t < KMAX; ++t)
                if (t == keep) rel = rels[t];
        }
        uint32_t sel[KMAX];
#pragma unroll
        for (int t = 0; t < KMAX; ++t) {
            sel[t] = 0xFFFFFFFFu;
            if constexpr (KMAX <= 16) sel[t] = t < keep ? vals[t] : 0xFFFFFFFFu;
        }
        int cnt = keep;
        bad = false;
        while (cnt < k && !bad) {
            const int j = min(rel >> 5, C32 - 2);
            const uint32_t win = __builtin_amdgcn_alignbit(M[j + 1], M[j], rel & 31) & (0u - (rel < lim));
            const int adv = __ffs(win);
            bad = adv == 0;
            rel += adv;
            const uint32_t val = w[a + max(rel - 1, 0)] >> sh;
            bool fresh = !bad;
#pragma unroll
            for (int t = 0; t < KMAX; ++t) fresh &= sel[t] != val;
#pragma unroll
            for (int t = KMAX - 1; t > 0; --t) sel[t] = fresh ? sel[t - 1] : sel[t];
            sel[0] = fresh ? val : sel[0];
            cnt += fresh;
        }
    }
    if (bad) return walk_words<KMAX>(w, nvalid, u, d, k, pool);
    return a + rel;
}

template <int KMAX>
__global__ __launch_bounds__(kMEntries) void draw_masked_kernel(const uint32_t* __restrict__ wr, Ctl* c, HopBufs hb,
                                                                int hop, int k, int setsize, int R) {
    GS_DS_BAIL(c);
    extern __shared__ uint64_t smem64[];
    __shared__ int s_d[256], s_moff[257];
    __shared__ int s_nsr;
    const HopCtl& h = c->hop[hop];
    if (static_cast<int>(blockIdx.x) >= h.n_wg) return;  // past the work list (hop_setup)
    const int item = hb.wg[blockIdx.x];
    const int b = item & 0xFFFF, part = item >> 16;
    const int Wst = h.W;
    const int bw = min(hb.bw[b], Wst);
    const int e0 = part * kMEntries;
    if (e0 >= bw) return;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int r0 = b * R, nr = min(R, h.n_dst - r0);
    const int ndr = hb.dbase[min(b + 1, h.n_blocks)] - hb.dbase[b];
    // phase stamps of one workgroup of the last hop (gs_dsampler_debug slots 56..61)
    const bool stamp = hop > 0 && b == h.n_blocks / 2 && part == 0 && tid == 0;
    if (stamp) c->dbg[56] = static_cast<int64_t>(__builtin_amdgcn_s_memrealtime());
    // masks: [node][draw][kMChunks] (pool: k draws, selected-set: 1), then the words
    uint64_t* masks = smem64;
    uint32_t* w = reinterpret_cast<uint32_t*>(masks + R * max(k, 1) * kMChunks);
    // words from this workgroup's first entry on (entry e0 starts at word e0 of the block)
    const int nw = kMEntries + ndr + 3 * R * max(k, 1) + 64;
    const int nvalid = load_words(wr, c, h.P0 + hb.dbase[b] + hb.blo[b] + e0, nw, w);
    if (tid < 64) {  // the sampled nodes in order, compacted by one wave
        int m = 0, off = 0;
        for (int q0 = 0; q0 < nr; q0 += 64) {
            const int q = q0 + lane;
            const int d = q < nr ? hb.deg[r0 + q] : 0;
            const bool smp = q < nr && k > 0 && d >= k;
            const uint64_t bal = __ballot(smp);
            const int at = m + __popcll(bal & ((1ull << lane) - 1ull));
            const int sz = smp ? (static_cast<uint32_t>(d) <= static_cast<uint32_t>(setsize) ? k : 1) * kMChunks : 0;
            // exclusive prefix of the mask sizes in this chunk of nodes
            int inc = sz;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const int t = __shfl_up(inc, o, 64);
                if (lane >= o) inc += t;
            }
            if (smp) {
                s_d[at] = d;
                s_moff[at] = off + inc - sz;
            }
            m += __popcll(bal);
            off += __shfl(inc, 63, 64);
        }
        if (lane == 0) {
            s_moff[m] = off;
            s_nsr = m;
        }
    }
    __syncthreads();
    const int nsr = s_nsr;
    if (stamp) c->dbg[57] = static_cast<int64_t>(__builtin_amdgcn_s_memrealtime());
    // build: node m's window starts at word m * k (entry e0, no rejections
    // yet).  One wave per node: its kMChunks words per lane read at once, then
    // a ballot per (draw bound, chunk).
    for (int q = wave; q < nsr; q += kMEntries / 64) {
        const uint32_t d = static_cast<uint32_t>(s_d[q]);
        uint64_t* M = masks + s_moff[q];
        uint32_t x[kMChunks];
        bool ok[kMChunks];
#pragma unroll
        for (int ch = 0; ch < kMChunks; ++ch) {
            const int pos = q * k + 64 * ch + lane;
            ok[ch] = pos < nvalid;
            x[ch] = w[max(0, min(pos, nvalid - 1))];
        }
        if (d <= static_cast<uint32_t>(setsize)) {
            for (int i = 0; i < k; ++i) {
                const uint32_t m = d - i;
                const int sh = __clz(m);
#pragma unroll
                for (int ch = 0; ch < kMChunks; ++ch) {
                    const uint64_t bal = __ballot(ok[ch] && (x[ch] >> sh) < m);
                    if (lane == 0) M[i * kMChunks + ch] = bal;
                }
            }
        } else {
            const int sh = __clz(d);
#pragma unroll
            for (int ch = 0; ch < kMChunks; ++ch) {
                const uint64_t bal = __ballot(ok[ch] && (x[ch] >> sh) < d);
                if (lane == 0) M[ch] = bal;
            }
        }
    }
    __syncthreads();
    if (stamp) c->dbg[58] = static_cast<int64_t>(__builtin_amdgcn_s_memrealtime());
    const int ent = e0 + tid;
    int u = ent < bw ? tid : -1;  // word index relative to e0
    uint8_t* rej = hb.rej + static_cast<int64_t>(b) * R * kWMax + ent;
    bool rej_over = false;
    for (int q = 0; q < nsr; ++q) {
        const uint32_t d = static_cast<uint32_t>(s_d[q]);
        const int u0 = u;
        u = walk_masked<KMAX>(reinterpret_cast<const uint32_t*>(masks + s_moff[q]), q * k, u, d, k,
                              d <= static_cast<uint32_t>(setsize), w, nvalid);
        // this node's rejections on this entry's path (the emit's node starts)
        if (u >= 0) {
            const int rj = u - u0 - k;
            rej_over |= rj > 254;
            rej[static_cast<int64_t>(q) * kWMax] = static_cast<uint8_t>(min(rj, 255));
        }
    }
    if (rej_over) atomicOr(&c->status, kStWords);  // a node with > 254 rejections: never seen, reported
    if (stamp) {
        c->dbg[59] = static_cast<int64_t>(__builtin_amdgcn_s_memrealtime());
        c->dbg[60] = nsr | (static_cast<int64_t>(bw) << 16) | (static_cast<int64_t>(h.n_blocks) << 32);
        c->dbg[61] = h.n_wg | (static_cast<int64_t>(h.W) << 16) | (static_cast<int64_t>(ndr) << 32);
    }
    if (ent < bw) {
        uint16_t* E = hb.tab + static_cast<int64_t>(b) * Wst;
        const int dr = u < 0 ? -1 : u - tid - ndr;
        E[ent] = (dr < 0 || dr >= 0xFFFF) ? 0xFFFF : static_cast<uint16_t>(dr);
    }
}

// Group maps: for every entry of the group's first block, the entries of each
// of its blocks (path) and the group's exit, relative to the next group's
// window (uint16; 0xFFFF outside it), or absolute for the last group.  The
// group's block maps are staged in LDS.
__global__ __launch_bounds__(256) void draw_compose_kernel(Ctl* c, HopBufs hb, int hop) {
    GS_DS_BAIL(c);
    extern __shared__ __attribute__((aligned(16))) uint16_t tabs[];
    __shared__ int los[kComposeEntries / 64 + 1], wid[kComposeEntries / 64 + 1];
    const HopCtl& h = c->hop[hop];
    const int gi = blockIdx.x;
    if (gi >= h.n_groups) return;
    const int W = h.W, G = h.G;
    const int b0 = gi * G, nbk = min(G, h.n_blocks - b0);
    const bool last_group = gi == h.n_groups - 1;
    for (int i = threadIdx.x; i <= nbk; i += blockDim.x) {  // blo[nb] exists (setup)
        los[i] = hb.blo[b0 + i];
        wid[i] = i < nbk ? min(hb.bw[b0 + i], W) : W;
    }
    __syncthreads();
    // The group's block maps are nbk consecutive rows of W entries in hb.tab
    // (an entry past a row's width is never read): one flat copy of 16-byte
    // chunks, every load of the thread in flight before its LDS stores (one
    // memory round instead of one per block).
    {
        const uint4* src = reinterpret_cast<const uint4*>(hb.tab + static_cast<int64_t>(b0) * W);
        uint4* dst = reinterpret_cast<uint4*>(tabs);
        const int n16 = nbk * W / 8;  // <= kComposeEntries / 8
        constexpr int kU = kComposeEntries / 8 / 256;
        uint4 v[kU];
#pragma unroll
        for (int u = 0; u < kU; ++u) v[u] = src[min(static_cast<int>(threadIdx.x) + 256 * u, n16 - 1)];
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            const int i = threadIdx.x + 256 * u;
            if (i < n16) dst[i] = v[u];
        }
    }
    __syncthreads();
    int32_t* path = hb.path + static_cast<int64_t>(b0) * W;
    // kPathIlp entries per thread walk their block chains together (each chain
    // is a dependent LDS lookup per block)
    constexpr int kPathIlp = 4;
    const int w0 = wid[0];
    const int bw_next = last_group ? 0 : hb.bw[b0 + nbk];
    for (int e0 = threadIdx.x; e0 < w0; e0 += kPathIlp * blockDim.x) {
        int j[kPathIlp];
#pragma unroll
        for (int u = 0; u < kPathIlp; ++u) j[u] = los[0] + e0 + u * static_cast<int>(blockDim.x);
        for (int q = 0; q < nbk; ++q) {
            const int lq = los[q], wq = wid[q];
#pragma unroll
            for (int u = 0; u < kPathIlp; ++u) {
                const int e = e0 + u * static_cast<int>(blockDim.x);
                if (e < w0) path[q * W + e] = j[u];
                const int t = j[u] - lq;
                const bool in = j[u] >= 0 && t >= 0 && t < wq;
                const uint16_t d = tabs[q * W + (in ? t : 0)];
                j[u] = (in && d != 0xFFFF) ? j[u] + d : -1;
            }
        }
#pragma unroll
        for (int u = 0; u < kPathIlp; ++u) {
            const int e = e0 + u * static_cast<int>(blockDim.x);
            if (e >= w0) break;
            if (last_group) {
                hb.gexit_last[e] = j[u];
            } else {
                const int t = j[u] - los[nbk];
                hb.gexit[static_cast<int64_t>(gi) * W + e] =
                    (j[u] < 0 || t < 0 || t >= bw_next) ? 0xFFFF : static_cast<uint16_t>(t);
            }
        }
    }
}

// One block: chain the group maps from j = 0 (staged in LDS when they fit),
// then every block's true entry (a lookup in its group's path) and the hop's
// end position.
__global__ __launch_bounds__(1024) void draw_chain_kernel(Ctl* c, HopBufs hb, int hop) {
    GS_DS_BAIL(c);
    extern __shared__ __attribute__((aligned(16))) uint16_t gx[];
    __shared__ int gentry[kMaxGroups + 1];
    HopCtl& h = c->hop[hop];
    const int W = h.W, G = h.G, ng = h.n_groups;
    if (ng > kMaxGroups) {
        if (threadIdx.x == 0) c->status |= kStWindow;
        return;
    }
    const int64_t n16 = static_cast<int64_t>(ng - 1) * W;
    const bool staged = n16 <= kChainEntries;
    if (staged) {  // W % 64 == 0: whole 16-byte chunks, every load of a thread before its stores
        const uint4* src = reinterpret_cast<const uint4*>(hb.gexit);
        uint4* dst = reinterpret_cast<uint4*>(gx);
        const int n8 = static_cast<int>(n16 / 8);
        constexpr int kU = (kChainEntries / 8 + 1023) / 1024;
        uint4 v[kU];
#pragma unroll
        for (int u = 0; u < kU; ++u) v[u] = src[max(0, min(static_cast<int>(threadIdx.x) + 1024 * u, n8 - 1))];
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            const int i = threadIdx.x + 1024 * u;
            if (i < n8) dst[i] = v[u];
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        int j = 0;
        for (int gi = 0; gi < ng; ++gi) {
            gentry[gi] = j;
            const int lo = hb.blo[gi * G];
            const int t = j - lo;
            if (j < 0 || t < 0 || t >= min(hb.bw[gi * G], W)) {
                j = -1;
                for (int q = gi + 1; q < ng; ++q) gentry[q] = -1;
                break;
            }
            if (gi == ng - 1) {
                j = hb.gexit_last[t];
            } else {
                const uint16_t d = staged ? gx[static_cast<int64_t>(gi) * W + t] : hb.gexit[static_cast<int64_t>(gi) * W + t];
                j = d == 0xFFFF ? -1 : hb.blo[(gi + 1) * G] + d;
            }
        }
        gentry[ng] = j;
        if (j < 0) c->status |= kStWindow;
        h.j_end = j;
        c->pos_cur = h.P0 + h.n_draws + max(j, 0);
    }
    __syncthreads();
    for (int b = threadIdx.x; b < h.n_blocks; b += blockDim.x) {
        const int gi = b / G;
        const int jg = gentry[gi];
        const int t = jg - hb.blo[gi * G];
        hb.entry[b] = (jg < 0 || t < 0 || t >= min(hb.bw[gi * G], W)) ? -1 : hb.path[static_cast<int64_t>(b) * W + t];
    }
}

// Every frontier node from its start on the true path, one wave per node:
// node m of block b starts m * k words plus the rejections of the block's
// earlier sampled nodes (recorded per entry by the table kernel) after the
// block's true entry.  The wave stages 256 of its words in LDS and walks
// them 64 at a time — a ballot of the words acceptable for the current draw
// finds the next accepted one — emitting random.sample's result order as
// absolute CSR entries: pool branch with the swapped pool slots in lanes
// (key, value), selected-set branch with the picks in lanes; rows below k
// whole.
constexpr int kEmitWaves = 4;
constexpr int kEmitWords = 256;
__global__ __launch_bounds__(64 * kEmitWaves) void draw_emit_kernel(const uint32_t* __restrict__ wr, Ctl* c, HopBufs hb,
                                                                    DevGraph g, int hop, int k, int setsize, int R,
                                                                    int last, int gcn, int32_t* __restrict__ pack) {
    GS_DS_BAIL(c);
    __shared__ uint32_t wbuf[kEmitWaves][kEmitWords];
    HopCtl& h = c->hop[hop];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int r = blockIdx.x * kEmitWaves + wave;
    if (r >= h.n_dst) return;
    const int b = r / R, r0 = b * R;
    const int j = hb.entry[b];
    if (j < 0) return;  // reported by the chain
    uint32_t* w = wbuf[wave];
    const int32_t v = hb.dst[r];
    const uint32_t d = static_cast<uint32_t>(hb.deg[r]);
    const int32_t base = static_cast<int32_t>(g.row_ptr[v]);
    int32_t* out = (last ? pack + h.off[GS_PK_POS] : hb.ent) + hb.pos_ptr[r];
    const bool sampled = k > 0 && d >= static_cast<uint32_t>(k);
    const int cnt = sampled ? k : static_cast<int>(d);
    bool over = false;
    if (!sampled) {
        for (int t = lane; t < cnt; t += 64) out[t] = base + t;
    } else {
        // this node's index among the block's sampled nodes, and their rejections
        const int e = j - hb.blo[b];
        const int qn = r - r0;
        int m = 0, rj = 0;
        for (int q0 = 0; q0 < qn; q0 += 64) {
            const int qq = q0 + lane;
            const bool smp = qq < qn && hb.deg[r0 + qq] >= k;
            const uint64_t bal = __ballot(smp);
            const int mm = m + __popcll(bal & ((1ull << lane) - 1ull));
            int x = smp ? hb.rej[(static_cast<int64_t>(b) * R + mm) * kWMax + e] : 0;
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
            m += __popcll(bal);
            rj += x;
        }
        const int64_t gen = c->gen_end;
        int64_t A = h.P0 + hb.dbase[b] + j + static_cast<int64_t>(m) * k + rj;  // the node's first word
        auto stage = [&](int64_t from) {  // kEmitWords words from `from` into the wave's buffer
            uint32_t t4[kEmitWords / 64];
#pragma unroll
            for (int u = 0; u < kEmitWords / 64; ++u) t4[u] = wr[(from + lane + 64 * u) & kRingMask];
#pragma unroll
            for (int u = 0; u < kEmitWords / 64; ++u) w[lane + 64 * u] = t4[u];
        };
        stage(A);
        int u = 0;  // words of the buffer consumed
        auto refill = [&]() {  // keep 64 words ahead of u in the buffer
            if (u + 64 > kEmitWords) {
                A += u;
                u = 0;
                stage(A);
            }
            if (A + u + 64 > gen) over = true;
        };
        if (d <= static_cast<uint32_t>(setsize)) {
            uint32_t mk = 0, mv = 0;  // lane t < nm: pool slot mk holds mv
            int nm = 0;
            for (int i = 0; i < k && !over;) {
                refill();
                if (over) break;
                const uint32_t mm = d - i;
                const int sh = __clz(mm);
                const uint32_t x = w[u + lane] >> sh;
                const uint64_t acc = __ballot(x < mm);
                if (!acc) {
                    u += 64;
                    continue;
                }
                const int p = __ffsll(static_cast<unsigned long long>(acc)) - 1;
                const uint32_t xs = __shfl(x, p, 64);
                u += p + 1;
                const uint64_t hx = __ballot(lane < nm && mk == xs);
                const uint64_t hl = __ballot(lane < nm && mk == mm - 1);
                const uint32_t val = hx ? __shfl(mv, __ffsll(static_cast<unsigned long long>(hx)) - 1, 64) : xs;
                const uint32_t lastv = hl ? __shfl(mv, __ffsll(static_cast<unsigned long long>(hl)) - 1, 64) : mm - 1;
                if (hx) {
                    if (lane == __ffsll(static_cast<unsigned long long>(hx)) - 1) mv = lastv;
                } else {
                    if (lane == nm) {
                        mk = xs;
                        mv = lastv;
                    }
                    ++nm;
                }
                if (lane == 0) out[i] = base + static_cast<int32_t>(val);
                ++i;
            }
        } else {
            const int sh = __clz(d);
            uint32_t selv = 0xFFFFFFFFu;  // lane t < n_sel: the t-th selected value
            int n_sel = 0;
            while (n_sel < k && !over) {
                refill();
                if (over) break;
                const uint32_t x = w[u + lane] >> sh;
                uint64_t cand = __ballot(x < d);
                int consumed = 64;
                while (cand) {
                    const int p = __ffsll(static_cast<unsigned long long>(cand)) - 1;
                    cand &= cand - 1;
                    const uint32_t xs = __shfl(x, p, 64);
                    if (!__ballot(lane < n_sel && selv == xs)) {
                        if (lane == n_sel) selv = xs;
                        if (lane == 0) out[n_sel] = base + static_cast<int32_t>(xs);
                        ++n_sel;
                        if (n_sel == k) {
                            consumed = p + 1;
                            break;
                        }
                    }
                }
                u += consumed;
            }
        }
    }
    if (lane == 0) {
        // empty neighbourhood after the self rule (non-gcn): no entry, or a
        // lone entry that is the node itself
        if (!gcn && (cnt == 0 || (cnt == 1 && g.col[out[0]] == v))) atomicAdd(&h.n_empty, 1);
        if (last) {
            pack[h.off[GS_PK_DST_IDS] + r] = v;
            pack[h.off[GS_PK_POS_PTR] + r] = hb.pos_ptr[r];
            if (r == h.n_dst - 1) pack[h.off[GS_PK_POS_PTR] + h.n_dst] = hb.pos_ptr[h.n_dst];
        }
        if (over) atomicOr(&c->status, kStWords);
    }
}

// Roots after the pack (the host sampler's layout), totals for the host.
__global__ void finish_kernel(Ctl* c, const int32_t* __restrict__ roots, int n_roots, int32_t* __restrict__ pack,
                              int fail_empty, int n_hops) {
    GS_DS_BAIL(c);
    const int at = c->total;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n_roots; i += gridDim.x * blockDim.x)
        pack[at + i] = roots[i];
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        c->used = at + n_roots;
        if (fail_empty)
            for (int j = 0; j < n_hops; ++j)
                if (c->hop[j].n_empty) c->status |= kStEmpty;
    }
}

__global__ void begin_kernel(Ctl* c, const int32_t* __restrict__ roots, int32_t* __restrict__ dst0, int n_roots) {
    for (int i = threadIdx.x; i < n_roots; i += blockDim.x) dst0[i] = roots[i];
    if (threadIdx.x == 0) {
        c->total = 0;
        c->used = 0;
        c->pos_batch = c->pos_cur;
        // every run starts on a fresh mark epoch: a union reads epoch + 1 and
        // only finish_union advances it, so a run that failed before its
        // finish_union (kStTable / kStSize / kStSpin, then GS_DS_BAIL) left
        // marks at epoch + 1 that would outrank this run's own at that epoch
        c->epoch += 1;
    }
}

// Words [pos, pos + n) of the stream, for the known-answer helper.
__global__ void copy_words_kernel(const uint32_t* __restrict__ wr, int64_t pos, int64_t n, uint32_t* __restrict__ out) {
    for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < n; i += int64_t(gridDim.x) * blockDim.x)
        out[i] = wr[(pos + i) & kRingMask];
}

__global__ void copy_block_kernel(const uint32_t* __restrict__ xr, int64_t first, uint32_t* __restrict__ out) {
    for (int i = threadIdx.x; i < 624; i += blockDim.x) out[i] = xr[(first + i) & kRingMask];
}

}  // namespace ds
}  // namespace gs

// --------------------------------------------------------------- host side

using namespace gs::ds;

namespace {

void hip_ok(hipError_t e, const char* what) {
    if (e != hipSuccess) gs::fail(GS_EHIP, std::string(what) + ": " + hipGetErrorString(e));
}

int r_of(int k) { return k > 0 ? std::max(1, 256 / k) : 256; }

}  // namespace

struct gs_dsampler {
    int32_t n_hops = 0;
    int32_t fanouts[GS_MAX_HOPS] = {};
    int32_t flags = 0;
    int64_t max_roots = 0;
    int64_t nd_max[GS_MAX_HOPS] = {};   // frontier bound per hop
    int64_t npos_max[GS_MAX_HOPS] = {};
    const gs_graph* host_graph = nullptr;
    DevGraph g{};
    std::vector<void*> owned;
    uint32_t* xr = nullptr;   // raw words ring
    uint32_t* wr = nullptr;   // tempered words ring
    uint32_t* tmp = nullptr;  // small transfer buffer (state block, words)
    int64_t tmp_n = 0;
    Ctl* ctl = nullptr;       // device control block
    Ctl* ctl_host = nullptr;  // pinned mirrors, run i's copied into slot i % kResSlots at its end
    hipEvent_t run_done[kResSlots] = {};  // per slot: its run's end
    int64_t n_runs = 0;
    HopBufs hb[GS_MAX_HOPS];
    UnionBufs ub[GS_MAX_HOPS];
    int32_t* pack_cur = nullptr;
    uint64_t* mark = nullptr;  // first-occurrence marks of the frontier unions (shared by the hops)
    int32_t* lid = nullptr;    // union key -> frontier position (shared by the hops)
    hipEvent_t done = nullptr;
    hipStream_t last_stream = nullptr;
    // aux stream: the union's lists and the next run's words beside the
    // draws (GS_DS_AUX=0: everything on the caller's stream)
    hipStream_t aux = nullptr;
    hipEvent_t ev_gen = nullptr, ev_join = nullptr;
    bool ran = false;

    template <typename T>
    T* alloc(int64_t n) {
        void* p = nullptr;
        hip_ok(hipMalloc(&p, std::max<int64_t>(n, 1) * sizeof(T)), "hipMalloc(dsampler)");
        owned.push_back(p);
        return static_cast<T*>(p);
    }
    ~gs_dsampler() {
        if (done) (void)hipEventSynchronize(done);
        if (aux) (void)hipStreamSynchronize(aux);
        for (hipEvent_t e : {ev_gen, ev_join})
            if (e) (void)hipEventDestroy(e);
        if (aux) (void)hipStreamDestroy(aux);
        for (void* p : owned) (void)hipFree(p);
        if (ctl_host) (void)hipHostFree(ctl_host);
        for (hipEvent_t e : run_done)
            if (e) (void)hipEventDestroy(e);
        if (done) (void)hipEventDestroy(done);
    }
};

namespace {

void launch_hop_draws(gs_dsampler* ds, int hop, bool last, int n_roots, hipStream_t st) {
    const int k = ds->fanouts[hop];
    const int setsize = static_cast<int>(gs::sample_setsize(k));
    const int R = r_of(k);
    const int gcn = (ds->flags & GS_SAMPLE_GCN) ? 1 : 0;
    const HopBufs& hb = ds->hb[hop];
    hop_setup_kernel<<<1, 1024, 0, st>>>(ds->g, ds->ctl, hb, hop, k, setsize, R, last ? 1 : 0, n_roots, gcn);
    gs::check_launch("hop_setup_kernel");
    mt_gen_kernel<<<1, kGenThreads, 0, st>>>(ds->xr, ds->wr, ds->ctl, 0, hop);
    gs::check_launch("mt_gen_kernel");
    if (last && ds->aux) {  // the previous hop's lists and the next run's words, beside this hop's draws
        hip_ok(hipEventRecord(ds->ev_gen, st), "hipEventRecord(dsampler fork)");
        hip_ok(hipStreamWaitEvent(ds->aux, ds->ev_gen, 0), "hipStreamWaitEvent(dsampler fork)");
        if (hop > 0)
            gs::ds::launch_hop_lists(ds->ctl, ds->hb[hop - 1], ds->ub[hop - 1], hop - 1, ds->nd_max[hop - 1],
                                     ds->nd_max[hop], ds->flags, ds->pack_cur, ds->aux);
        mt_gen_kernel<<<1, kGenThreads, 0, ds->aux>>>(ds->xr, ds->wr, ds->ctl, kGenAhead, hop, 1);
        gs::check_launch("mt_gen_kernel(ahead)");
    }
    const int nb_max = static_cast<int>((ds->nd_max[hop] + R - 1) / R);
    const size_t mask_lds = static_cast<size_t>(R) * std::max(k, 1) * kMChunks * sizeof(uint64_t) +
                            (kMEntries + 4 * R * std::max(k, 1) + 64) * sizeof(uint32_t);
    // selected-set values in registers: the unrolled duplicate test costs KMAX per accepted word
    const dim3 grid(static_cast<unsigned>(nb_max * (kWMax / kMEntries)));  // the work list's bound
    if (k <= 8)
        draw_masked_kernel<8><<<grid, kMEntries, mask_lds, st>>>(ds->wr, ds->ctl, hb, hop, k, setsize, R);
    else if (k <= 10)  // the bench's and Pubmed's last hop
        draw_masked_kernel<10><<<grid, kMEntries, mask_lds, st>>>(ds->wr, ds->ctl, hb, hop, k, setsize, R);
    else if (k <= 12)
        draw_masked_kernel<12><<<grid, kMEntries, mask_lds, st>>>(ds->wr, ds->ctl, hb, hop, k, setsize, R);
    else if (k <= 16)
        draw_masked_kernel<16><<<grid, kMEntries, mask_lds, st>>>(ds->wr, ds->ctl, hb, hop, k, setsize, R);
    else if (k <= 25)
        draw_masked_kernel<25><<<grid, kMEntries, mask_lds, st>>>(ds->wr, ds->ctl, hb, hop, k, setsize, R);
    else
        draw_masked_kernel<32><<<grid, kMEntries, mask_lds, st>>>(ds->wr, ds->ctl, hb, hop, k, setsize, R);
    gs::check_launch("draw_masked_kernel");
    const int ng_max = (nb_max + kMinG - 1) / kMinG;
    draw_compose_kernel<<<ng_max, 256, kComposeEntries * sizeof(uint16_t), st>>>(ds->ctl, hb, hop);
    gs::check_launch("draw_compose_kernel");
    draw_chain_kernel<<<1, 1024, kChainEntries * sizeof(uint16_t), st>>>(ds->ctl, hb, hop);
    gs::check_launch("draw_chain_kernel");
    draw_emit_kernel<<<static_cast<unsigned>((ds->nd_max[hop] + kEmitWaves - 1) / kEmitWaves), 64 * kEmitWaves, 0, st>>>(
        ds->wr, ds->ctl, hb, ds->g, hop, k, setsize, R, last ? 1 : 0, gcn, ds->pack_cur);
    gs::check_launch("draw_emit_kernel");
}

void ensure_tmp(gs_dsampler* ds, int64_t n) {
    if (ds->tmp_n >= n) return;
    ds->tmp = ds->alloc<uint32_t>(n);
    ds->tmp_n = n;
}

int64_t pos_now(gs_dsampler* ds, hipStream_t st) {
    int64_t p = 0;
    hip_ok(hipMemcpyAsync(&p, &ds->ctl->pos_cur, sizeof(p), hipMemcpyDeviceToHost, st), "hipMemcpyAsync");
    hip_ok(hipStreamSynchronize(st), "hipStreamSynchronize");
    return p;
}

void check_status(int status) {
    if (!status) return;
    if (status & kStEmpty) gs::fail(GS_EEMPTY, "empty neighbourhood");
    // invariant breaks: loud, never retried
    if (status & kStOrder) gs::fail(GS_EINVAL, "device sampler: block states out of order");
    if (status & kStSpin)
        gs::fail(GS_EINVAL, "device sampler: a set-table insert exceeded its probe bound (table invariant broken)");
    // capacities of the device path (the batch is valid; the host sampler takes it)
    if (status & kStWindow)
        gs::fail(GS_ELIMIT, "device sampler: a rejection count fell outside its block window (batch too large "
                            "for the device windows; sample it on the host)");
    if (status & kStWords) gs::fail(GS_ELIMIT, "device sampler: a walk ran past its loaded words");
    if (status & kStTable) gs::fail(GS_ELIMIT, "device sampler: frontier union outgrew the device table");
    if (status & kStSize) gs::fail(GS_ELIMIT, "device sampler: frontier outgrew its bound");
    gs::fail(GS_EINVAL, "device sampler: status " + std::to_string(status));
}

}  // namespace

namespace gs {
bool dsampler_run_ready(gs_dsampler* ds, int64_t run) {
    if (!ds || run < ds->n_runs - kResSlots) return true;
    if (run >= ds->n_runs) return false;
    const hipError_t e = hipEventQuery(ds->run_done[run % kResSlots]);
    if (e == hipErrorNotReady) return false;
    hip_ok(e, "hipEventQuery(dsampler run)");
    return true;
}
bool dsampler_ready(gs_dsampler* ds) {
    if (!ds || !ds->ran) return true;
    const hipError_t e = hipEventQuery(ds->done);
    if (e == hipErrorNotReady) return false;
    hip_ok(e, "hipEventQuery(dsampler)");
    return true;
}
}  // namespace gs

extern "C" {

int gs_dsampler_create(const gs_graph* gp, const int32_t* fanouts, int32_t n_hops, int64_t max_roots, int32_t flags,
                       gs_dsampler** out) {
    GS_API_BEGIN
    GS_REQUIRE(gp && out, GS_EINVAL, "NULL argument");
    GS_REQUIRE(n_hops >= 1 && n_hops <= GS_MAX_HOPS, GS_EINVAL, "n_hops out of [1, 8]");
    GS_REQUIRE(max_roots >= 1 && max_roots < (int64_t(1) << 24), GS_EINVAL, "max_roots out of range");
    const auto& g = *reinterpret_cast<const gs::Graph*>(gp);
    GS_REQUIRE(g.n_entries < (int64_t(1) << 31) && g.n_nodes < (int64_t(1) << 31), GS_ERANGE,
               "graph too large for int32 entries");
    std::unique_ptr<gs_dsampler> ds(new gs_dsampler());
    ds->n_hops = n_hops;
    ds->flags = flags;
    ds->max_roots = max_roots;
    ds->host_graph = gp;
    for (int32_t j = 0; j < n_hops; ++j) {
        ds->fanouts[j] = fanouts ? fanouts[j] : 10;
        GS_REQUIRE(ds->fanouts[j] <= 32, GS_EINVAL, "device sampler: fanouts above 32 are not supported");
    }
    int64_t nd = max_roots;
    for (int32_t j = 0; j < n_hops; ++j) {
        const int64_t k = ds->fanouts[j];
        const int64_t per = k > 0 ? std::min<int64_t>(k, g.max_degree) : g.max_degree;
        ds->nd_max[j] = nd;
        ds->npos_max[j] = nd * per;
        GS_REQUIRE(ds->npos_max[j] < (int64_t(1) << 31), GS_ERANGE, "sampled entries exceed int32");
        nd = std::min<int64_t>(g.n_nodes, nd + nd * per);
    }
    // graph
    auto up = [&](const void* src, size_t bytes) {
        void* p = nullptr;
        hip_ok(hipMalloc(&p, std::max<size_t>(bytes, 1)), "hipMalloc(graph)");
        ds->owned.push_back(p);
        if (bytes) hip_ok(hipMemcpy(p, src, bytes, hipMemcpyHostToDevice), "hipMemcpy(graph)");
        return p;
    };
    ds->g.n_nodes = g.n_nodes;
    ds->g.row_ptr = static_cast<const int64_t*>(up(g.row_ptr.data(), g.row_ptr.size() * sizeof(int64_t)));
    ds->g.col = static_cast<const int32_t*>(up(g.col.data(), g.col.size() * sizeof(int32_t)));
    ds->g.slot = static_cast<const uint32_t*>(up(g.slot.data(), g.slot.size() * sizeof(uint32_t)));
    ds->g.log2size = static_cast<const uint8_t*>(up(g.log2size.data(), g.log2size.size()));
    ds->g.dirty = g.dirty.empty() ? nullptr : static_cast<const uint8_t*>(up(g.dirty.data(), g.dirty.size()));
    ds->xr = ds->alloc<uint32_t>(kRing);
    ds->wr = ds->alloc<uint32_t>(kRing);
    ds->ctl = ds->alloc<Ctl>(1);
    hip_ok(hipMemset(ds->ctl, 0, sizeof(Ctl)), "hipMemset");
    hip_ok(hipHostMalloc(reinterpret_cast<void**>(&ds->ctl_host), kResSlots * sizeof(Ctl), hipHostMallocDefault),
           "hipHostMalloc");
    std::memset(ds->ctl_host, 0, kResSlots * sizeof(Ctl));
    for (hipEvent_t& e : ds->run_done) hip_ok(hipEventCreateWithFlags(&e, hipEventDisableTiming), "hipEventCreate");
    for (int32_t j = 0; j < n_hops; ++j) {
        const int k = ds->fanouts[j];
        const int64_t ndj = ds->nd_max[j];
        const int64_t nb = (ndj + r_of(k) - 1) / r_of(k);
        const int64_t ng = (nb + kMinG - 1) / kMinG;
        HopBufs& h = ds->hb[j];
        h.dst = ds->alloc<int32_t>(ndj);
        h.deg = ds->alloc<int32_t>(ndj);
        h.mv = ds->alloc<float2>(ndj);
        h.pos_ptr = ds->alloc<int32_t>(ndj + 1);
        h.blo = ds->alloc<int32_t>(nb + 1);
        h.bw = ds->alloc<int32_t>(nb + 1);
        h.dbase = ds->alloc<int32_t>(nb + 1);
        h.tab = ds->alloc<uint16_t>(nb * kWMax);
        h.path = ds->alloc<int32_t>(nb * kWMax);
        h.gexit = ds->alloc<uint16_t>(ng * kWMax);
        h.gexit_last = ds->alloc<int32_t>(kWMax);
        h.entry = ds->alloc<int32_t>(nb);
        h.rej = ds->alloc<uint8_t>(nb * r_of(k) * kWMax);
        h.wg = ds->alloc<int32_t>(nb * (kWMax / kMEntries));
        h.ent = j + 1 < n_hops ? ds->alloc<int32_t>(ds->npos_max[j]) : nullptr;
        if (j + 1 < n_hops) {
            GS_REQUIRE(k >= 1, GS_EINVAL, "device sampler: hops before the last need a fanout >= 1");
            UnionBufs& u = ds->ub[j];
            u.set_cnt = ds->alloc<int32_t>(ndj);
            u.set_items = ds->alloc<int32_t>(ds->npos_max[j] + ndj);
            u.first_tab = ds->alloc<int32_t>(kSmallSet);
            u.first_meta = ds->alloc<int32_t>(2);
            u.tpre = ds->alloc<int32_t>(ndj + 1);
            u.ubef = ds->alloc<int32_t>(ndj + 1);
            u.fresh = ds->alloc<int32_t>(ds->npos_max[j] + ndj);
            u.tcnt = ds->alloc<int32_t>(ds->nd_max[j + 1] + 1);
            u.longs = ds->alloc<int32_t>(ds->nd_max[j + 1] + 1);
            u.fmask = ds->alloc<uint64_t>(ndj);
            u.sched = ds->alloc<int32_t>(2 * (kMaxStages + 1));
            u.skeys = ds->alloc<int32_t>(2 * static_cast<int64_t>(kBigKeys));
            if (!ds->mark) {
                ds->mark = ds->alloc<uint64_t>(g.n_nodes);
                hip_ok(hipMemset(ds->mark, 0, g.n_nodes * sizeof(uint64_t)), "hipMemset(mark)");
                ds->lid = ds->alloc<int32_t>(g.n_nodes);
            }
            u.mark = ds->mark;
            u.lid = ds->lid;
        }
    }
    hip_ok(hipEventCreateWithFlags(&ds->done, hipEventDisableTiming), "hipEventCreate");
    const char* aux_env = std::getenv("GS_DS_AUX");
    if (!(flags & GS_DSAMPLER_NO_AUX) && !(aux_env && std::string(aux_env) == "0")) {
        hip_ok(hipStreamCreateWithFlags(&ds->aux, hipStreamNonBlocking), "hipStreamCreate(dsampler aux)");
        for (hipEvent_t* e : {&ds->ev_gen, &ds->ev_join})
            hip_ok(hipEventCreateWithFlags(e, hipEventDisableTiming), "hipEventCreate");
    }
    // the stream starts as random.seed(0) would leave it; callers set it
    gs::MT19937 mt;
    const uint32_t zero = 0;
    mt.init_by_array(&zero, 1);
    *out = ds.release();
    GS_REQUIRE(gs_dsampler_set_rng(*out, mt.mt, mt.index, nullptr) == GS_OK, GS_EHIP, gs_last_error());
    GS_API_END
}

void gs_dsampler_destroy(gs_dsampler* ds) { delete ds; }

int gs_dsampler_set_rng(gs_dsampler* ds, const uint32_t* mt624, int64_t pos, void* stream) {
    GS_API_BEGIN
    GS_REQUIRE(ds && mt624, GS_EINVAL, "NULL argument");
    GS_REQUIRE(pos >= 0 && pos <= 624, GS_EINVAL, "state index out of range");
    hipStream_t st = gs::as_stream(stream);
    if (ds->ran) hip_ok(hipEventSynchronize(ds->done), "hipEventSynchronize");
    ensure_tmp(ds, 624);
    hip_ok(hipMemcpyAsync(ds->tmp, mt624, 624 * sizeof(uint32_t), hipMemcpyHostToDevice, st), "hipMemcpyAsync");
    mt_seed_kernel<<<1, 256, 0, st>>>(ds->tmp, pos, ds->xr, ds->wr, ds->ctl);
    gs::check_launch("mt_seed_kernel");
    hip_ok(hipStreamSynchronize(st), "hipStreamSynchronize");
    GS_API_END
}

int gs_dsampler_get_rng(gs_dsampler* ds, uint32_t* mt624, int64_t* pos, void* stream) {
    GS_API_BEGIN
    GS_REQUIRE(ds && mt624 && pos, GS_EINVAL, "NULL argument");
    hipStream_t st = gs::as_stream(stream);
    if (ds->ran) hip_ok(hipEventSynchronize(ds->done), "hipEventSynchronize");
    const int64_t p = pos_now(ds, st);
    int64_t blk = p / 624, idx = p % 624;
    if (p > 0 && idx == 0) {
        blk -= 1;
        idx = 624;
    }
    mt_gen_kernel<<<1, kGenThreads, 0, st>>>(ds->xr, ds->wr, ds->ctl, 624 * (blk + 1), -1);
    gs::check_launch("mt_gen_kernel");
    ensure_tmp(ds, 624);
    copy_block_kernel<<<1, 256, 0, st>>>(ds->xr, 624 * blk, ds->tmp);
    gs::check_launch("copy_block_kernel");
    hip_ok(hipMemcpyAsync(mt624, ds->tmp, 624 * sizeof(uint32_t), hipMemcpyDeviceToHost, st), "hipMemcpyAsync");
    hip_ok(hipStreamSynchronize(st), "hipStreamSynchronize");
    *pos = idx;
    GS_API_END
}

int gs_dsampler_words(gs_dsampler* ds, int64_t n, uint32_t* out, void* stream) {
    GS_API_BEGIN
    GS_REQUIRE(ds && out && n >= 0 && n < kRing / 2, GS_EINVAL, "bad arguments");
    hipStream_t st = gs::as_stream(stream);
    if (ds->ran) hip_ok(hipEventSynchronize(ds->done), "hipEventSynchronize");
    const int64_t p = pos_now(ds, st);
    mt_gen_kernel<<<1, kGenThreads, 0, st>>>(ds->xr, ds->wr, ds->ctl, p + n, -1);
    gs::check_launch("mt_gen_kernel");
    ensure_tmp(ds, n);
    copy_words_kernel<<<64, 256, 0, st>>>(ds->wr, p, n, ds->tmp);
    gs::check_launch("copy_words_kernel");
    if (n) hip_ok(hipMemcpyAsync(out, ds->tmp, n * sizeof(uint32_t), hipMemcpyDeviceToHost, st), "hipMemcpyAsync");
    hip_ok(hipStreamSynchronize(st), "hipStreamSynchronize");
    GS_API_END
}

int64_t gs_dsampler_pack_bound(const gs_dsampler* ds, int64_t n_roots) {
    if (!ds || n_roots < 1 || n_roots > ds->max_roots) return -1;
    return gs_sample_pack_bound(ds->host_graph, n_roots, ds->fanouts, ds->n_hops) + n_roots;
}

int gs_dsampler_run(gs_dsampler* ds, const int32_t* roots, int64_t n_roots, int32_t* pack, int64_t cap, void* stream) {
    GS_API_BEGIN
    GS_REQUIRE(ds && roots && pack, GS_EINVAL, "NULL argument");
    GS_REQUIRE(n_roots >= 1 && n_roots <= ds->max_roots, GS_EINVAL, "n_roots out of [1, max_roots]");
    GS_REQUIRE(cap >= gs_dsampler_pack_bound(ds, n_roots), GS_EINVAL, "pack buffer below gs_dsampler_pack_bound");
    hipStream_t st = gs::as_stream(stream);
    ds->pack_cur = pack;
    begin_kernel<<<1, 256, 0, st>>>(ds->ctl, roots, ds->hb[0].dst, static_cast<int>(n_roots));
    gs::check_launch("begin_kernel");
    for (int32_t j = 0; j < ds->n_hops; ++j) {
        const bool last = j == ds->n_hops - 1;
        launch_hop_draws(ds, j, last, static_cast<int>(n_roots), st);
        if (!last) gs::ds::launch_hop_union(ds->g, ds->ctl, ds->hb[j], ds->ub[j], ds->hb[j + 1], j, ds->fanouts[j],
                                            ds->nd_max[j], ds->nd_max[j + 1], ds->flags, pack, st,
                                            !(ds->aux && j + 2 == ds->n_hops));
    }
    if (ds->aux) {  // join: the lists are in the pack, the words ahead are in the ring
        hip_ok(hipEventRecord(ds->ev_join, ds->aux), "hipEventRecord(dsampler join)");
        hip_ok(hipStreamWaitEvent(st, ds->ev_join, 0), "hipStreamWaitEvent(dsampler join)");
    }
    finish_kernel<<<8, 256, 0, st>>>(ds->ctl, roots, static_cast<int>(n_roots), pack,
                                     (ds->flags & GS_SAMPLE_FAIL_EMPTY) ? 1 : 0, ds->n_hops);
    gs::check_launch("finish_kernel");
    const int slot = static_cast<int>(ds->n_runs % kResSlots);
    hip_ok(hipMemcpyAsync(ds->ctl_host + slot, ds->ctl, sizeof(Ctl), hipMemcpyDeviceToHost, st), "hipMemcpyAsync(ctl)");
    hip_ok(hipEventRecord(ds->run_done[slot], st), "hipEventRecord");
    hip_ok(hipEventRecord(ds->done, st), "hipEventRecord");
    ds->ran = true;
    ++ds->n_runs;
    GS_API_END
}

int gs_dsampler_debug(gs_dsampler* ds, int64_t* out, int32_t n) {
    GS_API_BEGIN
    GS_REQUIRE(ds && ds->ran && out && n >= 0 && n <= 64, GS_EINVAL, "bad arguments");
    hip_ok(hipEventSynchronize(ds->done), "hipEventSynchronize");
    std::memcpy(out, ds->ctl_host[(ds->n_runs - 1) % kResSlots].dbg, n * sizeof(int64_t));
    GS_API_END
}

namespace {
// The layout of the run whose Ctl mirror is `c`, as the host sampler reports it.
void report(const gs_dsampler* ds, const Ctl& c, int64_t* hop_sizes, int64_t* offsets, int64_t* used) {
    check_status(c.status);
    for (int32_t j = 0; j < GS_MAX_HOPS; ++j) {
        const bool on = j < ds->n_hops;
        const bool last = j == ds->n_hops - 1;
        if (hop_sizes) {
            hop_sizes[4 * j] = on ? c.hop[j].n_dst : 0;
            hop_sizes[4 * j + 1] = on ? c.hop[j].n_pos : 0;
            // as the host sampler: -1 = not materialised (the last hop), 0 past the hops
            hop_sizes[4 * j + 2] = on ? (last ? -1 : c.hop[j].n_src) : 0;
            hop_sizes[4 * j + 3] = on ? (last ? -1 : c.hop[j].n_nbr) : 0;
        }
        if (offsets)
            for (int f = 0; f < GS_PK_NFIELDS; ++f) {
                const bool lastf = f == GS_PK_POS_PTR || f == GS_PK_POS || f == GS_PK_DST_IDS;
                offsets[j * GS_PK_NFIELDS + f] = on && (last == lastf) ? c.hop[j].off[f] : -1;
            }
    }
    if (used) *used = c.used;
}
}  // namespace

int gs_dsampler_result(gs_dsampler* ds, int64_t* hop_sizes, int64_t* offsets, int64_t* used) {
    GS_API_BEGIN
    GS_REQUIRE(ds && ds->ran, GS_EINVAL, "no run to report");
    hip_ok(hipEventSynchronize(ds->done), "hipEventSynchronize");
    report(ds, ds->ctl_host[(ds->n_runs - 1) % kResSlots], hop_sizes, offsets, used);
    GS_API_END
}

int64_t gs_dsampler_runs(const gs_dsampler* ds) { return ds ? ds->n_runs : -1; }

int gs_dsampler_result_of(gs_dsampler* ds, int64_t run, int64_t* hop_sizes, int64_t* offsets, int64_t* used) {
    GS_API_BEGIN
    GS_REQUIRE(ds, GS_EINVAL, "NULL argument");
    GS_REQUIRE(run >= 0 && run < ds->n_runs && run >= ds->n_runs - kResSlots, GS_ERANGE,
               "device sampler: run not issued or no longer kept (the last " + std::to_string(kResSlots) +
                   " runs are)");
    const int slot = static_cast<int>(run % kResSlots);
    hip_ok(hipEventSynchronize(ds->run_done[slot]), "hipEventSynchronize");
    report(ds, ds->ctl_host[slot], hop_sizes, offsets, used);
    GS_API_END
}

}  // extern "C"
