#pragma once
// Segmented gather-aggregate for GraphSage.aggregate (models.py:291-330) and
// its backward.  The reference builds a dense [n_dst, n_src] 0/1 mask and
// multiplies (MEAN, :305-314) or loops rows in Python (MAX, :316-326); here
// each destination is owned by a group of G lanes of one wavefront that
// streams its neighbours' feature rows straight from HBM (16 B per lane, so a
// 1 KiB fp32 F=256 row is one coalesced wave load) and reduces in registers.
// Nothing of size n_dst x n_src is ever formed.

#include "kcommon.hpp"

namespace gs {

constexpr int kBlock = 256;
#ifndef GS_AGG_BWD_BATCH
#define GS_AGG_BWD_BATCH 1
#endif
constexpr int kRows = 16;  // neighbour rows in flight per lane group

// Lanes [lo, lo + G) of the wave's ballot.
template <int G>
__device__ __forceinline__ uint64_t group_bits(bool p) {
    const uint64_t m = __ballot(p);
    if constexpr (G == 64) return m;
    const int lo = (threadIdx.x & 63) & ~(G - 1);
    return (m >> lo) & ((uint64_t(1) << G) - 1);
}

// One group of G lanes per destination r.  EXPAND: the neighbourhood is the
// sampled positions idx[ptr[r]..ptr[r+1]) of node dst_ids[r]'s CSR row,
// expanded on the fly (col[row_ptr[node] + pos], or col[idx] when row_ptr is
// NULL and idx already holds absolute entries, as in the packed sample);
// self is skipped unless gcn,
// and gcn adds it once (models.py:285, :297-298).  Otherwise idx holds the
// source rows of X directly (already self-filtered and ascending).
//
// Every load is unconditional: slots past the neighbourhood re-read the
// chunk's first row (already in flight) and are masked when accumulated, so a
// group keeps all kRows rows of a chunk in flight instead of waiting on each.
template <int OP, typename T, int VEC, int G, bool EXPAND>
__global__ __launch_bounds__(kBlock) void agg_fwd_kernel(
    const T* __restrict__ X, int64_t ldx, int F, int n_dst, const int* __restrict__ ptr,
    const int* __restrict__ idx, const int64_t* __restrict__ row_ptr, const int* __restrict__ col,
    const int* __restrict__ dst_ids, int gcn, T* __restrict__ out, int64_t ldo,
    int* __restrict__ argmax) {
    const int gl = threadIdx.x % G;
    const int r = blockIdx.x * (kBlock / G) + threadIdx.x / G;
    if (r >= n_dst) return;  // whole lane groups leave together
    const int beg = ptr[r], end = ptr[r + 1];
    int node = 0;
    int64_t rs = 0;
    if (EXPAND) {
        node = dst_ids[r];
        if (row_ptr) rs = row_ptr[node];
    }
    // explicit lists (layers >= 2: fanout up to 25-30 per destination) keep
    // twice the rows in flight, so a whole neighbourhood is one memory round
    constexpr int NR = kRows * (EXPAND ? 1 : 2);
    const bool want_am = (OP == GS_AGG_MAX) && (argmax != nullptr);
    const int nf = (F + G * VEC - 1) / (G * VEC);
    for (int fi = 0; fi < nf; ++fi) {
        const int f0 = fi * G * VEC + gl * VEC;
        const bool act = f0 < F;
        const int f0c = act ? f0 : 0;
        float acc[VEC];
        int am[VEC];
#pragma unroll
        for (int v = 0; v < VEC; ++v) {
            acc[v] = (OP == GS_AGG_MAX) ? -INFINITY : 0.f;
            am[v] = -1;
        }
        int cnt = 0;
        bool self_seen = false;
        for (int base = beg; base < end; base += G) {
            const int m = min(G, end - base);
            const bool mine = gl < m;
            const int e = idx[mine ? base + gl : base];
            int my;
            if (EXPAND) {
                const int nb = col[rs + e];
                self_seen |= group_bits<G>(mine && nb == node) != 0;
                my = (mine && (gcn || nb != node)) ? nb : -1;
            } else {
                my = mine ? e : -1;
            }
            for (int j = 0; j < m; j += NR) {
                int rows[NR];
                bool ok[NR];
#pragma unroll
                for (int u = 0; u < NR; ++u) {
                    rows[u] = __shfl(my, j + u < m ? j + u : j, G);
                    ok[u] = (j + u < m) && rows[u] >= 0;
                }
                const int fallback = rows[0] >= 0 ? rows[0] : (EXPAND ? node : 0);
                float x[NR][VEC];
#pragma unroll
                for (int u = 0; u < NR; ++u)
                    RowIO<T, VEC>::load(X + static_cast<int64_t>(ok[u] ? rows[u] : fallback) * ldx + f0c, x[u]);
#pragma unroll
                for (int u = 0; u < NR; ++u) {
                    cnt += ok[u];
#pragma unroll
                    for (int v = 0; v < VEC; ++v) {
                        if (OP == GS_AGG_MEAN) {
                            acc[v] += ok[u] ? x[u][v] : 0.f;
                        } else {
                            const bool take = ok[u] && x[u][v] > acc[v];  // strict: first index wins ties
                            acc[v] = take ? x[u][v] : acc[v];
                            am[v] = take ? rows[u] : am[v];
                        }
                    }
                }
            }
        }
        if (EXPAND && gcn && !self_seen) {  // gcn keeps self exactly once (set semantics)
            ++cnt;
            float x[VEC];
            RowIO<T, VEC>::load(X + static_cast<int64_t>(node) * ldx + f0c, x);
#pragma unroll
            for (int v = 0; v < VEC; ++v) {
                if (OP == GS_AGG_MEAN) acc[v] += x[v];
                else if (x[v] > acc[v]) { acc[v] = x[v]; am[v] = node; }
            }
        }
        if (!act) continue;
        if (OP == GS_AGG_MEAN) {
            const float inv = 1.0f / static_cast<float>(cnt);  // cnt == 0 -> NaN row, as 0/0 in :313
#pragma unroll
            for (int v = 0; v < VEC; ++v) acc[v] *= inv;
        }
        RowIO<T, VEC>::store(out + static_cast<int64_t>(r) * ldo + f0, acc);
        if (want_am) {
#pragma unroll
            for (int v = 0; v < VEC; ++v) argmax[static_cast<int64_t>(r) * F + f0 + v] = am[v];
        }
    }
}

// Backward over source rows c (transposed neighbourhood lists, GS_PK_TIDX
// encoding): self-row gradient + mean/max routing, then the relu mask of the
// layer that produced these rows.  Fixed order, no atomics.
template <int OP, int VEC, int G, bool PAIR = false>
__device__ __forceinline__ void agg_bwd_body(
    int bx, int n_src, int F, const int* __restrict__ tptr, const int* __restrict__ tidx,
    const int* __restrict__ ptr, const float* __restrict__ dA, const float* __restrict__ dSelf,
    int64_t ldd, const int* __restrict__ argmax, const float* __restrict__ Hprev, int64_t ldh,
    float* __restrict__ dH, int64_t off2 = 0) {
    // PAIR: the input gradient arrives as two partial sums (the top launch's
    // pair form), the second off2 floats past the first; each row is their
    // sum, first + second (a separate instance: no second loads otherwise)
    constexpr bool pair = PAIR;
    const int gl = threadIdx.x % G;
    const int c = bx * (kBlock / G) + threadIdx.x / G;
    if (c >= n_src) return;
    const int beg = tptr[c], end = tptr[c + 1];
    for (int f0 = gl * VEC; f0 < ((F + G * VEC - 1) / (G * VEC)) * G * VEC; f0 += G * VEC) {
        const bool act = f0 < F;
        float g[VEC];
#pragma unroll
        for (int v = 0; v < VEC; ++v) g[v] = 0.f;
#if GS_AGG_BWD_BATCH
        // Entries in groups of 8: the group's transposed indices in one load
        // round, then every row (and MEAN count / MAX argmax) of the group in
        // one more, then the adds in entry order (the same sums as one entry
        // at a time).  Addresses are clamped, values selected at use.
        const int f0c = act ? f0 : 0;
        for (int t0 = beg; t0 < end; t0 += 8) {
            int e[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) e[u] = tidx[min(t0 + u, end - 1)];
            float x[8][VEC], y[8][VEC], w[8];
            int am[8][VEC];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int eu = e[u];
                const bool self_e = eu < 0;
                const int row = self_e ? -eu - 1 : eu;
                const float* src = (self_e && dSelf) ? dSelf : dA;
                RowIO<float, VEC>::load(src + static_cast<int64_t>(row) * ldd + f0c, x[u]);
                if constexpr (PAIR) RowIO<float, VEC>::load(src + static_cast<int64_t>(row) * ldd + f0c + off2, y[u]);
                if (OP == GS_AGG_MEAN) {
                    const int re = self_e ? 0 : eu;
                    w[u] = 1.0f / static_cast<float>(ptr[re + 1] - ptr[re]);
                } else {
#pragma unroll
                    for (int v = 0; v < VEC; ++v)
                        am[u][v] = argmax[static_cast<int64_t>(self_e ? 0 : eu) * F + f0c + v];
                }
            }
            if (!act) continue;
#pragma unroll
            for (int u = 0; u < 8; ++u)
#pragma unroll
                for (int v = 0; v < VEC; ++v) x[u][v] = pair ? x[u][v] + y[u][v] : x[u][v];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                if (t0 + u >= end) break;
                if (e[u] < 0) {
                    if (!dSelf) continue;  // gcn: self rows feed no linear input
#pragma unroll
                    for (int v = 0; v < VEC; ++v) g[v] += x[u][v];
                } else if (OP == GS_AGG_MEAN) {
#pragma unroll
                    for (int v = 0; v < VEC; ++v) g[v] += x[u][v] * w[u];
                } else {
#pragma unroll
                    for (int v = 0; v < VEC; ++v)
                        if (am[u][v] == c) g[v] += x[u][v];
                }
            }
        }
#else
        for (int t = beg; t < end; ++t) {
            const int e = tidx[t];
            if (!act) continue;
            float x[VEC];
            float x2[VEC];
            if (e < 0) {
                if (!dSelf) continue;  // gcn: self rows feed no linear input
                RowIO<float, VEC>::load(dSelf + static_cast<int64_t>(-e - 1) * ldd + f0, x);
                if constexpr (PAIR) RowIO<float, VEC>::load(dSelf + static_cast<int64_t>(-e - 1) * ldd + f0 + off2, x2);
#pragma unroll
                for (int v = 0; v < VEC; ++v) g[v] += pair ? x[v] + x2[v] : x[v];
            } else if (OP == GS_AGG_MEAN) {
                const float w = 1.0f / static_cast<float>(ptr[e + 1] - ptr[e]);
                RowIO<float, VEC>::load(dA + static_cast<int64_t>(e) * ldd + f0, x);
                if constexpr (PAIR) RowIO<float, VEC>::load(dA + static_cast<int64_t>(e) * ldd + f0 + off2, x2);
#pragma unroll
                for (int v = 0; v < VEC; ++v) g[v] += (pair ? x[v] + x2[v] : x[v]) * w;
            } else {
                RowIO<float, VEC>::load(dA + static_cast<int64_t>(e) * ldd + f0, x);
                if constexpr (PAIR) RowIO<float, VEC>::load(dA + static_cast<int64_t>(e) * ldd + f0 + off2, x2);
#pragma unroll
                for (int v = 0; v < VEC; ++v)
                    if (argmax[static_cast<int64_t>(e) * F + f0 + v] == c) g[v] += pair ? x[v] + x2[v] : x[v];
            }
        }
#endif
        if (!act) continue;
        if (Hprev) {
            float h[VEC];
            RowIO<float, VEC>::load(Hprev + static_cast<int64_t>(c) * ldh + f0, h);
#pragma unroll
            for (int v = 0; v < VEC; ++v) g[v] = h[v] > 0.f ? g[v] : 0.f;
        }
        RowIO<float, VEC>::store(dH + static_cast<int64_t>(c) * ldh + f0, g);
    }
}

// The same backward from per-row records written a step ahead by the side
// stream (resolve_top_kernel's third role): int4 pair {n, beg, e0 .. e5} per
// source row c = its transposed-list length, offset and first six entries.
// The record and the row's relu-mask quad load in one round, the entries'
// rows (+ MEAN counts / MAX argmax) in the next; entries past the sixth
// (hub rows) follow one at a time from tidx.  Entries are added in list order
// with agg_bwd_body's expressions: bitwise its result.
constexpr int kTrec = 6;  // entries inline in a record
template <int OP, int VEC, int G, bool PAIR = false>
__device__ __forceinline__ void agg_bwd_rec_body(
    int bx, int n_src, int F, const int4* __restrict__ rec, const int* __restrict__ tidx,
    const int* __restrict__ ptr, const float* __restrict__ dA, const float* __restrict__ dSelf,
    int64_t ldd, const int* __restrict__ argmax, const float* __restrict__ Hprev, int64_t ldh,
    float* __restrict__ dH, int64_t off2 = 0) {
    constexpr bool pair = PAIR;  // two partial input gradients (agg_bwd_body)
    const int gl = threadIdx.x % G;
    const int c = bx * (kBlock / G) + threadIdx.x / G;
    if (c >= n_src) return;
    const int4 ra = rec[2 * static_cast<int64_t>(c)], rb = rec[2 * static_cast<int64_t>(c) + 1];
    const int n = ra.x, beg = ra.y;
    const int e[kTrec] = {ra.z, ra.w, rb.x, rb.y, rb.z, rb.w};
    for (int f0 = gl * VEC; f0 < ((F + G * VEC - 1) / (G * VEC)) * G * VEC; f0 += G * VEC) {
        const bool act = f0 < F;
        const int f0c = act ? f0 : 0;
        float h[VEC];
        if (Hprev) RowIO<float, VEC>::load(Hprev + static_cast<int64_t>(c) * ldh + f0c, h);
        float g[VEC];
#pragma unroll
        for (int v = 0; v < VEC; ++v) g[v] = 0.f;
        float x[kTrec][VEC], y[kTrec][VEC], w[kTrec];
        int am[kTrec][VEC], pa[kTrec], pb[kTrec];
#pragma unroll
        for (int u = 0; u < kTrec; ++u) {
            const int eu = e[u];
            const bool self_e = eu < 0;
            const int row = self_e ? -eu - 1 : eu;
            const float* src = (self_e && dSelf) ? dSelf : dA;
            RowIO<float, VEC>::load(src + static_cast<int64_t>(row) * ldd + f0c, x[u]);
            if constexpr (PAIR) RowIO<float, VEC>::load(src + static_cast<int64_t>(row) * ldd + f0c + off2, y[u]);
            if (OP == GS_AGG_MEAN) {
                const int re = self_e ? 0 : eu;
                pa[u] = ptr[re];
                pb[u] = ptr[re + 1];
            } else {
#pragma unroll
                for (int v = 0; v < VEC; ++v) am[u][v] = argmax[static_cast<int64_t>(self_e ? 0 : eu) * F + f0c + v];
            }
        }
        // every load of the round issued before the first use waits on one
        // (the counts' divisions had the compiler wait inside the load loop)
        __builtin_amdgcn_sched_barrier(0);
        if (OP == GS_AGG_MEAN) {
#pragma unroll
            for (int u = 0; u < kTrec; ++u) w[u] = 1.0f / static_cast<float>(pb[u] - pa[u]);
        }
        if (!act) continue;
#pragma unroll
        for (int u = 0; u < kTrec; ++u)
#pragma unroll
            for (int v = 0; v < VEC; ++v) x[u][v] = pair ? x[u][v] + y[u][v] : x[u][v];
#pragma unroll
        for (int u = 0; u < kTrec; ++u) {
            if (u >= n) break;
            if (e[u] < 0) {
                if (!dSelf) continue;  // gcn: self rows feed no linear input
#pragma unroll
                for (int v = 0; v < VEC; ++v) g[v] += x[u][v];
            } else if (OP == GS_AGG_MEAN) {
#pragma unroll
                for (int v = 0; v < VEC; ++v) g[v] += x[u][v] * w[u];
            } else {
#pragma unroll
                for (int v = 0; v < VEC; ++v)
                    if (am[u][v] == c) g[v] += x[u][v];
            }
        }
        for (int t = beg + kTrec; t < beg + n; ++t) {  // hub rows: the rest of the list
            const int et = tidx[t];
            float xt[VEC], yt[VEC];
            if (et < 0) {
                if (!dSelf) continue;
                RowIO<float, VEC>::load(dSelf + static_cast<int64_t>(-et - 1) * ldd + f0, xt);
                if constexpr (PAIR) RowIO<float, VEC>::load(dSelf + static_cast<int64_t>(-et - 1) * ldd + f0 + off2, yt);
#pragma unroll
                for (int v = 0; v < VEC; ++v) g[v] += pair ? xt[v] + yt[v] : xt[v];
            } else if (OP == GS_AGG_MEAN) {
                const float wt = 1.0f / static_cast<float>(ptr[et + 1] - ptr[et]);
                RowIO<float, VEC>::load(dA + static_cast<int64_t>(et) * ldd + f0, xt);
                if constexpr (PAIR) RowIO<float, VEC>::load(dA + static_cast<int64_t>(et) * ldd + f0 + off2, yt);
#pragma unroll
                for (int v = 0; v < VEC; ++v) g[v] += (pair ? xt[v] + yt[v] : xt[v]) * wt;
            } else {
                RowIO<float, VEC>::load(dA + static_cast<int64_t>(et) * ldd + f0, xt);
                if constexpr (PAIR) RowIO<float, VEC>::load(dA + static_cast<int64_t>(et) * ldd + f0 + off2, yt);
#pragma unroll
                for (int v = 0; v < VEC; ++v)
                    if (argmax[static_cast<int64_t>(et) * F + f0 + v] == c) g[v] += pair ? xt[v] + yt[v] : xt[v];
            }
        }
        if (Hprev) {
#pragma unroll
            for (int v = 0; v < VEC; ++v) g[v] = h[v] > 0.f ? g[v] : 0.f;
        }
        RowIO<float, VEC>::store(dH + static_cast<int64_t>(c) * ldh + f0, g);
    }
}

template <int OP, int VEC, int G>
__global__ __launch_bounds__(kBlock) void agg_bwd_kernel(
    int n_src, int F, const int* __restrict__ tptr, const int* __restrict__ tidx,
    const int* __restrict__ ptr, const float* __restrict__ dA, const float* __restrict__ dSelf,
    int64_t ldd, const int* __restrict__ argmax, const float* __restrict__ Hprev, int64_t ldh,
    float* __restrict__ dH) {
    agg_bwd_body<OP, VEC, G>(blockIdx.x, n_src, F, tptr, tidx, ptr, dA, dSelf, ldd, argmax, Hprev, ldh, dH);
}

inline int pick_group(int F, int vec) {
    const int lanes = (F + vec - 1) / vec;
    int g = 16;
    while (g < lanes && g < 64) g <<= 1;
    return g;
}

}  // namespace gs
