// C-ABI launchers of the gather-aggregate kernels (kernels/agg_dev.hpp), and
// the runner's two-step layer-1 gather: resolve the sampled positions into
// padded neighbour ids, then gather rows through them.
#include "agg_dev.hpp"
#include "internal.hpp"

#include <algorithm>
#include <cstdlib>

namespace gs {

// ids[r·k + j] = node of destination r's j-th sampled position
// (col[ent[ptr[r] + j]]), or -1 past its count and, unless gcn, for r's own
// node (models.py:297-298: the aggregate skips self).  One thread per slot;
// this is the gather's dependent index chain, run ahead of it.
__global__ __launch_bounds__(kBlock) void resolve_ids_kernel(int n_dst, int k, const int* __restrict__ ptr,
                                                             const int* __restrict__ ent,
                                                             const int* __restrict__ col,
                                                             const int* __restrict__ dst_ids, int gcn,
                                                             int* __restrict__ ids) {
    const int64_t t = blockIdx.x * int64_t(kBlock) + threadIdx.x;
    if (t >= static_cast<int64_t>(n_dst) * k) return;
    const int r = static_cast<int>(t / k), j = static_cast<int>(t - static_cast<int64_t>(r) * k);
    const int e = ptr[r] + j;
    int nb = -1;
    if (e < ptr[r + 1]) nb = col[ent[e]];
    if (!gcn && nb == dst_ids[r]) nb = -1;
    ids[t] = nb;
}

// The same resolve, plus a second role for the fused top launch (top.hip):
// the roots' hop-1 lists padded to `tk` slots behind their self row, one
// record of 1 + tk ids per root (-1 past the list), so the top launch loads a
// root's whole neighbourhood in one round instead of three (ptr, list, rows);
// and a third for the layer-2 backward's gather (agg_bwd_rec_body): per
// layer-1 row c, {n, beg, e0 .. e5} of its transposed hop-1 list (n_rec rows,
// from the pack's GS_PK_TPTR / TIDX of hop 1; entries past n are 0).
__global__ __launch_bounds__(kBlock) void resolve_top_kernel(int n_dst, int k, const int* __restrict__ ptr,
                                                             const int* __restrict__ ent,
                                                             const int* __restrict__ col,
                                                             const int* __restrict__ dst_ids, int gcn,
                                                             int* __restrict__ ids, int n_top, int tk,
                                                             const int* __restrict__ tptr,
                                                             const int* __restrict__ tnbr,
                                                             const int* __restrict__ tself, int* __restrict__ tout,
                                                             int n_rec, const int* __restrict__ rptr,
                                                             const int* __restrict__ ridx, int* __restrict__ rout) {
    const int64_t t = blockIdx.x * int64_t(kBlock) + threadIdx.x;
    const int64_t n1 = static_cast<int64_t>(n_dst) * k;
    if (t < n1) {
        const int r = static_cast<int>(t / k), j = static_cast<int>(t - static_cast<int64_t>(r) * k);
        const int e = ptr[r] + j;
        int nb = -1;
        if (e < ptr[r + 1]) nb = col[ent[e]];
        if (!gcn && nb == dst_ids[r]) nb = -1;
        ids[t] = nb;
        return;
    }
    const int64_t u = t - n1;
    const int64_t n2 = static_cast<int64_t>(n_top) * (tk + 1);
    if (u >= n2) {  // third role: the backward's records, 8 ints per row
        const int64_t q = u - n2;
        if (q >= static_cast<int64_t>(n_rec) * 8) return;
        const int c = static_cast<int>(q >> 3), j = static_cast<int>(q & 7);
        const int b = rptr[c], n = rptr[c + 1] - b;
        rout[q] = j == 0 ? n : j == 1 ? b : (j - 2 < n ? ridx[b + j - 2] : 0);
        return;
    }
    const int r = static_cast<int>(u / (tk + 1)), j = static_cast<int>(u - static_cast<int64_t>(r) * (tk + 1));
    int v;
    if (j == 0) {
        v = tself[r];
    } else {
        const int e = tptr[r] + j - 1;
        v = e < tptr[r + 1] ? tnbr[e] : -1;
    }
    tout[u] = v;
}

// A row chunk as loaded (one 16-byte vector per lane, or a scalar), unpacked
// to floats only when accumulated.
template <typename T, int VEC>
struct RawVec {
    using type = T;
    static __device__ __forceinline__ void unpack(const T& r, float (&v)[VEC]) {
        RowIO<T, VEC>::load(&r, v);
    }
};
template <>
struct RawVec<float, 4> {
    using type = float4;
    static __device__ __forceinline__ void unpack(const float4& r, float (&v)[4]) {
        v[0] = r.x; v[1] = r.y; v[2] = r.z; v[3] = r.w;
    }
};
template <>
struct RawVec<bf16_t, 8> {
    using type = uint4;
    static __device__ __forceinline__ void unpack(const uint4& r, float (&v)[8]) {
        const uint32_t w[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            v[2 * i] = __uint_as_float(w[i] << 16);
            v[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
        }
    }
};

// The layer-1 gather over resolved ids (k slots per destination, -1 = skip).
// Same lane groups, chunking and accumulation order as agg_fwd_kernel's
// expand mode (empty slots add +0 / never win a max), so the output is
// bitwise that kernel's; the only index load is the destination's k ids.
// SELF: also copy each destination's own feature row X[dst_ids[r]] to
// self_out[r] (its load in the same memory round as the neighbours'), so the
// layer-1 GEMMs read [self | agg] as one dense block instead of gathering the
// self rows through their index (GS_SELF_ROWS).
// ONE (the launcher's choice when F == G·VEC, k <= kRows, no gcn and a grid
// with a lane group per destination): each destination in two load rounds —
// its k ids and its own id together, then the self row and every neighbour
// row together — written straight-line, with no loop around the loads (the
// general form's loops had the compiler drain the self row's load before the
// id load and split the rows into two waits: five dependent rounds).  Same
// rows, same order of adds: bitwise the general form.  NR1: the row loads of
// that form, k rounded up to a multiple of 4 (the adds run in chunks of 4 up
// to k, so rows loaded past that chunk were never added).
template <int OP, typename T, int VEC, int G, bool SELF, bool ONE, int NR1 = kRows>
__global__ __launch_bounds__(kBlock) void agg_ids_kernel(const T* __restrict__ X, int64_t ldx, int F, int n_dst, int k,
                                                         const int* __restrict__ ids, const int* __restrict__ dst_ids,
                                                         int gcn, T* __restrict__ out, int64_t ldo,
                                                         T* __restrict__ self_out, int64_t ldso) {
    const int gl = threadIdx.x % G;
    if constexpr (ONE) {
        using Raw = typename RawVec<T, VEC>::type;
        constexpr int NR = NR1;
        static_assert(NR % 4 == 0 && NR <= kRows, "row loads: whole chunks of 4");
        const int r = blockIdx.x * (kBlock / G) + threadIdx.x / G;
        if (r >= n_dst) return;
        const int f0 = gl * VEC;
        const int node = SELF ? dst_ids[r] : 0;
        const int nb = gl < k ? ids[static_cast<int64_t>(r) * k + gl] : -1;
        int rows[NR];
        bool ok[NR];
#pragma unroll
        for (int u = 0; u < NR; ++u) {
            rows[u] = __shfl(nb, u, G);
            ok[u] = u < k && rows[u] >= 0;
        }
        const int fallback = SELF ? node : (rows[0] >= 0 ? rows[0] : 0);
        Raw xself{};
        if (SELF) xself = *reinterpret_cast<const Raw*>(X + static_cast<int64_t>(node) * ldx + f0);
        // every slot loaded (past k: the fallback row's line again), the adds in
        // chunks of 4 up to k (uniform: slots past k add nothing)
        Raw x[NR];
#pragma unroll
        for (int u = 0; u < NR; ++u)
            x[u] = *reinterpret_cast<const Raw*>(X + static_cast<int64_t>(ok[u] ? rows[u] : fallback) * ldx + f0);
        __builtin_amdgcn_sched_barrier(0);  // every row load issued before the first add waits on one
        float acc[VEC];
#pragma unroll
        for (int v = 0; v < VEC; ++v) acc[v] = (OP == GS_AGG_MAX) ? -INFINITY : 0.f;
        int cnt = 0;
        int ka = k;
        asm volatile("" : "+s"(ka));  // (kept opaque: the adds stay behind the loads)
#pragma unroll
        for (int q = 0; q < NR / 4; ++q)
            if (4 * q < ka) {
#pragma unroll
                for (int u = 4 * q; u < 4 * q + 4; ++u) {
                    cnt += ok[u];
                    float xv[VEC];
                    RawVec<T, VEC>::unpack(x[u], xv);
#pragma unroll
                    for (int v = 0; v < VEC; ++v) {
                        if (OP == GS_AGG_MEAN) {
                            acc[v] += ok[u] ? xv[v] : 0.f;
                        } else {
                            const bool take = ok[u] && xv[v] > acc[v];
                            acc[v] = take ? xv[v] : acc[v];
                        }
                    }
                }
            }
        if (SELF) *reinterpret_cast<Raw*>(self_out + static_cast<int64_t>(r) * ldso + f0) = xself;
        if (OP == GS_AGG_MEAN) {
            const float inv = 1.0f / static_cast<float>(cnt);
#pragma unroll
            for (int v = 0; v < VEC; ++v) acc[v] *= inv;
        }
        RowIO<T, VEC>::store(out + static_cast<int64_t>(r) * ldo + f0, acc);
        return;
    }
    // grid-stride over destinations (the launch caps the grid: agg_ids_block_cap)
    for (int r = blockIdx.x * (kBlock / G) + threadIdx.x / G; r < n_dst; r += gridDim.x * (kBlock / G)) {
    const int node = (gcn || SELF) ? dst_ids[r] : 0;
    const int* rid = ids + static_cast<int64_t>(r) * k;
    // 16 rows in flight for 16-byte fp32 and bf16 vectors alike, so a fanout
    // <= 16 neighbourhood is one memory round (8 for bf16 split a 10-slot
    // neighbourhood into two dependent rounds: 0.28 of HBM peak, round 1)
    constexpr int NR = kRows;
    const int nf = (F + G * VEC - 1) / (G * VEC);
    for (int fi = 0; fi < nf; ++fi) {
        const int f0 = fi * G * VEC + gl * VEC;
        const bool act = f0 < F;
        const int f0c = act ? f0 : 0;
        using Raw = typename RawVec<T, VEC>::type;
        Raw xself{};
        if (SELF) xself = *reinterpret_cast<const Raw*>(X + static_cast<int64_t>(node) * ldx + f0c);
        float acc[VEC];
#pragma unroll
        for (int v = 0; v < VEC; ++v) acc[v] = (OP == GS_AGG_MAX) ? -INFINITY : 0.f;
        int cnt = 0;
        bool self_seen = false;
        for (int base = 0; base < k; base += G) {
            const int m = min(G, k - base);
            const bool mine = gl < m;
            const int nb = rid[mine ? base + gl : base];
            if (gcn) self_seen |= group_bits<G>(mine && nb == node) != 0;
            const int my = mine ? nb : -1;
            for (int j = 0; j < m; j += NR) {
                int rows[NR];
                bool ok[NR];
#pragma unroll
                for (int u = 0; u < NR; ++u) {
                    rows[u] = __shfl(my, j + u < m ? j + u : j, G);
                    ok[u] = (j + u < m) && rows[u] >= 0;
                }
                const int fallback = rows[0] >= 0 ? rows[0] : node;
                Raw x[NR];
#pragma unroll
                for (int u = 0; u < NR; ++u)
                    x[u] = *reinterpret_cast<const Raw*>(X + static_cast<int64_t>(ok[u] ? rows[u] : fallback) * ldx + f0c);
#pragma unroll
                for (int u = 0; u < NR; ++u) {
                    cnt += ok[u];
                    float xv[VEC];
                    RawVec<T, VEC>::unpack(x[u], xv);
#pragma unroll
                    for (int v = 0; v < VEC; ++v) {
                        if (OP == GS_AGG_MEAN) {
                            acc[v] += ok[u] ? xv[v] : 0.f;
                        } else {
                            const bool take = ok[u] && xv[v] > acc[v];
                            acc[v] = take ? xv[v] : acc[v];
                        }
                    }
                }
            }
        }
        if (gcn && !self_seen) {  // gcn keeps self exactly once (set semantics)
            ++cnt;
            float x[VEC];
            RowIO<T, VEC>::load(X + static_cast<int64_t>(node) * ldx + f0c, x);
#pragma unroll
            for (int v = 0; v < VEC; ++v) {
                if (OP == GS_AGG_MEAN) acc[v] += x[v];
                else acc[v] = x[v] > acc[v] ? x[v] : acc[v];
            }
        }
        if (!act) continue;
        if (SELF) *reinterpret_cast<Raw*>(self_out + static_cast<int64_t>(r) * ldso + f0) = xself;
        if (OP == GS_AGG_MEAN) {
            const float inv = 1.0f / static_cast<float>(cnt);
#pragma unroll
            for (int v = 0; v < VEC; ++v) acc[v] *= inv;
        }
        RowIO<T, VEC>::store(out + static_cast<int64_t>(r) * ldo + f0, acc);
    }
    }
}

void resolve_ids_launch(int64_t n_dst, int k, const int32_t* ptr, const int32_t* ent, const int32_t* col,
                        const int32_t* dst_ids, int gcn, int32_t* ids, hipStream_t st) {
    GS_REQUIRE(n_dst >= 0 && k >= 1 && n_dst * k < (int64_t(1) << 31), GS_EINVAL, "bad sizes");
    if (n_dst == 0) return;
    const int64_t total = n_dst * k;
    resolve_ids_kernel<<<dim3(static_cast<unsigned>((total + kBlock - 1) / kBlock)), kBlock, 0, st>>>(
        static_cast<int>(n_dst), k, ptr, ent, col, dst_ids, gcn, ids);
    check_launch("resolve_ids");
}

void resolve_top_launch(int64_t n_dst, int k, const int32_t* ptr, const int32_t* ent, const int32_t* col,
                        const int32_t* dst_ids, int gcn, int32_t* ids, int64_t n_top, int tk, const int32_t* tptr,
                        const int32_t* tnbr, const int32_t* tself, int32_t* tout, hipStream_t st, int64_t n_rec,
                        const int32_t* rptr, const int32_t* ridx, int32_t* rout) {
    GS_REQUIRE(n_dst >= 0 && k >= 1 && n_dst * k < (int64_t(1) << 31) && n_top >= 0 && tk >= 1 &&
                   n_top * (tk + 1) < (int64_t(1) << 30) && n_rec >= 0 && n_rec < (int64_t(1) << 27) &&
                   (n_rec == 0 || (rptr && ridx && rout)),
               GS_EINVAL, "bad sizes");
    const int64_t total = n_dst * k + n_top * (tk + 1) + n_rec * 8;
    if (total == 0) return;
    resolve_top_kernel<<<dim3(static_cast<unsigned>((total + kBlock - 1) / kBlock)), kBlock, 0, st>>>(
        static_cast<int>(n_dst), k, ptr, ent, col, dst_ids, gcn, ids, static_cast<int>(n_top), tk, tptr, tnbr, tself,
        tout, static_cast<int>(n_rec), rptr, ridx, rout);
    check_launch("resolve_top");
}

// One pass, a block per 256/G destinations (a grid capped at one block per
// CU made the side-stream gather 10 -> 17 us without moving the step).
static int agg_ids_block_cap() { return 1 << 30; }

void agg_ids_launch(gs_agg op, gs_dtype dt, const void* X, int64_t ldx, int64_t F, int64_t n_dst, int k,
                    const int32_t* ids, const int32_t* dst_ids, int gcn, void* out, int64_t ldo, hipStream_t st,
                    void* self_out, int64_t ldso) {
    GS_REQUIRE(op == GS_AGG_MEAN || op == GS_AGG_MAX, GS_EINVAL, "agg_func must be MEAN or MAX");
    GS_REQUIRE(F >= 1 && n_dst >= 0 && k >= 1 && ldx >= F && ldo >= F, GS_EINVAL, "bad sizes");
    GS_REQUIRE(!self_out || (dst_ids && ldso >= F), GS_EINVAL, "self rows need dst_ids and ldso >= F");
    if (n_dst == 0) return;
    const int V = dt == GS_F32 ? 4 : 8;
    const bool vec = F % V == 0 && ldx % V == 0 && ldo % V == 0 && aligned16(X) && aligned16(out) &&
                     (!self_out || (ldso % V == 0 && aligned16(self_out)));
    const int f = static_cast<int>(F), n = static_cast<int>(n_dst);
    static const int cap = agg_ids_block_cap();
#define GS_IDS2(OPV, TT, VV, GG, ONE, NRV)                                                                       \
    do {                                                                                                         \
        const dim3 grid_(std::min((n + (kBlock / GG) - 1) / (kBlock / GG), cap));                                \
        if (self_out)                                                                                            \
            launch_k(agg_ids_kernel<OPV, TT, VV, GG, true, ONE, NRV>, grid_, dim3(kBlock), 0, st,                \
                     static_cast<const TT*>(X), ldx, f, n, k, ids, dst_ids, gcn, static_cast<TT*>(out), ldo,      \
                     static_cast<TT*>(self_out), ldso);                                                          \
        else                                                                                                     \
            launch_k(agg_ids_kernel<OPV, TT, VV, GG, false, ONE, NRV>, grid_, dim3(kBlock), 0, st,               \
                     static_cast<const TT*>(X), ldx, f, n, k, ids, dst_ids, gcn, static_cast<TT*>(out), ldo,      \
                     static_cast<TT*>(nullptr), ldso);                                                           \
    } while (0)
    // the one-pass form loads k rounded up to 4 rows (a 10-neighbour hop: 12, not 16)
#define GS_IDS1(OPV, TT, VV, GG, ONE)                                                                            \
    do {                                                                                                         \
        if (!(ONE)) GS_IDS2(OPV, TT, VV, GG, false, kRows);                                                      \
        else if (k <= 4) GS_IDS2(OPV, TT, VV, GG, true, 4);                                                      \
        else if (k <= 8) GS_IDS2(OPV, TT, VV, GG, true, 8);                                                      \
        else if (k <= 12) GS_IDS2(OPV, TT, VV, GG, true, 12);                                                    \
        else GS_IDS2(OPV, TT, VV, GG, true, kRows);                                                              \
    } while (0)
    // one lane group per destination (no grid cap), one vector per lane, at
    // most kRows ids, no gcn: the two-round form
    const bool one_ok = !gcn && k <= kRows && static_cast<int64_t>(n + 1) * 64 < (int64_t(1) << 31) &&
                        cap >= (n + 3) / 4;
#define GS_IDS(OPV, TT, VV, GG)                                      \
    do {                                                             \
        if (one_ok && f == (GG) * (VV)) GS_IDS1(OPV, TT, VV, GG, true); \
        else GS_IDS1(OPV, TT, VV, GG, false);                        \
    } while (0)
#define GS_IDS_T(OPV, TT)                                                     \
    do {                                                                      \
        constexpr int VV = sizeof(TT) == 4 ? 4 : 8;                           \
        if (!vec) GS_IDS(OPV, TT, 1, 64);                                     \
        else {                                                                \
            const int G = pick_group(f, VV);                                  \
            if (G == 16) GS_IDS(OPV, TT, VV, 16);                             \
            else if (G == 32) GS_IDS(OPV, TT, VV, 32);                        \
            else GS_IDS(OPV, TT, VV, 64);                                     \
        }                                                                     \
    } while (0)
    if (op == GS_AGG_MEAN) {
        if (dt == GS_F32) GS_IDS_T(GS_AGG_MEAN, float);
        else GS_IDS_T(GS_AGG_MEAN, bf16_t);
    } else {
        if (dt == GS_F32) GS_IDS_T(GS_AGG_MAX, float);
        else GS_IDS_T(GS_AGG_MAX, bf16_t);
    }
#undef GS_IDS_T
#undef GS_IDS
#undef GS_IDS1
#undef GS_IDS2
    check_launch("agg_ids");
}

template <int OP, typename T, bool EXPAND>
static void launch_fwd(int vec, const T* X, int64_t ldx, int F, int n_dst, const int* ptr,
                       const int* idx, const int64_t* row_ptr, const int* col, const int* dst_ids,
                       int gcn, T* out, int64_t ldo, int* am, hipStream_t st) {
    constexpr int V = sizeof(T) == 4 ? 4 : 8;
    if (vec == 1) {
        const dim3 grid((n_dst + (kBlock / 64) - 1) / (kBlock / 64));
        launch_k(agg_fwd_kernel<OP, T, 1, 64, EXPAND>, grid, dim3(kBlock), 0, st, X, ldx, F, n_dst, ptr, idx, row_ptr,
                 col, dst_ids, gcn, out, ldo, am);
        return;
    }
    const int G = pick_group(F, V);
    const dim3 grid((n_dst + (kBlock / G) - 1) / (kBlock / G));
#define GS_AGG_FWD(GG)                                                                                   \
    launch_k(agg_fwd_kernel<OP, T, V, GG, EXPAND>, grid, dim3(kBlock), 0, st, X, ldx, F, n_dst, ptr, idx, row_ptr, \
             col, dst_ids, gcn, out, ldo, am)
    if (G == 16) GS_AGG_FWD(16);
    else if (G == 32) GS_AGG_FWD(32);
    else GS_AGG_FWD(64);
#undef GS_AGG_FWD
}

template <int OP>
static void launch_bwd(int vec, int n_src, int F, const int* tptr, const int* tidx, const int* ptr,
                       const float* dA, const float* dSelf, int64_t ldd, const int* am,
                       const float* Hprev, int64_t ldh, float* dH, hipStream_t st) {
    if (vec == 1) {
        const dim3 grid((n_src + 3) / 4);
        agg_bwd_kernel<OP, 1, 64><<<grid, kBlock, 0, st>>>(n_src, F, tptr, tidx, ptr, dA, dSelf, ldd, am,
                                                           Hprev, ldh, dH);
        return;
    }
    const int G = pick_group(F, 4);
    const dim3 grid((n_src + (kBlock / G) - 1) / (kBlock / G));
#define GS_AGG_BWD(GG)                                                                          \
    agg_bwd_kernel<OP, 4, GG><<<grid, kBlock, 0, st>>>(n_src, F, tptr, tidx, ptr, dA, dSelf, ldd, am, \
                                                       Hprev, ldh, dH)
    if (G == 16) GS_AGG_BWD(16);
    else if (G == 32) GS_AGG_BWD(32);
    else GS_AGG_BWD(64);
#undef GS_AGG_BWD
}

}  // namespace gs

extern "C" {

int gs_agg_fwd(gs_agg op, gs_dtype xdt, const void* X, int64_t ldx, int64_t F, int64_t n_dst,
               const int32_t* ptr, const int32_t* idx, const int64_t* row_ptr, const int32_t* col,
               const int32_t* dst_ids, int32_t gcn, void* out, gs_dtype odt, int64_t ldo,
               int32_t* argmax, void* stream) {
    GS_API_BEGIN
    using namespace gs;
    GS_REQUIRE(op == GS_AGG_MEAN || op == GS_AGG_MAX, GS_EINVAL, "agg_func must be MEAN or MAX");
    GS_REQUIRE(xdt == odt, GS_EINVAL, "output dtype must equal feature dtype");
    GS_REQUIRE(F >= 1 && F < (1 << 30) && n_dst >= 0 && n_dst < (int64_t(1) << 31), GS_EINVAL, "bad sizes");
    GS_REQUIRE(ldx >= F && ldo >= F, GS_EINVAL, "leading dimension smaller than F");
    if (n_dst == 0) return GS_OK;
    GS_REQUIRE(X && ptr && idx && out, GS_EINVAL, "NULL device pointer");
    const bool expand = col != nullptr;
    GS_REQUIRE(!expand || dst_ids, GS_EINVAL, "expand mode needs dst_ids");
    GS_REQUIRE(!(argmax && expand), GS_EINVAL, "argmax is only produced in explicit mode");
    const int V = xdt == GS_F32 ? 4 : 8;
    const int vec = (F % V == 0 && ldx % V == 0 && ldo % V == 0 && aligned16(X) && aligned16(out)) ? V : 1;
    hipStream_t st = as_stream(stream);
    const int f = static_cast<int>(F), n = static_cast<int>(n_dst);
#define GS_DISPATCH(OPV, TT)                                                                              \
    do {                                                                                                  \
        if (expand)                                                                                       \
            launch_fwd<OPV, TT, true>(vec, static_cast<const TT*>(X), ldx, f, n, ptr, idx, row_ptr, col,  \
                                      dst_ids, gcn, static_cast<TT*>(out), ldo, nullptr, st);             \
        else                                                                                              \
            launch_fwd<OPV, TT, false>(vec, static_cast<const TT*>(X), ldx, f, n, ptr, idx, nullptr,      \
                                       nullptr, nullptr, 0, static_cast<TT*>(out), ldo, argmax, st);      \
    } while (0)
    if (op == GS_AGG_MEAN) {
        if (xdt == GS_F32) GS_DISPATCH(GS_AGG_MEAN, float);
        else GS_DISPATCH(GS_AGG_MEAN, bf16_t);
    } else {
        if (xdt == GS_F32) GS_DISPATCH(GS_AGG_MAX, float);
        else GS_DISPATCH(GS_AGG_MAX, bf16_t);
    }
#undef GS_DISPATCH
    check_launch("gs_agg_fwd");
    GS_API_END
}

int gs_agg_bwd(gs_agg op, int64_t n_src, int64_t F, const int32_t* tptr, const int32_t* tidx,
               const int32_t* ptr, const float* dA, const float* dSelf, int64_t ldd,
               const int32_t* argmax, const float* Hprev, int64_t ldh, float* dH, void* stream) {
    GS_API_BEGIN
    using namespace gs;
    GS_REQUIRE(op == GS_AGG_MEAN || op == GS_AGG_MAX, GS_EINVAL, "agg_func must be MEAN or MAX");
    GS_REQUIRE(F >= 1 && n_src >= 0 && n_src < (int64_t(1) << 31), GS_EINVAL, "bad sizes");
    GS_REQUIRE(ldd >= F && ldh >= F, GS_EINVAL, "leading dimension smaller than F");
    if (n_src == 0) return GS_OK;
    GS_REQUIRE(tptr && tidx && ptr && dA && dH, GS_EINVAL, "NULL device pointer");
    GS_REQUIRE(op != GS_AGG_MAX || argmax, GS_EINVAL, "MAX backward needs argmax");
    const int vec = (F % 4 == 0 && ldd % 4 == 0 && ldh % 4 == 0 && aligned16(dA) && (!dSelf || aligned16(dSelf)) &&
                     aligned16(dH) && (!Hprev || aligned16(Hprev)))
                        ? 4
                        : 1;
    hipStream_t st = as_stream(stream);
    if (op == GS_AGG_MEAN)
        launch_bwd<GS_AGG_MEAN>(vec, static_cast<int>(n_src), static_cast<int>(F), tptr, tidx, ptr, dA, dSelf,
                                ldd, argmax, Hprev, ldh, dH, st);
    else
        launch_bwd<GS_AGG_MAX>(vec, static_cast<int>(n_src), static_cast<int>(F), tptr, tidx, ptr, dA, dSelf,
                               ldd, argmax, Hprev, ldh, dH, st);
    check_launch("gs_agg_bwd");
    GS_API_END
}

}  // extern "C"
