// Layer 1 of GraphSage.forward (models.py:255-260) as ONE kernel: the
// gather-aggregate of the sampled neighbourhoods (aggregate, models.py:291-330)
// feeding SageLayer's concat-linear-relu (models.py:209-220) through LDS.
//
// Per block of 16 destinations (8 wavefronts):
//   gather : wave w reduces destinations 2w, 2w+1 — self row X[dst] and the
//            mean / max of its sampled neighbour rows X[col[entry]] (absolute
//            CSR entries from the pack, self dropped unless gcn) — into the
//            block's LDS tile A = [self | agg] (16 x K), and writes the agg rows
//            to HBM for the weight gradient.  All loads are unconditional
//            (clamped, masked at use) so 16 neighbour rows stay in flight, and
//            the second destination's index chain is issued with the first's.
//   linear : wave w owns output columns 16w.. (+128 per extra pass); its W
//            slots stream from L2 two K-chunks ahead of its MFMAs, A comes from
//            LDS; relu epilogue (NaN kept, as torch.relu).
// Versus the two-kernel path this drops the A round trip through HBM and
// one launch, and overlaps the gather's latency chain with other blocks'
// MFMA work.
#include "kcommon.hpp"

namespace gs {

constexpr int kS1Threads = 512;  // 8 wavefronts
constexpr int kS1Rows = 16;      // destinations per block
constexpr int kS1Inflight = 16;  // neighbour rows in flight per wave (8 for bf16's 8-element vectors)

// LDS bytes of the A tile for K elements of T (pitch K + one 16-B slot).
inline size_t sage1_lds(int64_t K, size_t esz) {
    return static_cast<size_t>(kS1Rows) * (K + 16 / esz) * esz;
}

template <typename T>
__device__ __forceinline__ void store_vec(T* p, const float (&v)[16 / sizeof(T)]) {
    RowIO<T, 16 / sizeof(T)>::store(p, v);
}

template <int OP, typename T, bool HAS_SELF, bool RELU>
__global__ __launch_bounds__(kS1Threads) void sage1_fwd_kernel(
    const T* __restrict__ X, int64_t ldx, int F, int H, int n_dst, const int* __restrict__ ptr,
    const int* __restrict__ ent, const int* __restrict__ col, const int* __restrict__ dst_ids, int gcn,
    const T* __restrict__ W, T* __restrict__ agg_out, int64_t ld_agg, float* __restrict__ out, int64_t ldo) {
    constexpr int EPV = 16 / sizeof(T);
    constexpr int BK = 16 * EPV;  // K elements per chunk (16 slots of 16 B)
    constexpr int NR = sizeof(T) == 4 ? kS1Inflight : kS1Inflight / 2;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    T* sA = reinterpret_cast<T*>(smem);
    const int K = HAS_SELF ? 2 * F : F;
    const int SA = K + EPV;  // elements
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int m0 = blockIdx.x * kS1Rows;

    // ------------------------------------------------------------ gather
    {
        int rr[2], beg[2], end[2], node[2];
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            rr[q] = 2 * wave + q;
            const int r = min(m0 + rr[q], n_dst - 1);
            beg[q] = ptr[r];
            end[q] = ptr[r + 1];
            node[q] = dst_ids[r];
        }
        // neighbour ids of both destinations (first 64 of each; longer
        // neighbourhoods continue in the loop below)
        // expand mode (col != NULL): ent holds absolute CSR entries, self is
        // dropped unless gcn; explicit mode (col == NULL): ent holds the
        // source rows themselves, already self-filtered (gcn lists include self)
        const bool expand = col != nullptr;
        if (!expand) gcn = 0;
        int my[2];
        bool selfhit[2];
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            const int m = min(64, end[q] - beg[q]);
            const bool mine = lane < m;
            const int e = m > 0 ? ent[mine ? beg[q] + lane : beg[q]] : 0;
            const int nb = expand ? col[e] : e;
            my[q] = (mine && (!expand || gcn || nb != node[q])) ? nb : -1;
            selfhit[q] = __ballot(mine && nb == node[q]) != 0;
        }
        for (int q = 0; q < 2; ++q) {
            const bool live = m0 + rr[q] < n_dst;
            // wave-uniform trip count: every lane takes part in the shuffles
            // and ballots below (ids of neighbour j live in lane j), lanes
            // past F work on a clamped column and store nothing
            const int nf = (F + 64 * EPV - 1) / (64 * EPV);
            for (int fi = 0; fi < nf; ++fi) {
                const int fr = fi * 64 * EPV + lane * EPV;
                const bool act = fr < F;
                const int f0 = act ? fr : 0;
                float self[EPV];  // issued first: lands with the neighbour rows
                RowIO<T, EPV>::load(X + static_cast<int64_t>(node[q]) * ldx + f0, self);
                float acc[EPV];
#pragma unroll
                for (int v = 0; v < EPV; ++v) acc[v] = (OP == GS_AGG_MAX) ? -INFINITY : 0.f;
                int cnt = 0;
                bool self_seen = selfhit[q];
                for (int base = beg[q]; base < end[q]; base += 64) {
                    const int m = min(64, end[q] - base);
                    int mine_id = my[q];
                    if (base != beg[q]) {  // rare: more than 64 sampled entries
                        const bool mine = lane < m;
                        const int e = ent[mine ? base + lane : base];
                        const int nb = expand ? col[e] : e;
                        mine_id = (mine && (!expand || gcn || nb != node[q])) ? nb : -1;
                        self_seen |= __ballot(mine && nb == node[q]) != 0;
                    }
                    for (int j = 0; j < m; j += NR) {
                        int rows[NR];
                        bool ok[NR];
#pragma unroll
                        for (int u = 0; u < NR; ++u) {
                            rows[u] = __shfl(mine_id, j + u < m ? j + u : j, 64);
                            ok[u] = (j + u < m) && rows[u] >= 0;
                        }
                        const int fb = rows[0] >= 0 ? rows[0] : node[q];
                        float x[NR][EPV];
#pragma unroll
                        for (int u = 0; u < NR; ++u)
                            RowIO<T, EPV>::load(X + static_cast<int64_t>(ok[u] ? rows[u] : fb) * ldx + f0, x[u]);
#pragma unroll
                        for (int u = 0; u < NR; ++u) {
                            cnt += ok[u];
#pragma unroll
                            for (int v = 0; v < EPV; ++v) {
                                if (OP == GS_AGG_MEAN) acc[v] += ok[u] ? x[u][v] : 0.f;
                                else acc[v] = (ok[u] && x[u][v] > acc[v]) ? x[u][v] : acc[v];
                            }
                        }
                    }
                }
                if (gcn && !self_seen) {  // gcn keeps self exactly once (models.py:285)
                    ++cnt;
#pragma unroll
                    for (int v = 0; v < EPV; ++v) {
                        if (OP == GS_AGG_MEAN) acc[v] += self[v];
                        else acc[v] = self[v] > acc[v] ? self[v] : acc[v];
                    }
                }
                if (OP == GS_AGG_MEAN) {
                    const float inv = 1.0f / static_cast<float>(cnt);  // 0 neighbours -> NaN, as 0/0 at :313
#pragma unroll
                    for (int v = 0; v < EPV; ++v) acc[v] *= inv;
                }
                // the agg row as the tile holds it (rounded to T), the self row verbatim
                if (!act) continue;
                T* arow = sA + rr[q] * SA;
                store_vec<T>(arow + (HAS_SELF ? F : 0) + f0, acc);
                if (HAS_SELF) store_vec<T>(arow + f0, self);
                if (live) store_vec<T>(agg_out + static_cast<int64_t>(m0 + rr[q]) * ld_agg + f0, acc);
            }
        }
    }
    __syncthreads();

    // ------------------------------------------------------------ linear
    const int r = lane & 15, kq = lane >> 4;
    const int nC = (K + BK - 1) / BK;
    for (int ct = wave; ct * 16 < H; ct += kS1Threads / 64) {
        const T* wrow = W + static_cast<int64_t>(ct * 16 + r) * K;
        auto wslot = [&](int c, int g) -> uint4 {
            const int k = c * BK + (4 * g + kq) * EPV;
            const uint4 v = *reinterpret_cast<const uint4*>(wrow + (k < K ? k : 0));
            return k < K ? v : make_uint4(0, 0, 0, 0);
        };
        uint4 w0[4], w1[4];
#pragma unroll
        for (int g = 0; g < 4; ++g) w0[g] = wslot(0, g);
#pragma unroll
        for (int g = 0; g < 4; ++g) w1[g] = wslot(min(1, nC - 1), g);
        f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
        for (int c = 0; c < nC; ++c) {
            uint4 wc[4];
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                wc[g] = w0[g];
                w0[g] = w1[g];
            }
            const int cn = min(c + 2, nC - 1);
#pragma unroll
            for (int g = 0; g < 4; ++g) w1[g] = wslot(cn, g);  // two chunks ahead
            __builtin_amdgcn_sched_barrier(0);
            uint4 av[4];
#pragma unroll
            for (int g = 0; g < 4; ++g) {  // slots past K read zeros (not the next row / stale LDS)
                const int k = c * BK + (4 * g + kq) * EPV;
                const uint4 v = *reinterpret_cast<const uint4*>(sA + r * SA + (k < K ? k : 0));
                av[g] = k < K ? v : make_uint4(0, 0, 0, 0);
            }
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                if constexpr (sizeof(T) == 4) {
                    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(av[g].x), __uint_as_float(wc[g].x), acc, 0, 0, 0);
                    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(av[g].y), __uint_as_float(wc[g].y), acc, 0, 0, 0);
                    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(av[g].z), __uint_as_float(wc[g].z), acc, 0, 0, 0);
                    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(av[g].w), __uint_as_float(wc[g].w), acc, 0, 0, 0);
                } else {
                    s16x8 a8, b8;
                    __builtin_memcpy(&a8, &av[g], 16);
                    __builtin_memcpy(&b8, &wc[g], 16);
                    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a8, b8, acc, 0, 0, 0);
                }
            }
            __builtin_amdgcn_sched_barrier(0);
        }
        const int colx = ct * 16 + r;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int row = m0 + 4 * kq + j;
            if (row < n_dst) {
                const float v = acc[j];
                out[static_cast<int64_t>(row) * ldo + colx] = (RELU && !(v > 0.f) && v == v) ? 0.f : v;
            }
        }
    }
}

}  // namespace gs

extern "C" {

int gs_sage1_fwd_supported(gs_dtype dt, int64_t F, int64_t H, int32_t gcn) {
    if (dt != GS_F32 && dt != GS_BF16) return 0;
    const int64_t EPV = dt == GS_F32 ? 4 : 8;
    const int64_t K = gcn ? F : 2 * F;
    if (F % EPV != 0 || H < 16 || H % 16 != 0 || H > 256) return 0;
    return gs::sage1_lds(K, dt == GS_F32 ? 4 : 2) <= 64 * 1024 ? 1 : 0;
}

int gs_sage1_fwd(gs_agg op, gs_dtype dt, const void* X, int64_t ldx, int64_t F, int64_t H, int64_t n_dst,
                 const int32_t* ptr, const int32_t* ent, const int32_t* col, const int32_t* dst_ids, int32_t gcn,
                 const void* W, void* agg_out, int64_t ld_agg, float* out, int64_t ldo, int32_t relu,
                 void* stream) {
    GS_API_BEGIN
    using namespace gs;
    GS_REQUIRE(op == GS_AGG_MEAN || op == GS_AGG_MAX, GS_EINVAL, "agg_func must be MEAN or MAX");
    GS_REQUIRE(gs_sage1_fwd_supported(dt, F, H, gcn), GS_EINVAL, "shape not supported by the fused layer-1 kernel");
    GS_REQUIRE(n_dst >= 0 && n_dst < (int64_t(1) << 31) && F < (1 << 28), GS_EINVAL, "bad sizes");
    if (n_dst == 0) return GS_OK;
    const int64_t EPV = dt == GS_F32 ? 4 : 8;
    GS_REQUIRE(X && ptr && ent && dst_ids && W && agg_out && out, GS_EINVAL, "NULL device pointer");
    GS_REQUIRE(ldx % EPV == 0 && ld_agg % EPV == 0 && aligned16(X) && aligned16(W) && aligned16(agg_out),
               GS_EINVAL, "X / W / agg_out must be 16-byte aligned with aligned strides");
    GS_REQUIRE(ldx >= F && ld_agg >= F && ldo >= H, GS_EINVAL, "leading dimension too small");
    const int64_t K = gcn ? F : 2 * F;
    const size_t smem = sage1_lds(K, dt == GS_F32 ? 4 : 2);
    const dim3 grid(static_cast<unsigned>((n_dst + kS1Rows - 1) / kS1Rows));
    hipStream_t st = as_stream(stream);
    const int f = static_cast<int>(F), h = static_cast<int>(H), n = static_cast<int>(n_dst);
#define GS_S1(OPV, TT, SELF, RELU)                                                                       \
    launch_k(sage1_fwd_kernel<OPV, TT, SELF, RELU>, grid, dim3(kS1Threads), static_cast<uint32_t>(smem), st, \
             static_cast<const TT*>(X), ldx, f, h, n, ptr, ent, col, dst_ids, gcn, static_cast<const TT*>(W), \
             static_cast<TT*>(agg_out), ld_agg, out, ldo)
#define GS_S1_R(OPV, TT, SELF) \
    do { if (relu) GS_S1(OPV, TT, SELF, true); else GS_S1(OPV, TT, SELF, false); } while (0)
#define GS_S1_S(OPV, TT) \
    do { if (gcn) GS_S1_R(OPV, TT, false); else GS_S1_R(OPV, TT, true); } while (0)
#define GS_S1_T(OPV) \
    do { if (dt == GS_F32) GS_S1_S(OPV, float); else GS_S1_S(OPV, bf16_t); } while (0)
    if (op == GS_AGG_MEAN) GS_S1_T(GS_AGG_MEAN);
    else GS_S1_T(GS_AGG_MAX);
#undef GS_S1_T
#undef GS_S1_S
#undef GS_S1_R
#undef GS_S1
    check_launch("gs_sage1_fwd");
    GS_API_END
}

}  // extern "C"
