// UnsupervisedLoss.get_loss_sage (models.py:65-96) and get_loss_margin
// (models.py:98-132), forward and backward, over the index plan built on the
// host by gs_unsup_loss_plan (host/unsup.cpp).
//
// Forward, launch 1 (pair_scores_kernel): one 256-lane block per scored node.
// Its pairs are spread over sixteen 16-lane groups (pair j -> group j % 16);
// a group reads the two embedding rows of a pair as float4 chunks and reduces
// dot, |a|^2, |b|^2 across its 16 lanes.  cos follows F.cosine_similarity
// (eps = 1e-8 clamps each norm).  The block then folds the groups' partials in
// a fixed order into the node score and writes, per pair g, {c_g, cos_g, n1,
// n2}: c_g = d loss / d cos_g for d loss = 1.
//   sage  : score = -mean_p log σ(cos⁺_p) - Q · mean_n log σ(-cos⁻_n)
//           c⁺ = -(1 - σ(cos⁺)) / (M P_m),  c⁻ = Q σ(cos⁻) / (M N_m)
//   margin: score = max(0, max_n log σ(cos⁻) - min_p log σ(cos⁺) + MARGIN)
//           only the arg-min positive and arg-max negative (first index on
//           ties, like torch.min/max over dim 0) carry ∓(1 - σ(cos)) / M,
//           halved when the hinge sits exactly at 0 (torch.maximum's tie rule).
// Forward, launch 2 (loss_reduce_kernel): loss = Σ_m score_m / M, fixed order.
// Backward (row_grad_kernel): one block per embedding row r; its pair
// memberships (tptr/tidx, ascending) are spread over the 16 groups, each adds
//   c_g · (other / (m_r m_o) - [n_r > eps] cos_g · row / (n_r m_r))
// and the 16 partial rows are added in group order, times d loss.  No atomics:
// the result is deterministic.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>

#include "kcommon.hpp"

namespace gs {
namespace {

constexpr int kUnsupThreads = 256;
constexpr int kGroup = 16;
constexpr int kGroups = kUnsupThreads / kGroup;
constexpr float kCosEps = 1e-8f;

struct Plan {
    const int32_t *pos_ptr, *neg_ptr, *pa, *pb, *na, *nb, *tptr, *tidx;
    int64_t M, P, N, U;
};

__device__ __forceinline__ float group_sum(float v) {
#pragma unroll
    for (int o = kGroup / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, kGroup);
    return v;
}

__device__ __forceinline__ float sigmoidf(float x) { return 1.0f / (1.0f + __expf(-x)); }

// dot / squared norms of rows a and b over D = 4 * nq floats, 16 lanes.
template <int NC>
__device__ __forceinline__ void pair_dots(const float* __restrict__ E, int64_t lde, int nq, int ra, int rb,
                                          int lane, float& dot, float& sa, float& sb) {
    const float4* A = reinterpret_cast<const float4*>(E + static_cast<int64_t>(ra) * lde);
    const float4* B = reinterpret_cast<const float4*>(E + static_cast<int64_t>(rb) * lde);
    float4 x[NC], y[NC];
#pragma unroll
    for (int c = 0; c < NC; ++c) {
        const int q = lane + c * kGroup;
        const bool ok = q < nq;
        x[c] = A[ok ? q : 0];
        y[c] = B[ok ? q : 0];
        if (!ok) x[c] = y[c] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
    float d = 0.f, s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
        d += x[c].x * y[c].x + x[c].y * y[c].y + x[c].z * y[c].z + x[c].w * y[c].w;
        s1 += x[c].x * x[c].x + x[c].y * x[c].y + x[c].z * x[c].z + x[c].w * x[c].w;
        s2 += y[c].x * y[c].x + y[c].y * y[c].y + y[c].z * y[c].z + y[c].w * y[c].w;
    }
    dot = group_sum(d);
    sa = group_sum(s1);
    sb = group_sum(s2);
}

__device__ __forceinline__ float cos_of(float dot, float n1, float n2) {
    return dot / (fmaxf(n1, kCosEps) * fmaxf(n2, kCosEps));
}

// Per-group running state folded in group order afterwards.
struct Acc {
    float sum;  // sage: Σ log σ(±cos)
    float ext;  // margin: min (pos) / max (neg) of log σ(cos)
    int arg;    // pair index of ext (first on ties)
    float cos;  // cos of that pair
};

template <int NC, bool MARGIN_LOSS>
__global__ __launch_bounds__(kUnsupThreads) void pair_scores_kernel(Plan pl, const float* __restrict__ E,
                                                                     int64_t lde, int nq, float q, float margin,
                                                                     float4* __restrict__ info,
                                                                     float* __restrict__ score) {
    __shared__ Acc acc[2][kGroups];
    const int m = blockIdx.x;
    const int grp = threadIdx.x / kGroup, lane = threadIdx.x % kGroup;
    const float invM = 1.0f / static_cast<float>(pl.M);
    for (int side = 0; side < 2; ++side) {  // 0: positive pairs, 1: negative pairs
        const int32_t* ptr = side == 0 ? pl.pos_ptr : pl.neg_ptr;
        const int32_t* ia = side == 0 ? pl.pa : pl.na;
        const int32_t* ib = side == 0 ? pl.pb : pl.nb;
        const int lo = ptr[m], hi = ptr[m + 1];
        Acc a{0.f, side == 0 ? INFINITY : -INFINITY, -1, 0.f};
        for (int j = lo + grp; j < hi; j += kGroups) {
            float dot, s1, s2;
            pair_dots<NC>(E, lde, nq, ia[j], ib[j], lane, dot, s1, s2);
            const float n1 = sqrtf(s1), n2 = sqrtf(s2);
            const float c = cos_of(dot, n1, n2);
            if (MARGIN_LOSS) {
                const float ls = __logf(sigmoidf(c));
                const bool better = side == 0 ? ls < a.ext : ls > a.ext;
                if (better) {
                    a.ext = ls;
                    a.arg = j;
                    a.cos = c;
                }
            } else {
                a.sum += side == 0 ? __logf(sigmoidf(c)) : __logf(sigmoidf(-c));
            }
            if (lane == 0) {
                const int64_t g = side == 0 ? j : pl.P + j;
                float coef = 0.f;
                if (!MARGIN_LOSS)
                    coef = side == 0 ? -(1.0f - sigmoidf(c)) * invM / static_cast<float>(hi - lo)
                                     : q * sigmoidf(c) * invM / static_cast<float>(hi - lo);
                info[g] = make_float4(coef, c, n1, n2);
            }
        }
        if (lane == 0) acc[side][grp] = a;
    }
    __syncthreads();
    if (threadIdx.x != 0) return;
    if (!MARGIN_LOSS) {
        float sp = 0.f, sn = 0.f;
        for (int g = 0; g < kGroups; ++g) {
            sp += acc[0][g].sum;
            sn += acc[1][g].sum;
        }
        const float np = static_cast<float>(pl.pos_ptr[m + 1] - pl.pos_ptr[m]);
        const float nn = static_cast<float>(pl.neg_ptr[m + 1] - pl.neg_ptr[m]);
        score[m] = -sp / np - q * (sn / nn);
        return;
    }
    Acc p = acc[0][0], n = acc[1][0];
    for (int g = 1; g < kGroups; ++g) {  // earlier pair index wins ties
        const Acc& x = acc[0][g];
        if (x.arg >= 0 && (x.ext < p.ext || (x.ext == p.ext && x.arg < p.arg))) p = x;
        const Acc& y = acc[1][g];
        if (y.arg >= 0 && (y.ext > n.ext || (y.ext == n.ext && y.arg < n.arg))) n = y;
    }
    const float h = n.ext - p.ext + margin;
    score[m] = fmaxf(h, 0.f);
    const float f = h > 0.f ? 1.f : (h == 0.f ? 0.5f : 0.f);
    // coefficients: only the two selected pairs are non-zero (the group loop
    // wrote 0 into every pair's .x)
    reinterpret_cast<float*>(info + p.arg)[0] = -f * (1.0f - sigmoidf(p.cos)) * invM;
    reinterpret_cast<float*>(info + pl.P + n.arg)[0] = f * (1.0f - sigmoidf(n.cos)) * invM;
}

__global__ __launch_bounds__(64) void loss_reduce_kernel(const float* __restrict__ score, int64_t M,
                                                         float* __restrict__ loss) {
    float s = 0.f;
    for (int64_t i = threadIdx.x; i < M; i += 64) s += score[i];
    s = wave_sum(s);
    if (threadIdx.x == 0) loss[0] = s / static_cast<float>(M);
}

template <int NC>
__global__ __launch_bounds__(kUnsupThreads) void row_grad_kernel(Plan pl, const float* __restrict__ E, int64_t lde,
                                                                  int nq, const float4* __restrict__ info,
                                                                  const float* __restrict__ dloss,
                                                                  float* __restrict__ dE, int64_t ldd) {
    __shared__ float4 part[kGroups][kGroup * NC];
    const int r = blockIdx.x;
    const int grp = threadIdx.x / kGroup, lane = threadIdx.x % kGroup;
    const float4* X = reinterpret_cast<const float4*>(E + static_cast<int64_t>(r) * lde);
    float4 x[NC], acc[NC];
#pragma unroll
    for (int c = 0; c < NC; ++c) {
        const int qq = lane + c * kGroup;
        x[c] = qq < nq ? X[qq] : make_float4(0.f, 0.f, 0.f, 0.f);
        acc[c] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
    const int lo = pl.tptr[r], hi = pl.tptr[r + 1];
    for (int t = lo + grp; t < hi; t += kGroups) {
        const int code = pl.tidx[t];
        const int64_t g = code >> 1;
        const int side = code & 1;
        const int32_t* ia = g < pl.P ? pl.pa : pl.na - pl.P;
        const int32_t* ib = g < pl.P ? pl.pb : pl.nb - pl.P;
        const int other = side == 0 ? ib[g] : ia[g];
        const float4 in = info[g];
        const float ns = side == 0 ? in.z : in.w, no = side == 0 ? in.w : in.z;
        const float ms = fmaxf(ns, kCosEps), mo = fmaxf(no, kCosEps);
        const float a = in.x / (ms * mo);
        const float b = ns > kCosEps ? in.x * in.y / (ns * ms) : 0.f;
        const float4* O = reinterpret_cast<const float4*>(E + static_cast<int64_t>(other) * lde);
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            const int qq = lane + c * kGroup;
            const float4 o = qq < nq ? O[qq] : make_float4(0.f, 0.f, 0.f, 0.f);
            acc[c].x += a * o.x - b * x[c].x;
            acc[c].y += a * o.y - b * x[c].y;
            acc[c].z += a * o.z - b * x[c].z;
            acc[c].w += a * o.w - b * x[c].w;
        }
    }
#pragma unroll
    for (int c = 0; c < NC; ++c) part[grp][lane + c * kGroup] = acc[c];
    __syncthreads();
    const float s = dloss[0];
    float4* out = reinterpret_cast<float4*>(dE + static_cast<int64_t>(r) * ldd);
    for (int qq = threadIdx.x; qq < nq; qq += kUnsupThreads) {
        float4 v = part[0][qq];
        for (int g = 1; g < kGroups; ++g) {
            const float4 w = part[g][qq];
            v.x += w.x;
            v.y += w.y;
            v.z += w.z;
            v.w += w.w;
        }
        out[qq] = make_float4(v.x * s, v.y * s, v.z * s, v.w * s);
    }
}

Plan make_plan(const int32_t* plan, int64_t M, int64_t P, int64_t N, int64_t U) {
    Plan pl;
    pl.pos_ptr = plan;
    pl.neg_ptr = pl.pos_ptr + (M + 1);
    pl.pa = pl.neg_ptr + (M + 1);
    pl.pb = pl.pa + P;
    pl.na = pl.pb + P;
    pl.nb = pl.na + N;
    pl.tptr = pl.nb + N;
    pl.tidx = pl.tptr + (U + 1);
    pl.M = M;
    pl.P = P;
    pl.N = N;
    pl.U = U;
    return pl;
}

int chunks_for(int64_t D) {
    const int64_t nq = D / 4;
    if (nq <= 2 * kGroup) return 2;
    if (nq <= 4 * kGroup) return 4;
    if (nq <= 8 * kGroup) return 8;
    return 16;
}

void check_rows(int64_t D, const float* p, int64_t ld, const char* what) {
    GS_REQUIRE(D >= 4 && D % 4 == 0 && D <= 4 * 16 * kGroup, GS_EINVAL, "embedding width must be a multiple of 4, <= 1024");
    GS_REQUIRE(ld >= D && ld % 4 == 0 && (reinterpret_cast<uintptr_t>(p) & 15) == 0, GS_EINVAL,
               std::string(what) + " rows must be 16-byte aligned");
}

}  // namespace
}  // namespace gs

extern "C" {

int64_t gs_unsup_loss_ws_floats(int64_t M, int64_t P, int64_t N) { return 4 * (P + N) + M + 4; }

int gs_unsup_loss_fwd(int32_t kind, int64_t M, int64_t P, int64_t N, int64_t U, int64_t D, const float* emb,
                      int64_t lde, const int32_t* plan, float q, float margin, float* loss, float* ws,
                      void* stream) {
    GS_API_BEGIN
    using namespace gs;
    GS_REQUIRE(kind == 0 || kind == 1, GS_EINVAL, "kind: 0 = sage, 1 = margin");
    GS_REQUIRE(M >= 1 && P >= M && N >= M && U >= 1 && M < (1 << 30), GS_EINVAL, "bad plan sizes");
    GS_REQUIRE(emb && plan && loss && ws, GS_EINVAL, "NULL device pointer");
    check_rows(D, emb, lde, "embedding");
    GS_REQUIRE((reinterpret_cast<uintptr_t>(ws) & 15) == 0, GS_EINVAL, "workspace must be 16-byte aligned");
    hipStream_t st = as_stream(stream);
    const Plan pl = make_plan(plan, M, P, N, U);
    float4* info = reinterpret_cast<float4*>(ws);
    float* score = ws + 4 * (P + N);
    const int nq = static_cast<int>(D / 4);
    const dim3 grid(static_cast<unsigned>(M));
#define GS_PAIR(NC)                                                                                               \
    (kind ? pair_scores_kernel<NC, true><<<grid, kUnsupThreads, 0, st>>>(pl, emb, lde, nq, q, margin, info, score) \
          : pair_scores_kernel<NC, false><<<grid, kUnsupThreads, 0, st>>>(pl, emb, lde, nq, q, margin, info, score))
    switch (chunks_for(D)) {
        case 2: GS_PAIR(2); break;
        case 4: GS_PAIR(4); break;
        case 8: GS_PAIR(8); break;
        default: GS_PAIR(16); break;
    }
#undef GS_PAIR
    loss_reduce_kernel<<<1, 64, 0, st>>>(score, M, loss);
    check_launch("gs_unsup_loss_fwd");
    GS_API_END
}

int gs_unsup_loss_bwd(int64_t M, int64_t P, int64_t N, int64_t U, int64_t D, const float* emb, int64_t lde,
                      const int32_t* plan, const float* ws, const float* dloss, float* dE, int64_t ldd,
                      void* stream) {
    GS_API_BEGIN
    using namespace gs;
    GS_REQUIRE(M >= 1 && P >= M && N >= M && U >= 1 && U < (int64_t(1) << 31), GS_EINVAL, "bad plan sizes");
    GS_REQUIRE(emb && plan && ws && dloss && dE, GS_EINVAL, "NULL device pointer");
    check_rows(D, emb, lde, "embedding");
    check_rows(D, dE, ldd, "gradient");
    hipStream_t st = as_stream(stream);
    const Plan pl = make_plan(plan, M, P, N, U);
    const float4* info = reinterpret_cast<const float4*>(ws);
    const int nq = static_cast<int>(D / 4);
    const dim3 grid(static_cast<unsigned>(U));
    switch (chunks_for(D)) {
        case 2: row_grad_kernel<2><<<grid, kUnsupThreads, 0, st>>>(pl, emb, lde, nq, info, dloss, dE, ldd); break;
        case 4: row_grad_kernel<4><<<grid, kUnsupThreads, 0, st>>>(pl, emb, lde, nq, info, dloss, dE, ldd); break;
        case 8: row_grad_kernel<8><<<grid, kUnsupThreads, 0, st>>>(pl, emb, lde, nq, info, dloss, dE, ldd); break;
        default: row_grad_kernel<16><<<grid, kUnsupThreads, 0, st>>>(pl, emb, lde, nq, info, dloss, dE, ldd); break;
    }
    check_launch("gs_unsup_loss_bwd");
    GS_API_END
}

}  // extern "C"
