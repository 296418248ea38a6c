// Layer-1 SageLayer forward GEMM lab: out[n,H] = relu([X[sidx] | A] · Wᵀ) at
// the rmat2m shape (n ≈ 4.4k, F = 256, K = 512, H = 128, fp32), timing kernel
// variants against the library's default (linear_fwd_wide_kernel<32>) with
// HIP events, cold (MALL flushed between launches) and warm.  Every variant
// must equal the default bitwise (same MFMA operands in the same order).
// Developer tool, not part of the library:
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 -I include tools/lab/gemm_lab.hip -o /tmp/gemm_lab
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "../../graphsage-pytorch_amd/csrc/kernels/linear_dev.hpp"

#define CK(x)                                                                      \
    do {                                                                           \
        hipError_t e_ = (x);                                                       \
        if (e_ != hipSuccess) {                                                    \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            std::exit(2);                                                          \
        }                                                                          \
    } while (0)

namespace lab {
using gs::f32x4;

// Block = 16 rows x NW·CW columns.  The block's 16 concat rows (K floats
// each) are loaded into LDS in one round; each wave then streams its own CW W
// rows straight into registers, D groups of 16 k ahead, and runs NT = CW/16
// accumulators.  Accumulation order = the chunked kernel's (k ascending in
// groups of 16, element j of lane kq's slot in MFMA j).
// PACKED: W given as Wp[g][ct][lane] uint4 (one 1 KiB coalesced read per
// group and 16-column tile) instead of row-major.
template <int NG, int CW, int NW, int D, bool PACKED>
__global__ __launch_bounds__(NW * 64) void fwd_rows_kernel(int n, int F, int H, const float* __restrict__ Xs,
                                                            int64_t ldxs, const int* __restrict__ sidx,
                                                            const float* __restrict__ A, int64_t lda,
                                                            const float* __restrict__ W, float* __restrict__ out,
                                                            int64_t ldo, unsigned long long* __restrict__ stamps) {
    unsigned long long t_start = 0;
    if (stamps) t_start = __builtin_amdgcn_s_memrealtime();
    constexpr int K = NG * 16;
    constexpr int NT = CW / 16;
    constexpr int PITCH = K + 4;  // floats; rows 4 banks apart
    constexpr int NTH = NW * 64;
    __shared__ float sA[16 * PITCH];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int r = lane & 15, kq = lane >> 4;
    const int m0 = blockIdx.x * 16;
    const int cb = blockIdx.y * (CW * NW) + wave * CW;  // first column of this wave
    // W ring: group g of tile t
    uint4 wv[D][NT];
    auto wload = [&](int g, int u) {
#pragma unroll
        for (int t = 0; t < NT; ++t) {
            const int ct = (cb >> 4) + t;
            if constexpr (PACKED) {
                wv[u][t] = reinterpret_cast<const uint4*>(W)[((int64_t)g * (H >> 4) + ct) * 64 + lane];
            } else {
                const int c = min(cb + 16 * t + r, H - 1);
                wv[u][t] = *reinterpret_cast<const uint4*>(W + (int64_t)c * K + 16 * g + 4 * kq);
            }
        }
    };
#pragma unroll
    for (int u = 0; u < D; ++u) wload(u, u);
    // A tile: 16 rows x 2 halves (self | agg) of F floats; one row-half per
    // wave instruction (F/4 = 64 lanes x 16 B), wave-uniform row and half, so
    // the self index is a scalar load and no lane branches.  All of a wave's
    // row-half loads are issued before the first is stored.
    static_assert(K == 512, "lab: F = 256");
    constexpr int RH = 32 / NW;  // row-halves per wave
    uint4 av[RH];
    int srow_[RH];
#pragma unroll
    for (int q = 0; q < RH; ++q) {
        const int rh = wave * RH + q, row = rh >> 1;
        srow_[q] = sidx[min(m0 + row, n - 1)];
    }
#pragma unroll
    for (int q = 0; q < RH; ++q) {
        const int rh = wave * RH + q, row = rh >> 1, half = rh & 1;
        const int gr = min(m0 + row, n - 1);
        const float* p = half ? A + (int64_t)gr * lda : Xs + (int64_t)srow_[q] * ldxs;
        av[q] = reinterpret_cast<const uint4*>(p)[lane];
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int q = 0; q < RH; ++q) {
        const int rh = wave * RH + q, row = rh >> 1, half = rh & 1;
        *reinterpret_cast<uint4*>(sA + row * PITCH + half * 256 + lane * 4) = av[q];
    }
    __syncthreads();
    unsigned long long t_a = 0;
    if (stamps) t_a = __builtin_amdgcn_s_memrealtime();
    f32x4 acc[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int g = 0; g < NG; ++g) {
        const int u = g % D;
        const uint4 a = *reinterpret_cast<const uint4*>(sA + r * PITCH + 16 * g + 4 * kq);
        uint4 w[NT];
#pragma unroll
        for (int t = 0; t < NT; ++t) w[t] = wv[u][t];
        if (g + D < NG) wload(g + D, u);
        __builtin_amdgcn_sched_barrier(0);  // the prefetch stays D groups ahead, ahead of these MFMAs
#pragma unroll
        for (int t = 0; t < NT; ++t) acc[t] = gs::mfma_slot<float>(a, w[t], acc[t]);
        __builtin_amdgcn_sched_barrier(0);
    }
    if (stamps && lane == 0) {
        const unsigned long long t_e = __builtin_amdgcn_s_memrealtime();
        unsigned long long* p = stamps + 3 * (((int64_t)blockIdx.y * gridDim.x + blockIdx.x) * NW + wave);
        p[0] = t_start; p[1] = t_a; p[2] = t_e;
    }
#pragma unroll
    for (int t = 0; t < NT; ++t) {
        const int col = cb + 16 * t + r;
        if (col >= H) continue;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int row = m0 + 4 * kq + j;
            if (row < n) {
                const float v = acc[t][j];
                out[(int64_t)row * ldo + col] = (!(v > 0.f) && v == v) ? 0.f : v;
            }
        }
    }
}


// Block = 32 rows x 64 columns (the traffic-optimal tile at 256 CUs: per
// block 64 KiB of A rows + 128 KiB of W).  A (32 concat rows) is loaded into
// LDS in one round; W is packed (Wp[g][ct][lane]) and streamed per wave
// straight into registers, D groups ahead.
//   KS = 1: 4 waves, wave w owns columns 16w.. for both 16-row tiles (two
//           accumulators sharing each W operand); k ascending: bitwise the
//           chunked kernel.
//   KS = 2: 8 waves, wave (w & 3, w >> 2) = (column tile, K half); the two
//           halves' tiles are added in LDS (half 0 + half 1): not bitwise.
// XCD-aware 1-D grid: blocks b and b + 8 (one XCD) are the two column halves
// of one row tile, so its A rows come from HBM once.
template <int KS, int D>
__global__ __launch_bounds__(256 * KS) void fwd_t32_kernel(int n, int F, int H, const float* __restrict__ Xs,
                                                           int64_t ldxs, const int* __restrict__ sidx,
                                                           const float* __restrict__ A, int64_t lda,
                                                           const float* __restrict__ Wp, float* __restrict__ out,
                                                           int64_t ldo, unsigned long long* __restrict__ stamps) {
    constexpr int K = 512, NG = K / 16, PITCH = K + 4, NW = 4 * KS;
    constexpr int GH = NG / KS;  // groups per wave
    __shared__ float sA[32 * PITCH];
    unsigned long long t_start = 0;
    if (stamps) t_start = __builtin_amdgcn_s_memrealtime();
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int r = lane & 15, kq = lane >> 4;
    const int b = blockIdx.x, x = b & 7, q = b >> 3;
    const int tile = (q >> 1) * 8 + x, ch = q & 1;
    const int m0 = tile * 32;
    if (m0 >= n) return;
    const int wc = wave & 3, kh = KS == 2 ? wave >> 2 : 0;
    const int ct = ch * 4 + wc;  // 16-column tile
    const int g0 = kh * GH;
    uint4 wv[D];
    auto wload = [&](int g, int u) {
        wv[u] = reinterpret_cast<const uint4*>(Wp)[((int64_t)g * (H >> 4) + ct) * 64 + lane];
    };
#pragma unroll
    for (int u = 0; u < D; ++u) wload(g0 + u, u);
    constexpr int RH = 64 / NW;  // row-halves per wave
    int srow_[RH];
#pragma unroll
    for (int i = 0; i < RH; ++i) {
        const int rh = wave * RH + i;
        srow_[i] = sidx[min(m0 + (rh >> 1), n - 1)];
    }
    uint4 av[RH];
#pragma unroll
    for (int i = 0; i < RH; ++i) {
        const int rh = wave * RH + i, row = rh >> 1;
        const int gr = min(m0 + row, n - 1);
        const float* p = (rh & 1) ? A + (int64_t)gr * lda : Xs + (int64_t)srow_[i] * ldxs;
        av[i] = reinterpret_cast<const uint4*>(p)[lane];
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < RH; ++i) {
        const int rh = wave * RH + i;
        *reinterpret_cast<uint4*>(sA + (rh >> 1) * PITCH + (rh & 1) * 256 + lane * 4) = av[i];
    }
    __syncthreads();
    unsigned long long t_a = 0;
    if (stamps) t_a = __builtin_amdgcn_s_memrealtime();
    f32x4 acc0 = f32x4{0.f, 0.f, 0.f, 0.f}, acc1 = acc0;
#pragma unroll
    for (int gi = 0; gi < GH; ++gi) {
        const int g = g0 + gi, u = gi % D;
        const uint4 a0 = *reinterpret_cast<const uint4*>(sA + r * PITCH + 16 * g + 4 * kq);
        const uint4 a1 = *reinterpret_cast<const uint4*>(sA + (16 + r) * PITCH + 16 * g + 4 * kq);
        const uint4 w = wv[u];
        if (gi + D < GH) wload(g + D, u);
        __builtin_amdgcn_sched_barrier(0);
        acc0 = gs::mfma_slot<float>(a0, w, acc0);
        acc1 = gs::mfma_slot<float>(a1, w, acc1);
        __builtin_amdgcn_sched_barrier(0);
    }
    if constexpr (KS == 2) {  // half 1 hands its tiles to half 0 through LDS (A no longer read)
        __syncthreads();
        float* red = sA;
        if (kh == 1) {
            *reinterpret_cast<f32x4*>(red + (wc * 64 + lane) * 8) = acc0;
            *reinterpret_cast<f32x4*>(red + (wc * 64 + lane) * 8 + 4) = acc1;
        }
        __syncthreads();
        if (kh == 1) return;
        const f32x4 p0 = *reinterpret_cast<const f32x4*>(red + (wc * 64 + lane) * 8);
        const f32x4 p1 = *reinterpret_cast<const f32x4*>(red + (wc * 64 + lane) * 8 + 4);
        acc0 += p0;
        acc1 += p1;
    }
    if (stamps && lane == 0) {
        const unsigned long long t_e = __builtin_amdgcn_s_memrealtime();
        unsigned long long* p = stamps + 3 * ((int64_t)blockIdx.x * NW + wave);
        p[0] = t_start; p[1] = t_a; p[2] = t_e;
    }
    const int col = ct * 16 + r;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int row0 = m0 + 4 * kq + j, row1 = row0 + 16;
        const float v0 = acc0[j], v1 = acc1[j];
        if (row0 < n) out[(int64_t)row0 * ldo + col] = (!(v0 > 0.f) && v0 == v0) ? 0.f : v0;
        if (row1 < n) out[(int64_t)row1 * ldo + col] = (!(v1 > 0.f) && v1 == v1) ? 0.f : v1;
    }
}


// 16 rows x (16·NW) columns, packed W in registers (D groups ahead), A in
// LDS loaded in one round but consumed in two halves: the self half's rows
// (K 0..F) are stored and published first, so the MFMAs over K < F run while
// the agg half (stored after them) is still arriving.  k ascending: bitwise.
template <int NW, int D>
__global__ __launch_bounds__(NW * 64) void fwd_2ph_kernel(int n, int F, int H, const float* __restrict__ Xs,
                                                          int64_t ldxs, const int* __restrict__ sidx,
                                                          const float* __restrict__ A, int64_t lda,
                                                          const float* __restrict__ Wp, float* __restrict__ out,
                                                          int64_t ldo, unsigned long long* __restrict__ stamps) {
    constexpr int K = 512, NG = 32, PITCH = K + 4;
    __shared__ float sA[16 * PITCH];
    unsigned long long t_start = 0;
    if (stamps) t_start = __builtin_amdgcn_s_memrealtime();
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int r = lane & 15, kq = lane >> 4;
    const int m0 = blockIdx.x * 16;
    const int ct = blockIdx.y * NW + wave;
    constexpr int RPW = 16 / NW;  // rows per wave (each: a self row-half and an agg row-half)
    int srow_[RPW];
#pragma unroll
    for (int i = 0; i < RPW; ++i) srow_[i] = sidx[min(m0 + wave * RPW + i, n - 1)];
    uint4 sv[RPW], gv[RPW];
#pragma unroll
    for (int i = 0; i < RPW; ++i) sv[i] = reinterpret_cast<const uint4*>(Xs + (int64_t)srow_[i] * ldxs)[lane];
#pragma unroll
    for (int i = 0; i < RPW; ++i)
        gv[i] = reinterpret_cast<const uint4*>(A + (int64_t)min(m0 + wave * RPW + i, n - 1) * lda)[lane];
    uint4 wv[D];
    auto wload = [&](int g, int u) {
        wv[u] = reinterpret_cast<const uint4*>(Wp)[((int64_t)g * (H >> 4) + ct) * 64 + lane];
    };
#pragma unroll
    for (int u = 0; u < D; ++u) wload(u, u);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < RPW; ++i) *reinterpret_cast<uint4*>(sA + (wave * RPW + i) * PITCH + lane * 4) = sv[i];
    __syncthreads();
    unsigned long long t_a = 0;
    if (stamps) t_a = __builtin_amdgcn_s_memrealtime();
    f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int g = 0; g < NG; ++g) {
        if (g == NG / 2) {  // the agg half: store (its loads have had the self half's MFMAs to land), publish
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int i = 0; i < RPW; ++i)
                *reinterpret_cast<uint4*>(sA + (wave * RPW + i) * PITCH + 256 + lane * 4) = gv[i];
            __syncthreads();
        }
        const int u = g % D;
        const uint4 a = *reinterpret_cast<const uint4*>(sA + r * PITCH + 16 * g + 4 * kq);
        const uint4 w = wv[u];
        if (g + D < NG) wload(g + D, u);
        __builtin_amdgcn_sched_barrier(0);
        acc = gs::mfma_slot<float>(a, w, acc);
        __builtin_amdgcn_sched_barrier(0);
    }
    if (stamps && lane == 0) {
        const unsigned long long t_e = __builtin_amdgcn_s_memrealtime();
        unsigned long long* p = stamps + 3 * (((int64_t)blockIdx.y * gridDim.x + blockIdx.x) * NW + wave);
        p[0] = t_start; p[1] = t_a; p[2] = t_e;
    }
    const int col = ct * 16 + r;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int row = m0 + 4 * kq + j;
        const float v = acc[j];
        if (row < n) out[(int64_t)row * ldo + col] = (!(v > 0.f) && v == v) ? 0.f : v;
    }
}

// W-stationary: a wave owns one 16-column tile; its W slice (16 columns x K)
// sits in registers for the whole launch, and the wave walks row tiles
// t = bx, bx + RG, ..., loading each tile's A rows (self | agg) straight into
// registers in the MFMA operand layout (lane (r, kq): quad 4g + kq of row r
// for k group g), no LDS and no barriers.  Same operands in the same order as
// the chunked kernel: bitwise equal.  PF: the next tile's A is loaded under
// the current tile's MFMAs.
template <bool PF>
__global__ __launch_bounds__(256, 2) void fwd_wreg_kernel(int n, int F, int H, const float* __restrict__ Xs,
                                                          int64_t ldxs, const int* __restrict__ sidx,
                                                          const float* __restrict__ A, int64_t lda,
                                                          const float* __restrict__ W, float* __restrict__ out,
                                                          int64_t ldo, unsigned long long* __restrict__ stamps) {
    unsigned long long t_start = 0;
    if (stamps) t_start = __builtin_amdgcn_s_memrealtime();
    constexpr int K = 512, NG = 32, R = 16;  // A ring: 16 groups = one half (self or agg) of a tile
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int r = lane & 15, kq = lane >> 4;
    const int ct = blockIdx.y * 4 + wave;
    uint4 w[NG];
    {
        const float* wrow = W + (int64_t)(16 * ct + r) * K + 4 * kq;
#pragma unroll
        for (int g = 0; g < NG; ++g) w[g] = *reinterpret_cast<const uint4*>(wrow + 16 * g);
    }
    const int ntiles = (n + 15) / 16;
    uint4 a[R];
    unsigned long long t_a = 0;
    int t = blockIdx.x;
    if (t >= ntiles) return;
    // half h of tile t: h = 0 the self row X[sidx], 1 the aggregate row
    auto src = [&](int tt, int h) -> const float* {
        const int row = min(16 * tt + r, n - 1);
        return (h ? A + (int64_t)row * lda : Xs + (int64_t)sidx[row] * ldxs) + 4 * kq;
    };
    {
        const float* p = src(t, 0);
#pragma unroll
        for (int g = 0; g < R; ++g) a[g] = *reinterpret_cast<const uint4*>(p + 16 * g);
    }
    for (; t < ntiles; t += gridDim.x) {
        const int tn = t + gridDim.x;
        f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
        const float* p1 = src(t, 1);
#pragma unroll
        for (int g = 0; g < R; ++g) {  // self half; refill with the agg half
            acc = gs::mfma_slot<float>(a[g], w[g], acc);
            a[g] = *reinterpret_cast<const uint4*>(p1 + 16 * g);
        }
        const bool more = PF && tn < ntiles;
        const float* p0 = more ? src(tn, 0) : p1;
#pragma unroll
        for (int g = 0; g < R; ++g) {  // agg half; refill with the next tile's self half
            acc = gs::mfma_slot<float>(a[g], w[R + g], acc);
            if (more) a[g] = *reinterpret_cast<const uint4*>(p0 + 16 * g);
        }
        if (stamps && t_a == 0) t_a = __builtin_amdgcn_s_memrealtime();
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int row = 16 * t + 4 * kq + j;
            if (row < n) {
                const float v = acc[j];
                out[(int64_t)row * ldo + 16 * ct + r] = (!(v > 0.f) && v == v) ? 0.f : v;
            }
        }
        if (!PF && tn < ntiles) {
            const float* q = src(tn, 0);
#pragma unroll
            for (int g = 0; g < R; ++g) a[g] = *reinterpret_cast<const uint4*>(q + 16 * g);
        }
    }
    if (stamps && lane == 0) {
        const unsigned long long t_e = __builtin_amdgcn_s_memrealtime();
        unsigned long long* p = stamps + 3 * (((int64_t)blockIdx.y * gridDim.x + blockIdx.x) * 4 + wave);
        p[0] = t_start; p[1] = t_a ? t_a : t_e; p[2] = t_e;
    }
}

template <int N>
__device__ __forceinline__ void wait_vm() {  // s_waitcnt vmcnt(N), other counters untouched
    static_assert(N >= 0 && N < 64, "vmcnt range");
    __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}

// W-stationary, one block per CU: block b owns column half h = (b >> 3) & 1
// and the row tiles p, p + NP, p + 2 NP of pair p = (b >> 4) * 8 + (b & 7)
// (blocks b and b + 8 -- one XCD under round-robin placement -- are the two
// halves of a pair, so a tile's A rows come from HBM once).  Wave w keeps its
// 16-column slice of W (all K) in registers, loaded once; the block's tiles
// (16 rows of [X[sidx] | A], 2 KiB each) land in LDS by DMA (one 1 KiB
// row-half per wave instruction: waves 0, 2 the self halves, 1, 3 the agg
// halves), issued tile 0 first, then W, then the rest; every count is a
// compile-time constant (CNT tiles) so the waits are exact.  Same MFMA
// operands in the same order as the chunked kernel: bitwise equal.
template <int CNT, bool PACKED>
__device__ __forceinline__ void wstat_body(int n, int H, const float* __restrict__ Xs, int64_t ldxs,
                                           const int* __restrict__ sidx, const float* __restrict__ A, int64_t lda,
                                           const float* __restrict__ W, float* __restrict__ out, int64_t ldo,
                                           int h, int p, int NP, float* sA, unsigned long long* stamp) {
    constexpr int K = 512, NG = 32, PITCH = K + 4;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int r = lane & 15, kq = lane >> 4;
    const int half = wave & 1;
    // this wave's source rows: lane l < 8 * CNT -> tile l >> 3, row (wave >> 1) + 2 (l & 7)
    int myrow = 0;
    {
        const int li = min(lane, 8 * CNT - 1);
        const int gr = min(16 * (p + (li >> 3) * NP) + (wave >> 1) + 2 * (li & 7), n - 1);
        myrow = half ? gr : sidx[gr];
    }
    const float* base = half ? A : Xs;
    const int64_t ld = half ? lda : ldxs;
    // register staging: tile i's 8 row-halves of this wave, 16 B per lane
    // each, two tiles in flight (tile 2 reuses tile 0's registers once they
    // are in LDS)
    // (eight named registers per tile: no private array for the compiler to
    // leave in scratch)
#define GS_LAB_STG(M) M(0) M(1) M(2) M(3) M(4) M(5) M(6) M(7)
    uint4 s0_0, s0_1, s0_2, s0_3, s0_4, s0_5, s0_6, s0_7;
    uint4 s1_0, s1_1, s1_2, s1_3, s1_4, s1_5, s1_6, s1_7;
#define GS_LAB_LD(q) dst##q = *reinterpret_cast<const uint4*>(base + (int64_t)__builtin_amdgcn_readlane(myrow, 8 * i + q) * ld + 4 * lane);
#define GS_LAB_ST(q) *reinterpret_cast<uint4*>(sA + (i * 16 + (wave >> 1) + 2 * q) * PITCH + half * (K / 2) + 4 * lane) = src##q;
    auto load_tile = [&](int i, uint4& dst0, uint4& dst1, uint4& dst2, uint4& dst3, uint4& dst4, uint4& dst5,
                         uint4& dst6, uint4& dst7) __attribute__((always_inline)) { GS_LAB_STG(GS_LAB_LD) };
    auto stage = [&](int i, const uint4& src0, const uint4& src1, const uint4& src2, const uint4& src3,
                     const uint4& src4, const uint4& src5, const uint4& src6, const uint4& src7)
                     __attribute__((always_inline)) {
        GS_LAB_STG(GS_LAB_ST)
        __syncthreads();
    };
#define GS_LAB_S0 s0_0, s0_1, s0_2, s0_3, s0_4, s0_5, s0_6, s0_7
#define GS_LAB_S1 s1_0, s1_1, s1_2, s1_3, s1_4, s1_5, s1_6, s1_7
    load_tile(0, GS_LAB_S0);
    uint4 w[NG];
    if constexpr (PACKED) {  // Wp[g][ct][lane]: one coalesced 1 KiB read per group
        const uint4* wp = reinterpret_cast<const uint4*>(W) + (4 * h + wave) * 64 + lane;
#pragma unroll
        for (int g = 0; g < NG; ++g) w[g] = wp[(int64_t)g * (H / 16) * 64];
    } else {
        const float* wrow = W + (int64_t)(64 * h + 16 * wave + r) * K + 4 * kq;
#pragma unroll
        for (int g = 0; g < NG; ++g) w[g] = *reinterpret_cast<const uint4*>(wrow + 16 * g);
    }
    if constexpr (CNT > 1) load_tile(1, GS_LAB_S1);
    auto compute = [&](int i) __attribute__((always_inline)) {
        const float* ar = sA + (i * 16 + r) * PITCH + 4 * kq;
        f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int g = 0; g < NG; ++g) {
            const uint4 a = *reinterpret_cast<const uint4*>(ar + 16 * g);
            acc = gs::mfma_slot<float>(a, w[g], acc);
        }
        const int t = p + i * NP;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int row = 16 * t + 4 * kq + j;
            if (row < n) {
                const float v = acc[j];
                out[(int64_t)row * ldo + 64 * h + 16 * wave + r] = (!(v > 0.f) && v == v) ? 0.f : v;
            }
        }
    };
    stage(0, GS_LAB_S0);
    if (stamp && (threadIdx.x & 63) == 0) stamp[1] = __builtin_amdgcn_s_memrealtime();
    if constexpr (CNT > 2) load_tile(2, GS_LAB_S0);
    compute(0);
    if constexpr (CNT > 1) {
        stage(1, GS_LAB_S1);
        compute(1);
    }
    if constexpr (CNT > 2) {
        stage(2, GS_LAB_S0);
        compute(2);
    }
}

template <int MAXT, bool PACKED>
__global__ __launch_bounds__(256, 1) void fwd_wstat_kernel(int n, int F, int H, const float* __restrict__ Xs,
                                                           int64_t ldxs, const int* __restrict__ sidx,
                                                           const float* __restrict__ A, int64_t lda,
                                                           const float* __restrict__ W, float* __restrict__ out,
                                                           int64_t ldo, unsigned long long* __restrict__ stamps) {
    static_assert(MAXT >= 1 && MAXT <= 3, "tiles per block");
    unsigned long long t_start = 0;
    if (stamps) t_start = __builtin_amdgcn_s_memrealtime();
    unsigned long long* ta = stamps ? stamps + 3 * ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) : nullptr;
    extern __shared__ __attribute__((aligned(16))) float sA[];  // [MAXT * 16][K + 4]
    const int b = blockIdx.x, NP = gridDim.x >> 1;
    const int h = (b >> 3) & 1, p = (b >> 4) * 8 + (b & 7);
    const int ntiles = (n + 15) / 16;
    const int cnt = p < ntiles ? min(MAXT, (ntiles - p + NP - 1) / NP) : 0;
    switch (cnt) {
        case 1: wstat_body<1, PACKED>(n, H, Xs, ldxs, sidx, A, lda, W, out, ldo, h, p, NP, sA, ta); break;
        case 2: if constexpr (MAXT >= 2) wstat_body<2, PACKED>(n, H, Xs, ldxs, sidx, A, lda, W, out, ldo, h, p, NP, sA, ta); break;
        case 3: if constexpr (MAXT >= 3) wstat_body<3, PACKED>(n, H, Xs, ldxs, sidx, A, lda, W, out, ldo, h, p, NP, sA, ta); break;
        default: break;
    }
    if (stamps && (threadIdx.x & 63) == 0) {
        const unsigned long long t_e = __builtin_amdgcn_s_memrealtime();
        unsigned long long* q = stamps + 3 * ((int64_t)b * 4 + (threadIdx.x >> 6));
        q[0] = t_start; if (cnt == 0) q[1] = t_e; q[2] = t_e;
    }
}

}  // namespace lab

static unsigned long long* g_stamps = nullptr;  // set for one instrumented launch

struct Variant {
    const char* name;
    void (*launch)(int n, int F, int H, const float* X, const int* sidx, const float* A, const float* W,
                   const float* Wp, float* out, hipStream_t st);
    int nw = 0;  // waves per block of an instrumented variant (0: none)
};

static void run_default(int n, int F, int H, const float* X, const int* sidx, const float* A, const float* W,
                        const float* Wp, float* out, hipStream_t st) {
    const int K = 2 * F;
    dim3 grid((n + 31) / 32, (H + 63) / 64);
    gs::linear_fwd_wide_kernel<32, true, true><<<grid, 512, 0, st>>>(n, F, H, K, X, F, sidx, A, F, W, out, H);
}

template <int CW, int NW, int D, bool PACKED>
static void run_rows(int n, int F, int H, const float* X, const int* sidx, const float* A, const float* W,
                     const float* Wp, float* out, hipStream_t st) {
    dim3 grid((n + 15) / 16, H / (CW * NW));
    lab::fwd_rows_kernel<32, CW, NW, D, PACKED><<<grid, NW * 64, 0, st>>>(n, F, H, X, F, sidx, A, F,
                                                                         PACKED ? Wp : W, out, H, g_stamps);
}

template <int KS, int D>
static void run_t32(int n, int F, int H, const float* X, const int* sidx, const float* A, const float* W,
                    const float* Wp, float* out, hipStream_t st) {
    const int tiles = (n + 31) / 32;
    const int nb = ((tiles + 7) / 8) * 16;
    lab::fwd_t32_kernel<KS, D><<<nb, 256 * KS, 0, st>>>(n, F, H, X, F, sidx, A, F, Wp, out, H, g_stamps);
}

template <bool PF, int RG>
static void run_wreg(int n, int F, int H, const float* X, const int* sidx, const float* A, const float* W,
                     const float* Wp, float* out, hipStream_t st) {
    const int tiles = (n + 15) / 16;
    dim3 grid(std::min(tiles, RG), H / 64);
    lab::fwd_wreg_kernel<PF><<<grid, 256, 0, st>>>(n, F, H, X, F, sidx, A, F, W, out, H, g_stamps);
}

template <int MAXT, bool FILL, bool PACKED = false>
static void run_wstat(int n, int F, int H, const float* X, const int* sidx, const float* A, const float* W,
                      const float* Wp, float* out, hipStream_t st) {
    static bool attr = false;
    const int smem = MAXT * 16 * 516 * 4;
    if (!attr) {
        CK(hipFuncSetAttribute(reinterpret_cast<const void*>(lab::fwd_wstat_kernel<MAXT, PACKED>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, smem));
        attr = true;
    }
    const int tiles = (n + 15) / 16;
    int np = FILL ? 128 : ((tiles + MAXT - 1) / MAXT + 7) / 8 * 8;  // pairs (FILL: one block per CU)
    while (np * MAXT < tiles) np += 8;
    lab::fwd_wstat_kernel<MAXT, PACKED><<<2 * np, 256, smem, st>>>(n, F, H, X, F, sidx, A, F, PACKED ? Wp : W, out, H,
                                                                   g_stamps);
}

template <int NW, int D>
static void run_2ph(int n, int F, int H, const float* X, const int* sidx, const float* A, const float* W,
                    const float* Wp, float* out, hipStream_t st) {
    dim3 grid((n + 15) / 16, H / 16 / NW);
    lab::fwd_2ph_kernel<NW, D><<<grid, NW * 64, 0, st>>>(n, F, H, X, F, sidx, A, F, Wp, out, H, g_stamps);
}

int main(int argc, char** argv) {
    const int n = argc > 1 ? std::atoi(argv[1]) : 4400;
    const int reps = argc > 2 ? std::atoi(argv[2]) : 50;
    const int64_t N = int64_t(1) << 21;
    const int F = 256, H = 128, K = 512;
    std::mt19937 gen(7);
    std::uniform_real_distribution<float> U(-1.f, 1.f);
    std::vector<float> hX(N * F), hA((size_t)n * F), hW((size_t)H * K);
    for (auto& v : hX) v = U(gen);
    for (auto& v : hA) v = U(gen);
    for (auto& v : hW) v = U(gen) * 0.05f;
    std::vector<int> hs(n);
    const int mode = argc > 3 ? std::atoi(argv[3]) : 0;  // 0 random rows, 1 rows 0..n-1, 2 random of the first 64Ki rows
    for (int i = 0; i < n; ++i)
        hs[i] = mode == 1 ? i : mode == 2 ? static_cast<int>(gen() % 65536) : static_cast<int>(gen() % N);
    std::printf("self rows: %s\n", mode == 1 ? "contiguous" : mode == 2 ? "random of 64Ki rows (64 MiB)" : "random of 2Mi rows (2 GiB)");
    // packed W: Wp[g][ct][lane] = W[16ct + (lane&15)][16g + 4(lane>>4) .. +3]
    std::vector<float> hWp((size_t)H * K);
    for (int g = 0; g < K / 16; ++g)
        for (int ct = 0; ct < H / 16; ++ct)
            for (int l = 0; l < 64; ++l)
                for (int e = 0; e < 4; ++e)
                    hWp[(((size_t)g * (H / 16) + ct) * 64 + l) * 4 + e] =
                        hW[(size_t)(16 * ct + (l & 15)) * K + 16 * g + 4 * (l >> 4) + e];
    float *X, *A, *W, *Wp, *out, *ref;
    int* sidx;
    char* flush;
    const size_t FL = size_t(512) << 20;
    CK(hipMalloc(&X, hX.size() * 4));
    CK(hipMalloc(&A, hA.size() * 4));
    CK(hipMalloc(&W, hW.size() * 4));
    CK(hipMalloc(&Wp, hWp.size() * 4));
    CK(hipMalloc(&out, (size_t)n * H * 4));
    CK(hipMalloc(&ref, (size_t)n * H * 4));
    CK(hipMalloc(&sidx, n * 4));
    CK(hipMalloc(&flush, FL));
    CK(hipMemcpy(X, hX.data(), hX.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(A, hA.data(), hA.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(W, hW.data(), hW.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(Wp, hWp.data(), hWp.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(sidx, hs.data(), n * 4, hipMemcpyHostToDevice));
    hipStream_t st;
    CK(hipStreamCreate(&st));
    run_default(n, F, H, X, sidx, A, W, Wp, ref, st);
    CK(hipStreamSynchronize(st));
    std::vector<float> hr((size_t)n * H), ho((size_t)n * H);
    CK(hipMemcpy(hr.data(), ref, hr.size() * 4, hipMemcpyDeviceToHost));
    {  // fp64 check of the default on a few rows
        double maxe = 0;
        for (int i = 0; i < n; i += 97)
            for (int c = 0; c < H; ++c) {
                double s = 0;
                for (int k = 0; k < K; ++k)
                    s += double(hW[(size_t)c * K + k]) * (k < F ? hX[(size_t)hs[i] * F + k] : hA[(size_t)i * F + k - F]);
                s = s > 0 ? s : 0;
                maxe = std::max(maxe, std::fabs(s - hr[(size_t)i * H + c]));
            }
        std::printf("default vs fp64: max abs err %.3g\n", maxe);
    }
    Variant vs[] = {
        {"default wide<32>", run_default},
        {"rows packed CW16 NW4 D8 (64 cols)", run_rows<16, 4, 8, true>},
        {"rows packed CW16 NW4 D2 (64 cols)", run_rows<16, 4, 2, true>},
        {"t32 KS1 D2", run_t32<1, 2>, -4},
        {"t32 KS2 D2", run_t32<2, 2>, -8},
        {"2ph NW8 D4", run_2ph<8, 4>, 8},
        {"wstat MAXT3 256 blocks", run_wstat<3, true>, 4},
        {"wstat MAXT3 184 blocks", run_wstat<3, false>, 4},
        {"wstat packed MAXT3 256 blocks", run_wstat<3, true, true>, 4},
        {"wstat packed MAXT3 184 blocks", run_wstat<3, false, true>, 4},
        {"wreg RG256", run_wreg<false, 256>, 4},
        {"wreg PF RG256", run_wreg<true, 256>, 4},
    };
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (auto& v : vs) {
        CK(hipMemset(out, 0, (size_t)n * H * 4));
        v.launch(n, F, H, X, sidx, A, W, Wp, out, st);
        CK(hipStreamSynchronize(st));
        CK(hipGetLastError());
        CK(hipMemcpy(ho.data(), out, ho.size() * 4, hipMemcpyDeviceToHost));
        const bool same = std::memcmp(ho.data(), hr.data(), ho.size() * 4) == 0;
        double t[2];
        for (int cold = 0; cold < 2; ++cold) {
            std::vector<float> ms;
            for (int i = 0; i < reps; ++i) {
                if (cold) CK(hipMemsetAsync(flush, i & 0xff, FL, st));
                CK(hipEventRecord(e0, st));
                v.launch(n, F, H, X, sidx, A, W, Wp, out, st);
                CK(hipEventRecord(e1, st));
                CK(hipEventSynchronize(e1));
                float m;
                CK(hipEventElapsedTime(&m, e0, e1));
                ms.push_back(m);
            }
            std::sort(ms.begin(), ms.end());
            t[cold] = ms[ms.size() / 2] * 1e3;
        }
        if (v.nw) {  // one cold instrumented launch: per-wave phase times (s_memrealtime, 100 MHz)
            const int nwv = v.nw > 0 ? v.nw : -v.nw;
            const int nb = v.nw > 0 ? ((n + 15) / 16) * (H / 16 / v.nw) * v.nw : (((n + 31) / 32 + 7) / 8) * 16 * nwv;
            unsigned long long* ds;
            CK(hipMalloc(&ds, (size_t)nb * 3 * 8));
            CK(hipMemset(ds, 0, (size_t)nb * 3 * 8));
            CK(hipMemsetAsync(flush, 7, FL, st));
            g_stamps = ds;
            v.launch(n, F, H, X, sidx, A, W, Wp, out, st);
            g_stamps = nullptr;
            CK(hipStreamSynchronize(st));
            std::vector<unsigned long long> hs3((size_t)nb * 3);
            CK(hipMemcpy(hs3.data(), ds, hs3.size() * 8, hipMemcpyDeviceToHost));
            CK(hipFree(ds));
            unsigned long long t0 = ~0ull, t1 = 0, smax = 0;
            std::vector<double> pa, pk;
            CK(hipMemset(ds, 0, 0));
            for (int i = 0; i < nb; ++i) {
                if (hs3[3 * i] == 0) continue;  // spare block / non-stamping wave
                t0 = std::min(t0, hs3[3 * i]);
                t1 = std::max(t1, hs3[3 * i + 2]);
                smax = std::max(smax, hs3[3 * i]);
                pa.push_back((hs3[3 * i + 1] - hs3[3 * i]) * 0.01);
                pk.push_back((hs3[3 * i + 2] - hs3[3 * i + 1]) * 0.01);
            }
            std::sort(pa.begin(), pa.end());
            std::sort(pk.begin(), pk.end());
            std::printf("   phases (us): span %.2f, last wave start %.2f; A-load med %.2f p90 %.2f; K-loop med %.2f p90 %.2f max %.2f\n",
                        (t1 - t0) * 0.01, (smax - t0) * 0.01, pa[pa.size() / 2], pa[pa.size() * 9 / 10],
                        pk[pk.size() / 2], pk[pk.size() * 9 / 10], pk.back());
        }
        const double fl = 2.0 * n * K * H;
        std::printf("%-36s %s  warm %7.2f us (%5.1f TF)  cold %7.2f us (%5.1f TF)\n", v.name,
                    same ? "bitwise=default" : "DIFFERS        ", t[0], fl / t[0] / 1e6, t[1], fl / t[1] / 1e6);
    }
    return 0;
}
