#pragma once
// Loss-head slab reduce and the clip/SGD parameter groups, shared by the
// C-ABI launchers (misc.hip) and the fused backward launches (bwd.hip).
#include "kcommon.hpp"

namespace gs {

constexpr int kClsRedThreads = 256;

// Element t of the [C][D+1] (+ loss) classifier partials summed over the
// row blocks' slabs (cls_rows_kernel writes them): dWc, dbc and the mean NLL.
// Block = 64 elements x 4 waves; wave q adds the slabs of its quarter of the
// row blocks in order and wave 0 adds the four part sums in wave order (fixed,
// no atomics): at B = 512 (128 row blocks) one round of 32 loads per thread
// instead of four (GS_CLS_RED_SEQ: one thread per element over every slab).
// With `part`, block bx also writes Σ of its dWc/dbc elements squared to
// part[bx].
#ifndef GS_CLS_RED_SEQ
#define GS_CLS_RED_SEQ 0
#endif
constexpr int kClsRedCols = GS_CLS_RED_SEQ ? kClsRedThreads : 64;
__device__ __forceinline__ void cls_reduce_body(int bx, int B, int D, int C, int n_blocks,
                                                const float* __restrict__ slab, float* __restrict__ dWc,
                                                float* __restrict__ dbc, float* __restrict__ loss,
                                                float* __restrict__ part) {
    const int per = C * (D + 1);
    constexpr int P = kClsRedThreads / kClsRedCols;  // slab parts per element
    const int q = threadIdx.x / kClsRedCols;
    const int t = bx * kClsRedCols + threadIdx.x % kClsRedCols;
    const int tc = min(t, per);
    const int nq = (n_blocks + P - 1) / P;
    const int k0 = min(n_blocks, q * nq), k1 = min(n_blocks, k0 + nq);
    float s = 0.f;
#pragma unroll 32  // one round of loads for the usual <= 32 row blocks per part
    for (int k = k0; k < k1; ++k) s += slab[static_cast<int64_t>(k) * (per + 1) + tc];
    if constexpr (P > 1) {
        __shared__ float red[P > 1 ? P - 1 : 1][kClsRedCols];
        if (q > 0) red[q - 1][threadIdx.x % kClsRedCols] = s;
        __syncthreads();
        if (q == 0)
#pragma unroll
            for (int p = 0; p < P - 1; ++p) s += red[p][threadIdx.x];
    }
    const bool own = q == 0;
    if (own && t == per) loss[0] = s / static_cast<float>(B);  // -sum(logp[i, y_i]) / B  (utils.py:162-163)
    if (own && t < per) {
        const int c = t / (D + 1), d = t - c * (D + 1);
        if (d < D) dWc[static_cast<int64_t>(c) * D + d] = s;
        else dbc[c] = s;
    }
    if (part) block_sum_to(own && t < per ? s * s : 0.f, part + bx);
}

inline int cls_reduce_blocks(int64_t C, int64_t D) {
    return static_cast<int>((C * (D + 1) + 1 + kClsRedCols - 1) / kClsRedCols);
}

// Parameter groups of the clip (utils.py:186-187: one clip_grad_norm_ per
// model): flat offsets, and per group npart norm partials at part + g·pstride.
struct Groups {
    int64_t off[9];
    int npart[8];
    int n, pstride;
    bf16_t* sh = nullptr;  // bf16 shadow of params [sh_lo, sh_hi) (g_lowp_shadow), or none
    int64_t sh_lo = 0, sh_hi = 0;
};

// Host-visible step-completion flag (kcommon.hpp DoneFlag), stored by the
// first thread of the launch.
__device__ __forceinline__ void signal_done(int64_t* done, int64_t value) {
    if (done && blockIdx.x == 0 && threadIdx.x == 0)
        __hip_atomic_store(done, value, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// One group's squared norm from its np partials, as every clip of this
// library folds them (lane-strided, then a fixed xor tree; identical on every
// lane, in every kernel, for any block size).
__device__ __forceinline__ float clip_fold(const float* __restrict__ pg, int np, int lane) {
    float t = 0.f;
    constexpr int kPre = 8;
    if (np > 0 && np <= 64 * kPre) {
        // every partial of the lane loaded before the first add (clamped
        // addresses, the count tested after the loads): one memory round;
        // adding +0 past the count leaves t unchanged
        float v[kPre];
#pragma unroll
        for (int u = 0; u < kPre; ++u) v[u] = pg[min(lane + 64 * u, np - 1)];
#pragma unroll
        for (int u = 0; u < kPre; ++u) t += lane + 64 * u < np ? v[u] : 0.f;
    } else {
#pragma unroll 4
        for (int b = lane; b < np; b += 64) t += pg[b];
    }
    return wave_sum(t);
}

// clip_fold in two halves, for a kernel that issues the partials' loads
// ahead of its own (np <= 512: one load per lane and u; clip_fold's sums).
struct FoldLoads {
    float v[8];
};
__device__ __forceinline__ void clip_fold_issue(const float* __restrict__ pg, int np, int lane, FoldLoads& f) {
#pragma unroll
    for (int u = 0; u < 8; ++u) f.v[u] = pg[min(lane + 64 * u, max(np, 1) - 1)];  // np >= 1 (the caller's)
}
__device__ __forceinline__ float clip_fold_finish(int np, int lane, const FoldLoads& f) {
    float t = 0.f;
#pragma unroll
    for (int u = 0; u < 8; ++u) t += lane + 64 * u < np ? f.v[u] : 0.f;
    return wave_sum(t);
}

// clip_grad_norm_'s coefficient (utils.py:186), times the gradient scale.
__device__ __forceinline__ float clip_mult(float sumsq, float scale, float max_norm) {
    const float norm = sqrtf(sumsq) * scale;
    return scale * fminf(max_norm / (norm + 1e-6f), 1.0f);
}

// One parameter's clip + SGD step: the clipped gradient to gi, the new value
// returned (p.add_(g, alpha=-lr), utils.py:190; one rounding, as contracted).
__device__ __forceinline__ float sgd_elem(float p, float g, float m, float lr, float& gi) {
    gi = g * m;
    return fmaf(-lr, gi, p);
}

// Clip (per group, utils.py:186-187) + SGD (utils.py:187-190) on float4
// (every group offset a multiple of 4, 16-B aligned arrays), block bx of
// nblk: wave w folds group w's norm partials (lane-strided loads, then a
// fixed xor-tree: the same order in every block and for any block size),
// then each thread updates its quads; each thread's first g / p quads are
// loaded before the fold, so the two dependent rounds overlap.  With G.sh the
// new params of [sh_lo, sh_hi) also go to the bf16 shadow.
__device__ __forceinline__ void sgd4_body(const Groups& G, float* __restrict__ p, float* __restrict__ g,
                                          const float* __restrict__ part, float scale, float max_norm, float lr,
                                          int bx, int nblk) {
    __shared__ float mult[8];
    const int nthr = static_cast<int>(blockDim.x);
    const int64_t n4 = G.off[G.n] / 4;
    const int64_t i0 = bx * int64_t(nthr) + threadIdx.x;
    float4* g4 = reinterpret_cast<float4*>(g);
    float4* p4 = reinterpret_cast<float4*>(p);
    float4 gv = make_float4(0.f, 0.f, 0.f, 0.f), pv = gv;
    if (i0 < n4) {
        gv = g4[i0];
        pv = p4[i0];
    }
    const int lane = threadIdx.x & 63;
    // the group index wave-uniform in an SGPR: its npart is a scalar kernarg
    // load, not a vector load whose wait would also drain the g / p loads above
    for (int grp = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); grp < G.n; grp += nthr / 64) {
        const float t = clip_fold(part + grp * G.pstride, G.npart[grp], lane);
        if (lane == 0) mult[grp] = clip_mult(t, scale, max_norm);
    }
    __syncthreads();
    for (int64_t i = i0; i < n4; i += int64_t(nblk) * nthr) {
        if (i != i0) {
            gv = g4[i];
            pv = p4[i];
        }
        int grp = 0;
        while (4 * i >= G.off[grp + 1]) ++grp;
        const float m = mult[grp];
        float4 gi, pn;
        pn.x = sgd_elem(pv.x, gv.x, m, lr, gi.x);
        pn.y = sgd_elem(pv.y, gv.y, m, lr, gi.y);
        pn.z = sgd_elem(pv.z, gv.z, m, lr, gi.z);
        pn.w = sgd_elem(pv.w, gv.w, m, lr, gi.w);
        g4[i] = gi;
        p4[i] = pn;
        if (G.sh && 4 * i >= G.sh_lo && 4 * i < G.sh_hi) {  // sh_lo, sh_hi multiples of 4
            uint2 b;
            b.x = static_cast<uint32_t>(f2bf(pn.x)) | (static_cast<uint32_t>(f2bf(pn.y)) << 16);
            b.y = static_cast<uint32_t>(f2bf(pn.z)) | (static_cast<uint32_t>(f2bf(pn.w)) << 16);
            *reinterpret_cast<uint2*>(G.sh + (4 * i - G.sh_lo)) = b;
        }
    }
}

}  // namespace gs
