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

}  // namespace gs
