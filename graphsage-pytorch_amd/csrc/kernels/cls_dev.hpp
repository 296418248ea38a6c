#pragma once
// Loss-head slab reduce and the clip/SGD parameter groups, shared by the
// C-ABI launchers (misc.hip) and the fused backward launches (bwd.hip).
#include "kcommon.hpp"

namespace gs {

constexpr int kClsRedThreads = 256;

// Element t of the [C][D+1] (+ loss) classifier partials summed over the
// row blocks' slabs in block order (cls_rows_kernel writes them): dWc, dbc
// and the mean NLL.  With `part`, block bx also writes Σ of its dWc/dbc
// elements squared to part[bx].
__device__ __forceinline__ void cls_reduce_body(int bx, int B, int D, int C, int n_blocks,
                                                const float* __restrict__ slab, float* __restrict__ dWc,
                                                float* __restrict__ dbc, float* __restrict__ loss,
                                                float* __restrict__ part) {
    const int per = C * (D + 1);
    const int t = bx * kClsRedThreads + threadIdx.x;
    const int tc = min(t, per);
    float s = 0.f;
#pragma unroll 32  // one round of loads for the usual <= 32 row blocks
    for (int k = 0; k < n_blocks; ++k) s += slab[static_cast<int64_t>(k) * (per + 1) + tc];
    if (t == per) loss[0] = s / static_cast<float>(B);  // -sum(logp[i, y_i]) / B  (utils.py:162-163)
    if (t < per) {
        const int c = t / (D + 1), d = t - c * (D + 1);
        if (d < D) dWc[static_cast<int64_t>(c) * D + d] = s;
        else dbc[c] = s;
    }
    if (part) block_sum_to(t < per ? s * s : 0.f, part + bx);
}

inline int cls_reduce_blocks(int64_t C, int64_t D) {
    return static_cast<int>((C * (D + 1) + 1 + kClsRedThreads - 1) / kClsRedThreads);
}

// Parameter groups of the clip (utils.py:186-187: one clip_grad_norm_ per
// model): flat offsets, and per group npart norm partials at part + g·pstride.
struct Groups {
    int64_t off[9];
    int npart[8];
    int n, pstride;
};

}  // namespace gs
