// Small kernels around the hot path: the synthetic feature table, the
// classification head + NLL loss (models.py:8-27, utils.py:159-164), gradient
// clipping + SGD (utils.py:185-187) and the f32 -> bf16 weight cast.
#include <algorithm>
#include <cmath>

#include "kcommon.hpp"

namespace gs {

constexpr int kTb = 256;

// Counter hash of (seed, row, col) -> U(-1, 1) with 2^-23 resolution (exact in
// fp32).  Mirrored in gs_uniform_host and in the Python/numpy test helpers.
__host__ __device__ __forceinline__ float uniform_hash(uint64_t seed, uint64_t row, uint64_t col) {
    uint64_t z = seed * 0x9E3779B97F4A7C15ull + row * 0xBF58476D1CE4E5B9ull + col * 0x94D049BB133111EBull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    const int32_t m = static_cast<int32_t>(z >> 40) - (1 << 23);
    return static_cast<float>(m) * (1.0f / 8388608.0f);
}

template <typename T>
__global__ __launch_bounds__(kTb) void fill_uniform_kernel(T* X, int64_t N, int64_t F, int64_t ld, uint64_t seed) {
    const int64_t total = N * F;
    for (int64_t i = blockIdx.x * int64_t(kTb) + threadIdx.x; i < total; i += int64_t(gridDim.x) * kTb) {
        const int64_t r = i / F, c = i - r * F;
        const float v = uniform_hash(seed, r, c);
        if constexpr (sizeof(T) == 4) X[r * ld + c] = v;
        else X[r * ld + c] = f2bf(v);
    }
}

__global__ __launch_bounds__(kTb) void cast_bf16_kernel(const float* in, bf16_t* out, int64_t n) {
    for (int64_t i = blockIdx.x * int64_t(kTb) + threadIdx.x; i < n; i += int64_t(gridDim.x) * kTb)
        out[i] = f2bf(in[i]);
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    return v;
}
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// One wavefront per row: logits (lanes over D, one wave reduction per class),
// log_softmax (max-shifted, as torch), the row's NLL term, dlogits =
// (softmax - onehot) / B, and dE[i] = dlogits · Wc (lanes over D again).
constexpr int kClsMaxC = 1024;
__global__ __launch_bounds__(kTb) void cls_rows_kernel(int B, int D, int C, const float* __restrict__ E,
                                                       const float* __restrict__ Wc, const float* __restrict__ bc,
                                                       const int* __restrict__ labels, float* __restrict__ dl,
                                                       float* __restrict__ rowloss, float* __restrict__ dE) {
    __shared__ float zs[kTb / 64][kClsMaxC];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int i = blockIdx.x * (kTb / 64) + w;
    if (i >= B) return;
    const float* e = E + static_cast<int64_t>(i) * D;
    const int y = labels[i];
    float mx = -INFINITY;
    for (int c = 0; c < C; ++c) {
        const float* wr = Wc + static_cast<int64_t>(c) * D;
        float p = 0.f;
        for (int d = lane; d < D; d += 64) p = fmaf(e[d], wr[d], p);
        const float z = wave_sum(p) + bc[c];
        if (lane == 0) zs[w][c] = z;
        mx = fmaxf(mx, z);
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the row's logits are in LDS
    __builtin_amdgcn_wave_barrier();
    float se = 0.f;
    for (int c = lane; c < C; c += 64) se += expf(zs[w][c] - mx);
    const float lse = logf(wave_sum(se));
    const float invB = 1.0f / static_cast<float>(B);
    for (int c = lane; c < C; c += 64) {
        const float lp = zs[w][c] - mx - lse;
        if (c == y) rowloss[i] = -lp;
        const float g = (expf(lp) - (c == y ? 1.f : 0.f)) * invB;
        dl[static_cast<int64_t>(i) * C + c] = g;
        zs[w][c] = g;
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_wave_barrier();
    for (int d = lane; d < D; d += 64) {
        float s = 0.f;
        for (int c = 0; c < C; ++c) s = fmaf(zs[w][c], Wc[static_cast<int64_t>(c) * D + d], s);
        dE[static_cast<int64_t>(i) * D + d] = s;
    }
}

// Partial dWc / dbc over a 32-row chunk: slab[chunk][c][0..D) and [c][D] (bias).
constexpr int kClsChunk = 32;
__global__ __launch_bounds__(kTb) void cls_dW_partial_kernel(int B, int D, int C, const float* __restrict__ dl,
                                                             const float* __restrict__ E, float* __restrict__ slab) {
    const int chunk = blockIdx.y;
    const int64_t t = blockIdx.x * int64_t(kTb) + threadIdx.x;
    const int64_t per = static_cast<int64_t>(C) * (D + 1);
    if (t >= per) return;
    const int c = static_cast<int>(t / (D + 1)), d = static_cast<int>(t - static_cast<int64_t>(c) * (D + 1));
    const int i0 = chunk * kClsChunk, i1 = min(B, i0 + kClsChunk);
    float s = 0.f;
#pragma unroll 8
    for (int i = i0; i < i1; ++i) {
        const float g = dl[static_cast<int64_t>(i) * C + c];
        s += (d < D) ? g * E[static_cast<int64_t>(i) * D + d] : g;
    }
    slab[chunk * per + t] = s;
}

__global__ __launch_bounds__(kTb) void cls_dW_reduce_kernel(int B, int D, int C, int n_chunks,
                                                            const float* __restrict__ slab,
                                                            const float* __restrict__ rowloss, float* __restrict__ dWc,
                                                            float* __restrict__ dbc, float* __restrict__ loss) {
    const int64_t t = blockIdx.x * int64_t(kTb) + threadIdx.x;
    const int64_t per = static_cast<int64_t>(C) * (D + 1);
    if (t < per) {
        float s = 0.f;
        for (int k = 0; k < n_chunks; ++k) s += slab[k * per + t];
        const int c = static_cast<int>(t / (D + 1)), d = static_cast<int>(t - static_cast<int64_t>(c) * (D + 1));
        if (d < D) dWc[static_cast<int64_t>(c) * D + d] = s;
        else dbc[c] = s;
    }
    if (blockIdx.x == 0 && threadIdx.x < 64) {  // -sum(logp[i, y_i]) / B  (utils.py:162-163)
        float s = 0.f;
        for (int i = threadIdx.x; i < B; i += 64) s += rowloss[i];
        s = wave_sum(s);
        if (threadIdx.x == 0) loss[0] = s / static_cast<float>(B);
    }
}

struct Groups {
    int64_t off[9];
    int n;
};

constexpr int kNormBlocks = 64;

__global__ __launch_bounds__(kTb) void group_sumsq_kernel(Groups G, const float* __restrict__ g, float* __restrict__ part) {
    __shared__ float red[kTb / 64];
    const int grp = blockIdx.y;
    const int64_t lo = G.off[grp], hi = G.off[grp + 1];
    float s = 0.f;
    for (int64_t i = lo + blockIdx.x * int64_t(kTb) + threadIdx.x; i < hi; i += int64_t(kNormBlocks) * kTb) {
        const float v = g[i];
        s = fmaf(v, v, s);
    }
    s = wave_sum(s);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        float t = 0.f;
        for (int w = 0; w < kTb / 64; ++w) t += red[w];
        part[grp * kNormBlocks + blockIdx.x] = t;
    }
}

// clip_coef = max_norm / (||scale·g|| + 1e-6), clamped to 1; mult = scale · coef.
__global__ void group_coef_kernel(int n, const float* __restrict__ part, float scale, float max_norm,
                                  float* __restrict__ mult) {
    const int grp = threadIdx.x;
    if (grp >= n) return;
    float t = 0.f;
    for (int b = 0; b < kNormBlocks; ++b) t += part[grp * kNormBlocks + b];
    const float norm = sqrtf(t) * scale;
    const float coef = fminf(max_norm / (norm + 1e-6f), 1.0f);
    mult[grp] = scale * coef;
}

__global__ __launch_bounds__(kTb) void sgd_kernel(Groups G, float* __restrict__ p, float* __restrict__ g,
                                                  const float* __restrict__ mult, float lr) {
    const int64_t total = G.off[G.n];
    for (int64_t i = blockIdx.x * int64_t(kTb) + threadIdx.x; i < total; i += int64_t(gridDim.x) * kTb) {
        int grp = 0;
        while (i >= G.off[grp + 1]) ++grp;
        const float gi = g[i] * mult[grp];
        g[i] = gi;
        p[i] = p[i] - lr * gi;
    }
}

}  // namespace gs

extern "C" {

int gs_fill_uniform(void* X, gs_dtype dt, int64_t N, int64_t F, int64_t ld, uint64_t seed, void* stream) {
    GS_API_BEGIN
    using namespace gs;
    GS_REQUIRE(X && N >= 0 && F >= 1 && ld >= F, GS_EINVAL, "bad arguments");
    const int64_t total = N * F;
    if (total == 0) return GS_OK;
    const dim3 grid(static_cast<unsigned>(std::min<int64_t>((total + kTb - 1) / kTb, 65536)));
    if (dt == GS_F32)
        fill_uniform_kernel<float><<<grid, kTb, 0, as_stream(stream)>>>(static_cast<float*>(X), N, F, ld, seed);
    else
        fill_uniform_kernel<bf16_t><<<grid, kTb, 0, as_stream(stream)>>>(static_cast<bf16_t*>(X), N, F, ld, seed);
    check_launch("gs_fill_uniform");
    GS_API_END
}

int gs_uniform_host(uint64_t seed, int64_t row0, int64_t F, int64_t n_rows, float* out) {
    GS_API_BEGIN
    GS_REQUIRE(out && F >= 1 && n_rows >= 0, GS_EINVAL, "bad arguments");
    for (int64_t r = 0; r < n_rows; ++r)
        for (int64_t c = 0; c < F; ++c) out[r * F + c] = gs::uniform_hash(seed, row0 + r, c);
    GS_API_END
}

int gs_cast_f32_bf16(const float* in, void* out, int64_t n, void* stream) {
    GS_API_BEGIN
    using namespace gs;
    GS_REQUIRE(in && out && n >= 0, GS_EINVAL, "bad arguments");
    if (n == 0) return GS_OK;
    const dim3 grid(static_cast<unsigned>(std::min<int64_t>((n + kTb - 1) / kTb, 4096)));
    cast_bf16_kernel<<<grid, kTb, 0, as_stream(stream)>>>(in, static_cast<bf16_t*>(out), n);
    check_launch("gs_cast_f32_bf16");
    GS_API_END
}

int gs_cls_nll_fwd_bwd(int64_t B, int64_t D, int64_t C, const float* E, const float* Wc, const float* bc,
                       const int32_t* labels, float* loss, float* dE, float* dWc, float* dbc, float* ws,
                       void* stream) {
    GS_API_BEGIN
    using namespace gs;
    GS_REQUIRE(B >= 1 && D >= 1 && C >= 1 && B < (1 << 30), GS_EINVAL, "bad sizes");
    GS_REQUIRE(C <= kClsMaxC, GS_EINVAL, "at most 1024 classes");
    GS_REQUIRE(E && Wc && bc && labels && loss && dE && dWc && dbc && ws, GS_EINVAL, "NULL device pointer");
    hipStream_t st = as_stream(stream);
    const int b = static_cast<int>(B), d = static_cast<int>(D), c = static_cast<int>(C);
    float* dl = ws;
    float* rowloss = ws + B * C;
    const int n_chunks = (b + kClsChunk - 1) / kClsChunk;
    float* slab = rowloss + B;
    cls_rows_kernel<<<dim3((b + 3) / 4), kTb, 0, st>>>(b, d, c, E, Wc, bc, labels, dl, rowloss, dE);
    const int64_t per = C * (D + 1);
    cls_dW_partial_kernel<<<dim3(static_cast<unsigned>((per + kTb - 1) / kTb), n_chunks), kTb, 0, st>>>(b, d, c, dl,
                                                                                                       E, slab);
    cls_dW_reduce_kernel<<<dim3(static_cast<unsigned>((per + kTb - 1) / kTb)), kTb, 0, st>>>(b, d, c, n_chunks, slab,
                                                                                             rowloss, dWc, dbc, loss);
    check_launch("gs_cls_nll_fwd_bwd");
    GS_API_END
}

int64_t gs_cls_nll_ws_floats(int64_t B, int64_t D, int64_t C) {
    const int64_t n_chunks = (B + gs::kClsChunk - 1) / gs::kClsChunk;
    return B * C + B + n_chunks * C * (D + 1);
}

int gs_clip_sgd(int32_t n_groups, const int64_t* goff_host, float* params, float* grads, float grad_scale,
                float max_norm, float lr, float* ws, void* stream) {
    GS_API_BEGIN
    using namespace gs;
    GS_REQUIRE(n_groups >= 1 && n_groups <= 8 && goff_host, GS_EINVAL, "1..8 parameter groups");
    GS_REQUIRE(params && grads && ws, GS_EINVAL, "NULL device pointer");
    Groups G;
    G.n = n_groups;
    for (int i = 0; i <= n_groups; ++i) G.off[i] = goff_host[i];
    for (int i = 0; i < n_groups; ++i) GS_REQUIRE(G.off[i] <= G.off[i + 1], GS_EINVAL, "group offsets not sorted");
    hipStream_t st = as_stream(stream);
    float* part = ws;
    float* mult = ws + n_groups * kNormBlocks;
    group_sumsq_kernel<<<dim3(kNormBlocks, n_groups), kTb, 0, st>>>(G, grads, part);
    group_coef_kernel<<<1, 64, 0, st>>>(n_groups, part, grad_scale, max_norm, mult);
    const int64_t total = G.off[n_groups];
    const dim3 grid(static_cast<unsigned>(std::max<int64_t>(1, std::min<int64_t>((total + kTb - 1) / kTb, 1024))));
    sgd_kernel<<<grid, kTb, 0, st>>>(G, params, grads, mult, lr);
    check_launch("gs_clip_sgd");
    GS_API_END
}

}  // extern "C"
