// Small kernels around the hot path: the synthetic feature table, the
// classification head + NLL loss (models.py:8-27, utils.py:159-164), gradient
// clipping + SGD (utils.py:185-187) and the f32 -> bf16 weight cast.
#include <algorithm>
#include <cmath>
#include <cstdlib>

#include "cls_dev.hpp"

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


// ------------------------------------------------------- classifier + NLL
// One block of 16 waves per R <= kClsRowsMax rows, one wave per row.  Wc is staged in LDS
// (row pitch D + 1) when it fits.  Per row, lane (cl, dq) = (lane & 15,
// lane >> 4) computes the dot product of class c0 + cl over one quarter of D
// and two xor-shuffles add the quarters, so a group of 16 classes costs one
// short FMA chain instead of a wave reduction per class.  Then log_softmax
// (max-shifted, as torch), the row's NLL term, dlogits = (softmax - onehot)
// / B and dE = dlogits · Wc, optionally masked by E > 0 (the relu of the layer
// that produced E, so the caller gets dZ directly).  Labels are read through
// the roots (labels[roots[i]]).  The block then reduces its rows' dWc / dbc /
// loss into one partial slab; cls_reduce_kernel adds the slabs in a fixed
// order.
constexpr int kClsThreads = 1024;
constexpr int64_t kClsLdsFloats = 16 * 1024;  // 64 KiB
constexpr int64_t kClsWcLds = 8 * 1024;
// Rows per block.  Fewer rows per block means more blocks in flight and a
// shorter per-block partial-slab phase: at B = 512 the kernel took 12.1 us
// with 16 rows (32 blocks), 8.3 us with 8 or 4 (rocprof, in-step); the step
// ran 81.5-82.3 us with 4 against 86.9-89.1 us with 16.
// Large batches (Pubmed trains on B ~ 9.7k roots in one step) grow the rows
// per block up to kClsRowsBig until about kClsSlabTarget slabs remain: at four
// rows the slab sum read 2.4k slabs per element on 7 blocks (161 us).
constexpr int kClsRowsMax = 4;
constexpr int kClsRowsBig = 32;
constexpr int64_t kClsSlabTarget = 384;

struct ClsPlan {
    int rows;
    bool wc_lds;
    size_t smem;
};

inline ClsPlan cls_plan(int64_t B, int64_t C, int64_t D) {
    ClsPlan p;
    p.wc_lds = C * (D + 1) <= kClsWcLds;
    const int64_t fixed = p.wc_lds ? C * (D + 1) : 0;
    p.rows = 1;
    for (int r = kClsRowsMax; r > 1; r >>= 1)
        if (fixed + r * (C + D + 1) <= kClsLdsFloats) {
            p.rows = r;
            break;
        }
    // keep the one-float4-per-thread E tile (FAST) while growing
    while (p.rows >= kClsRowsMax && p.rows < kClsRowsBig && (B + p.rows - 1) / p.rows > kClsSlabTarget &&
           fixed + 2 * p.rows * (C + D + 1) <= kClsLdsFloats && 2 * p.rows * D <= 4 * kClsThreads)
        p.rows *= 2;
    p.smem = static_cast<size_t>(fixed + p.rows * (C + D + 1)) * sizeof(float);
    return p;
}

// FAST: the block's E rows and Wc are at most one float4 per thread each and
// 16-byte aligned, so the prologue is straight-line: the roots load, the E
// and Wc loads and the bias issue together, the labels load follows the roots
// alone, and nothing waits before the LDS stores (two dependent rounds).
template <bool FAST>
__global__ __launch_bounds__(kClsThreads) void cls_rows_kernel(
    int B, int D, int C, int R, int wc_lds, const float* __restrict__ E, const float* __restrict__ Wc,
    const float* __restrict__ bc, const int* __restrict__ labels, const int* __restrict__ roots, int mask_relu,
    float* __restrict__ dE, float* __restrict__ slab) {
    extern __shared__ __attribute__((aligned(16))) float sm[];
    float* sdl = sm;             // [R][C]
    float* sE = sdl + R * C;     // [R][D]
    float* sloss = sE + R * D;   // [R]
    float* sW = sloss + R;       // [C][D + 1] when wc_lds
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int cl = lane & 15, dq = lane >> 4;
    const int r0 = blockIdx.x * R;
    const int nr = min(R, B - r0);
    const float invB = 1.0f / static_cast<float>(B);
    // every global read is issued before the first barrier: the label chain
    // (roots -> labels) and the bias overlap the E / Wc tile loads
    // (addresses clamped, values selected afterwards: no load sits behind a
    // branch, so they all overlap instead of each waiting for the previous)
    const int wr_ = min(w, nr - 1);
    const int nE = nr * D, nW = wc_lds ? C * D : 0;
    const int tid = static_cast<int>(threadIdx.x);
    int y_w;
    float b_lane;
    if constexpr (FAST) {
        // stores are unconditional (out-of-range threads write a dump slot):
        // a predicated store would let the compiler sink its load behind a
        // branch, and the branch join would wait for every load in flight
        __shared__ float dump[4];
        const int root = roots[r0 + wr_];
        const float4 ev = reinterpret_cast<const float4*>(E + static_cast<int64_t>(r0) * D)[min(tid, nE / 4 - 1)];
        const float4 wv = reinterpret_cast<const float4*>(Wc)[min(tid, C * D / 4 - 1)];
        b_lane = bc[min(cl, C - 1)];
        y_w = labels[root];
        const int t = 4 * tid;
        const bool in = t < nE;
        float* de = t < R * D ? sE + t : dump;
        de[0] = in ? ev.x : 0.f;
        de[1] = in ? ev.y : 0.f;
        de[2] = in ? ev.z : 0.f;
        de[3] = in ? ev.w : 0.f;
        float* dw = t < nW ? sW + t + t / D : dump;  // D % 4 == 0: the quad stays in one row
        dw[0] = wv.x;
        dw[1] = wv.y;
        dw[2] = wv.z;
        dw[3] = wv.w;
    } else {
    y_w = labels[roots ? roots[r0 + wr_] : r0 + wr_];
    b_lane = bc[min(cl, C - 1)];
    for (int t0 = 0; t0 < R * D; t0 += 4 * kClsThreads) {
        float v[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] = E[static_cast<int64_t>(r0) * D + min(t0 + q * kClsThreads + tid, nE - 1)];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int t = t0 + q * kClsThreads + tid;
            if (t < R * D) sE[t] = t < nE ? v[q] : 0.f;
        }
    }
    for (int t0 = 0; t0 < nW; t0 += 4 * kClsThreads) {
        float v[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] = Wc[min(t0 + q * kClsThreads + tid, nW - 1)];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int t = t0 + q * kClsThreads + tid;
            if (t < nW) sW[t + t / D] = v[q];
        }
    }
    }
    __syncthreads();
    const float* W = wc_lds ? sW : Wc;
    const int wp = wc_lds ? D + 1 : D;  // row pitch of W
    const int DQ = (D + 3) / 4;
    const int d_lo = min(D, dq * DQ), d_hi = min(D, d_lo + DQ);
    for (int ii = w; ii < nr; ii += kClsThreads / 64) {
        const float* e = sE + ii * D;
        const int y = ii == w ? y_w : labels[roots ? roots[r0 + ii] : r0 + ii];
        float mx = -INFINITY;
        for (int c0 = 0; c0 < C; c0 += 16) {
            const int c = c0 + cl;
            const float* wr = W + static_cast<int64_t>(min(c, C - 1)) * wp;
            float p = 0.f;
            for (int d = d_lo; d < d_hi; ++d) p = fmaf(e[d], wr[d], p);
            p += __shfl_xor(p, 16, 64);
            p += __shfl_xor(p, 32, 64);
            const float z = p + (c0 == 0 ? b_lane : bc[min(c, C - 1)]);
            if (dq == 0 && c < C) sdl[ii * C + c] = z;
            if (c < C) mx = fmaxf(mx, z);
        }
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 64));
        __builtin_amdgcn_wave_barrier();
        float se = 0.f;
        for (int c = lane; c < C; c += 64) se += expf(sdl[ii * C + c] - mx);
        const float lse = logf(wave_sum(se));
        for (int c = lane; c < C; c += 64) {
            const float lp = sdl[ii * C + c] - mx - lse;
            if (c == y) sloss[ii] = -lp;
            sdl[ii * C + c] = (expf(lp) - (c == y ? 1.f : 0.f)) * invB;
        }
        __builtin_amdgcn_wave_barrier();
        for (int d = lane; d < D; d += 64) {
            float s = 0.f;
            for (int c = 0; c < C; ++c) s = fmaf(sdl[ii * C + c], W[static_cast<int64_t>(c) * wp + d], s);
            if (mask_relu && !(e[d] > 0.f)) s = 0.f;
            dE[static_cast<int64_t>(r0 + ii) * D + d] = s;
        }
    }
    __syncthreads();
    // block partials: [C][D+1] (column D = bias) + 1 loss term
    const int per = C * (D + 1);
    float* out = slab + static_cast<int64_t>(blockIdx.x) * (per + 1);
    for (int t = threadIdx.x; t < per; t += kClsThreads) {
        const int c = t / (D + 1), d = t - c * (D + 1);
        float s = 0.f;
        for (int ii = 0; ii < nr; ++ii) s = fmaf(sdl[ii * C + c], d < D ? sE[ii * D + d] : 1.f, s);
        out[t] = s;
    }
    if (threadIdx.x < 64) {
        float s = 0.f;
        for (int ii = threadIdx.x; ii < nr; ii += 64) s += sloss[ii];
        s = wave_sum(s);
        if (threadIdx.x == 0) out[per] = s;
    }
}

__global__ __launch_bounds__(kClsRedThreads) void cls_reduce_kernel(int B, int D, int C, int n_blocks,
                                                                    const float* __restrict__ slab,
                                                                    float* __restrict__ dWc, float* __restrict__ dbc,
                                                                    float* __restrict__ loss) {
    cls_reduce_body(blockIdx.x, B, D, C, n_blocks, slab, dWc, dbc, loss, nullptr);
}

// ------------------------------------------------------- clip + SGD
constexpr int kNormBlocks = 64;

__global__ __launch_bounds__(kTb) void group_sumsq_kernel(Groups G, const float* __restrict__ g, float* __restrict__ part) {
    __shared__ float red[kTb / 64];
    const int grp = blockIdx.y;
    const int64_t lo = G.off[grp], hi = G.off[grp + 1];
    float s = 0.f;
#pragma unroll 8
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
        part[grp * G.pstride + blockIdx.x] = t;
    }
}

// group_sumsq_kernel with the deferred update's speculative W1 (after an
// all-reduce, gs_trainer_update in deferred mode): the elements [0, n1) of
// group 0 also get S = P - lr·(scale·g) (sgd_elem with m = scale: the update
// when the clip coefficient is 1; + its bf16 copy), and the launch stores
// the step's done flag (it is the step's last).
struct SumsqSpec {
    const float* P;
    float* S;
    uint16_t* S_lp;
    int64_t n1;
    float lr, scale;
    int64_t* done;
    int64_t done_value;
};
__global__ __launch_bounds__(kTb) void group_sumsq_spec_kernel(Groups G, const float* __restrict__ g,
                                                               float* __restrict__ part, SumsqSpec sp) {
    signal_done(sp.done, sp.done_value);
    __shared__ float red[kTb / 64];
    const int grp = blockIdx.y;
    const int64_t lo = G.off[grp], hi = G.off[grp + 1];
    float s = 0.f;
#pragma unroll 8
    for (int64_t i = lo + blockIdx.x * int64_t(kTb) + threadIdx.x; i < hi; i += int64_t(kNormBlocks) * kTb) {
        const float v = g[i];
        s = fmaf(v, v, s);
        if (i < sp.n1) {
            float gi;
            const float pn = sgd_elem(sp.P[i], v, sp.scale, sp.lr, gi);
            sp.S[i] = pn;
            if (sp.S_lp) sp.S_lp[i] = f2bf(pn);
        }
    }
    s = wave_sum(s);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        float t = 0.f;
        for (int w = 0; w < kTb / 64; ++w) t += red[w];
        part[grp * G.pstride + blockIdx.x] = t;
    }
}

int sumsq_spec_launch(int32_t n_groups, const int64_t* goff_host, const float* grads, float* part, const float* P,
                      float* S, uint16_t* S_lp, int64_t n1, float lr, float scale, hipStream_t st) {
    GS_REQUIRE(n_groups >= 1 && n_groups <= 8 && goff_host && grads && part && P && S, GS_EINVAL, "sumsq_spec: bad args");
    GS_REQUIRE(goff_host[0] == 0 && n1 <= goff_host[1], GS_EINVAL, "sumsq_spec: W1 not at the front of group 0");
    Groups G;
    G.n = n_groups;
    G.pstride = kNormBlocks;
    for (int i = 0; i < n_groups; ++i) G.npart[i] = kNormBlocks;
    for (int i = 0; i <= n_groups; ++i) G.off[i] = goff_host[i];
    const SumsqSpec sp{P, S, S_lp, n1, lr, scale, g_done_flag.ptr, g_done_flag.value};
    g_done_flag = {};
    group_sumsq_spec_kernel<<<dim3(kNormBlocks, n_groups), kTb, 0, st>>>(G, grads, part, sp);
    check_launch("sumsq_spec");
    return kNormBlocks;
}

// Each block first folds the per-group partial sums (same fixed order in
// every block) into clip_coef = max_norm / (||scale·g|| + 1e-6) clamped to 1,
// then p -= lr · (scale · coef) · g and g is left scaled like torch's in-place
// clip.
__global__ __launch_bounds__(kTb) void sgd_kernel(Groups G, float* __restrict__ p, float* __restrict__ g,
                                                  const float* __restrict__ part, float scale, float max_norm,
                                                  float lr, int64_t* done, int64_t done_value) {
    signal_done(done, done_value);
    __shared__ float mult[8];
    // wave w folds group w (lane-strided loads, all in flight, then a fixed
    // xor-tree): the same order in every block
    const int lane = threadIdx.x & 63;
    for (int grp = threadIdx.x >> 6; grp < G.n; grp += kTb / 64) {
        const float* pg = part + grp * G.pstride;
        const int np = G.npart[grp];
        float t = 0.f;
#pragma unroll 4
        for (int b = lane; b < np; b += 64) t += pg[b];
        t = wave_sum(t);
        if (lane == 0) {
            const float norm = sqrtf(t) * scale;
            mult[grp] = scale * fminf(max_norm / (norm + 1e-6f), 1.0f);
        }
    }
    __syncthreads();
    const int64_t total = G.off[G.n];
    for (int64_t i = blockIdx.x * int64_t(kTb) + threadIdx.x; i < total; i += int64_t(gridDim.x) * kTb) {
        int grp = 0;
        while (i >= G.off[grp + 1]) ++grp;
        const float gi = g[i] * mult[grp];
        g[i] = gi;
        const float pn = p[i] - lr * gi;
        p[i] = pn;
        if (G.sh && i >= G.sh_lo && i < G.sh_hi) G.sh[i - G.sh_lo] = f2bf(pn);
    }
}

// sgd_kernel on float4 (sgd4_body, cls_dev.hpp).
__global__ __launch_bounds__(kTb) void sgd4_kernel(Groups G, float* __restrict__ p, float* __restrict__ g,
                                                   const float* __restrict__ part, float scale, float max_norm,
                                                   float lr, int64_t* done, int64_t done_value) {
    signal_done(done, done_value);
    sgd4_body(G, p, g, part, scale, max_norm, lr, blockIdx.x, gridDim.x);
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

int64_t gs_cls_nll_ws_floats(int64_t B, int64_t D, int64_t C) {
    const int r = gs::cls_plan(B, C, D).rows;
    const int64_t nb = (B + r - 1) / r;
    return nb * (C * (D + 1) + 1);
}

}  // extern "C"

namespace gs {

int cls_rows_launch(int64_t B, int64_t D, int64_t C, const float* E, const float* Wc, const float* bc,
                    const int32_t* labels, const int32_t* roots, int32_t mask_relu, float* dE, float* ws,
                    hipStream_t st) {
    GS_REQUIRE(B >= 1 && D >= 1 && C >= 1 && B < (1 << 30), GS_EINVAL, "bad sizes");
    GS_REQUIRE(C + D + 1 <= kClsLdsFloats, GS_EINVAL, "classes + embedding dims too large");
    GS_REQUIRE(E && Wc && bc && labels && dE && ws, GS_EINVAL, "NULL device pointer");
    const int b = static_cast<int>(B), d = static_cast<int>(D), c = static_cast<int>(C);
    const ClsPlan plan = cls_plan(B, C, D);
    const int nb = (b + plan.rows - 1) / plan.rows;
    const bool fast = roots && D % 4 == 0 && plan.rows * D <= 4 * kClsThreads && C * D <= 4 * kClsThreads &&
                      aligned16(E) && aligned16(Wc);
    if (fast)
        cls_rows_kernel<true><<<dim3(nb), kClsThreads, plan.smem, st>>>(b, d, c, plan.rows, plan.wc_lds ? 1 : 0, E, Wc,
                                                                        bc, labels, roots, mask_relu, dE, ws);
    else
        cls_rows_kernel<false><<<dim3(nb), kClsThreads, plan.smem, st>>>(b, d, c, plan.rows, plan.wc_lds ? 1 : 0, E,
                                                                         Wc, bc, labels, roots, mask_relu, dE, ws);
    check_launch("cls_rows");
    return nb;
}

void sgd_with_parts(int32_t n_groups, const int64_t* goff_host, const int* npart, int pstride, float* params,
                    float* grads, const float* part, float grad_scale, float max_norm, float lr, hipStream_t st) {
    GS_REQUIRE(n_groups >= 1 && n_groups <= 8, GS_EINVAL, "1..8 parameter groups");
    Groups G;
    G.n = n_groups;
    G.pstride = pstride;
    for (int i = 0; i < n_groups; ++i) G.npart[i] = npart[i];
    for (int i = 0; i <= n_groups; ++i) G.off[i] = goff_host[i];
    const int64_t total = G.off[n_groups];
    const LowpShadow sh = g_lowp_shadow;
    g_lowp_shadow = {};
    G.sh = sh.p;
    G.sh_lo = sh.lo;
    G.sh_hi = sh.hi;
    bool vec = aligned16(params) && aligned16(grads);
    for (int i = 0; i <= n_groups; ++i) vec = vec && G.off[i] % 4 == 0;
    vec = vec && (!sh.p || (sh.lo % 4 == 0 && sh.hi % 4 == 0 && reinterpret_cast<uintptr_t>(sh.p) % 8 == 0));
    if (vec) {  // 4.9 us -> see DESIGN §4 (rmat2m, ~100k parameters)
        const int64_t n4 = total / 4;
        const dim3 grid(static_cast<unsigned>(std::max<int64_t>(1, std::min<int64_t>((n4 + kTb - 1) / kTb, 512))));
        sgd4_kernel<<<grid, kTb, 0, st>>>(G, params, grads, part, grad_scale, max_norm, lr, g_done_flag.ptr,
                                          g_done_flag.value);
    } else {
        const dim3 grid(static_cast<unsigned>(std::max<int64_t>(1, std::min<int64_t>((total + kTb - 1) / kTb, 512))));
        sgd_kernel<<<grid, kTb, 0, st>>>(G, params, grads, part, grad_scale, max_norm, lr, g_done_flag.ptr,
                                         g_done_flag.value);
    }
    g_done_flag = {};
    check_launch("sgd");
}

}  // namespace gs

extern "C" {

int gs_cls_nll_fwd_bwd(int64_t B, int64_t D, int64_t C, const float* E, const float* Wc, const float* bc,
                       const int32_t* labels, const int32_t* roots, int32_t mask_relu, float* loss, float* dE,
                       float* dWc, float* dbc, float* ws, void* stream) {
    GS_API_BEGIN
    using namespace gs;
    GS_REQUIRE(B >= 1 && D >= 1 && C >= 1 && B < (1 << 30), GS_EINVAL, "bad sizes");
    GS_REQUIRE(C + D + 1 <= kClsLdsFloats, GS_EINVAL, "classes + embedding dims too large");
    GS_REQUIRE(E && Wc && bc && labels && loss && dE && dWc && dbc && ws, GS_EINVAL, "NULL device pointer");
    hipStream_t st = as_stream(stream);
    const int b = static_cast<int>(B), d = static_cast<int>(D), c = static_cast<int>(C);
    const int nb = cls_rows_launch(B, D, C, E, Wc, bc, labels, roots, mask_relu, dE, ws, st);
    cls_reduce_kernel<<<dim3(cls_reduce_blocks(C, D)), kClsRedThreads, 0, st>>>(b, d, c, nb, ws, dWc, dbc, loss);
    check_launch("gs_cls_nll_fwd_bwd");
    GS_API_END
}

int gs_clip_sgd(int32_t n_groups, const int64_t* goff_host, float* params, float* grads, float grad_scale,
                float max_norm, float lr, float* ws, void* stream) {
    GS_API_BEGIN
    using namespace gs;
    GS_REQUIRE(n_groups >= 1 && n_groups <= 8 && goff_host, GS_EINVAL, "1..8 parameter groups");
    GS_REQUIRE(params && grads && ws, GS_EINVAL, "NULL device pointer");
    const LowpShadow sh = g_lowp_shadow;
    g_lowp_shadow = {};
    Groups G;
    G.n = n_groups;
    G.pstride = kNormBlocks;
    G.sh = sh.p;
    G.sh_lo = sh.lo;
    G.sh_hi = sh.hi;
    for (int i = 0; i < n_groups; ++i) G.npart[i] = kNormBlocks;
    for (int i = 0; i <= n_groups; ++i) G.off[i] = goff_host[i];
    for (int i = 0; i < n_groups; ++i) GS_REQUIRE(G.off[i] <= G.off[i + 1], GS_EINVAL, "group offsets not sorted");
    hipStream_t st = as_stream(stream);
    group_sumsq_kernel<<<dim3(kNormBlocks, n_groups), kTb, 0, st>>>(G, grads, ws);
    const int64_t total = G.off[n_groups];
    const dim3 grid(static_cast<unsigned>(std::max<int64_t>(1, std::min<int64_t>((total + kTb - 1) / kTb, 512))));
    sgd_kernel<<<grid, kTb, 0, st>>>(G, params, grads, ws, grad_scale, max_norm, lr, g_done_flag.ptr,
                                     g_done_flag.value);
    g_done_flag = {};
    check_launch("gs_clip_sgd");
    GS_API_END
}

}  // extern "C"
