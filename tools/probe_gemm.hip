// Ablation probe of the layer-1 GEMM loops at the bench shape (n = 4,400
// rows, F = 256, K = 512, H = 128, fp32, self rows gathered from a 2M-row
// table).  Copies of linear_dw's and linear_fwd's loops with parts switched
// off, each timed over many launches with HIP events:
//   mode 0  as shipped
//   mode 1  no global loads inside the chunk loop (chunk 0's data reused)
//   mode 2  no MFMA (LDS operands summed with VALU adds instead)
//   mode 3  no LDS operand reads and no MFMA (loads, LDS stores, barriers)
// Developer tool, not part of the library:
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -I include tools/probe_gemm.hip -o tools/bin/probe_gemm
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#include "../graphsage-pytorch_amd/csrc/kernels/linear_dev.hpp"

using namespace gs;

#define CK(x)                                                                    \
    do {                                                                         \
        hipError_t e_ = (x);                                                     \
        if (e_ != hipSuccess) {                                                  \
            std::printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            return 1;                                                            \
        }                                                                        \
    } while (0)

template <int MODE>
__global__ __launch_bounds__(kThreads) void dw_probe(int n, int F, int H, int K, int rows_per_split,
                                                     const float* __restrict__ Xs, int64_t ldxs,
                                                     const int* __restrict__ sidx, const float* __restrict__ A,
                                                     int64_t lda, const float* __restrict__ dout, int64_t ldo,
                                                     float* __restrict__ dst, int64_t split_stride) {
    __shared__ float sZ[2][16 * kDwPitch];
    __shared__ float sI[2][16 * kDwPitch];
    __shared__ int sIdx[kDwMaxSlab];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int r = lane & 15, kq = lane >> 4;
    const int k0 = blockIdx.x * 64, h0 = blockIdx.y * 64;
    const int i_beg = blockIdx.z * rows_per_split;
    const int i_end = min(n, i_beg + rows_per_split);
    const int nC = (i_end - i_beg + 15) / 16;
    const int lr = tid >> 4, lq = (tid & 15) * 4;
    for (int t = tid; t < i_end - i_beg; t += kThreads) sIdx[t] = sidx[i_beg + t];
    __syncthreads();
    auto load = [&](int c, float4& z, float4& x) {
        const int t = min(16 * c + lr, i_end - i_beg - 1);
        const int ic = i_beg + t;
        z = row_quad_raw<true>(dout + static_cast<int64_t>(ic) * ldo, h0 + lq, H);
        const float* arow = A + static_cast<int64_t>(ic) * lda;
        const float* srow = Xs + static_cast<int64_t>(sIdx[t]) * ldxs;
        x = concat_quad_raw<float, true, true>(srow, arow, F, K, k0 + lq);
    };
    auto stash = [&](int c, int buf, float4 z, float4 x) {
        if (16 * c + lr >= i_end - i_beg) z = x = make_float4(0.f, 0.f, 0.f, 0.f);
        *reinterpret_cast<float4*>(&sZ[buf][lr * kDwPitch + lq]) = z;
        *reinterpret_cast<float4*>(&sI[buf][lr * kDwPitch + lq]) = x;
    };
    float4 z, x;
    load(0, z, x);
    stash(0, 0, z, x);
    f32x4 acc[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int c = 0; c < nC; ++c) {
        __syncthreads();
        const int cn = min(c + 1, nC - 1);
        if (MODE != 1) load(cn, z, x);
        __builtin_amdgcn_sched_barrier(0);
        const float* tz = sZ[c & 1];
        const float* ti = sI[c & 1];
        if (MODE != 3) {
            float a[4], b[4][4];
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                const int row = 4 * s + kq;
                a[s] = tz[row * kDwPitch + wave * 16 + r];
#pragma unroll
                for (int t = 0; t < 4; ++t) b[s][t] = ti[row * kDwPitch + t * 16 + r];
            }
            if (MODE == 2) {
#pragma unroll
                for (int s = 0; s < 4; ++s)
#pragma unroll
                    for (int t = 0; t < 4; ++t) acc[t][s] += a[s] * b[s][t];
            } else {
#pragma unroll
                for (int s = 0; s < 4; ++s)
#pragma unroll
                    for (int t = 0; t < 4; ++t)
                        acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[s], b[s][t], acc[t], 0, 0, 0);
            }
        }
        __builtin_amdgcn_sched_barrier(0);
        stash(cn, (c + 1) & 1, z, x);
    }
    float* slab = dst + static_cast<int64_t>(blockIdx.z) * split_stride;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        const int k = k0 + t * 16 + r;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int h = h0 + wave * 16 + 4 * kq + j;
            if (h < H && k < K) slab[static_cast<int64_t>(h) * K + k] = acc[t][j];
        }
    }
}

template <int MODE>
__global__ __launch_bounds__(kThreads) void fwd_probe(int n, int F, int H, int K, const float* __restrict__ Xs,
                                                      int64_t ldxs, const int* __restrict__ sidx,
                                                      const float* __restrict__ A, int64_t lda,
                                                      const float* __restrict__ W, float* __restrict__ out,
                                                      int64_t ldo) {
    constexpr int SA = kSlots + 1;
    __shared__ uint4 sA[2][16 * SA];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int r = lane & 15, kq = lane >> 4;
    const int m0 = blockIdx.x * 16;
    const int ct = blockIdx.y * 4 + wave;
    const int ar = tid >> 4, as = tid & 15;
    const int arow_i = min(m0 + ar, n - 1);
    const float* arow = A + static_cast<int64_t>(arow_i) * lda;
    const float* srow = Xs + static_cast<int64_t>(sidx[arow_i]) * ldxs;
    const float* wrow = W + static_cast<int64_t>(min(ct * 16 + r, H - 1)) * K;
    const int nC = (K + 63) / 64;
    uint4 a_nx = concat_slot<float, true, true>(srow, arow, F, K, as * 4);
    uint4 w_nx[4];
#pragma unroll
    for (int g = 0; g < 4; ++g) w_nx[g] = concat_slot<float, false, true>(nullptr, wrow, K, K, (4 * g + kq) * 4);
    sA[0][ar * SA + as] = a_nx;
    f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int c = 0; c < nC; ++c) {
        uint4 w_cur[4];
#pragma unroll
        for (int g = 0; g < 4; ++g) w_cur[g] = w_nx[g];
        __syncthreads();
        const int kn = min(c + 1, nC - 1) * 64;
        if (MODE != 1) {
            a_nx = concat_slot<float, true, true>(srow, arow, F, K, kn + as * 4);
#pragma unroll
            for (int g = 0; g < 4; ++g)
                w_nx[g] = concat_slot<float, false, true>(nullptr, wrow, K, K, kn + (4 * g + kq) * 4);
        }
        __builtin_amdgcn_sched_barrier(0);
        const uint4* tile = sA[c & 1];
        if (MODE != 3) {
            uint4 av[4];
#pragma unroll
            for (int g = 0; g < 4; ++g) av[g] = tile[r * SA + 4 * g + kq];
            if (MODE == 2) {
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    acc[0] += __uint_as_float(av[g].x) * __uint_as_float(w_cur[g].x);
                    acc[1] += __uint_as_float(av[g].y) * __uint_as_float(w_cur[g].y);
                    acc[2] += __uint_as_float(av[g].z) * __uint_as_float(w_cur[g].z);
                    acc[3] += __uint_as_float(av[g].w) * __uint_as_float(w_cur[g].w);
                }
            } else {
#pragma unroll
                for (int g = 0; g < 4; ++g) acc = mfma_slot<float>(av[g], w_cur[g], acc);
            }
        } else {
            acc[0] += __uint_as_float(w_cur[0].x);
        }
        __builtin_amdgcn_sched_barrier(0);
        sA[(c + 1) & 1][ar * SA + as] = a_nx;
    }
    const int col = ct * 16 + r;
    if (col >= H) return;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int row = m0 + 4 * kq + j;
        if (row < n) out[static_cast<int64_t>(row) * ldo + col] = acc[j];
    }
}


// mode 4: the chunk's 20 LDS operands read before its MFMAs (one wait), 1 chunk ahead
// mode 5: mode 4 with global loads 2 chunks ahead (register double buffer)
template <int MODE>
__global__ __launch_bounds__(kThreads) void dw_probe2(int n, int F, int H, int K, int rows_per_split,
                                                      const float* __restrict__ Xs, int64_t ldxs,
                                                      const int* __restrict__ sidx, const float* __restrict__ A,
                                                      int64_t lda, const float* __restrict__ dout, int64_t ldo,
                                                      float* __restrict__ dst, int64_t split_stride) {
    __shared__ float sZ[2][16 * kDwPitch];
    __shared__ float sI[2][16 * kDwPitch];
    __shared__ int sIdx[kDwMaxSlab];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int r = lane & 15, kq = lane >> 4;
    const int k0 = blockIdx.x * 64, h0 = blockIdx.y * 64;
    const int i_beg = blockIdx.z * rows_per_split;
    const int i_end = min(n, i_beg + rows_per_split);
    const int nC = (i_end - i_beg + 15) / 16;
    const int lr = tid >> 4, lq = (tid & 15) * 4;
    for (int t = tid; t < i_end - i_beg; t += kThreads) sIdx[t] = sidx[i_beg + t];
    __syncthreads();
    auto load = [&](int c, float4& z, float4& x) {
        const int t = min(16 * min(c, nC - 1) + lr, i_end - i_beg - 1);
        const int ic = i_beg + t;
        z = row_quad_raw<true>(dout + static_cast<int64_t>(ic) * ldo, h0 + lq, H);
        const float* arow = A + static_cast<int64_t>(ic) * lda;
        const float* srow = Xs + static_cast<int64_t>(sIdx[t]) * ldxs;
        x = concat_quad_raw<float, true, true>(srow, arow, F, K, k0 + lq);
    };
    auto stash = [&](int c, float4 z, float4 x) {
        if (16 * c + lr >= i_end - i_beg) z = x = make_float4(0.f, 0.f, 0.f, 0.f);
        *reinterpret_cast<float4*>(&sZ[c & 1][lr * kDwPitch + lq]) = z;
        *reinterpret_cast<float4*>(&sI[c & 1][lr * kDwPitch + lq]) = x;
    };
    f32x4 acc[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
    auto compute = [&](int c) {
        const float* tz = sZ[c & 1];
        const float* ti = sI[c & 1];
        float a[4], b[4][4];
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            const int row = 4 * s + kq;
            a[s] = tz[row * kDwPitch + wave * 16 + r];
#pragma unroll
            for (int t = 0; t < 4; ++t) b[s][t] = ti[row * kDwPitch + t * 16 + r];
        }
        __builtin_amdgcn_sched_barrier(0);  // all 20 LDS reads issued before the first MFMA
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
            for (int t = 0; t < 4; ++t) acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[s], b[s][t], acc[t], 0, 0, 0);
    };
    if (MODE == 4) {
        float4 z, x;
        load(0, z, x);
        stash(0, z, x);
        for (int c = 0; c < nC; ++c) {
            __syncthreads();
            load(c + 1, z, x);
            __builtin_amdgcn_sched_barrier(0);
            compute(c);
            __builtin_amdgcn_sched_barrier(0);
            stash(c + 1, z, x);
        }
    } else {
        float4 z0, x0, z1, x1;  // chunk c+1 in (z1,x1) when c even ... two named register sets
        load(0, z0, x0);
        stash(0, z0, x0);
        load(1, z1, x1);
        int c = 0;
        for (; c + 1 < nC; c += 2) {
            __syncthreads();
            load(c + 2, z0, x0);  // chunk c+2 (chunk c was stashed from z0/x0 already)
            __builtin_amdgcn_sched_barrier(0);
            compute(c);
            __builtin_amdgcn_sched_barrier(0);
            stash(c + 1, z1, x1);
            __syncthreads();
            load(c + 3, z1, x1);
            __builtin_amdgcn_sched_barrier(0);
            compute(c + 1);
            __builtin_amdgcn_sched_barrier(0);
            stash(c + 2, z0, x0);
        }
        if (c < nC) {
            __syncthreads();
            compute(c);
        }
    }
    float* slab = dst + static_cast<int64_t>(blockIdx.z) * split_stride;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        const int k = k0 + t * 16 + r;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int h = h0 + wave * 16 + 4 * kq + j;
            if (h < H && k < K) slab[static_cast<int64_t>(h) * K + k] = acc[t][j];
        }
    }
}

// mode 4: two accumulator chains (even / odd slots), 1 chunk ahead
// mode 5: two chains, W and A slots 2 chunks ahead (register double buffer)
template <int MODE>
__global__ __launch_bounds__(kThreads) void fwd_probe2(int n, int F, int H, int K, const float* __restrict__ Xs,
                                                       int64_t ldxs, const int* __restrict__ sidx,
                                                       const float* __restrict__ A, int64_t lda,
                                                       const float* __restrict__ W, float* __restrict__ out,
                                                       int64_t ldo) {
    constexpr int SA = kSlots + 1;
    __shared__ uint4 sA[2][16 * SA];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int r = lane & 15, kq = lane >> 4;
    const int m0 = blockIdx.x * 16;
    const int ct = blockIdx.y * 4 + wave;
    const int ar = tid >> 4, as = tid & 15;
    const int arow_i = min(m0 + ar, n - 1);
    const float* arow = A + static_cast<int64_t>(arow_i) * lda;
    const float* srow = Xs + static_cast<int64_t>(sidx[arow_i]) * ldxs;
    const float* wrow = W + static_cast<int64_t>(min(ct * 16 + r, H - 1)) * K;
    const int nC = (K + 63) / 64;
    auto lda_ = [&](int c) { return concat_slot<float, true, true>(srow, arow, F, K, min(c, nC - 1) * 64 + as * 4); };
    auto ldw = [&](int c, uint4 (&w)[4]) {
#pragma unroll
        for (int g = 0; g < 4; ++g)
            w[g] = concat_slot<float, false, true>(nullptr, wrow, K, K, min(c, nC - 1) * 64 + (4 * g + kq) * 4);
    };
    f32x4 acc0 = f32x4{0.f, 0.f, 0.f, 0.f}, acc1 = acc0;
    auto compute = [&](int c, const uint4 (&w)[4]) {
        const uint4* tile = sA[c & 1];
        uint4 av[4];
#pragma unroll
        for (int g = 0; g < 4; ++g) av[g] = tile[r * SA + 4 * g + kq];
        __builtin_amdgcn_sched_barrier(0);
        acc0 = mfma_slot<float>(av[0], w[0], acc0);
        acc1 = mfma_slot<float>(av[1], w[1], acc1);
        acc0 = mfma_slot<float>(av[2], w[2], acc0);
        acc1 = mfma_slot<float>(av[3], w[3], acc1);
    };
    if (MODE == 4) {
        uint4 a_nx = lda_(0), w_nx[4], w_cur[4];
        ldw(0, w_nx);
        sA[0][ar * SA + as] = a_nx;
        for (int c = 0; c < nC; ++c) {
#pragma unroll
            for (int g = 0; g < 4; ++g) w_cur[g] = w_nx[g];
            __syncthreads();
            a_nx = lda_(c + 1);
            ldw(c + 1, w_nx);
            __builtin_amdgcn_sched_barrier(0);
            compute(c, w_cur);
            __builtin_amdgcn_sched_barrier(0);
            sA[(c + 1) & 1][ar * SA + as] = a_nx;
        }
    } else {
        uint4 a0 = lda_(0), a1 = lda_(1), w0[4], w1[4];
        ldw(0, w0);
        ldw(1, w1);
        sA[0][ar * SA + as] = a0;
        int c = 0;
        for (; c + 1 < nC; c += 2) {
            __syncthreads();
            a0 = lda_(c + 2);
            __builtin_amdgcn_sched_barrier(0);
            compute(c, w0);
            ldw(c + 2, w0);
            __builtin_amdgcn_sched_barrier(0);
            sA[(c + 1) & 1][ar * SA + as] = a1;
            __syncthreads();
            a1 = lda_(c + 3);
            __builtin_amdgcn_sched_barrier(0);
            compute(c + 1, w1);
            ldw(c + 3, w1);
            __builtin_amdgcn_sched_barrier(0);
            sA[c & 1][ar * SA + as] = a0;
        }
        if (c < nC) {
            __syncthreads();
            compute(c, w0);
        }
    }
    const f32x4 acc = acc0 + acc1;
    const int col = ct * 16 + r;
    if (col >= H) return;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int row = m0 + 4 * kq + j;
        if (row < n) out[static_cast<int64_t>(row) * ldo + col] = acc[j];
    }
}


// Pure MFMA: each wave runs `iters` x 16 MFMAs on 4 independent accumulators
// (the dW loop's shape without memory); block 0 / wave 0 stamps the shader
// clock (s_memtime) and the 100 MHz wall clock (s_memrealtime) around it.
__global__ __launch_bounds__(kThreads) void mfma_only(int iters, float* out, unsigned long long* clk) {
    const int lane = threadIdx.x & 63;
    f32x4 acc[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
    float a = lane * 1e-3f, b = 1.0f - lane * 1e-3f;
    const unsigned long long c0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
            for (int t = 0; t < 4; ++t) acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[t], 0, 0, 0);
        a += 1e-7f;
    }
    const f32x4 v = acc[0] + acc[1] + acc[2] + acc[3];
    const unsigned long long c1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        clk[0] = c1 - c0;
        clk[1] = r1 - r0;
    }
    out[blockIdx.x * kThreads + threadIdx.x] = v[0] + v[1] + v[2] + v[3];
}


// mode 6: 64-row chunks (4 sub-chunks of 16 per barrier), one chunk ahead;
// inside a chunk the next sub-chunk's 20 LDS operands are read before the
// current sub-chunk's 16 MFMAs
template <int CR>
__global__ __launch_bounds__(kThreads) void dw_probe3(int n, int F, int H, int K, int rows_per_split,
                                                      const float* __restrict__ Xs, int64_t ldxs,
                                                      const int* __restrict__ sidx, const float* __restrict__ A,
                                                      int64_t lda, const float* __restrict__ dout, int64_t ldo,
                                                      float* __restrict__ dst, int64_t split_stride) {
    constexpr int RW = 16 * CR;  // rows per chunk
    __shared__ float sZ[2][RW * kDwPitch];
    __shared__ float sI[2][RW * kDwPitch];
    __shared__ int sIdx[kDwMaxSlab];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int r = lane & 15, kq = lane >> 4;
    const int k0 = blockIdx.x * 64, h0 = blockIdx.y * 64;
    const int i_beg = blockIdx.z * rows_per_split;
    const int i_end = min(n, i_beg + rows_per_split);
    const int nrow = i_end - i_beg;
    const int nC = (nrow + RW - 1) / RW;
    const int lr = tid >> 4, lq = (tid & 15) * 4;
    for (int t = tid; t < nrow; t += kThreads) sIdx[t] = sidx[i_beg + t];
    __syncthreads();
    auto load = [&](int c, float4 (&z)[CR], float4 (&x)[CR]) {
#pragma unroll
        for (int q = 0; q < CR; ++q) {
            const int t = min(RW * min(c, nC - 1) + 16 * q + lr, nrow - 1);
            const int ic = i_beg + t;
            z[q] = row_quad_raw<true>(dout + static_cast<int64_t>(ic) * ldo, h0 + lq, H);
            const float* arow = A + static_cast<int64_t>(ic) * lda;
            const float* srow = Xs + static_cast<int64_t>(sIdx[t]) * ldxs;
            x[q] = concat_quad_raw<float, true, true>(srow, arow, F, K, k0 + lq);
        }
    };
    auto stash = [&](int c, float4 (&z)[CR], float4 (&x)[CR]) {
#pragma unroll
        for (int q = 0; q < CR; ++q) {
            float4 zz = z[q], xx = x[q];
            if (RW * c + 16 * q + lr >= nrow) zz = xx = make_float4(0.f, 0.f, 0.f, 0.f);
            *reinterpret_cast<float4*>(&sZ[c & 1][(16 * q + lr) * kDwPitch + lq]) = zz;
            *reinterpret_cast<float4*>(&sI[c & 1][(16 * q + lr) * kDwPitch + lq]) = xx;
        }
    };
    f32x4 acc[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
    auto read_ops = [&](int c, int q, float (&a)[4], float (&b)[4][4]) {
        const float* tz = sZ[c & 1] + 16 * q * kDwPitch;
        const float* ti = sI[c & 1] + 16 * q * kDwPitch;
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            const int row = 4 * s + kq;
            a[s] = tz[row * kDwPitch + wave * 16 + r];
#pragma unroll
            for (int t = 0; t < 4; ++t) b[s][t] = ti[row * kDwPitch + t * 16 + r];
        }
    };
    auto mfmas = [&](const float (&a)[4], const float (&b)[4][4]) {
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
            for (int t = 0; t < 4; ++t) acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[s], b[s][t], acc[t], 0, 0, 0);
    };
    float4 z[CR], x[CR];
    load(0, z, x);
    stash(0, z, x);
    for (int c = 0; c < nC; ++c) {
        __syncthreads();
        load(c + 1, z, x);
        __builtin_amdgcn_sched_barrier(0);
        float a0[4], b0[4][4], a1[4], b1[4][4];
        read_ops(c, 0, a0, b0);
#pragma unroll
        for (int q = 0; q < CR; q += 2) {
            if (q + 1 < CR) read_ops(c, q + 1, a1, b1);
            __builtin_amdgcn_sched_barrier(0);
            mfmas(a0, b0);
            __builtin_amdgcn_sched_barrier(0);
            if (q + 2 < CR) read_ops(c, q + 2, a0, b0);
            __builtin_amdgcn_sched_barrier(0);
            if (q + 1 < CR) mfmas(a1, b1);
            __builtin_amdgcn_sched_barrier(0);
        }
        stash(c + 1, z, x);
    }
    float* slab = dst + static_cast<int64_t>(blockIdx.z) * split_stride;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        const int k = k0 + t * 16 + r;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int h = h0 + wave * 16 + 4 * kq + j;
            if (h < H && k < K) slab[static_cast<int64_t>(h) * K + k] = acc[t][j];
        }
    }
}

__global__ void fill(float* p, int64_t n, uint32_t seed) {
    for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < n; i += int64_t(gridDim.x) * blockDim.x) {
        uint32_t h = static_cast<uint32_t>(i) * 2654435761u ^ seed;
        h ^= h >> 13;
        h *= 0x5bd1e995u;
        p[i] = static_cast<float>(h & 0xffff) / 65536.f - 0.5f;
    }
}

int main() {
    const int n = 4400, F = 256, K = 512, H = 128;
    const int64_t NX = int64_t(1) << 21;
    float *X, *A, *dZ, *W, *out, *slabs;
    int* sidx;
    CK(hipMalloc(&X, NX * F * 4));
    CK(hipMalloc(&A, int64_t(n) * F * 4));
    CK(hipMalloc(&dZ, int64_t(n) * H * 4));
    CK(hipMalloc(&W, int64_t(H) * K * 4));
    CK(hipMalloc(&out, int64_t(n) * H * 4));
    const int S = dw_splits(n, K, H), rps = dw_rows_per_split(n, K, H);
    CK(hipMalloc(&slabs, int64_t(S) * H * K * 4));
    CK(hipMalloc(&sidx, n * 4));
    fill<<<4096, 256>>>(X, NX * F, 1);
    fill<<<256, 256>>>(A, int64_t(n) * F, 2);
    fill<<<256, 256>>>(dZ, int64_t(n) * H, 3);
    fill<<<256, 256>>>(W, int64_t(H) * K, 4);
    std::vector<int> hs(n);
    uint64_t s = 88172645463325252ull;
    for (int i = 0; i < n; ++i) {
        s ^= s << 13; s ^= s >> 7; s ^= s << 17;
        hs[i] = static_cast<int>(s % NX);
    }
    CK(hipMemcpy(sidx, hs.data(), n * 4, hipMemcpyHostToDevice));
    CK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int reps = 200;
    auto time_it = [&](auto launch) -> float {
        for (int i = 0; i < 10; ++i) launch();
        (void)hipEventRecord(e0);
        for (int i = 0; i < reps; ++i) launch();
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, e0, e1);
        return ms * 1e3f / reps;
    };
    const dim3 gdw((K + 63) / 64, (H + 63) / 64, S);
    const dim3 gfw((n + 15) / 16, (H + 63) / 64);
    std::printf("dw: S=%d rps=%d grid=(%u,%u,%u)\n", S, rps, gdw.x, gdw.y, gdw.z);
    const char* names[4] = {"as shipped", "no loop loads", "no MFMA", "no LDS reads, no MFMA"};
    float t;
    t = time_it([&] { dw_probe<0><<<gdw, kThreads>>>(n, F, H, K, rps, X, F, sidx, A, F, dZ, H, slabs, int64_t(H) * K); });
    std::printf("  dw  mode 0 %-24s %7.2f us/launch\n", names[0], t);
    t = time_it([&] { dw_probe<1><<<gdw, kThreads>>>(n, F, H, K, rps, X, F, sidx, A, F, dZ, H, slabs, int64_t(H) * K); });
    std::printf("  dw  mode 1 %-24s %7.2f us/launch\n", names[1], t);
    t = time_it([&] { dw_probe<2><<<gdw, kThreads>>>(n, F, H, K, rps, X, F, sidx, A, F, dZ, H, slabs, int64_t(H) * K); });
    std::printf("  dw  mode 2 %-24s %7.2f us/launch\n", names[2], t);
    t = time_it([&] { dw_probe<3><<<gdw, kThreads>>>(n, F, H, K, rps, X, F, sidx, A, F, dZ, H, slabs, int64_t(H) * K); });
    std::printf("  dw  mode 3 %-24s %7.2f us/launch\n", names[3], t);
    t = time_it([&] { fwd_probe<0><<<gfw, kThreads>>>(n, F, H, K, X, F, sidx, A, F, W, out, H); });
    std::printf("  fwd mode 0 %-24s %7.2f us/launch\n", names[0], t);
    t = time_it([&] { fwd_probe<1><<<gfw, kThreads>>>(n, F, H, K, X, F, sidx, A, F, W, out, H); });
    std::printf("  fwd mode 1 %-24s %7.2f us/launch\n", names[1], t);
    t = time_it([&] { fwd_probe<2><<<gfw, kThreads>>>(n, F, H, K, X, F, sidx, A, F, W, out, H); });
    std::printf("  fwd mode 2 %-24s %7.2f us/launch\n", names[2], t);
    t = time_it([&] { fwd_probe<3><<<gfw, kThreads>>>(n, F, H, K, X, F, sidx, A, F, W, out, H); });
    std::printf("  fwd mode 3 %-24s %7.2f us/launch\n", names[3], t);
    t = time_it([&] { dw_probe2<4><<<gdw, kThreads>>>(n, F, H, K, rps, X, F, sidx, A, F, dZ, H, slabs, int64_t(H) * K); });
    std::printf("  dw  mode 4 %-24s %7.2f us/launch\n", "LDS reads first", t);
    t = time_it([&] { dw_probe2<5><<<gdw, kThreads>>>(n, F, H, K, rps, X, F, sidx, A, F, dZ, H, slabs, int64_t(H) * K); });
    std::printf("  dw  mode 5 %-24s %7.2f us/launch\n", "LDS first + 2 ahead", t);
    t = time_it([&] { dw_probe3<2><<<gdw, kThreads>>>(n, F, H, K, rps, X, F, sidx, A, F, dZ, H, slabs, int64_t(H) * K); });
    std::printf("  dw  mode 6 %-24s %7.2f us/launch\n", "32-row chunks", t);
    t = time_it([&] { dw_probe3<4><<<gdw, kThreads>>>(n, F, H, K, rps, X, F, sidx, A, F, dZ, H, slabs, int64_t(H) * K); });
    std::printf("  dw  mode 6 %-24s %7.2f us/launch\n", "64-row chunks", t);
    {
        const int S2 = 32, rps2 = (n + S2 - 1) / S2 / 16 * 16 + 16;
        const dim3 g2((K + 63) / 64, (H + 63) / 64, (n + rps2 - 1) / rps2);
        t = time_it([&] { dw_probe3<4><<<g2, kThreads>>>(n, F, H, K, rps2, X, F, sidx, A, F, dZ, H, slabs, int64_t(H) * K); });
        std::printf("  dw  mode 6 %-24s %7.2f us/launch (%u slabs)\n", "64-row chunks", t, g2.z);
    }
    t = time_it([&] { fwd_probe2<4><<<gfw, kThreads>>>(n, F, H, K, X, F, sidx, A, F, W, out, H); });
    std::printf("  fwd mode 4 %-24s %7.2f us/launch\n", "2 chains", t);
    t = time_it([&] { fwd_probe2<5><<<gfw, kThreads>>>(n, F, H, K, X, F, sidx, A, F, W, out, H); });
    std::printf("  fwd mode 5 %-24s %7.2f us/launch\n", "2 chains + 2 ahead", t);
    {
        unsigned long long* clk;
        float* o2;
        CK(hipMalloc(&clk, 16));
        CK(hipMalloc(&o2, 256 * kThreads * 4));
        for (int iters : {18, 180}) {
            t = time_it([&] { mfma_only<<<256, kThreads>>>(iters, o2, clk); });
            unsigned long long hc[2];
            CK(hipMemcpy(hc, clk, 16, hipMemcpyDeviceToHost));
            const double us = hc[1] / 100.0, mhz = hc[0] / us;
            std::printf("  MFMA only, %3d x 16 per wave, 1 wave/SIMD: %7.2f us/launch; in-kernel %.2f us, %.0f MHz "
                        "shader clock, %.1f cycles per MFMA\n", iters, t, us, mhz, double(hc[0]) / (iters * 16.0));
        }
    }
    t = time_it([&] { fill<<<1, 64>>>(out, 64, 5); });
    std::printf("  empty-ish launch            %7.2f us/launch\n", t);
    return 0;
}
