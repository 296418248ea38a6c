// SageLayer (models.py:189-220) on CDNA4 matrix cores.
//   forward : out = relu([Xs[sidx] | A] · Wᵀ)      (:216 cat self-first, :219)
//   backward: dW = dZᵀ · [Xs[sidx] | A],  dIn = dZ · W,  dZ = dOut ⊙ (out > 0)
// The concat is never materialised: the K loop reads its first F columns from
// the gathered self rows and the rest from the aggregate.  fp32 inputs run on
// v_mfma_f32_16x16x4_f32 (exact f32 products, fp32 accumulate); bf16 inputs on
// v_mfma_f32_16x16x32_bf16 with fp32 accumulate.
#include <algorithm>

#include "kcommon.hpp"

namespace gs {

constexpr int kThreads = 256;  // 4 wavefronts

// ---------------------------------------------------------------- forward
// Block = 16 output rows x all H columns; wave w owns column tiles w, w+4, ...
// K is walked in 128-byte chunks per row (32 fp32 / 64 bf16).  Each lane reads
// 16 B of a row from LDS and feeds 4 fp32 MFMAs (k-slots permuted identically
// for both operands) or one bf16 MFMA.
template <typename T, bool HAS_SELF, bool RELU, bool VLOAD, int NTW>
__global__ __launch_bounds__(kThreads) void linear_fwd_kernel(
    int n, int F, int H, int K, const T* __restrict__ Xs, int64_t ldxs, const int* __restrict__ sidx,
    const T* __restrict__ A, int64_t lda, const T* __restrict__ W, float* __restrict__ out, int64_t ldo) {
    constexpr int EPV = 16 / sizeof(T);
    constexpr int BK = 8 * EPV;
    constexpr int BM = 16;
    constexpr int SROW = BK + EPV;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    T* sA = reinterpret_cast<T*>(smem);
    T* sW = sA + BM * SROW;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int m0 = blockIdx.x * BM;

    const int a_row = tid >> 3, a_c = tid & 7;
    const bool a_ok = tid < 128 && m0 + a_row < n;
    const T* self_row = nullptr;
    const T* agg_row = nullptr;
    if (a_ok) {
        if (HAS_SELF) self_row = Xs + static_cast<int64_t>(sidx ? sidx[m0 + a_row] : m0 + a_row) * ldxs;
        agg_row = A + static_cast<int64_t>(m0 + a_row) * lda;
    }
    f32x4 acc[NTW];
#pragma unroll
    for (int t = 0; t < NTW; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};

    for (int k0 = 0; k0 < K; k0 += BK) {
        if (tid < 128) {
            const int k = k0 + a_c * EPV;
            T* dst = sA + a_row * SROW + a_c * EPV;
            if (VLOAD) {
                uint4 v = make_uint4(0, 0, 0, 0);
                if (a_ok && k < K) {
                    const T* src = (HAS_SELF && k < F) ? self_row + k : agg_row + (HAS_SELF ? k - F : k);
                    v = *reinterpret_cast<const uint4*>(src);
                }
                *reinterpret_cast<uint4*>(dst) = v;
            } else {
#pragma unroll
                for (int e = 0; e < EPV; ++e) {
                    const int kk = k + e;
                    T v = T(0);
                    if (a_ok && kk < K) v = (HAS_SELF && kk < F) ? self_row[kk] : agg_row[HAS_SELF ? kk - F : kk];
                    dst[e] = v;
                }
            }
        }
        for (int i = tid; i < H * 8; i += kThreads) {
            const int h = i >> 3, c = i & 7, k = k0 + c * EPV;
            T* dst = sW + h * SROW + c * EPV;
            if (VLOAD) {
                uint4 v = make_uint4(0, 0, 0, 0);
                if (k < K) v = *reinterpret_cast<const uint4*>(W + static_cast<int64_t>(h) * K + k);
                *reinterpret_cast<uint4*>(dst) = v;
            } else {
#pragma unroll
                for (int e = 0; e < EPV; ++e) dst[e] = (k + e < K) ? W[static_cast<int64_t>(h) * K + k + e] : T(0);
            }
        }
        __syncthreads();
        const int r = lane & 15, kq = lane >> 4;
#pragma unroll
        for (int g = 0; g < 2; ++g) {
            const uint4 av = *reinterpret_cast<const uint4*>(sA + r * SROW + (g * 4 + kq) * EPV);
#pragma unroll
            for (int t = 0; t < NTW; ++t) {
                const int ct = wave + 4 * t;
                if (ct * 16 >= H) break;
                const uint4 bv = *reinterpret_cast<const uint4*>(sW + (ct * 16 + r) * SROW + (g * 4 + kq) * EPV);
                if constexpr (sizeof(T) == 4) {
                    acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(av.x), __uint_as_float(bv.x), acc[t], 0, 0, 0);
                    acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(av.y), __uint_as_float(bv.y), acc[t], 0, 0, 0);
                    acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(av.z), __uint_as_float(bv.z), acc[t], 0, 0, 0);
                    acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(av.w), __uint_as_float(bv.w), acc[t], 0, 0, 0);
                } else {
                    s16x8 a8, b8;
                    __builtin_memcpy(&a8, &av, 16);
                    __builtin_memcpy(&b8, &bv, 16);
                    acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a8, b8, acc[t], 0, 0, 0);
                }
            }
        }
        __syncthreads();
    }
#pragma unroll
    for (int t = 0; t < NTW; ++t) {
        const int ct = wave + 4 * t;
        if (ct * 16 >= H) break;
        const int col = ct * 16 + (lane & 15);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int row = m0 + 4 * (lane >> 4) + j;
            if (row < n) {
                const float v = acc[t][j];
                out[static_cast<int64_t>(row) * ldo + col] = (RELU && !(v > 0.f) && v == v) ? 0.f : v;  // NaN kept, as torch.relu
            }
        }
    }
}

// ------------------------------------------------------------ weight grad
// dW[h][k] = Σ_i dZ[i][h] · In[i][k].  Block = one 64-column tile of K over a
// contiguous row range (split s); MFMA "k" runs over rows i, so both operands
// come straight from row-major LDS tiles.  Splits write fp32 slabs that a
// second kernel sums in a fixed order (deterministic, no atomics).
template <typename T, bool HAS_SELF, bool RELU, bool VLOAD, int HTW>
__global__ __launch_bounds__(kThreads) void linear_dw_kernel(
    int n, int F, int H, int K, int rows_per_split, const T* __restrict__ Xs, int64_t ldxs,
    const int* __restrict__ sidx, const T* __restrict__ A, int64_t lda, const float* __restrict__ dout,
    const float* __restrict__ out, int64_t ldo, float* __restrict__ dst, int64_t split_stride) {
    constexpr int BI = 16, BKC = 64, SA = BKC + 16;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int SZ = ((H + 31) / 32) * 32 + 16;
    float* sZ = reinterpret_cast<float*>(smem);
    float* sA = sZ + BI * SZ;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int kc0 = blockIdx.x * BKC;
    const int i_beg = blockIdx.y * rows_per_split;
    const int i_end = min(n, i_beg + rows_per_split);
    const int HT = (H + 15) / 16;

    f32x4 acc[HTW][4];
#pragma unroll
    for (int t = 0; t < HTW; ++t)
#pragma unroll
        for (int c = 0; c < 4; ++c) acc[t][c] = f32x4{0.f, 0.f, 0.f, 0.f};

    for (int i0 = i_beg; i0 < i_end; i0 += BI) {
        for (int e = tid; e < BI * H; e += kThreads) {
            const int ii = e / H, h = e - ii * H, i = i0 + ii;
            float z = 0.f;
            if (i < i_end) {
                z = dout[static_cast<int64_t>(i) * ldo + h];
                if (RELU && !(out[static_cast<int64_t>(i) * ldo + h] > 0.f)) z = 0.f;
            }
            sZ[ii * SZ + h] = z;
        }
        {
            const int ii = tid >> 4, c = (tid & 15) * 4, i = i0 + ii, k = kc0 + c;
            float v[4] = {0.f, 0.f, 0.f, 0.f};
            if (i < i_end) {
                const T* srow = HAS_SELF ? Xs + static_cast<int64_t>(sidx ? sidx[i] : i) * ldxs : nullptr;
                const T* arow = A + static_cast<int64_t>(i) * lda;
                if (VLOAD && k + 3 < K) {
                    const T* src = (HAS_SELF && k < F) ? srow + k : arow + (HAS_SELF ? k - F : k);
                    if constexpr (sizeof(T) == 4) {
                        const float4 q = *reinterpret_cast<const float4*>(src);
                        v[0] = q.x; v[1] = q.y; v[2] = q.z; v[3] = q.w;
                    } else {
                        const uint2 q = *reinterpret_cast<const uint2*>(src);
                        v[0] = __uint_as_float(q.x << 16); v[1] = __uint_as_float(q.x & 0xffff0000u);
                        v[2] = __uint_as_float(q.y << 16); v[3] = __uint_as_float(q.y & 0xffff0000u);
                    }
                } else {
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        const int kk = k + e;
                        if (kk >= K) break;
                        const T x = (HAS_SELF && kk < F) ? srow[kk] : arow[HAS_SELF ? kk - F : kk];
                        if constexpr (sizeof(T) == 4) v[e] = x;
                        else v[e] = bf2f(x);
                    }
                }
            }
#pragma unroll
            for (int e = 0; e < 4; ++e) sA[ii * SA + c + e] = v[e];
        }
        __syncthreads();
#pragma unroll
        for (int kk = 0; kk < BI; kk += 4) {
            const int ri = kk + (lane >> 4);
            float b[4];
#pragma unroll
            for (int c = 0; c < 4; ++c) b[c] = sA[ri * SA + c * 16 + (lane & 15)];
#pragma unroll
            for (int t = 0; t < HTW; ++t) {
                const int ht = wave + 4 * t;
                if (ht >= HT) break;
                const float a = sZ[ri * SZ + ht * 16 + (lane & 15)];
#pragma unroll
                for (int c = 0; c < 4; ++c) acc[t][c] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b[c], acc[t][c], 0, 0, 0);
            }
        }
        __syncthreads();
    }
    float* slab = dst + static_cast<int64_t>(blockIdx.y) * split_stride;
#pragma unroll
    for (int t = 0; t < HTW; ++t) {
        const int ht = wave + 4 * t;
        if (ht >= HT) break;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const int k = kc0 + c * 16 + (lane & 15);
            if (k >= K) continue;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int h = ht * 16 + 4 * (lane >> 4) + j;
                if (h < H) slab[static_cast<int64_t>(h) * K + k] = acc[t][c][j];
            }
        }
    }
}

__global__ __launch_bounds__(kThreads) void sum_slabs_kernel(const float* __restrict__ slabs, int S,
                                                             int64_t len, float* __restrict__ out) {
    for (int64_t i = blockIdx.x * int64_t(kThreads) + threadIdx.x; i < len; i += int64_t(gridDim.x) * kThreads) {
        float s = 0.f;
        for (int t = 0; t < S; ++t) s += slabs[t * len + i];
        out[i] = s;
    }
}

// ------------------------------------------------------------- input grad
// dIn[i][k] = Σ_h dZ[i][h] · W[h][k]; block = 16 rows x 64 columns of K.
template <bool HAS_SELF, bool RELU>
__global__ __launch_bounds__(kThreads) void linear_dx_kernel(
    int n, int F, int H, int K, const float* __restrict__ dout, const float* __restrict__ out, int64_t ldo,
    const float* __restrict__ W, float* __restrict__ dSelf, float* __restrict__ dA, int64_t ldd) {
    constexpr int BM = 16, BH = 32, BKC = 64, SZ = BH + 2, SW = BKC + 16;
    __shared__ float sZ[BM * SZ];
    __shared__ float sW[BH * SW];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int m0 = blockIdx.x * BM, kc0 = blockIdx.y * BKC;
    f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int h0 = 0; h0 < H; h0 += BH) {
        for (int e = tid; e < BM * BH; e += kThreads) {
            const int ii = e / BH, hh = e - ii * BH, i = m0 + ii, h = h0 + hh;
            float z = 0.f;
            if (i < n && h < H) {
                z = dout[static_cast<int64_t>(i) * ldo + h];
                if (RELU && !(out[static_cast<int64_t>(i) * ldo + h] > 0.f)) z = 0.f;
            }
            sZ[ii * SZ + hh] = z;
        }
        for (int e = tid; e < BH * BKC; e += kThreads) {
            const int hh = e / BKC, c = e - hh * BKC, h = h0 + hh, k = kc0 + c;
            sW[hh * SW + c] = (h < H && k < K) ? W[static_cast<int64_t>(h) * K + k] : 0.f;
        }
        __syncthreads();
#pragma unroll
        for (int hh = 0; hh < BH; hh += 4) {
            const float a = sZ[(lane & 15) * SZ + hh + (lane >> 4)];
            const float b = sW[(hh + (lane >> 4)) * SW + wave * 16 + (lane & 15)];
            acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc, 0, 0, 0);
        }
        __syncthreads();
    }
    const int k = kc0 + wave * 16 + (lane & 15);
    if (k >= K) return;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int i = m0 + 4 * (lane >> 4) + j;
        if (i >= n) continue;
        if (HAS_SELF && k < F) dSelf[static_cast<int64_t>(i) * ldd + k] = acc[j];
        else dA[static_cast<int64_t>(i) * ldd + (HAS_SELF ? k - F : k)] = acc[j];
    }
}

static int dw_splits(int64_t n) {
    int64_t s = (n + 127) / 128;
    if (s < 1) s = 1;
    if (s > 64) s = 64;
    return static_cast<int>(s);
}

}  // namespace gs

extern "C" {

int gs_sage_linear_fwd(gs_dtype dt, int64_t n, int64_t F, int64_t H, const void* Xs, int64_t ldxs,
                       const int32_t* sidx, const void* A, int64_t lda, const void* Wd, float* out,
                       int64_t ldo, int32_t relu, void* stream) {
    GS_API_BEGIN
    using namespace gs;
    GS_REQUIRE(dt == GS_F32 || dt == GS_BF16, GS_EINVAL, "dtype must be f32 or bf16");
    GS_REQUIRE(n >= 0 && n < (int64_t(1) << 31) && F >= 1 && F < (1 << 28), GS_EINVAL, "bad sizes");
    GS_REQUIRE(H >= 16 && H <= 256 && H % 16 == 0, GS_EINVAL, "out_size must be a multiple of 16 in [16, 256]");
    GS_REQUIRE(lda >= F && ldo >= H && (!Xs || ldxs >= F), GS_EINVAL, "leading dimension too small");
    if (n == 0) return GS_OK;
    GS_REQUIRE(A && Wd && out, GS_EINVAL, "NULL device pointer");
    const bool self = Xs != nullptr;
    const int K = static_cast<int>(self ? 2 * F : F);
    const int EPV = dt == GS_F32 ? 4 : 8;
    const bool vload = F % EPV == 0 && lda % EPV == 0 && (!self || (ldxs % EPV == 0 && aligned16(Xs))) &&
                       aligned16(A) && aligned16(Wd);
    const size_t esz = dt == GS_F32 ? 4 : 2;
    const size_t smem = static_cast<size_t>(16 + H) * (8 * EPV + EPV) * esz;
    const dim3 grid(static_cast<unsigned>((n + 15) / 16));
    hipStream_t st = as_stream(stream);
    const int nn = static_cast<int>(n), ff = static_cast<int>(F), hh = static_cast<int>(H);
#define GS_LFWD1(TT, SELF, RELU, VL, NT)                                                                  \
    linear_fwd_kernel<TT, SELF, RELU, VL, NT><<<grid, kThreads, smem, st>>>(                              \
        nn, ff, hh, K, static_cast<const TT*>(Xs), ldxs, sidx, static_cast<const TT*>(A), lda,            \
        static_cast<const TT*>(Wd), out, ldo)
#define GS_LFWD(TT, SELF, RELU, VL) \
    do { if (hh <= 128) GS_LFWD1(TT, SELF, RELU, VL, 2); else GS_LFWD1(TT, SELF, RELU, VL, 4); } while (0)
#define GS_LFWD_V(TT, SELF, RELU) \
    do { if (vload) GS_LFWD(TT, SELF, RELU, true); else GS_LFWD(TT, SELF, RELU, false); } while (0)
#define GS_LFWD_R(TT, SELF) \
    do { if (relu) GS_LFWD_V(TT, SELF, true); else GS_LFWD_V(TT, SELF, false); } while (0)
#define GS_LFWD_S(TT) \
    do { if (self) GS_LFWD_R(TT, true); else GS_LFWD_R(TT, false); } while (0)
    if (dt == GS_F32) GS_LFWD_S(float);
    else GS_LFWD_S(bf16_t);
#undef GS_LFWD_S
#undef GS_LFWD_R
#undef GS_LFWD_V
#undef GS_LFWD
#undef GS_LFWD1
    check_launch("gs_sage_linear_fwd");
    GS_API_END
}

int64_t gs_sage_linear_bwd_weight_ws(int64_t n, int64_t K, int64_t H) {
    const int S = gs::dw_splits(n);
    return S > 1 ? static_cast<int64_t>(S) * K * H * 4 : 0;
}

int gs_sage_linear_bwd_weight(gs_dtype dt, int64_t n, int64_t F, int64_t H, const void* Xs, int64_t ldxs,
                              const int32_t* sidx, const void* A, int64_t lda, const float* dout,
                              const float* out, int64_t ldo, int32_t relu, float* dW, void* ws,
                              int64_t ws_bytes, void* stream) {
    GS_API_BEGIN
    using namespace gs;
    GS_REQUIRE(dt == GS_F32 || dt == GS_BF16, GS_EINVAL, "dtype must be f32 or bf16");
    GS_REQUIRE(n >= 0 && n < (int64_t(1) << 31) && F >= 1 && H >= 1 && H <= 256, GS_EINVAL, "bad sizes");
    const bool self = Xs != nullptr;
    const int64_t K = self ? 2 * F : F;
    hipStream_t st = as_stream(stream);
    if (n == 0) {
        GS_REQUIRE(hipMemsetAsync(dW, 0, H * K * 4, st) == hipSuccess, GS_EHIP, "memset failed");
        return GS_OK;
    }
    GS_REQUIRE(A && dout && out && dW, GS_EINVAL, "NULL device pointer");
    const int S = dw_splits(n);
    const int64_t need = gs_sage_linear_bwd_weight_ws(n, K, H);
    GS_REQUIRE(ws_bytes >= need && (need == 0 || ws), GS_EINVAL, "workspace too small");
    const int rps = static_cast<int>(((n + S - 1) / S + 15) / 16 * 16);
    const int Sx = static_cast<int>((n + rps - 1) / rps);
    float* target = (Sx > 1) ? static_cast<float*>(ws) : dW;
    const bool vload = F % 4 == 0 && lda % 4 == 0 && aligned16(A) && (!self || (ldxs % 4 == 0 && aligned16(Xs)));
    const int SZ = static_cast<int>(((H + 31) / 32) * 32 + 16);
    const size_t smem = (16 * SZ + 16 * 80) * sizeof(float);
    const dim3 grid(static_cast<unsigned>((K + 63) / 64), static_cast<unsigned>(Sx));
    const int nn = static_cast<int>(n), ff = static_cast<int>(F), hh = static_cast<int>(H), kk = static_cast<int>(K);
#define GS_LDW1(TT, SELF, RELU, VL, HW)                                                                   \
    linear_dw_kernel<TT, SELF, RELU, VL, HW><<<grid, kThreads, smem, st>>>(                               \
        nn, ff, hh, kk, rps, static_cast<const TT*>(Xs), ldxs, sidx, static_cast<const TT*>(A), lda, dout, \
        out, ldo, target, H * K)
#define GS_LDW(TT, SELF, RELU, VL) \
    do { if (hh <= 128) GS_LDW1(TT, SELF, RELU, VL, 2); else GS_LDW1(TT, SELF, RELU, VL, 4); } while (0)
#define GS_LDW_V(TT, SELF, RELU) \
    do { if (vload) GS_LDW(TT, SELF, RELU, true); else GS_LDW(TT, SELF, RELU, false); } while (0)
#define GS_LDW_R(TT, SELF) \
    do { if (relu) GS_LDW_V(TT, SELF, true); else GS_LDW_V(TT, SELF, false); } while (0)
#define GS_LDW_S(TT) \
    do { if (self) GS_LDW_R(TT, true); else GS_LDW_R(TT, false); } while (0)
    if (dt == GS_F32) GS_LDW_S(float);
    else GS_LDW_S(bf16_t);
#undef GS_LDW_S
#undef GS_LDW_R
#undef GS_LDW_V
#undef GS_LDW
#undef GS_LDW1
    check_launch("gs_sage_linear_bwd_weight");
    if (Sx > 1) {
        const int64_t len = H * K;
        const dim3 g2(static_cast<unsigned>(std::min<int64_t>((len + kThreads - 1) / kThreads, 2048)));
        sum_slabs_kernel<<<g2, kThreads, 0, st>>>(target, Sx, len, dW);
        check_launch("gs_sage_linear_bwd_weight(sum)");
    }
    GS_API_END
}

int gs_sage_linear_bwd_input(int64_t n, int64_t F, int64_t H, const float* dout, const float* out, int64_t ldo,
                             int32_t relu, const float* W, float* dSelf, float* dA, int64_t ldd, void* stream) {
    GS_API_BEGIN
    using namespace gs;
    GS_REQUIRE(n >= 0 && n < (int64_t(1) << 31) && F >= 1 && H >= 1, GS_EINVAL, "bad sizes");
    if (n == 0) return GS_OK;
    GS_REQUIRE(dout && out && W && dA, GS_EINVAL, "NULL device pointer");
    const bool self = dSelf != nullptr;
    const int64_t K = self ? 2 * F : F;
    const dim3 grid(static_cast<unsigned>((n + 15) / 16), static_cast<unsigned>((K + 63) / 64));
    hipStream_t st = as_stream(stream);
    const int nn = static_cast<int>(n), ff = static_cast<int>(F), hh = static_cast<int>(H), kk = static_cast<int>(K);
#define GS_LDX(SELF, RELU) \
    linear_dx_kernel<SELF, RELU><<<grid, kThreads, 0, st>>>(nn, ff, hh, kk, dout, out, ldo, W, dSelf, dA, ldd)
    if (self) { if (relu) GS_LDX(true, true); else GS_LDX(true, false); }
    else { if (relu) GS_LDX(false, true); else GS_LDX(false, false); }
#undef GS_LDX
    check_launch("gs_sage_linear_bwd_input");
    GS_API_END
}

}  // extern "C"
