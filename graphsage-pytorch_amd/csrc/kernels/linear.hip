// SageLayer (models.py:189-220) on CDNA4 matrix cores.
//   forward : out = relu([Xs[sidx] | A] · Wᵀ)      (:216 cat self-first, :219)
//   backward: dW = dZᵀ · [Xs[sidx] | A],  dIn = dZ · W,  dZ = dOut ⊙ (out > 0)
// The concat is never materialised: the K loop reads its first F columns from
// the gathered self rows and the rest from the aggregate.  fp32 inputs run on
// v_mfma_f32_16x16x4_f32 (exact f32 products, fp32 accumulate); bf16 inputs on
// v_mfma_f32_16x16x32_bf16 with fp32 accumulate.
//
// These GEMMs are skinny (n ~ 0.5-30k rows, H = 128) and so latency-bound,
// not MFMA-bound, when written as a K loop of dependent chunk loads.  Both
// kernels therefore issue the block's whole row tile in one burst (every
// load in flight at once) and only stream the small, L2-resident weight
// through a double-buffered LDS ring whose next chunk is fetched while the
// MFMAs of the current one run.
#include <algorithm>
#include <mutex>
#include <unordered_set>

#include "kcommon.hpp"

namespace gs {

constexpr int kThreads = 256;  // 4 wavefronts
// Dynamic-LDS budget per workgroup: the runtime torch ships rejects requests
// near the 160 KiB hardware size (hipFuncSetAttribute: invalid argument at
// ~156 KB), so every layout below stays within 128 KiB.
constexpr int kLdsMax = 128 * 1024;

// Raise a kernel's dynamic-LDS limit once (the attribute call costs host
// time on every launch otherwise); kLdsMax is always requested so one call
// covers every shape.
template <typename K>
static void allow_smem(K kernel, size_t bytes) {
    if (bytes <= 64 * 1024) return;
    GS_REQUIRE(bytes <= static_cast<size_t>(kLdsMax), GS_EINVAL, "LDS request above budget");
    static std::mutex mu;
    static std::unordered_set<const void*> done;
    const void* key = reinterpret_cast<const void*>(kernel);
    std::lock_guard<std::mutex> lock(mu);
    if (done.count(key)) return;
    const hipError_t e = hipFuncSetAttribute(key, hipFuncAttributeMaxDynamicSharedMemorySize, kLdsMax);
    if (e != hipSuccess) {
        (void)hipGetLastError();  // do not leave a sticky error for the caller's next HIP call
        fail(GS_EHIP, std::string("hipFuncSetAttribute: ") + hipGetErrorString(e));
    }
    done.insert(key);
}

// 16 B of row `row` at element k of the virtual concat [self | agg] (zeros
// past K or past n).  VLOAD: F, K, strides and bases are 16-byte aligned.
template <typename T, bool HAS_SELF, bool VLOAD>
__device__ __forceinline__ uint4 concat_chunk(const T* self_row, const T* agg_row, int F, int K, int k,
                                              bool ok) {
    constexpr int EPV = 16 / sizeof(T);
    uint4 v = make_uint4(0, 0, 0, 0);
    if (!ok) return v;
    if (VLOAD) {
        if (k < K) {
            const T* src = (HAS_SELF && k < F) ? self_row + k : agg_row + (HAS_SELF ? k - F : k);
            v = *reinterpret_cast<const uint4*>(src);
        }
    } else {
        T e[EPV];
#pragma unroll
        for (int q = 0; q < EPV; ++q) {
            const int kk = k + q;
            e[q] = kk < K ? ((HAS_SELF && kk < F) ? self_row[kk] : agg_row[HAS_SELF ? kk - F : kk]) : T(0);
        }
        __builtin_memcpy(&v, e, 16);
    }
    return v;
}

template <typename T, bool VLOAD>
__device__ __forceinline__ uint4 w_chunk(const T* W, int K, int h, int k) {
    constexpr int EPV = 16 / sizeof(T);
    uint4 v = make_uint4(0, 0, 0, 0);
    if (VLOAD) {
        if (k < K) v = *reinterpret_cast<const uint4*>(W + static_cast<int64_t>(h) * K + k);
    } else {
        T e[EPV];
#pragma unroll
        for (int q = 0; q < EPV; ++q) e[q] = (k + q < K) ? W[static_cast<int64_t>(h) * K + k + q] : T(0);
        __builtin_memcpy(&v, e, 16);
    }
    return v;
}

// ---------------------------------------------------------------- forward
// Block = 16 output rows x all H columns; wave w owns column tiles w, w+4, ...
// The A tile (16 rows x KP columns of the concat) sits in LDS; W streams in
// 256-byte-per-row chunks (64 fp32 / 128 bf16) through two LDS buffers.  Each
// lane reads 16 B of a row and feeds 4 fp32 MFMAs (k-slots permuted
// identically for both operands) or one bf16 MFMA.
template <typename T, bool HAS_SELF, bool RELU, bool VLOAD, int NTW>
__global__ __launch_bounds__(kThreads) void linear_fwd_kernel(
    int n, int F, int H, int K, int KP, const T* __restrict__ Xs, int64_t ldxs, const int* __restrict__ sidx,
    const T* __restrict__ A, int64_t lda, const T* __restrict__ W, float* __restrict__ out, int64_t ldo) {
    constexpr int EPV = 16 / sizeof(T);
    constexpr int CH = NTW <= 2 ? 16 : 8;  // 16-byte chunks per W row per step (LDS budget at H = 256)
    constexpr int BK = CH * EPV;
    constexpr int BM = 16;
    constexpr int SW = BK + EPV;
    const int SA = KP + EPV;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    T* sA = reinterpret_cast<T*>(smem);
    T* sW[2] = {sA + BM * SA, sA + BM * SA + H * SW};
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int m0 = blockIdx.x * BM;
    const int nW = (K + BK - 1) / BK;
    const int wper = (H * CH) / kThreads;  // W chunks (16 B) per thread per step: H/16

    uint4 wreg[16];
    auto fetch_w = [&](int c) {
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            if (q >= wper) break;
            const int i = tid + q * kThreads;
            wreg[q] = w_chunk<T, VLOAD>(W, K, i / CH, c * BK + (i % CH) * EPV);
        }
    };
    auto stash_w = [&](int buf) {
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            if (q >= wper) break;
            const int i = tid + q * kThreads;
            *reinterpret_cast<uint4*>(sW[buf] + (i / CH) * SW + (i % CH) * EPV) = wreg[q];
        }
    };

    f32x4 acc[NTW];
#pragma unroll
    for (int t = 0; t < NTW; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
    fetch_w(0);
    const int r = lane & 15, kq = lane >> 4;
    int c = 0;
    for (int p0 = 0; p0 < K; p0 += KP) {
        // the whole A tile of this phase, every load in flight at once
        const int a_chunks = KP / EPV;
        const int a_total = BM * a_chunks;
        for (int base = tid; base < a_total; base += 8 * kThreads) {
            uint4 v[8];  // 8 loads in flight per lane before the first LDS store
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int i = base + u * kThreads;
                const int row = i / a_chunks, cc = i - row * a_chunks;
                const bool ok = i < a_total && m0 + row < n;
                const T* srow = nullptr;
                const T* arow = nullptr;
                if (ok) {
                    if (HAS_SELF) srow = Xs + static_cast<int64_t>(sidx ? sidx[m0 + row] : m0 + row) * ldxs;
                    arow = A + static_cast<int64_t>(m0 + row) * lda;
                }
                v[u] = concat_chunk<T, HAS_SELF, VLOAD>(srow, arow, F, K, p0 + cc * EPV, ok);
            }
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int i = base + u * kThreads;
                if (i >= a_total) break;
                const int row = i / a_chunks, cc = i - row * a_chunks;
                *reinterpret_cast<uint4*>(sA + row * SA + cc * EPV) = v[u];
            }
        }
        const int c_end = min(nW, (p0 + KP) / BK);
        for (; c < c_end; ++c) {
            stash_w(c & 1);
            __syncthreads();
            if (c + 1 < nW) fetch_w(c + 1);  // in flight under this chunk's MFMAs
            const T* a_base = sA + r * SA + (c * BK - p0);
            const T* w_base = sW[c & 1];
#pragma unroll
            for (int g = 0; g < CH / 4; ++g) {
                const uint4 av = *reinterpret_cast<const uint4*>(a_base + (g * 4 + kq) * EPV);
#pragma unroll
                for (int t = 0; t < NTW; ++t) {
                    const int ct = wave + 4 * t;
                    if (ct * 16 >= H) break;
                    const uint4 bv = *reinterpret_cast<const uint4*>(w_base + (ct * 16 + r) * SW + (g * 4 + kq) * EPV);
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
        }
        __syncthreads();  // before the next phase overwrites sA
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
// slab of up to kRS rows (split s): the slab's dZ (relu-masked dOut) and input
// columns are loaded into LDS in one burst, then the MFMA "k" runs over rows,
// both operands read straight from row-major LDS tiles.  Splits write fp32
// partials that sum_slabs_kernel adds in a fixed order (no atomics).
constexpr int kRS = 128;  // slab rows for H <= 128; 64 above (LDS budget)
static inline int dw_rows(int64_t H) { return H <= 128 ? kRS : kRS / 2; }
constexpr int kBKC = 64;
constexpr int kSAc = kBKC + 16;

template <typename T, bool HAS_SELF, bool RELU, bool VLOAD, int HTW>
__global__ __launch_bounds__(kThreads) void linear_dw_kernel(
    int n, int F, int H, int K, int rows_per_split, const T* __restrict__ Xs, int64_t ldxs,
    const int* __restrict__ sidx, const T* __restrict__ A, int64_t lda, const float* __restrict__ dout,
    const float* __restrict__ out, int64_t ldo, bool zvec, float* __restrict__ dst, int64_t split_stride) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int SZ = ((H + 31) / 32) * 32 + 16;  // bank-spread rows for the b32 fragment reads
    float* sZ = reinterpret_cast<float*>(smem);
    const int RS = rows_per_split;  // LDS slab height
    float* sA = sZ + RS * SZ;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int kc0 = blockIdx.x * kBKC;
    const int i_beg = blockIdx.y * rows_per_split;
    const int rows = min(n, i_beg + rows_per_split) - i_beg;
    const int HT = (H + 15) / 16;

    // dZ slab [rows][H]
    if (zvec) {
        const int q4 = H / 4;
        const int total = RS * q4;
        for (int base = tid; base < total; base += 8 * kThreads) {
            float4 z[8], o[8];  // 8 (16 with the relu mask) loads in flight per lane
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int e = base + u * kThreads;
                const int ii = e / q4, h = (e - ii * q4) * 4;
                z[u] = o[u] = make_float4(1.f, 1.f, 1.f, 1.f);
                if (e < total && ii < rows) {
                    const int64_t off = static_cast<int64_t>(i_beg + ii) * ldo + h;
                    z[u] = *reinterpret_cast<const float4*>(dout + off);
                    if (RELU) o[u] = *reinterpret_cast<const float4*>(out + off);
                } else {
                    z[u] = make_float4(0.f, 0.f, 0.f, 0.f);
                }
            }
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int e = base + u * kThreads;
                if (e >= total) break;
                const int ii = e / q4, h = (e - ii * q4) * 4;
                float4 zz = z[u];
                if (RELU) {
                    zz.x = o[u].x > 0.f ? zz.x : 0.f; zz.y = o[u].y > 0.f ? zz.y : 0.f;
                    zz.z = o[u].z > 0.f ? zz.z : 0.f; zz.w = o[u].w > 0.f ? zz.w : 0.f;
                }
                *reinterpret_cast<float4*>(sZ + ii * SZ + h) = zz;
            }
        }
    } else {
        for (int e = tid; e < RS * H; e += kThreads) {
            const int ii = e / H, h = e - ii * H;
            float z = 0.f;
            if (ii < rows) {
                const int64_t off = static_cast<int64_t>(i_beg + ii) * ldo + h;
                z = dout[off];
                if (RELU && !(out[off] > 0.f)) z = 0.f;
            }
            sZ[ii * SZ + h] = z;
        }
    }
    // input slab [rows][64 columns of the concat]
#pragma unroll 8
    for (int e = tid; e < RS * (kBKC / 4); e += kThreads) {
        const int ii = e >> 4, c = (e & 15) * 4, k = kc0 + c;
        float v[4] = {0.f, 0.f, 0.f, 0.f};
        if (ii < rows) {
            const int i = i_beg + ii;
            const T* srow = HAS_SELF ? Xs + static_cast<int64_t>(sidx ? sidx[i] : i) * ldxs : nullptr;
            const T* arow = A + static_cast<int64_t>(i) * lda;
            if (VLOAD && k < K) {
                const T* src = (HAS_SELF && k < F) ? srow + k : arow + (HAS_SELF ? k - F : k);
                if constexpr (sizeof(T) == 4) {
                    const float4 q = *reinterpret_cast<const float4*>(src);
                    v[0] = q.x; v[1] = q.y; v[2] = q.z; v[3] = q.w;
                } else {
                    const uint2 q = *reinterpret_cast<const uint2*>(src);
                    v[0] = __uint_as_float(q.x << 16); v[1] = __uint_as_float(q.x & 0xffff0000u);
                    v[2] = __uint_as_float(q.y << 16); v[3] = __uint_as_float(q.y & 0xffff0000u);
                }
            } else if (!VLOAD) {
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int kk = k + q;
                    if (kk >= K) break;
                    const T x = (HAS_SELF && kk < F) ? srow[kk] : arow[HAS_SELF ? kk - F : kk];
                    if constexpr (sizeof(T) == 4) v[q] = x;
                    else v[q] = bf2f(x);
                }
            }
        }
        *reinterpret_cast<float4*>(sA + ii * kSAc + c) = make_float4(v[0], v[1], v[2], v[3]);
    }
    __syncthreads();

    f32x4 acc[HTW][4];
#pragma unroll
    for (int t = 0; t < HTW; ++t)
#pragma unroll
        for (int c = 0; c < 4; ++c) acc[t][c] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int steps = (rows + 3) / 4;
    for (int s = 0; s < steps; ++s) {
        const int ri = 4 * s + (lane >> 4);
        float b[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) b[c] = sA[ri * kSAc + c * 16 + (lane & 15)];
#pragma unroll
        for (int t = 0; t < HTW; ++t) {
            const int ht = wave + 4 * t;
            if (ht >= HT) break;
            const float a = sZ[ri * SZ + ht * 16 + (lane & 15)];
#pragma unroll
            for (int c = 0; c < 4; ++c) acc[t][c] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b[c], acc[t][c], 0, 0, 0);
        }
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

// out[i] = Σ_s slabs[s][i], fixed order; 4 elements per thread.
__global__ __launch_bounds__(kThreads) void sum_slabs_kernel(const float* __restrict__ slabs, int S,
                                                             int64_t len, float* __restrict__ out) {
    const int64_t n4 = len / 4;
    for (int64_t i = blockIdx.x * int64_t(kThreads) + threadIdx.x; i < n4; i += int64_t(gridDim.x) * kThreads) {
        float4 s = *reinterpret_cast<const float4*>(slabs + 4 * i);
        for (int t = 1; t < S; ++t) {
            const float4 v = *reinterpret_cast<const float4*>(slabs + t * len + 4 * i);
            s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
        }
        *reinterpret_cast<float4*>(out + 4 * i) = s;
    }
    for (int64_t i = 4 * n4 + blockIdx.x * int64_t(kThreads) + threadIdx.x; i < len; i += int64_t(gridDim.x) * kThreads) {
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

static int dw_splits(int64_t n, int64_t H) {
    const int rs = dw_rows(H);
    return static_cast<int>(std::max<int64_t>(1, (n + rs - 1) / rs));
}

// Phase width of the forward's LDS-resident A tile (elements, multiple of the
// W chunk) so that A + two W buffers fit in 160 KiB.
static int fwd_chunks(int H) { return H <= 128 ? 16 : 8; }

static int fwd_phase(int K, int H, size_t esz) {
    const int EPV = static_cast<int>(16 / esz), BK = fwd_chunks(H) * EPV;
    const size_t w_bytes = 2 * static_cast<size_t>(H) * (BK + EPV) * esz;
    const size_t a_budget = kLdsMax - w_bytes - 1024;
    int KP = ((K + BK - 1) / BK) * BK;
    while (KP > BK && 16 * static_cast<size_t>(KP + EPV) * esz > a_budget) KP -= BK;
    return KP;
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
    const int KP = fwd_phase(K, static_cast<int>(H), esz);
    const size_t smem =
        (16 * static_cast<size_t>(KP + EPV) + 2 * static_cast<size_t>(H) * (fwd_chunks(static_cast<int>(H)) * EPV + EPV)) * esz;
    const dim3 grid(static_cast<unsigned>((n + 15) / 16));
    hipStream_t st = as_stream(stream);
    const int nn = static_cast<int>(n), ff = static_cast<int>(F), hh = static_cast<int>(H);
#define GS_LFWD1(TT, SELF, RELU, VL, NT)                                                                  \
    do {                                                                                                  \
        auto kern = linear_fwd_kernel<TT, SELF, RELU, VL, NT>;                                            \
        allow_smem(kern, smem);                                                                           \
        kern<<<grid, kThreads, smem, st>>>(nn, ff, hh, K, KP, static_cast<const TT*>(Xs), ldxs, sidx,     \
                                           static_cast<const TT*>(A), lda, static_cast<const TT*>(Wd),    \
                                           out, ldo);                                                     \
    } while (0)
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
    const int S = gs::dw_splits(n, H);
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
    const int S = dw_splits(n, H);
    const int64_t need = gs_sage_linear_bwd_weight_ws(n, K, H);
    GS_REQUIRE(ws_bytes >= need && (need == 0 || ws), GS_EINVAL, "workspace too small");
    float* target = (S > 1) ? static_cast<float*>(ws) : dW;
    const bool vload = F % 4 == 0 && lda % 4 == 0 && aligned16(A) && (!self || (ldxs % 4 == 0 && aligned16(Xs)));
    const bool zvec = H % 4 == 0 && ldo % 4 == 0 && aligned16(dout) && aligned16(out);
    const int SZ = static_cast<int>(((H + 31) / 32) * 32 + 16);
    const int RS = dw_rows(H);
    const size_t smem = static_cast<size_t>(RS) * (SZ + kSAc) * sizeof(float);
    const dim3 grid(static_cast<unsigned>((K + kBKC - 1) / kBKC), static_cast<unsigned>(S));
    const int nn = static_cast<int>(n), ff = static_cast<int>(F), hh = static_cast<int>(H), kk = static_cast<int>(K);
#define GS_LDW1(TT, SELF, RELU, VL, HW)                                                                   \
    do {                                                                                                  \
        auto kern = linear_dw_kernel<TT, SELF, RELU, VL, HW>;                                             \
        allow_smem(kern, smem);                                                                           \
        kern<<<grid, kThreads, smem, st>>>(nn, ff, hh, kk, RS, static_cast<const TT*>(Xs), ldxs, sidx,    \
                                           static_cast<const TT*>(A), lda, dout, out, ldo, zvec, target,  \
                                           H * K);                                                        \
    } while (0)
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
    if (S > 1) {
        const int64_t len = H * K;
        const dim3 g2(static_cast<unsigned>(std::min<int64_t>((len / 4 + kThreads - 1) / kThreads + 1, 2048)));
        sum_slabs_kernel<<<g2, kThreads, 0, st>>>(target, S, len, dW);
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
