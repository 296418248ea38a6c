#pragma once
// SageLayer (models.py:189-220) on CDNA4 matrix cores.
//   forward : out = relu([Xs[sidx] | A] · Wᵀ)      (:216 cat self-first, :219)
//   backward: dW = dZᵀ · [Xs[sidx] | A],  dIn = dZ · W,  dZ = dOut ⊙ (out > 0)
// The concat is never materialised: a K chunk reads its first F columns from
// the gathered self rows and the rest from the aggregate.  fp32 inputs run on
// v_mfma_f32_16x16x4_f32 (exact f32 products, fp32 accumulate); bf16 inputs on
// v_mfma_f32_16x16x32_bf16 with fp32 accumulate.
//
// These GEMMs are skinny (n ~ 0.5-30k rows, H <= 256, K <= a few thousand),
// so what sets their time is how many dependent memory round trips a wave
// waits through, not MFMA issue.  Every load below is therefore branch-free
// (addresses clamped into range, values masked with a select afterwards) so
// the compiler can keep a whole chunk's loads in flight, and each K (or row)
// chunk's loads are issued one chunk ahead, under the MFMAs of the current
// one, with a single workgroup barrier per chunk.

#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "cls_dev.hpp"

#include "kcommon.hpp"

namespace gs {

constexpr int kThreads = 256;  // 4 wavefronts
constexpr int kSlots = 16;     // 16-byte slots per row per K chunk (64 fp32 / 128 bf16)

// One 16-byte slot of the virtual concat row [self | agg] starting at element
// k; zeros at and past K.  VLOAD: F, strides and bases are 16-byte aligned,
// so a slot never straddles the self/agg seam.
template <typename T, bool HAS_SELF, bool VLOAD>
__device__ __forceinline__ uint4 concat_slot(const T* srow, const T* arow, int F, int K, int k) {
    constexpr int EPV = 16 / sizeof(T);
    if constexpr (VLOAD) {
        const bool in = k < K;
        const int kk = in ? k : 0;
        const T* p = (HAS_SELF && kk < F) ? srow + kk : arow + (HAS_SELF ? kk - F : kk);
        const uint4 v = *reinterpret_cast<const uint4*>(p);
        return in ? v : make_uint4(0, 0, 0, 0);
    } else {
        T e[EPV];
#pragma unroll
        for (int q = 0; q < EPV; ++q) {
            const int k1 = k + q;
            const bool in = k1 < K;
            const int kk = in ? k1 : 0;
            const T x = (HAS_SELF && kk < F) ? srow[kk] : arow[HAS_SELF ? kk - F : kk];
            e[q] = in ? x : T(0);
        }
        uint4 v;
        __builtin_memcpy(&v, e, 16);
        return v;
    }
}

// concat_slot's load alone (VLOAD layout): the address clamped into the row,
// no select on the value.  A select right after a load lets the compiler turn
// it into an exec-masked load in its own basic block, and the wait-count pass
// then drains every load in flight (vmcnt(0)) at the next use of any of them:
// the K loop's prefetch ring would be gone.  Callers zero slots at and past K
// when they stash them (slot_in_range).
template <typename T, bool HAS_SELF>
__device__ __forceinline__ uint4 concat_slot_raw(const T* srow, const T* arow, int F, int K, int k) {
    const int kk = k < K ? k : 0;
    const T* p = (HAS_SELF && kk < F) ? srow + kk : arow + (HAS_SELF ? kk - F : kk);
    return *reinterpret_cast<const uint4*>(p);
}

__device__ __forceinline__ uint4 slot_in_range(uint4 v, int k, int K) {
    const bool in = k < K;
    v.x = in ? v.x : 0u; v.y = in ? v.y : 0u; v.z = in ? v.z : 0u; v.w = in ? v.w : 0u;
    return v;
}

// 4 consecutive elements of the concat row as floats (dW operand).
template <typename T, bool HAS_SELF, bool VLOAD>
__device__ __forceinline__ float4 concat_quad(const T* srow, const T* arow, int F, int K, int k) {
    float v[4];
    if constexpr (VLOAD) {
        const bool in = k < K;
        const int kk = in ? k : 0;
        const T* p = (HAS_SELF && kk < F) ? srow + kk : arow + (HAS_SELF ? kk - F : kk);
        if constexpr (sizeof(T) == 4) {
            const float4 q = *reinterpret_cast<const float4*>(p);
            v[0] = q.x; v[1] = q.y; v[2] = q.z; v[3] = q.w;
        } else {
            const uint2 q = *reinterpret_cast<const uint2*>(p);
            v[0] = __uint_as_float(q.x << 16); v[1] = __uint_as_float(q.x & 0xffff0000u);
            v[2] = __uint_as_float(q.y << 16); v[3] = __uint_as_float(q.y & 0xffff0000u);
        }
        if (!in) v[0] = v[1] = v[2] = v[3] = 0.f;
    } else {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int k1 = k + q;
            const bool in = k1 < K;
            const int kk = in ? k1 : 0;
            const T x = (HAS_SELF && kk < F) ? srow[kk] : arow[HAS_SELF ? kk - F : kk];
            float f;
            if constexpr (sizeof(T) == 4) f = x;
            else f = bf2f(x);
            v[q] = in ? f : 0.f;
        }
    }
    return make_float4(v[0], v[1], v[2], v[3]);
}

// 4 consecutive floats of a row at column c (< lim masked to 0).  VEC: the
// row, c and lim are multiples of 4 floats.
template <bool VEC>
__device__ __forceinline__ float4 row_quad(const float* row, int c, int lim) {
    if constexpr (VEC) {
        const bool in = c < lim;
        const float4 v = *reinterpret_cast<const float4*>(row + (in ? c : 0));
        return in ? v : make_float4(0.f, 0.f, 0.f, 0.f);
    } else {
        float v[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const bool in = c + q < lim;
            const float x = row[in ? c + q : 0];
            v[q] = in ? x : 0.f;
        }
        return make_float4(v[0], v[1], v[2], v[3]);
    }
}

// Unmasked variants for loops that issue loads well before using them: the
// address is clamped into range and mask_quad zeroes the out-of-range
// elements at the point of use (a select right after the load would force a
// wait for it there).
template <bool VEC>
__device__ __forceinline__ float4 row_quad_raw(const float* row, int c, int lim) {
    if constexpr (VEC) {
        return *reinterpret_cast<const float4*>(row + (c < lim ? c : 0));
    } else {
        float v[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] = row[c + q < lim ? c + q : 0];
        return make_float4(v[0], v[1], v[2], v[3]);
    }
}

template <typename T, bool HAS_SELF, bool VLOAD>
__device__ __forceinline__ float4 concat_quad_raw(const T* srow, const T* arow, int F, int K, int k) {
    float v[4];
    if constexpr (VLOAD) {
        const int kk = k < K ? k : 0;
        const T* p = (HAS_SELF && kk < F) ? srow + kk : arow + (HAS_SELF ? kk - F : kk);
        if constexpr (sizeof(T) == 4) {
            const float4 q = *reinterpret_cast<const float4*>(p);
            v[0] = q.x; v[1] = q.y; v[2] = q.z; v[3] = q.w;
        } else {
            const uint2 q = *reinterpret_cast<const uint2*>(p);
            v[0] = __uint_as_float(q.x << 16); v[1] = __uint_as_float(q.x & 0xffff0000u);
            v[2] = __uint_as_float(q.y << 16); v[3] = __uint_as_float(q.y & 0xffff0000u);
        }
    } else {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int kk = k + q < K ? k + q : 0;
            const T x = (HAS_SELF && kk < F) ? srow[kk] : arow[HAS_SELF ? kk - F : kk];
            if constexpr (sizeof(T) == 4) v[q] = x;
            else v[q] = bf2f(x);
        }
    }
    return make_float4(v[0], v[1], v[2], v[3]);
}

__device__ __forceinline__ float4 mask_quad(float4 v, int c, int lim) {
    v.x = c < lim ? v.x : 0.f; v.y = c + 1 < lim ? v.y : 0.f;
    v.z = c + 2 < lim ? v.z : 0.f; v.w = c + 3 < lim ? v.w : 0.f;
    return v;
}

__device__ __forceinline__ float4 relu_mask(float4 z, float4 o) {
    z.x = o.x > 0.f ? z.x : 0.f; z.y = o.y > 0.f ? z.y : 0.f;
    z.z = o.z > 0.f ? z.z : 0.f; z.w = o.w > 0.f ? z.w : 0.f;
    return z;
}

template <typename T>
__device__ __forceinline__ f32x4 mfma_slot(uint4 a, uint4 b, f32x4 acc) {
    if constexpr (sizeof(T) == 4) {
        // k-slots permuted identically on both operands: MFMA j sums element j
        // of the four kq lanes' slots, so the four MFMAs cover all 16 k.
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a.x), __uint_as_float(b.x), acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a.y), __uint_as_float(b.y), acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a.z), __uint_as_float(b.z), acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a.w), __uint_as_float(b.w), acc, 0, 0, 0);
    } else {
        s16x8 a8, b8;
        __builtin_memcpy(&a8, &a, 16);
        __builtin_memcpy(&b8, &b, 16);
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a8, b8, acc, 0, 0, 0);
    }
    return acc;
}

// ---------------------------------------------------------------- forward
// Block = 16 rows x 64 output columns (wave w: columns 16·(4·by + w) ..).
// Per K chunk each thread loads one slot of the 16-row concat tile into a
// two-buffer LDS ring (shared by the 4 waves) and each lane loads the four
// W slots its MFMAs consume straight into registers (W rows are private to a
// wave).  Lane (r, kq) feeds MFMA group g with slot 4g + kq of row r.
template <typename T, bool HAS_SELF, bool RELU, bool VLOAD>
__global__ __launch_bounds__(kThreads) void linear_fwd_kernel(
    int n, int F, int H, int K, const T* __restrict__ Xs, int64_t ldxs, const int* __restrict__ sidx,
    const T* __restrict__ A, int64_t lda, const T* __restrict__ W, float* __restrict__ out, int64_t ldo) {
    constexpr int EPV = 16 / sizeof(T);
    constexpr int BK = kSlots * EPV;
    constexpr int SA = kSlots + 1;  // LDS row pitch in slots: rows land 4 banks apart
    __shared__ uint4 sA[2][16 * SA];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int r = lane & 15, kq = lane >> 4;
    const int m0 = blockIdx.x * 16;
    const int ct = blockIdx.y * 4 + wave;
    const int ar = tid >> 4, as = tid & 15;
    const int arow_i = min(m0 + ar, n - 1);
    const T* arow = A + static_cast<int64_t>(arow_i) * lda;
    const T* srow = HAS_SELF ? Xs + static_cast<int64_t>(sidx ? sidx[arow_i] : arow_i) * ldxs : nullptr;
    const T* wrow = W + static_cast<int64_t>(min(ct * 16 + r, H - 1)) * K;
    const int nC = (K + BK - 1) / BK;

    uint4 a_nx = concat_slot<T, HAS_SELF, VLOAD>(srow, arow, F, K, as * EPV);
    uint4 w_nx[4];
#pragma unroll
    for (int g = 0; g < 4; ++g) w_nx[g] = concat_slot<T, false, VLOAD>(nullptr, wrow, K, K, (4 * g + kq) * EPV);
    sA[0][ar * SA + as] = a_nx;
    f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int c = 0; c < nC; ++c) {
        uint4 w_cur[4];
#pragma unroll
        for (int g = 0; g < 4; ++g) w_cur[g] = w_nx[g];
        __syncthreads();
        // next chunk (the last iteration re-reads its own chunk; discarded)
        const int kn = min(c + 1, nC - 1) * BK;
        a_nx = concat_slot<T, HAS_SELF, VLOAD>(srow, arow, F, K, kn + as * EPV);
#pragma unroll
        for (int g = 0; g < 4; ++g) w_nx[g] = concat_slot<T, false, VLOAD>(nullptr, wrow, K, K, kn + (4 * g + kq) * EPV);
        __builtin_amdgcn_sched_barrier(0);  // prefetch issued ahead of the chunk's LDS reads and MFMAs
        const uint4* tile = sA[c & 1];
        uint4 av[4];
#pragma unroll
        for (int g = 0; g < 4; ++g) av[g] = tile[r * SA + 4 * g + kq];
#pragma unroll
        for (int g = 0; g < 4; ++g) acc = mfma_slot<T>(av[g], w_cur[g], acc);
        __builtin_amdgcn_sched_barrier(0);  // keep the wait for the prefetch behind every MFMA
        sA[(c + 1) & 1][ar * SA + as] = a_nx;
    }
    if (ct * 16 >= H) return;
    const int col = ct * 16 + r;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int row = m0 + 4 * kq + j;
        if (row < n) {
            const float v = acc[j];
            out[static_cast<int64_t>(row) * ldo + col] = (RELU && !(v > 0.f) && v == v) ? 0.f : v;  // NaN kept, as torch.relu
        }
    }
}

// Forward, fp32, W staged in LDS ("wide" tiles).  Block = ROWS rows x 64
// output columns, ROWS/4 waves: wave (wr, wc) = (w % (ROWS/16), w / (ROWS/16))
// owns the 16 x 16 tile at rows 16·wr, cols 16·wc.  Per K chunk of 64 every
// thread loads one 16-byte slot of the A tile and 64/ROWS slots of the W tile
// into a two-buffer LDS ring, one chunk ahead.  Against the 16-row kernel
// this reads each W chunk once per ROWS rows instead of once per 16.  ROWS =
// 32 (8 waves, ~270 blocks at the rmat2m layer-1 shape) is the fp32 default:
// W traffic from L2 halves while the grid still covers the chip.
constexpr int kWideRows = 64;
#ifndef GS_FWD_STAMP  // stage stamps for tools/lab/fwd_lab.hip; no-ops in the library
#define GS_FWD_STAMP(i)
#endif
#ifndef GS_FWD_AHEAD
#define GS_FWD_AHEAD 2
#endif
constexpr int kFwdAhead = GS_FWD_AHEAD;  // K chunks in flight ahead of the MFMAs (wide kernels)
// T = bf16_t: the same tiles with 8 elements per slot (a chunk is 128 k) and
// the 16x16x32 bf16 MFMA per slot pair — operands and order of the chunked
// bf16 kernel (slots 4g + kq, chunks ascending), so bitwise its output.
// The pending clip + SGD of the previous step (sp.on, fp32 only; FwdSpec in
// kcommon.hpp), run in the forward's prologue.  fwd_pending_issue loads the
// norm partials and this thread's share of the other parameters (W2, Wc, bc:
// thread t of block b takes quad b + nblk·t) before the forward's own first
// loads, so waiting for them (vmcnt retires in order) never waits for a K
// chunk; fwd_pending_apply then folds the partials (clip_fold's sums: the
// coefficients sgd4 would compute), updates those parameters (their readers
// come after this launch) and returns whether W1 is not the speculative
// update sp.S (the coefficient of its group is not 1).  In that case the
// workgroup writes its own 64-row slice of the update into sp.Wn (= S's
// buffer; every workgroup of a column tile writes the same values there),
// releases it, and the caller reloads its first chunks: the same W1 the
// separate SGD launch would have left, so the same output bit for bit.
// One quad of the other parameters' update (clip coefficient m).
__device__ __forceinline__ void sgd_quad(float4* p4, float4* g4, int64_t i, float4 pv, float4 gv, float m, float lr) {
    float4 gi, pn;
    pn.x = sgd_elem(pv.x, gv.x, m, lr, gi.x);
    pn.y = sgd_elem(pv.y, gv.y, m, lr, gi.y);
    pn.z = sgd_elem(pv.z, gv.z, m, lr, gi.z);
    pn.w = sgd_elem(pv.w, gv.w, m, lr, gi.w);
    g4[i] = gi;
    p4[i] = pn;
}

// The rest of the pending update once the coefficients are known: the other
// parameters' quads past the first (only for grids of fewer threads than
// quads), then, if W1's coefficient is not 1, this column tile's rows of W1's
// update into sp.Wn, released and visible to the workgroup.  Returns whether
// it wrote them (the caller reloads its first chunks).
__device__ __forceinline__ bool fwd_pending_rest(const FwdSpec& sp, int64_t i0, float m0, float m1, int H, int K,
                                                 int c0) {
    const int64_t stride = int64_t(gridDim.x) * gridDim.y * blockDim.x;
    float4* p4 = reinterpret_cast<float4*>(sp.p);
    float4* g4 = reinterpret_cast<float4*>(sp.g);
    for (int64_t i = i0 + stride; i < sp.up_hi / 4; i += stride)
        sgd_quad(p4, g4, i, p4[i], g4[i], 4 * i >= sp.grp1_lo ? m1 : m0, sp.lr);
    if (m0 == sp.scale) return false;  // clip coefficient 1: S is the update
    const int k4 = K / 4, rows = min(64, H - c0);
    const float4* P4 = reinterpret_cast<const float4*>(sp.P) + int64_t(c0) * k4;
    const float4* G4 = reinterpret_cast<const float4*>(sp.G1) + int64_t(c0) * k4;
    float4* N4 = reinterpret_cast<float4*>(sp.Wn) + int64_t(c0) * k4;
    uint2* L4 = sp.Wn_lp ? reinterpret_cast<uint2*>(sp.Wn_lp) + int64_t(c0) * k4 : nullptr;
    for (int i = threadIdx.x; i < rows * k4; i += blockDim.x) {
        const float4 pv = P4[i], gv = G4[i];
        float4 gi, pn;
        pn.x = sgd_elem(pv.x, gv.x, m0, sp.lr, gi.x);
        pn.y = sgd_elem(pv.y, gv.y, m0, sp.lr, gi.y);
        pn.z = sgd_elem(pv.z, gv.z, m0, sp.lr, gi.z);
        pn.w = sgd_elem(pv.w, gv.w, m0, sp.lr, gi.w);
        N4[i] = pn;
        if (L4) {  // the bf16 W1 the forward reads (sgd4's shadow conversion)
            uint2 b;
            b.x = static_cast<uint32_t>(f2bf(pn.x)) | (static_cast<uint32_t>(f2bf(pn.y)) << 16);
            b.y = static_cast<uint32_t>(f2bf(pn.z)) | (static_cast<uint32_t>(f2bf(pn.w)) << 16);
            L4[i] = b;
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    __syncthreads();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");  // no stale L1 lines of the speculative S
    return true;
}

// W is not __restrict__: with PEND a recomputed W1 is written into W's buffer
// (sp.Wn) and read back through W by the second K loop.
// Row split of the wide forward: `groups` workgroups per column tile, the
// first `extra` of them take base + 1 row tiles of 16, the rest base (the
// launcher sizes groups to one workgroup per CU, so no CU runs two while
// others idle: with fixed 32-row tiles 276 workgroups on 256 CUs left 20 CUs
// with two, and the launch waited ~1.5x a workgroup's time for them).
struct FwdRows {
    int base = 0, extra = 0, groups = 0;
};

template <typename T, int ROWS, bool HAS_SELF, bool RELU, bool PEND = false>
__global__ __launch_bounds__(ROWS * 16) void linear_fwd_wide_kernel(
    int n, int F, int H, int K, const T* __restrict__ Xs, int64_t ldxs, const int* __restrict__ sidx,
    const T* __restrict__ A, int64_t lda, const T* W, float* __restrict__ out, int64_t ldo,
    FwdRows rs, FwdSpec sp) {
    GS_FWD_STAMP(0);
    kstamp_begin(sp.stamp);
    constexpr int EPV = 16 / sizeof(T);  // elements per 16-byte slot
    constexpr int BK = kSlots * EPV;     // k per chunk
    constexpr int SP = kSlots + 1;  // row pitch in 16-byte slots: 16 rows of one slot column hit distinct banks
    constexpr int RT = ROWS / 16;   // row tiles
    constexpr int WQ = (64 + ROWS - 1) / ROWS;  // W slots per thread (ROWS = 48: the second only for lr < 16)
    static_assert(ROWS % 16 == 0 && ROWS <= 64, "row tiles of 16, at most 64 rows");
    __shared__ uint4 sA[2][ROWS * SP];
    __shared__ uint4 sW[2][64 * SP];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int r = lane & 15, kq = lane >> 4;
    const int wr = wave % RT, wc = wave / RT;
    // 1-D grid (the launcher's XCD map): the gy column tiles of row tile x are
    // blocks 8 apart in dispatch order, i.e. on one XCD under round-robin
    // placement, so the second column tile re-reads the A rows from that
    // XCD's L2 instead of HBM / MALL.  2-D grid: x = row tile, y = column tile.
    int bx = blockIdx.x, by = blockIdx.y;
    if (gridDim.y == 1 && H > 64) {
        const int gy = (H + 63) / 64, b = blockIdx.x;
        bx = (b / (8 * gy)) * 8 + (b & 7);
        by = (b >> 3) % gy;
    }
    const int nt = rs.base + (bx < rs.extra ? 1 : 0);  // row tiles of this workgroup (<= RT)
    const int m0 = 16 * (bx * rs.base + min(bx, rs.extra)), c0 = by * 64;
    // PEND: the pending update's loads before the first chunk's, branch-free
    // (the launcher guarantees 1 <= np0, np1 <= 512: clip_fold's one round),
    // so the fold's waits count past the K chunks' loads: the norm partials
    // and this thread's quad of the other parameters (thread t of block b:
    // quad b + nblk·t; a thread past them reads the last one and stores nothing)
    FoldLoads f0, f1;
    float4 upv, ugv;
    const int64_t ui0 = sp.up_lo / 4 + (int64_t(blockIdx.y) * gridDim.x + blockIdx.x) +
                        int64_t(gridDim.x) * gridDim.y * threadIdx.x;
    if constexpr (PEND) {
        clip_fold_issue(sp.part0, sp.np0, lane, f0);
        clip_fold_issue(sp.part1, sp.np1, lane, f1);
        const int64_t ui = min(ui0, sp.up_hi / 4 - 1);
        upv = reinterpret_cast<const float4*>(sp.p)[ui];
        ugv = reinterpret_cast<const float4*>(sp.g)[ui];
    }
    // the coefficients and the update of this thread's quad (before W1 is read)
    auto pending_apply = [&]() -> bool {
        const float mm0 = clip_mult(clip_fold_finish(sp.np0, lane, f0), sp.scale, sp.max_norm);
        const float mm1 = clip_mult(clip_fold_finish(sp.np1, lane, f1), sp.scale, sp.max_norm);
        if (ui0 < sp.up_hi / 4)
            sgd_quad(reinterpret_cast<float4*>(sp.p), reinterpret_cast<float4*>(sp.g), ui0, upv, ugv,
                     4 * ui0 >= sp.grp1_lo ? mm1 : mm0, sp.lr);
        return fwd_pending_rest(sp, ui0, mm0, mm1, H, K, c0);
    };
    if (bx >= rs.groups || m0 >= n) {  // spare blocks of the last group of 8 (they still take their share of the update)
        if constexpr (PEND) pending_apply();
        kstamp_end(sp.stamp);
        return;
    }
    const int lr = tid >> 4, ls = tid & 15;  // this thread's load: row lr (+ ROWS·q of W), slot ls
    const int arow_i = min(m0 + min(lr, 16 * nt - 1), n - 1);  // rows past this workgroup's: its last one
    const T* arow = A + static_cast<int64_t>(arow_i) * lda;
    const T* srow = HAS_SELF ? Xs + static_cast<int64_t>(sidx ? sidx[arow_i] : arow_i) * ldxs : nullptr;
    const T* wrow[WQ];
#pragma unroll
    for (int q = 0; q < WQ; ++q) wrow[q] = W + static_cast<int64_t>(min(c0 + min(lr + ROWS * q, 63), H - 1)) * K;
    const int nC = (K + BK - 1) / BK;
    // register ring of kFwdAhead chunks: slot u holds chunk c (c = u mod
    // kFwdAhead) once it is in LDS and is then refilled with chunk c + kFwdAhead
    uint4 ar[kFwdAhead], wr_[kFwdAhead][WQ];
    auto load = [&](int c, int u) {
        const int kn = min(c, nC - 1) * BK;  // past the end: re-read the last chunk (never stored)
        ar[u] = concat_slot_raw<T, HAS_SELF>(srow, arow, F, K, kn + ls * EPV);
#pragma unroll
        for (int q = 0; q < WQ; ++q) wr_[u][q] = concat_slot_raw<T, false>(nullptr, wrow[q], K, K, kn + ls * EPV);
    };
    auto stash = [&](int c, int u) {
        const int k = c * BK + ls * EPV;  // slots at and past K are zeros (both operands)
        sA[c & 1][lr * SP + ls] = slot_in_range(ar[u], k, K);
#pragma unroll
        for (int q = 0; q < WQ; ++q)
            if (64 % ROWS == 0 || lr + ROWS * q < 64) sW[c & 1][(lr + ROWS * q) * SP + ls] = slot_in_range(wr_[u][q], k, K);
    };
    auto run_k = [&]() -> f32x4 {
#pragma unroll
        for (int u = 0; u < kFwdAhead; ++u) load(u, u);
        stash(0, 0);
        f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
        GS_FWD_STAMP(1);
        // Every load and stash is unconditional (past the end: the last
        // chunk's slots re-read, zeros stored into a buffer no wave reads
        // again); only the MFMAs of a chunk past the end are skipped.  A
        // guarded stash lets the compiler sink the slot's load into the
        // guarded block, next to its use, and a loop exit between the ring's
        // loads leaves paths with different loads in flight, which the
        // wait-count pass merges into a full drain at the loop head.
        for (int cb = 0; cb < nC; cb += kFwdAhead) {
#pragma unroll
            for (int u = 0; u < kFwdAhead; ++u) {
                const int c = cb + u;
                __syncthreads();
                load(c + kFwdAhead, u);
                __builtin_amdgcn_sched_barrier(0);
                if ((kFwdAhead == 1 || c < nC) && wr < nt) {
                    const uint4* ta = sA[c & 1] + (16 * wr + r) * SP;
                    const uint4* tw = sW[c & 1] + (16 * wc + r) * SP;
                    uint4 av[4], wv[4];
#pragma unroll
                    for (int g = 0; g < 4; ++g) {
                        av[g] = ta[4 * g + kq];
                        wv[g] = tw[4 * g + kq];
                    }
#pragma unroll
                    for (int g = 0; g < 4; ++g) acc = mfma_slot<T>(av[g], wv[g], acc);
                }
                __builtin_amdgcn_sched_barrier(0);
                stash(c + 1, (u + 1) % kFwdAhead);
            }
        }
        return acc;
    };
    f32x4 acc = run_k();  // PEND: on the speculative W1 (sp.S)
    GS_FWD_STAMP(2);
    if constexpr (PEND) {
        // the fold after the K loop (its loads long done): the coefficients,
        // the other parameters' update, and, when W1's coefficient is not 1,
        // the recomputed W1 in S's buffer and the whole product again
        if (pending_apply()) acc = run_k();
    }
    GS_FWD_STAMP(3);
    const int col = c0 + 16 * wc + r;
    if (col < H && wr < nt) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int row = m0 + 16 * wr + 4 * kq + j;
            if (row < n) {
                const float v = acc[j];
                out[static_cast<int64_t>(row) * ldo + col] = (RELU && !(v > 0.f) && v == v) ? 0.f : v;
            }
        }
    }
    GS_FWD_STAMP(4);
    kstamp_end(sp.stamp);
}

// ------------------------------------------------------------ weight grad
// dW[h][k] = Σ_i dZ[i][h] · In[i][k].  Block = 64 h x 64 k over one slab of
// rows (blockIdx.z); wave w owns h rows 16w.. of the tile and 4 k tiles.  Rows
// stream in chunks of 16 through a two-buffer LDS ring (thread: 4 dZ values
// and 4 inputs of one row per chunk); the MFMA "k" runs over rows.  Slabs
// write fp32 partials that sum_slabs_kernel adds in a fixed order.
constexpr int kDwPitch = 64 + 16;  // rows 16 banks apart: (kq, r) reads of a column hit distinct banks
constexpr int kDwMaxSlab = 2048;  // rows per slab (their self indices are staged in LDS)
#ifndef GS_DW_CHUNK
#define GS_DW_CHUNK 16
#endif
constexpr int kDwCh = GS_DW_CHUNK;  // rows per LDS chunk (one barrier each); 16 or 32
static_assert(kDwCh == 16 || kDwCh == 32, "dW chunk rows");
constexpr int kDwRpt = kDwCh / 16;  // rows each thread loads per chunk
constexpr int kDwAhead = 2;  // row chunks whose global loads are in flight ahead of their stash
#ifndef GS_DW_STAMP
#define GS_DW_STAMP(i) ((void)0)  // stage stamps of tools/lab/dw_lab.hip
#endif

// PH row phases (blockDim = 256·PH): the waves of phase ph run the chunks
// ph, ph + PH, ... of the slab on their own LDS ring (one barrier per
// iteration for the whole block), each into its own accumulators; at the end
// phase 1 hands its sums to phase 0 through LDS, which adds them (fixed order,
// so deterministic) and stores the slab.  PH = 2 puts twice the rows in a slab
// at the same chunk loop length: half the slabs (and half the split-K bytes
// the slab sum re-reads) for the same per-workgroup latency.
// The body's LDS, declared by the kernel (one object for every role of a
// fused launch: two roles' own static arrays would add up per block).
template <int PH>
struct DwSmem {
    float sbuf[PH][2][2][kDwCh * kDwPitch];  // [phase][dZ | inputs][ring buffer]
    int sIdx[kDwMaxSlab];                    // the slab's self indices (HAS_SELF)
};

template <typename T, bool HAS_SELF, bool RELU, bool VLOAD, bool ZVEC, int PH = 1>
__device__ __forceinline__ void linear_dw_body(
    int bx, int by, int bz, int n, int F, int H, int K, int rows_per_split, const T* __restrict__ Xs, int64_t ldxs,
    const int* __restrict__ sidx, const T* __restrict__ A, int64_t lda, const float* __restrict__ dout,
    const float* __restrict__ out, int64_t ldo, float* __restrict__ dst, int64_t split_stride, DwSmem<PH>& sm) {
    static_assert(PH == 1 || PH == 2, "one or two row phases");
    auto& sbuf = sm.sbuf;
    int* sIdx = sm.sIdx;
    const int ph = PH == 1 ? 0 : static_cast<int>(threadIdx.x >> 8);
    const int tid = threadIdx.x & (kThreads - 1), lane = tid & 63, wave = tid >> 6;
    float (&sZ)[2][kDwCh * kDwPitch] = sbuf[ph][0];
    float (&sI)[2][kDwCh * kDwPitch] = sbuf[ph][1];
    const int r = lane & 15, kq = lane >> 4;
    const int k0 = bx * 64, h0 = by * 64;
    const int i_beg = bz * rows_per_split;
    const int i_end = min(n, i_beg + rows_per_split);
    const int nC = (i_end - i_beg + kDwCh - 1) / kDwCh;
    const int nI = (nC + PH - 1) / PH;  // iterations: this phase's chunks (the last may be past the slab: zeros)
    const int lr = tid >> 4, lq = (tid & 15) * 4;
    GS_DW_STAMP(0);
    if (HAS_SELF)  // (PH = 1 indexes by tid: a 512-thread block may run two 256-thread bodies side by side)
        for (int t = PH == 1 ? tid : static_cast<int>(threadIdx.x); t < i_end - i_beg; t += kThreads * PH)
            sIdx[t] = sidx ? sidx[i_beg + t] : i_beg + t;
    __syncthreads();

    // Rows past the slab read a valid row and are zeroed at the LDS store
    // (both operands: 0 · NaN would not vanish).  Chunks past the end re-read
    // the last one (their data is never stashed).  Thread rows: lr + 16 q.
    struct Ld {
        float4 z[kDwRpt], o[kDwRpt], x[kDwRpt];
    };
    auto load = [&](int it, Ld& L) {
        const int c = PH * it + ph;
#pragma unroll
        for (int q = 0; q < kDwRpt; ++q) {
            const int t = min(kDwCh * min(c, nC - 1) + lr + 16 * q, i_end - i_beg - 1);
            const int ic = i_beg + t;
            L.z[q] = row_quad_raw<ZVEC>(dout + static_cast<int64_t>(ic) * ldo, h0 + lq, H);
            if (RELU) L.o[q] = row_quad_raw<ZVEC>(out + static_cast<int64_t>(ic) * ldo, h0 + lq, H);
            const T* arow = A + static_cast<int64_t>(ic) * lda;
            const T* srow = HAS_SELF ? Xs + static_cast<int64_t>(sIdx[t]) * ldxs : nullptr;
            L.x[q] = concat_quad_raw<T, HAS_SELF, VLOAD>(srow, arow, F, K, k0 + lq);
        }
    };
    auto stash = [&](int it, const Ld& L) {
        const int c = PH * it + ph;
#pragma unroll
        for (int q = 0; q < kDwRpt; ++q) {
            float4 z = mask_quad(L.z[q], h0 + lq, H);
            if (RELU) z = relu_mask(z, L.o[q]);
            float4 x = mask_quad(L.x[q], k0 + lq, K);
            const int row = lr + 16 * q;
            if (kDwCh * c + row >= i_end - i_beg) z = x = make_float4(0.f, 0.f, 0.f, 0.f);
            *reinterpret_cast<float4*>(&sZ[it & 1][row * kDwPitch + lq]) = z;
            *reinterpret_cast<float4*>(&sI[it & 1][row * kDwPitch + lq]) = x;
        }
    };
    f32x4 acc[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
    // A chunk's MFMA operands in registers: lane (r, kq) holds, for row group
    // s, the input X[4s + kq][k0 + 16t + r] of each k tile t and the gradient
    // dZ[4s + kq][h0 + 16·wave + r].  The MFMA takes the inputs as its A
    // operand, so lane (r, kq) of tile t ends with dW[h0 + 16·wave + r][k0 +
    // 16t + 4kq .. +3]: four consecutive k, one 16-byte store.  Rows in
    // ascending groups of 4 (the same sequence for any chunk size).
    constexpr int NS = kDwCh / 4;
    struct Ops {
        float z[NS], x[NS][4];
    };
    auto read_ops = [&](int it, Ops& o) {
        const float* tz = sZ[it & 1];
        const float* ti = sI[it & 1];
#pragma unroll
        for (int s = 0; s < NS; ++s) {
            const int row = 4 * s + kq;
            o.z[s] = tz[row * kDwPitch + wave * 16 + r];
#pragma unroll
            for (int t = 0; t < 4; ++t) o.x[s][t] = ti[row * kDwPitch + t * 16 + r];
        }
    };
    auto mfma_ops = [&](const Ops& o) {
#pragma unroll
        for (int s = 0; s < NS; ++s)
#pragma unroll
            for (int t = 0; t < 4; ++t) acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(o.x[s][t], o.z[s], acc[t], 0, 0, 0);
    };
    // Software pipeline, one LDS barrier per iteration: iteration `it` reads
    // chunk it + 1's operands from LDS into registers while the MFMAs of chunk
    // it (read the iteration before) run, then stashes chunk it + 2 into the
    // LDS buffer chunk it came from (every wave's reads of it completed before
    // the barrier: it waits on them) and refills that register slot with
    // chunk it + 4 from global memory (two chunks of loads in flight).  The
    // MFMAs are unconditional within a pair of iterations (a phase's chunk
    // past the slab: zero operands, zero products), so the compiler
    // interleaves the stash, the address math and the loads between them.
    // The loop runs whole pairs with the loads and stashes unconditional; an
    // odd last iteration's MFMAs follow it (they need no stash or load): a
    // break or a guarded stash inside the loop would let the compiler sink
    // each load to its consumer, and the waits then drain the ring every
    // iteration.
    static_assert(kDwAhead == 2, "a pair of register slots (the loop unrolls by two)");
    Ld ring[2];
    load(0, ring[0]);
    __builtin_amdgcn_sched_barrier(0);  // in chunk order (the loop's waits count on it)
    load(1, ring[1]);
    __builtin_amdgcn_sched_barrier(0);
    stash(0, ring[0]);
    load(2, ring[0]);
    stash(1, ring[1]);
    load(3, ring[1]);
    Ops ops[2];
    __syncthreads();  // (no stores in flight: an LDS wait and the barrier, which the wait-count pass sees)
    read_ops(0, ops[0]);
    GS_DW_STAMP(1);
    auto step = [&](int it, int u) {
        __syncthreads();
        read_ops(it + 1, ops[u ^ 1]);
        mfma_ops(ops[u]);
        stash(it + 2, ring[u]);
        load(it + 4, ring[u]);
    };
    int it = 0;
    for (; it + 1 < nI; it += 2) {
        step(it, 0);
        step(it + 1, 1);
    }
    if (it < nI) mfma_ops(ops[0]);  // odd nI: the last chunk, read into ops[0] by the last step
    GS_DW_STAMP(2);
    if constexpr (PH == 2) {
        // phase 1's sums to phase 0 through phase 1's ring (free: every
        // phase-1 wave is past its last compute once all reach the barrier)
        // (LDS-only barriers: the loop's last prefetches, of chunks past the
        // slab, may still be in flight, and a __syncthreads would wait for them)
        float* xch = &sbuf[1][0][0][0];
        static_assert(4 * kDwCh * kDwPitch >= kThreads * 16, "exchange area");
        lds_barrier();
        if (ph == 1)
#pragma unroll
            for (int t = 0; t < 4; ++t)
                *reinterpret_cast<f32x4*>(&xch[(t * kThreads + tid) * 4]) = acc[t];
        lds_barrier();
        if (ph == 1) return;
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const f32x4 o = *reinterpret_cast<const f32x4*>(&xch[(t * kThreads + tid) * 4]);
            acc[t] = acc[t] + o;
        }
    }
    float* slab = dst + static_cast<int64_t>(bz) * split_stride;
    const int h = h0 + wave * 16 + r;
    if (h < H) {
        float* srow = slab + static_cast<int64_t>(h) * K;
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const int k = k0 + t * 16 + 4 * kq;
            if (K % 4 == 0 && k < K) {
                *reinterpret_cast<f32x4*>(srow + k) = acc[t];
            } else {
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    if (k + j < K) srow[k + j] = acc[t][j];
            }
        }
    }
    GS_DW_STAMP(3);
}

template <typename T, bool HAS_SELF, bool RELU, bool VLOAD, bool ZVEC>
__global__ __launch_bounds__(kThreads) void linear_dw_kernel(
    int n, int F, int H, int K, int rows_per_split, const T* __restrict__ Xs, int64_t ldxs,
    const int* __restrict__ sidx, const T* __restrict__ A, int64_t lda, const float* __restrict__ dout,
    const float* __restrict__ out, int64_t ldo, float* __restrict__ dst, int64_t split_stride) {
    __shared__ DwSmem<1> sm;
    linear_dw_body<T, HAS_SELF, RELU, VLOAD, ZVEC>(blockIdx.x, blockIdx.y, blockIdx.z, n, F, H, K, rows_per_split,
                                                   Xs, ldxs, sidx, A, lda, dout, out, ldo, dst, split_stride, sm);
}

// The same tiles on a 1-D grid mapped XCD by XCD: workgroup w runs on XCD
// w % 8, and every tile of slab z is given to XCD z % 8, so a slab's dZ and
// input rows are fetched into one XCD's L2 once and re-read there by its
// other tiles (on the (k, h, slab) grid the k tile sets the XCD, and every
// XCD fetched every dZ row).  Grid: 8 · tiles · ceil(S / 8); spare
// workgroups exit.
constexpr int kXcds = 8;
template <typename T, bool HAS_SELF, bool RELU, bool VLOAD, bool ZVEC, int PH = 1>
__global__ __launch_bounds__(kThreads * PH) void linear_dw_xcd_kernel(
    int n, int F, int H, int K, int rows_per_split, int gx, int tiles, int S, const T* __restrict__ Xs,
    int64_t ldxs, const int* __restrict__ sidx, const T* __restrict__ A, int64_t lda,
    const float* __restrict__ dout, const float* __restrict__ out, int64_t ldo, float* __restrict__ dst,
    int64_t split_stride, KStamp ks) {
    kstamp_begin(ks);
    const int w = blockIdx.x;
    const int j = w / kXcds;
    const int z = w % kXcds + kXcds * (j / tiles);
    if (z >= S) return;
    const int t = j % tiles;
    __shared__ DwSmem<PH> sm;
    linear_dw_body<T, HAS_SELF, RELU, VLOAD, ZVEC, PH>(t % gx, t / gx, z, n, F, H, K, rows_per_split, Xs, ldxs, sidx,
                                                       A, lda, dout, out, ldo, dst, split_stride, sm);
    kstamp_end(ks);  // a timed launch's span (phase 1 of PH = 2 joins after handing its sums over)
}


// out[i] = Σ_s slabs[s][i] in one fixed order shared by every slab-sum
// kernel: the S slabs fall into kSlabParts consecutive groups of
// P = ceil(S / kSlabParts); each group is summed from zero in slab order, and
// the group sums are added in group order (empty groups add +0).  This is the
// order of sum_slabs_split_kernel (one wave per group), so the fused backward
// (which runs this body) and the standalone launch give bitwise the same
// gradients for any S.  4 elements per thread.  With `part`, block bx also
// writes Σ out[i]² over its elements to part[bx] (the clip norm's partial).
constexpr int kSlabParts = 8;

// `active` false: a thread of a wider block that only joins the partial's
// block reduction (adding +0 leaves it bitwise unchanged).
__device__ __forceinline__ void sum_slabs_body(int bx, int nblk, const float* __restrict__ slabs, int S,
                                               int64_t len, float* __restrict__ out, float* __restrict__ part,
                                               bool active = true) {
    const int64_t n4 = active ? len / 4 : 0;
    const int per = (S + kSlabParts - 1) / kSlabParts;
    float sq = 0.f;
    constexpr int kPre = 16;
    if (S <= kPre) {
        // every slab's quad loaded before the first add (clamped addresses,
        // the slab count tested after the loads): one memory round instead of
        // one per group.  The adds are the loop below's, in its order: each
        // group from zero in slab order, the group sums in group order (an
        // empty trailing group adds +0 there, which leaves the sum unchanged).
        for (int64_t i = bx * int64_t(kThreads) + threadIdx.x; i < n4; i += int64_t(nblk) * kThreads) {
            float4 v[kPre];
#pragma unroll
            for (int t = 0; t < kPre; ++t)
                v[t] = *reinterpret_cast<const float4*>(slabs + min(t, S - 1) * len + 4 * i);
            float4 s = make_float4(0.f, 0.f, 0.f, 0.f), g = s;
            bool first = true;
#pragma unroll
            for (int t = 0; t < kPre; ++t) {
                if (t < S) {
                    g.x += v[t].x; g.y += v[t].y; g.z += v[t].z; g.w += v[t].w;
                    if ((t + 1) % per == 0 || t + 1 == S) {
                        if (first) s = g;
                        else { s.x += g.x; s.y += g.y; s.z += g.z; s.w += g.w; }
                        first = false;
                        g = make_float4(0.f, 0.f, 0.f, 0.f);
                    }
                }
            }
            *reinterpret_cast<float4*>(out + 4 * i) = s;
            sq = fmaf(s.x, s.x, sq); sq = fmaf(s.y, s.y, sq); sq = fmaf(s.z, s.z, sq); sq = fmaf(s.w, s.w, sq);
        }
    }
    for (int64_t i = bx * int64_t(kThreads) + threadIdx.x; S > kPre && i < n4; i += int64_t(nblk) * kThreads) {
        float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
        for (int q = 0; q < kSlabParts; ++q) {
            const int t0 = min(S, q * per), t1 = min(S, t0 + per);
            float4 g = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll 4
            for (int t = t0; t < t1; ++t) {
                const float4 v = *reinterpret_cast<const float4*>(slabs + t * len + 4 * i);
                g.x += v.x; g.y += v.y; g.z += v.z; g.w += v.w;
            }
            if (q == 0) s = g;
            else { s.x += g.x; s.y += g.y; s.z += g.z; s.w += g.w; }
        }
        *reinterpret_cast<float4*>(out + 4 * i) = s;
        sq = fmaf(s.x, s.x, sq); sq = fmaf(s.y, s.y, sq); sq = fmaf(s.z, s.z, sq); sq = fmaf(s.w, s.w, sq);
    }
    for (int64_t i = 4 * (len / 4) + bx * int64_t(kThreads) + threadIdx.x; active && i < len;
         i += int64_t(nblk) * kThreads) {
        float s = 0.f;
        for (int q = 0; q < kSlabParts; ++q) {
            const int t0 = min(S, q * per), t1 = min(S, t0 + per);
            float g = 0.f;
            for (int t = t0; t < t1; ++t) g += slabs[t * len + i];
            s = q == 0 ? g : s + g;
        }
        out[i] = s;
        sq = fmaf(s, s, sq);
    }
    if (part) block_sum_to(sq, part + bx);
}

inline int sum_slabs_blocks(int64_t len) {
    return static_cast<int>(std::min<int64_t>((len / 4 + kThreads - 1) / kThreads + 1, 2048));
}

// ------------------------------------------------------------- input grad
// dIn[i][k] = Σ_h dZ[i][h] · W[h][k].  Wave = 16 rows x 16 k columns, block =
// 4 waves along k, no LDS: lane (r, kq) loads dZ[r][16g + 4kq ..+4] as one
// quad and the matching four W[h][k] values, 8 groups of h in flight at once.
template <bool HAS_SELF, bool RELU, bool ZVEC>
__device__ __forceinline__ void linear_dx_body(
    int bx, int by, int n, int F, int H, int K, const float* __restrict__ dout, const float* __restrict__ out,
    int64_t ldo, const float* __restrict__ W, float* __restrict__ dSelf, float* __restrict__ dA, int64_t ldd) {
    constexpr int G = 8;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int r = lane & 15, kq = lane >> 4;
    const int m0 = bx * 16;
    const int kt = by * 4 + wave;
    const int kc = min(kt * 16 + r, K - 1);
    const int row = min(m0 + r, n - 1);
    const float* zrow = dout + static_cast<int64_t>(row) * ldo;
    const float* orow = out + static_cast<int64_t>(row) * ldo;
    f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int h0 = 0; h0 < H; h0 += 16 * G) {
        float4 z[G];
        float w[G][4];
#pragma unroll
        for (int g = 0; g < G; ++g) {
            const int hb = h0 + 16 * g + 4 * kq;
            z[g] = row_quad<ZVEC>(zrow, hb, H);
            if (RELU) z[g] = relu_mask(z[g], row_quad<ZVEC>(orow, hb, H));
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const bool in = hb + j < H;
                const float v = W[static_cast<int64_t>(in ? hb + j : 0) * K + kc];
                w[g][j] = in ? v : 0.f;
            }
        }
#pragma unroll
        for (int g = 0; g < G; ++g) {
            acc = __builtin_amdgcn_mfma_f32_16x16x4f32(z[g].x, w[g][0], acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_16x16x4f32(z[g].y, w[g][1], acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_16x16x4f32(z[g].z, w[g][2], acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_16x16x4f32(z[g].w, w[g][3], acc, 0, 0, 0);
        }
    }
    const int k = kt * 16 + r;
    if (k >= K) return;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int i = m0 + 4 * kq + j;
        if (i >= n) continue;
        if (HAS_SELF && k < F) dSelf[static_cast<int64_t>(i) * ldd + k] = acc[j];
        else dA[static_cast<int64_t>(i) * ldd + (HAS_SELF ? k - F : k)] = acc[j];
    }
}

template <bool HAS_SELF, bool RELU, bool ZVEC>
__global__ __launch_bounds__(kThreads) void linear_dx_kernel(
    int n, int F, int H, int K, const float* __restrict__ dout, const float* __restrict__ out, int64_t ldo,
    const float* __restrict__ W, float* __restrict__ dSelf, float* __restrict__ dA, int64_t ldd) {
    linear_dx_body<HAS_SELF, RELU, ZVEC>(blockIdx.x, blockIdx.y, n, F, H, K, dout, out, ldo, W, dSelf, dA, ldd);
}

// Row slabs of the weight gradient: enough (64 h x 64 k) x slab workgroups to
// fill the chip, at least 64 rows per slab, slab heights a multiple of 16.
constexpr int kDwTargetBlocks = 512;  // two blocks per CU (measured best of 256 / 512 / 1024 in the step)

// phases = 2 (the layer-1 weight gradient): workgroups of 512 threads, half as many
inline int dw_target_blocks(int phases = 1) { return kDwTargetBlocks / phases; }

inline int dw_rows_per_split(int64_t n, int64_t K, int64_t H, int phases = 1) {
    const int64_t tiles = ((K + 63) / 64) * ((H + 63) / 64);
    const int64_t want = std::max<int64_t>(1, (dw_target_blocks(phases) + tiles - 1) / tiles);
    const int64_t cap = std::max<int64_t>(1, n / 64);
    const int64_t S = std::max(std::min(want, cap), (n + kDwMaxSlab - 1) / kDwMaxSlab);
    const int64_t rows = (n + S - 1) / S;
    return static_cast<int>(std::min<int64_t>(kDwMaxSlab, std::max<int64_t>(16, (rows + 15) / 16 * 16)));
}

inline int dw_splits(int64_t n, int64_t K, int64_t H, int phases = 1) {
    const int rps = dw_rows_per_split(n, K, H, phases);
    return static_cast<int>(std::max<int64_t>(1, (n + rps - 1) / rps));
}

}  // namespace gs
