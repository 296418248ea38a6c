// C-ABI launchers of the SageLayer kernels (kernels/linear_dev.hpp).
#include <algorithm>
#include <cstdlib>
#include <string>

#include "cls_dev.hpp"
#include "internal.hpp"
#include "linear_dev.hpp"

namespace gs {

__global__ __launch_bounds__(kThreads) void sum_slabs_kernel(const float* __restrict__ slabs, int S,
                                                             int64_t len, float* __restrict__ out,
                                                             float* __restrict__ part) {
    sum_slabs_body(blockIdx.x, gridDim.x, slabs, S, len, out, part);
}

// The slab sum with the slabs split over the block: 64 float4 columns per
// block, wave q of kSlabParts adds slabs [q·P, (q+1)·P) (P = ceil(S/parts))
// from zero, and wave 0 adds the part sums in wave order (fixed, no atomics;
// the order of sum_slabs_body).  Each thread then waits on ceil(S/parts)
// loads instead of S: at the layer-1 dW (31 slabs of 64 Ki floats) and 8
// waves, one round of 4 loads instead of eight rounds, over 256 blocks
// instead of 65.  len % 4 == 0.
// With spec (the trainer's deferred update): also S = P - lr·sum, W1's SGD
// step when its clip coefficient turns out to be 1 (sgd_elem with m = 1).
struct SlabSpec {
    const float* P = nullptr;
    float* S = nullptr;
    float lr = 0.f;
    uint16_t* S_lp = nullptr;  // bf16 features: S in bf16 too (sgd4's shadow conversion)
};
__device__ __forceinline__ void sum_slabs_split_body(int bx, const float* __restrict__ slabs, int S, int64_t len,
                                                     float* __restrict__ out, float* __restrict__ part,
                                                     SlabSpec spec = {}) {
    __shared__ float4 red[kSlabParts - 1][64];
    const int q = threadIdx.x >> 6, c = threadIdx.x & 63;
    const int64_t n4 = len / 4;
    const int64_t i = bx * int64_t(64) + c;
    float4 pv = make_float4(0.f, 0.f, 0.f, 0.f);
    if (spec.S && q == 0 && i < n4) pv = reinterpret_cast<const float4*>(spec.P)[i];  // with the slab loads
    const int per = (S + kSlabParts - 1) / kSlabParts;
    const int t0 = min(S, q * per), t1 = min(S, t0 + per);
    float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
    constexpr int kPre = 8;
    if (i < n4 && t1 - t0 <= kPre && t1 > t0) {
        // the group's quads loaded before the first add (clamped addresses,
        // the count tested after the loads): one memory round
        float4 v[kPre];
#pragma unroll
        for (int u = 0; u < kPre; ++u)
            v[u] = *reinterpret_cast<const float4*>(slabs + min(t0 + u, t1 - 1) * len + 4 * i);
#pragma unroll
        for (int u = 0; u < kPre; ++u)
            if (u < t1 - t0) { s.x += v[u].x; s.y += v[u].y; s.z += v[u].z; s.w += v[u].w; }
    } else if (i < n4) {
#pragma unroll 8
        for (int t = t0; t < t1; ++t) {
            const float4 v = *reinterpret_cast<const float4*>(slabs + t * len + 4 * i);
            s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
        }
    }
    if (q > 0) red[q - 1][c] = s;
    __syncthreads();
    float sq = 0.f;
    if (q == 0 && i < n4) {
#pragma unroll
        for (int p = 0; p < kSlabParts - 1; ++p) {
            const float4 v = red[p][c];
            s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
        }
        *reinterpret_cast<float4*>(out + 4 * i) = s;
        sq = fmaf(s.x, s.x, sq); sq = fmaf(s.y, s.y, sq); sq = fmaf(s.z, s.z, sq); sq = fmaf(s.w, s.w, sq);
        if (spec.S) {
            float4 pn, gi;
            pn.x = sgd_elem(pv.x, s.x, 1.0f, spec.lr, gi.x);
            pn.y = sgd_elem(pv.y, s.y, 1.0f, spec.lr, gi.y);
            pn.z = sgd_elem(pv.z, s.z, 1.0f, spec.lr, gi.z);
            pn.w = sgd_elem(pv.w, s.w, 1.0f, spec.lr, gi.w);
            reinterpret_cast<float4*>(spec.S)[i] = pn;
            if (spec.S_lp) {
                uint2 b;
                b.x = static_cast<uint32_t>(f2bf(pn.x)) | (static_cast<uint32_t>(f2bf(pn.y)) << 16);
                b.y = static_cast<uint32_t>(f2bf(pn.z)) | (static_cast<uint32_t>(f2bf(pn.w)) << 16);
                reinterpret_cast<uint2*>(spec.S_lp)[i] = b;
            }
        }
    }
    if (part) block_sum_to(sq, part + bx);
}

__global__ __launch_bounds__(kSlabParts * 64) void sum_slabs_split_kernel(const float* __restrict__ slabs, int S,
                                                                          int64_t len, float* __restrict__ out,
                                                                          float* __restrict__ part) {
    sum_slabs_split_body(blockIdx.x, slabs, S, len, out, part);
}

// Two slab sums in one launch (the 2-layer step after the fused top layer):
// blocks [nb2, nb2 + nb1) sum the layer-1 dW slabs as sum_slabs_split_kernel,
// blocks [0, nb2) the layer-2 dW slabs as sum_slabs_body over nb2 blocks of
// kThreads (the other threads of these wider blocks only join the partial's
// reduction) -- each bitwise its standalone kernel, partials where those write.
// With spec.S (the trainer's deferred update) the layer-1 sum also writes W1's
// speculative update, and the launch stores the step's done flag (the
// runner's completion signal, otherwise stored by the SGD launch).
__global__ __launch_bounds__(kSlabParts * 64) void sum_slabs_pair_kernel(SlabSum s1, int nb1, SlabSum s2, int nb2,
                                                                         SlabSpec spec, int64_t* done,
                                                                         int64_t done_value) {
    signal_done(done, done_value);
    const int bx = blockIdx.x;
    if (bx < nb2) {  // the longer per-block chains first
        sum_slabs_body(bx, nb2, s2.slabs, s2.S, s2.len, s2.out, s2.part, threadIdx.x < kThreads);
        return;
    }
    sum_slabs_split_body(bx - nb2, s1.slabs, s1.S, s1.len, s1.out, s1.part, spec);
}

// sum_slabs_pair_kernel, then every block waits at a grid barrier (all
// gradients and norm partials written) and runs its share of the clip + SGD
// (sgd4_body: the same fold and per-element arithmetic as sgd4_kernel, so
// the parameters are bitwise those of the two-launch sequence).  The barrier
// is a never-reset arrival counter: launch g waits for g · grid arrivals.
// Every block of the grid is resident once earlier work drains (289 blocks
// of 8 waves at the 2-layer step); a block that has waited ~1 s regardless
// records it in *bar_err and goes on (the step is then wrong, never hung).
struct SgdLaunch {
    Groups G;
    float* p;
    float* g;
    const float* part;
    float max_norm, lr;
    int64_t* done;
    int64_t done_value;
    unsigned long long* bar;
    unsigned long long target;
    int* bar_err;
};
__global__ __launch_bounds__(kSlabParts * 64) void sum_slabs_pair_sgd_kernel(SlabSum s1, int nb1, SlabSum s2, int nb2,
                                                                             SgdLaunch u) {
    signal_done(u.done, u.done_value);
    const int bx = blockIdx.x;
    if (bx < nb2) sum_slabs_body(bx, nb2, s2.slabs, s2.S, s2.len, s2.out, s2.part, threadIdx.x < kThreads);
    else sum_slabs_split_body(bx - nb2, s1.slabs, s1.S, s1.len, s1.out, s1.part);
    __syncthreads();  // the block's sums and partials written; thread 0 publishes them
    if (threadIdx.x == 0) {
        __hip_atomic_fetch_add(u.bar, 1ull, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();  // 100 MHz
        while (__hip_atomic_load(u.bar, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < u.target) {
            __builtin_amdgcn_s_sleep(1);
            if (__builtin_amdgcn_s_memrealtime() - t0 > 100000000ull) {
                __hip_atomic_store(u.bar_err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                break;
            }
        }
    }
    __syncthreads();  // thread 0's acquire covers the block (as a cooperative grid sync)
    sgd4_body(u.G, u.p, u.g, u.part, 1.0f, u.max_norm, u.lr, bx, gridDim.x);
}

// ------------------------------------------------- W-stationary forward
// Layer-1 shape only (K = 512, H = 128, fp32, self rows): one block per CU.
// Block b owns column half h = (b >> 3) & 1 and the row tiles p, p + NP,
// p + 2 NP of pair p = (b >> 4) * 8 + (b & 7) (blocks b and b + 8, one XCD
// under round-robin placement, are the two halves of a pair, so a tile's A
// rows come from HBM once).  Wave w keeps its 16-column slice of W (all K)
// in registers, loaded once; the block's 16-row tiles of [X[sidx] | A] are
// register-staged into LDS (one 1 KiB row-half per wave instruction: waves 0
// and 2 the self halves, 1 and 3 the aggregate halves), two tiles in flight.
// Every count is a compile-time constant (CNT tiles), so the compiler's
// waits are exact.  Same MFMA operands in the same order as the chunked
// kernel: bitwise equal (tools/lab/gemm_lab.hip measured it 16.2 against
// 16.8 us for the default 32-row kernel, warm, in the lab).
constexpr int kWstatK = 512, kWstatPitch = kWstatK + 4, kWstatMaxTiles = 3;

template <int CNT, bool RELU>
__device__ __forceinline__ void wstat_body(int n, const float* __restrict__ Xs, int64_t ldxs,
                                           const int* __restrict__ sidx, const float* __restrict__ A, int64_t lda,
                                           const float* __restrict__ W, float* __restrict__ out, int64_t ldo, int h,
                                           int p, int NP, float* sA) {
    constexpr int K = kWstatK, NG = K / 16, PITCH = kWstatPitch;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int r = lane & 15, kq = lane >> 4;
    const int half = wave & 1;
    // this wave's source rows: lane l < 8 * CNT -> tile l >> 3, row (wave >> 1) + 2 (l & 7)
    int myrow;
    {
        const int li = min(lane, 8 * CNT - 1);
        const int gr = min(16 * (p + (li >> 3) * NP) + (wave >> 1) + 2 * (li & 7), n - 1);
        myrow = half ? gr : sidx[gr];
    }
    const float* base = half ? A : Xs;
    const int64_t ld = half ? lda : ldxs;
    // eight named registers per staged tile (a private array would stay in scratch)
#define GS_WST8(M) M(0) M(1) M(2) M(3) M(4) M(5) M(6) M(7)
    uint4 s0_0, s0_1, s0_2, s0_3, s0_4, s0_5, s0_6, s0_7;
    uint4 s1_0, s1_1, s1_2, s1_3, s1_4, s1_5, s1_6, s1_7;
#define GS_WST_LD(q) \
    d##q = *reinterpret_cast<const uint4*>(base + (int64_t)__builtin_amdgcn_readlane(myrow, 8 * i + q) * ld + 4 * lane);
#define GS_WST_ST(q) \
    *reinterpret_cast<uint4*>(sA + (i * 16 + (wave >> 1) + 2 * q) * PITCH + half * (K / 2) + 4 * lane) = v##q;
    auto load_tile = [&](int i, uint4& d0, uint4& d1, uint4& d2, uint4& d3, uint4& d4, uint4& d5, uint4& d6,
                         uint4& d7) __attribute__((always_inline)) { GS_WST8(GS_WST_LD) };
    auto stage = [&](int i, const uint4& v0, const uint4& v1, const uint4& v2, const uint4& v3, const uint4& v4,
                     const uint4& v5, const uint4& v6, const uint4& v7) __attribute__((always_inline)) {
        GS_WST8(GS_WST_ST)
        __syncthreads();
    };
#define GS_WST_S0 s0_0, s0_1, s0_2, s0_3, s0_4, s0_5, s0_6, s0_7
#define GS_WST_S1 s1_0, s1_1, s1_2, s1_3, s1_4, s1_5, s1_6, s1_7
    load_tile(0, GS_WST_S0);
    uint4 w[NG];
    {
        const float* wrow = W + (int64_t)(64 * h + 16 * wave + r) * K + 4 * kq;
#pragma unroll
        for (int g = 0; g < NG; ++g) w[g] = *reinterpret_cast<const uint4*>(wrow + 16 * g);
    }
    if constexpr (CNT > 1) load_tile(1, GS_WST_S1);
    auto compute = [&](int i) __attribute__((always_inline)) {
        const float* ar = sA + (i * 16 + r) * PITCH + 4 * kq;
        f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int g = 0; g < NG; ++g) {
            const uint4 a = *reinterpret_cast<const uint4*>(ar + 16 * g);
            acc = mfma_slot<float>(a, w[g], acc);
        }
        const int t = p + i * NP;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int row = 16 * t + 4 * kq + j;
            if (row < n) {
                const float v = acc[j];
                out[(int64_t)row * ldo + 64 * h + 16 * wave + r] = (RELU && !(v > 0.f) && v == v) ? 0.f : v;
            }
        }
    };
    stage(0, GS_WST_S0);
    if constexpr (CNT > 2) load_tile(2, GS_WST_S0);  // tile 0's registers are in LDS now
    compute(0);
    if constexpr (CNT > 1) {
        stage(1, GS_WST_S1);
        compute(1);
    }
    if constexpr (CNT > 2) {
        stage(2, GS_WST_S0);
        compute(2);
    }
#undef GS_WST8
#undef GS_WST_LD
#undef GS_WST_ST
#undef GS_WST_S0
#undef GS_WST_S1
}

template <bool RELU>
__global__ __launch_bounds__(256, 1) void linear_fwd_wstat_kernel(int n, const float* __restrict__ Xs, int64_t ldxs,
                                                                  const int* __restrict__ sidx,
                                                                  const float* __restrict__ A, int64_t lda,
                                                                  const float* __restrict__ W, float* __restrict__ out,
                                                                  int64_t ldo) {
    extern __shared__ __attribute__((aligned(16))) float sA[];  // [kWstatMaxTiles * 16][kWstatPitch]
    const int b = blockIdx.x, NP = gridDim.x >> 1;
    const int h = (b >> 3) & 1, p = (b >> 4) * 8 + (b & 7);
    const int ntiles = (n + 15) / 16;
    const int cnt = p < ntiles ? min(kWstatMaxTiles, (ntiles - p + NP - 1) / NP) : 0;
    if (cnt == 1) wstat_body<1, RELU>(n, Xs, ldxs, sidx, A, lda, W, out, ldo, h, p, NP, sA);
    else if (cnt == 2) wstat_body<2, RELU>(n, Xs, ldxs, sidx, A, lda, W, out, ldo, h, p, NP, sA);
    else if (cnt == 3) wstat_body<3, RELU>(n, Xs, ldxs, sidx, A, lda, W, out, ldo, h, p, NP, sA);
}

static bool wstat_lds_ready() {
    static int ok = -1;
    if (ok < 0) {
        const int want = kWstatMaxTiles * 16 * kWstatPitch * static_cast<int>(sizeof(float));
        const bool a = hipFuncSetAttribute(reinterpret_cast<const void*>(linear_fwd_wstat_kernel<true>),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, want) == hipSuccess;
        const bool b = hipFuncSetAttribute(reinterpret_cast<const void*>(linear_fwd_wstat_kernel<false>),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, want) == hipSuccess;
        (void)hipGetLastError();
        ok = (a && b) ? 1 : 0;
    }
    return ok == 1;
}

// Pairs of blocks for n rows: at least one block per CU (256), at most three
// 16-row tiles per block, whole groups of 8 pairs (the XCD pairing above).
static int wstat_pairs(int64_t n) {
    const int64_t tiles = (n + 15) / 16;
    int64_t np = std::max<int64_t>(128, (tiles + kWstatMaxTiles - 1) / kWstatMaxTiles);
    return static_cast<int>((np + 7) / 8 * 8);
}

static bool slab_split_on(int64_t len) {
    static const bool off = std::getenv("GS_SLAB_SEQ") != nullptr;  // A/B: the sequential slab sum
    return !off && len % 4 == 0;
}
static int64_t slab_split_blocks(int64_t len) { return (len / 4 + 63) / 64; }

// 64 KiB of dynamic LDS per block for the W-resident forward: raise the
// launch limit once (the default dynamic limit is lower); refused -> the
// 32-row tiles.
static bool wres_lds_ready(int K) {
    static int ok = -1;
    if (ok < 0) {
        const int want = kWresCols * 512 * static_cast<int>(sizeof(float));
        bool good = true;
        const void* ks[4] = {reinterpret_cast<const void*>(linear_fwd_wres_kernel<true, true>),
                             reinterpret_cast<const void*>(linear_fwd_wres_kernel<true, false>),
                             reinterpret_cast<const void*>(linear_fwd_wres_kernel<false, true>),
                             reinterpret_cast<const void*>(linear_fwd_wres_kernel<false, false>)};
        for (const void* k : ks)
            good = good && hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, want) == hipSuccess;
        (void)hipGetLastError();
        ok = good ? 1 : 0;
    }
    return ok == 1 && K <= 512;
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
    GS_REQUIRE(n > 0 || !g_fwd_spec.on, GS_EINVAL, "pending update with no rows");
    if (n == 0) return GS_OK;
    GS_REQUIRE(A && Wd && out, GS_EINVAL, "NULL device pointer");
    const bool self = Xs != nullptr;
    const int K = static_cast<int>(self ? 2 * F : F);
    const int EPV = dt == GS_F32 ? 4 : 8;
    const bool vload = F % EPV == 0 && lda % EPV == 0 && (!self || (ldxs % EPV == 0 && aligned16(Xs))) &&
                       aligned16(A) && aligned16(Wd);
    hipStream_t st = as_stream(stream);
    const int nn = static_cast<int>(n), ff = static_cast<int>(F), hh = static_cast<int>(H);
    // a pending clip + SGD (the trainer's deferred update): the fp32 wide kernel applies it
    FwdSpec sp = g_fwd_spec;
    g_fwd_spec = {};
    GS_REQUIRE(!sp.on || ((dt == GS_F32 ? (Wd == sp.S && !sp.Wn_lp) : (Wd == sp.S_lp && sp.Wn_lp != nullptr)) &&
                          K % 4 == 0 && self && relu && sp.np0 >= 1 && sp.np0 <= 512 && sp.np1 >= 1 &&
                          sp.np1 <= 512 && sp.up_hi > sp.up_lo),
               GS_EINVAL, "pending update: bad forward");
    // read per call (tests switch it between launches): wres | wide32 | wide | sk | chunked
    const std::string fwd_mode = std::getenv("GS_LIN_FWD") ? std::getenv("GS_LIN_FWD") : "";
    GS_REQUIRE(!sp.on || fwd_mode.empty() || fwd_mode == "wide" || fwd_mode == "wide32", GS_EINVAL,
               "pending update needs the wide forward");
    // fp32 default: 32-row W-in-LDS tiles (bitwise the chunked kernel's sums:
    // same MFMA operands in the same order).  In-step at rmat2m the step ran
    // 80.2-80.7 us against 82.3-82.4 us with the 16-row chunked kernel, which
    // GS_LIN_FWD=chunked (and bf16) still select; "wide" = 64-row tiles.
    const bool wide_on = fwd_mode == "wide";
    const bool wide32_on = fwd_mode != "wide" && fwd_mode != "sk" && fwd_mode != "chunked";
    if (fwd_mode == "sk" && dt == GS_F32 && vload) {
        const dim3 gs2(static_cast<unsigned>((n + 15) / 16), static_cast<unsigned>((H + 31) / 32));
        const float* xs = static_cast<const float*>(Xs);
        const float* a = static_cast<const float*>(A);
        const float* w = static_cast<const float*>(Wd);
        if (self) {
            if (relu) launch_k(linear_fwd_sk_kernel<true, true>, gs2, dim3(kThreads), 0, st, nn, ff, hh, K, xs, ldxs, sidx, a, lda, w, out, ldo);
            else launch_k(linear_fwd_sk_kernel<true, false>, gs2, dim3(kThreads), 0, st, nn, ff, hh, K, xs, ldxs, sidx, a, lda, w, out, ldo);
        } else {
            if (relu) launch_k(linear_fwd_sk_kernel<false, true>, gs2, dim3(kThreads), 0, st, nn, ff, hh, K, xs, ldxs, sidx, a, lda, w, out, ldo);
            else launch_k(linear_fwd_sk_kernel<false, false>, gs2, dim3(kThreads), 0, st, nn, ff, hh, K, xs, ldxs, sidx, a, lda, w, out, ldo);
        }
        check_launch("gs_sage_linear_fwd(sk)");
        return GS_OK;
    }
    // GS_LIN_FWD=wres: the W-resident kernel (a 32-column W slice per block
    // in LDS, filled once by LDS-DMA).  Bitwise the same sums, but slower at
    // the layer-1 shape (microbenchmark 14.5 against 10 us): each wave's
    // 16-row tile runs its whole K chain (2 x 128 MFMAs), and 1.1k such waves
    // on 1024 SIMDs leave a second round on some of them.  Opt-in.
    // GS_LIN_FWD=wstat: the W-stationary kernel above (layer-1 shape only).
    if (fwd_mode == "wstat" && dt == GS_F32 && vload && self && K == kWstatK && H == 128 && n < (int64_t(1) << 30) &&
        wstat_lds_ready()) {
        const int np = wstat_pairs(n);
        const uint32_t smem = kWstatMaxTiles * 16 * kWstatPitch * sizeof(float);
        const float* xs = static_cast<const float*>(Xs);
        const float* a = static_cast<const float*>(A);
        const float* w = static_cast<const float*>(Wd);
        if (relu) launch_k(linear_fwd_wstat_kernel<true>, dim3(2 * np), dim3(kThreads), smem, st, nn, xs, ldxs, sidx, a, lda, w, out, ldo);
        else launch_k(linear_fwd_wstat_kernel<false>, dim3(2 * np), dim3(kThreads), smem, st, nn, xs, ldxs, sidx, a, lda, w, out, ldo);
        check_launch("gs_sage_linear_fwd(wstat)");
        return GS_OK;
    }
    const bool wres_on = fwd_mode == "wres";
    if (wres_on && dt == GS_F32 && vload && K % 256 == 0 && K <= 512 && H % kWresCols == 0 &&
        wres_lds_ready(K)) {
        const int tiles = static_cast<int>((n + 15) / 16);
        const int tx = (tiles + 3) / 4;  // row-tile groups (4 tiles per block)
        const int nsl = hh / kWresCols;
        const int gx = ((tx + 7) / 8) * 8 * nsl;  // remap padding: whole groups of 8
        const size_t smem = static_cast<size_t>(kWresCols) * K * sizeof(float);
        const float* xs = static_cast<const float*>(Xs);
        const float* a = static_cast<const float*>(A);
        const float* w = static_cast<const float*>(Wd);
#define GS_LFWDR(SELF, RELU_) \
        launch_k(linear_fwd_wres_kernel<SELF, RELU_>, dim3(gx), dim3(kThreads), static_cast<uint32_t>(smem), st, nn, ff, hh, K, tx, xs, ldxs, sidx, a, lda, w, out, ldo)
        if (self) { if (relu) GS_LFWDR(true, true); else GS_LFWDR(true, false); }
        else { if (relu) GS_LFWDR(false, true); else GS_LFWDR(false, false); }
#undef GS_LFWDR
        check_launch("gs_sage_linear_fwd(wres)");
        return GS_OK;
    }
    // bf16 takes the wide tiles unless GS_LIN_FWD_BF16=chunked (A/B)
    static const bool bf16_chunked = std::getenv("GS_LIN_FWD_BF16") &&
                                     std::string(std::getenv("GS_LIN_FWD_BF16")) == "chunked";
    if ((wide_on || wide32_on) && vload && (dt == GS_F32 || !bf16_chunked)) {
        sp.stamp = take_kernel_stamp();  // a timed launch: the kernel stores its own span
        // Rows per tile: 32.  GS_FWD_ROWS=48 takes 48-row tiles when 32-row
        // tiles would need more than one workgroup per CU and 48-row ones fit
        // one: the round-3 default (with the self rows gathered through their
        // index, 32-row tiles measured 15.0 us at 264-300 workgroups against
        // 10.5 us at 256); with the dense [self | agg] slot the 32-row tiles
        // are faster in situ (sustained 9.10-9.12 against 8.67-9.00 M roots/s,
        // profiles/r04d_fwd_rows_ab.txt).  Every row tile runs the same MFMA
        // chain, so the output is bitwise the same.
        const char* rows_env = std::getenv("GS_FWD_ROWS");  // read per call (tests switch it)
        const bool rows32 = !(rows_env && std::string(rows_env) == "48");
        int R = wide32_on ? 32 : kWideRows;
        {
            static const int ncu = [] {
                int d = 0, c = 256;
                if (hipGetDevice(&d) != hipSuccess ||
                    hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, d) != hipSuccess)
                    c = 256;
                return c;
            }();
            const int64_t gyy = (H + 63) / 64;
            auto blocks = [&](int64_t rr) { return ((n + rr - 1) / rr + 7) / 8 * 8 * gyy; };
            if (wide32_on && !rows32 && blocks(32) > ncu && blocks(48) <= ncu) R = 48;
        }
        // XCD map (a 1-D grid, the kernel derives its tile): the column tiles of a row tile share
        // an XCD's L2; GS_FWD_NOXCD=1 restores the 2-D grid (A/B)
        static const bool noxcd = std::getenv("GS_FWD_NOXCD") != nullptr;
        const int64_t gx = (n + R - 1) / R, gy = (H + 63) / 64;
        const dim3 gw = (noxcd || gy == 1) ? dim3(static_cast<unsigned>(gx), static_cast<unsigned>(gy))
                                           : dim3(static_cast<unsigned>((gx + 7) / 8 * 8 * gy));
#define GS_LFWDW(TT, RR, SELF, RELU_)                                                                         \
        launch_k(linear_fwd_wide_kernel<TT, RR, SELF, RELU_>, gw, dim3(RR * 16), 0, st, nn, ff, hh, K,            \
                 static_cast<const TT*>(Xs), ldxs, sidx, static_cast<const TT*>(A), lda, static_cast<const TT*>(Wd), \
                 out, ldo, sp)
#define GS_LFWDW_R(TT, RR) \
        do { if (self) { if (relu) GS_LFWDW(TT, RR, true, true); else GS_LFWDW(TT, RR, true, false); } \
             else { if (relu) GS_LFWDW(TT, RR, false, true); else GS_LFWDW(TT, RR, false, false); } } while (0)
        if (sp.on) {  // self rows and relu (checked above): the pending-update instances
#define GS_LFWDP(TT, RR)                                                                                    \
            launch_k(linear_fwd_wide_kernel<TT, RR, true, true, true>, gw, dim3(RR * 16), 0, st, nn, ff, hh, K, \
                     static_cast<const TT*>(Xs), ldxs, sidx, static_cast<const TT*>(A), lda,                 \
                     static_cast<const TT*>(Wd), out, ldo, sp)
            if (dt == GS_F32) {
                if (R == 32) GS_LFWDP(float, 32);
                else if (R == 48) GS_LFWDP(float, 48);
                else GS_LFWDP(float, 64);
            } else {
                if (R == 32) GS_LFWDP(bf16_t, 32);
                else if (R == 48) GS_LFWDP(bf16_t, 48);
                else GS_LFWDP(bf16_t, 64);
            }
#undef GS_LFWDP
        } else if (dt == GS_F32) {
            if (R == 32) GS_LFWDW_R(float, 32);
            else if (R == 48) GS_LFWDW_R(float, 48);
            else GS_LFWDW_R(float, 64);
        } else {
            if (R == 32) GS_LFWDW_R(bf16_t, 32);
            else if (R == 48) GS_LFWDW_R(bf16_t, 48);
            else GS_LFWDW_R(bf16_t, 64);
        }
#undef GS_LFWDW_R
#undef GS_LFWDW
        check_launch("gs_sage_linear_fwd(wide)");
        return GS_OK;
    }
    GS_REQUIRE(!sp.on, GS_EINVAL, "pending update needs the wide forward (16-B aligned operands)");
    const dim3 grid(static_cast<unsigned>((n + 15) / 16), static_cast<unsigned>((H + 63) / 64));
#define GS_LFWD1(TT, SELF, RELU, VL)                                                                     \
    launch_k(linear_fwd_kernel<TT, SELF, RELU, VL>, grid, dim3(kThreads), 0, st,                        \
        nn, ff, hh, K, static_cast<const TT*>(Xs), ldxs, sidx, static_cast<const TT*>(A), lda,          \
        static_cast<const TT*>(Wd), out, ldo)
#define GS_LFWD_V(TT, SELF, RELU) \
    do { if (vload) GS_LFWD1(TT, SELF, RELU, true); else GS_LFWD1(TT, SELF, RELU, false); } while (0)
#define GS_LFWD_R(TT, SELF) \
    do { if (relu) GS_LFWD_V(TT, SELF, true); else GS_LFWD_V(TT, SELF, false); } while (0)
#define GS_LFWD_S(TT) \
    do { if (self) GS_LFWD_R(TT, true); else GS_LFWD_R(TT, false); } while (0)
    if (dt == GS_F32) GS_LFWD_S(float);
    else GS_LFWD_S(bf16_t);
#undef GS_LFWD_S
#undef GS_LFWD_R
#undef GS_LFWD_V
#undef GS_LFWD1
    check_launch("gs_sage_linear_fwd");
    GS_API_END
}

int64_t gs_sage_linear_bwd_weight_ws(int64_t n, int64_t K, int64_t H) {
    const int S = gs::dw_splits(n, K, H);
    return S > 1 ? static_cast<int64_t>(S) * K * H * 4 : 0;
}

}  // extern "C"

namespace gs {

// The row-slab launch of the weight gradient.  Returns the slab count S:
// S == 1 wrote dW directly, S > 1 left S partial slabs in ws for the caller
// to add (sum_slabs_kernel, or a fused launch in bwd.hip).
int linear_dw_slabs(gs_dtype dt, int64_t n, int64_t F, int64_t H, const void* Xs, int64_t ldxs,
                    const int32_t* sidx, const void* A, int64_t lda, const float* dout, const float* out,
                    int64_t ldo, int32_t relu, float* dW, void* ws, int64_t ws_bytes, hipStream_t st,
                    DwGroups* grp, int64_t H_split) {
    GS_REQUIRE(dt == GS_F32 || dt == GS_BF16, GS_EINVAL, "dtype must be f32 or bf16");
    static_assert(kDwGroupParts == kSlabParts && kDwGroupParts == kXcds, "group count = slab-sum parts = XCDs");
    if (grp) {
        grp->slabs = static_cast<const float*>(ws);
        grp->S = 0;
    }
    GS_REQUIRE(n >= 0 && n < (int64_t(1) << 31) && F >= 1 && H >= 1 && H <= 4096, GS_EINVAL, "bad sizes");
    const bool self = Xs != nullptr;
    const int64_t K = self ? 2 * F : F;
    if (n == 0) {
        GS_REQUIRE(hipMemsetAsync(dW, 0, H * K * 4, st) == hipSuccess, GS_EHIP, "memset failed");
        return 1;
    }
    GS_REQUIRE(A && dout && dW && (out || !relu), GS_EINVAL, "NULL device pointer");
    // H_split: the row slabs of an H_split-row gradient (a chunk of its rows
    // then has the whole gradient's slabs, hence its sums bit for bit)
    const int64_t Hs = H_split > 0 ? H_split : H;
    const int S = dw_splits(n, K, Hs);
    const int rps = dw_rows_per_split(n, K, Hs);
    const int64_t need = static_cast<int64_t>(S > 1 ? S : 0) * K * H * 4;
    GS_REQUIRE(ws_bytes >= need && (need == 0 || ws), GS_EINVAL, "workspace too small");
    float* target = (S > 1) ? static_cast<float*>(ws) : dW;
    // 4-element input reads: 16 B (fp32) / 8 B (bf16) aligned
    const uintptr_t amask = dt == GS_F32 ? 15u : 7u;
    const bool vload = F % 4 == 0 && lda % 4 == 0 && (!self || ldxs % 4 == 0) &&
                       (reinterpret_cast<uintptr_t>(A) & amask) == 0 &&
                       (!self || (reinterpret_cast<uintptr_t>(Xs) & amask) == 0);
    const bool zvec = H % 4 == 0 && ldo % 4 == 0 && aligned16(dout) && (!relu || aligned16(out));
    const dim3 grid(static_cast<unsigned>((K + 63) / 64), static_cast<unsigned>((H + 63) / 64),
                    static_cast<unsigned>(S));
    const int nn = static_cast<int>(n), ff = static_cast<int>(F), hh = static_cast<int>(H), kk = static_cast<int>(K);
    static const bool xcd_map = std::getenv("GS_DW_GRID3") == nullptr;
    // opt-in (read per call): measured slower -- the writers' agent-scope releases
    // took the launch from 13.9 to 24.2 us while the slab sum, now reading 2 MB
    // instead of 8, stayed at 9.0 us (rocprof, rmat2m)
    const bool no_group = std::getenv("GS_DW_GROUP") == nullptr;
    const int gx = static_cast<int>(grid.x), tiles = static_cast<int>(grid.x * grid.y);
    const dim3 grid_x(static_cast<unsigned>(kXcds * tiles * ((S + kXcds - 1) / kXcds)));
    const int P = (S + kSlabParts - 1) / kSlabParts;  // slabs per group (the slab sum's grouping)
    const bool grouped = grp && !no_group && P >= 2 && K % 4 == 0 && grp->cnt && grp->gpart &&
                         grp->n_cnt >= static_cast<int64_t>(kXcds) * tiles;
    if (grouped) {
        grp->slabs = grp->gpart;
        grp->S = (S + P - 1) / P;
    } else if (grp) {
        grp->S = S;
    }
#define GS_LDW1(TT, SELF, RELU, VL, ZV)                                                                  \
    do {                                                                                                 \
        if (grouped)                                                                                     \
            launch_k(linear_dw_grp_kernel<TT, SELF, RELU, VL, ZV>, grid_x, dim3(kThreads), 0, st,        \
                nn, ff, hh, kk, rps, gx, tiles, S, P, static_cast<const TT*>(Xs), ldxs, sidx,            \
                static_cast<const TT*>(A), lda, dout, out, ldo, target, H * K, grp->gpart, grp->cnt);    \
        else if (xcd_map)                                                                                \
            launch_k(linear_dw_xcd_kernel<TT, SELF, RELU, VL, ZV>, grid_x, dim3(kThreads), 0, st,        \
                nn, ff, hh, kk, rps, gx, tiles, S, static_cast<const TT*>(Xs), ldxs, sidx,               \
                static_cast<const TT*>(A), lda, dout, out, ldo, target, H * K);                          \
        else                                                                                             \
            launch_k(linear_dw_kernel<TT, SELF, RELU, VL, ZV>, grid, dim3(kThreads), 0, st,              \
                nn, ff, hh, kk, rps, static_cast<const TT*>(Xs), ldxs, sidx, static_cast<const TT*>(A),  \
                lda, dout, out, ldo, target, H * K);                                                     \
    } while (0)
#define GS_LDW_Z(TT, SELF, RELU, VL) \
    do { if (zvec) GS_LDW1(TT, SELF, RELU, VL, true); else GS_LDW1(TT, SELF, RELU, VL, false); } while (0)
#define GS_LDW_V(TT, SELF, RELU) \
    do { if (vload) GS_LDW_Z(TT, SELF, RELU, true); else GS_LDW_Z(TT, SELF, RELU, false); } while (0)
#define GS_LDW_R(TT, SELF) \
    do { if (relu) GS_LDW_V(TT, SELF, true); else GS_LDW_V(TT, SELF, false); } while (0)
#define GS_LDW_S(TT) \
    do { if (self) GS_LDW_R(TT, true); else GS_LDW_R(TT, false); } while (0)
    if (dt == GS_F32) GS_LDW_S(float);
    else GS_LDW_S(bf16_t);
#undef GS_LDW_S
#undef GS_LDW_R
#undef GS_LDW_V
#undef GS_LDW_Z
#undef GS_LDW1
    check_launch("gs_sage_linear_bwd_weight");
    return S;
}

int sum_slabs_launch(const float* slabs, int S, int64_t len, float* out, float* part, hipStream_t st) {
    if (slab_split_on(len)) {
        const int64_t nb = slab_split_blocks(len);
        // 8 waves (one round of 4 loads per thread at 31 slabs): 4.8 against 5.3 us for 4 waves,
        // step 75.8-77.2 against 77.9-78.5 us (rocprof / alternating runs, same box)
        sum_slabs_split_kernel<<<dim3(static_cast<unsigned>(nb)), kSlabParts * 64, 0, st>>>(slabs, S, len, out, part);
        check_launch("sum_slabs");
        return static_cast<int>(nb);
    }
    sum_slabs_kernel<<<dim3(sum_slabs_blocks(len)), kThreads, 0, st>>>(slabs, S, len, out, part);
    check_launch("sum_slabs");
    return sum_slabs_blocks(len);
}

bool sum_slabs_pair_ok(int64_t len1) { return slab_split_on(len1); }

int sum_slabs_pair_launch(const SlabSum& s1, const SlabSum& s2, hipStream_t st, const float* spec_P, float* spec_S,
                          float lr, uint16_t* spec_S_lp) {
    GS_REQUIRE(slab_split_on(s1.len) && s1.S > 1, GS_EINVAL, "slab pair: layer-1 sum not split");
    const int nb1 = static_cast<int>(slab_split_blocks(s1.len));
    const int nb2 = s2.S > 1 ? sum_slabs_blocks(s2.len) : 0;
    SlabSpec spec;
    DoneFlag done;
    if (spec_S) {  // the step's last launch: it carries the done flag
        GS_REQUIRE(spec_P && aligned16(spec_P) && aligned16(spec_S), GS_EINVAL, "slab pair: bad update buffers");
        GS_REQUIRE(!spec_S_lp || reinterpret_cast<uintptr_t>(spec_S_lp) % 8 == 0, GS_EINVAL, "slab pair: bad bf16 buffer");
        spec = SlabSpec{spec_P, spec_S, lr, spec_S_lp};
        done = g_done_flag;
        g_done_flag = {};
    }
    sum_slabs_pair_kernel<<<dim3(static_cast<unsigned>(nb1 + nb2)), kSlabParts * 64, 0, st>>>(s1, nb1, s2, nb2, spec,
                                                                                              done.ptr, done.value);
    check_launch("sum_slabs_pair");
    return nb1;
}

// The deferred update's last step (spec_finalize_launch): the groups' clip
// coefficients from the norm partials (clip_fold, as every clip here), W1 =
// S (coefficient 1) or P - lr·coef·G1 into w1_out with G1 scaled, and the
// clip + SGD of the other parameters: what sgd4_kernel would have left.
__global__ __launch_bounds__(kThreads) void spec_finalize_kernel(FwdSpec sp, float* __restrict__ w1_out,
                                                                 int64_t w1_floats) {
    const int lane = threadIdx.x & 63;
    const float m0 = clip_mult(clip_fold(sp.part0, sp.np0, lane), sp.scale, sp.max_norm);
    const float m1 = clip_mult(clip_fold(sp.part1, sp.np1, lane), sp.scale, sp.max_norm);
    const int64_t stride = int64_t(gridDim.x) * blockDim.x, t = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    float4* G1 = reinterpret_cast<float4*>(const_cast<float*>(sp.G1));
    const float4* S4 = reinterpret_cast<const float4*>(sp.S);
    const float4* P4 = reinterpret_cast<const float4*>(sp.P);
    float4* O4 = reinterpret_cast<float4*>(w1_out);
    for (int64_t i = t; i < w1_floats / 4; i += stride) {
        const float4 gv = G1[i];
        const bool spec = m0 == sp.scale;  // clip coefficient 1: S is the update
        const float4 pv = spec ? S4[i] : P4[i];
        float4 gi, pn;
        pn.x = sgd_elem(pv.x, gv.x, m0, sp.lr, gi.x);
        pn.y = sgd_elem(pv.y, gv.y, m0, sp.lr, gi.y);
        pn.z = sgd_elem(pv.z, gv.z, m0, sp.lr, gi.z);
        pn.w = sgd_elem(pv.w, gv.w, m0, sp.lr, gi.w);
        G1[i] = gi;
        O4[i] = spec ? pv : pn;
    }
    float4* p4 = reinterpret_cast<float4*>(sp.p);
    float4* g4 = reinterpret_cast<float4*>(sp.g);
    for (int64_t i = sp.up_lo / 4 + t; i < sp.up_hi / 4; i += stride) {
        const float m = 4 * i >= sp.grp1_lo ? m1 : m0;
        const float4 pv = p4[i], gv = g4[i];
        float4 gi, pn;
        pn.x = sgd_elem(pv.x, gv.x, m, sp.lr, gi.x);
        pn.y = sgd_elem(pv.y, gv.y, m, sp.lr, gi.y);
        pn.z = sgd_elem(pv.z, gv.z, m, sp.lr, gi.z);
        pn.w = sgd_elem(pv.w, gv.w, m, sp.lr, gi.w);
        g4[i] = gi;
        p4[i] = pn;
    }
}

void spec_finalize_launch(const FwdSpec& sp, float* w1_out, int64_t w1_floats, hipStream_t st) {
    GS_REQUIRE(sp.on && w1_floats % 4 == 0 && sp.up_lo % 4 == 0 && sp.up_hi % 4 == 0 && sp.grp1_lo % 4 == 0,
               GS_EINVAL, "spec finalize: bad layout");
    const int64_t n4 = std::max(w1_floats, sp.up_hi - sp.up_lo) / 4;
    const unsigned grid = static_cast<unsigned>(std::max<int64_t>(1, std::min<int64_t>((n4 + kThreads - 1) / kThreads, 256)));
    spec_finalize_kernel<<<dim3(grid), kThreads, 0, st>>>(sp, w1_out, w1_floats);
    check_launch("spec_finalize");
}

int sum_slabs_pair_sgd_launch(const SlabSum& s1, const SlabSum& s2, int np_before, const FusedSgd& u,
                              hipStream_t st) {
    GS_REQUIRE(slab_split_on(s1.len) && s1.S > 1, GS_EINVAL, "slab pair: layer-1 sum not split");
    GS_REQUIRE(u.n_groups >= 1 && u.n_groups <= 8, GS_EINVAL, "1..8 parameter groups");
    const int nb1 = static_cast<int>(slab_split_blocks(s1.len));
    const int nb2 = s2.S > 1 ? sum_slabs_blocks(s2.len) : 0;
    SgdLaunch a;
    a.G.n = u.n_groups;
    a.G.pstride = u.pstride;
    for (int i = 0; i < u.n_groups; ++i) a.G.npart[i] = u.npart[i];
    a.G.npart[0] = np_before + nb1;  // group 0: the partials before this launch and its layer-1 ones
    for (int i = 0; i <= u.n_groups; ++i) a.G.off[i] = u.goff_host[i];
    bool vec = aligned16(u.params) && aligned16(u.grads);
    for (int i = 0; i <= u.n_groups; ++i) vec = vec && a.G.off[i] % 4 == 0;
    const LowpShadow sh = g_lowp_shadow;
    vec = vec && (!sh.p || (sh.lo % 4 == 0 && sh.hi % 4 == 0 && reinterpret_cast<uintptr_t>(sh.p) % 8 == 0));
    GS_REQUIRE(vec, GS_EINVAL, "fused SGD needs 16-B aligned float4 groups");
    g_lowp_shadow = {};
    a.G.sh = sh.p;
    a.G.sh_lo = sh.lo;
    a.G.sh_hi = sh.hi;
    a.p = u.params;
    a.g = u.grads;
    a.part = u.part;
    a.max_norm = u.max_norm;
    a.lr = u.lr;
    a.done = g_done_flag.ptr;
    a.done_value = g_done_flag.value;
    g_done_flag = {};
    const unsigned nb = static_cast<unsigned>(nb1 + nb2);
    a.bar = u.bar;
    a.target = *u.bar_gen + nb;  // the host's count follows only a launch that went out
    a.bar_err = u.bar_err;
    sum_slabs_pair_sgd_kernel<<<dim3(nb), kSlabParts * 64, 0, st>>>(s1, nb1, s2, nb2, a);
    check_launch("sum_slabs_pair_sgd");
    *u.bar_gen = a.target;
    return nb1;
}

int sum_slabs_grid(int64_t len) {  // norm partials a slab sum of len floats may write (capacity bound)
    return static_cast<int>(std::max<int64_t>(sum_slabs_blocks(len), slab_split_blocks(len)));
}

}  // namespace gs

extern "C" {

int gs_sage_linear_bwd_weight(gs_dtype dt, int64_t n, int64_t F, int64_t H, const void* Xs, int64_t ldxs,
                              const int32_t* sidx, const void* A, int64_t lda, const float* dout,
                              const float* out, int64_t ldo, int32_t relu, float* dW, void* ws,
                              int64_t ws_bytes, void* stream) {
    GS_API_BEGIN
    using namespace gs;
    hipStream_t st = as_stream(stream);
    const int S = linear_dw_slabs(dt, n, F, H, Xs, ldxs, sidx, A, lda, dout, out, ldo, relu, dW, ws, ws_bytes, st);
    if (S > 1) sum_slabs_launch(static_cast<const float*>(ws), S, H * (Xs ? 2 * F : F), dW, nullptr, st);
    GS_API_END
}

int gs_sage_linear_bwd_input(int64_t n, int64_t F, int64_t H, const float* dout, const float* out, int64_t ldo,
                             int32_t relu, const float* W, float* dSelf, float* dA, int64_t ldd, void* stream) {
    GS_API_BEGIN
    using namespace gs;
    GS_REQUIRE(n >= 0 && n < (int64_t(1) << 31) && F >= 1 && H >= 1, GS_EINVAL, "bad sizes");
    if (n == 0) return GS_OK;
    GS_REQUIRE(dout && W && dA && (out || !relu), GS_EINVAL, "NULL device pointer");
    const bool self = dSelf != nullptr;
    const int64_t K = self ? 2 * F : F;
    const bool zvec = H % 4 == 0 && ldo % 4 == 0 && aligned16(dout) && (!relu || aligned16(out));
    const dim3 grid(static_cast<unsigned>((n + 15) / 16), static_cast<unsigned>((K + 63) / 64));
    hipStream_t st = as_stream(stream);
    const int nn = static_cast<int>(n), ff = static_cast<int>(F), hh = static_cast<int>(H), kk = static_cast<int>(K);
#define GS_LDX(SELF, RELU, ZV) \
    linear_dx_kernel<SELF, RELU, ZV><<<grid, kThreads, 0, st>>>(nn, ff, hh, kk, dout, out, ldo, W, dSelf, dA, ldd)
#define GS_LDX_Z(SELF, RELU) \
    do { if (zvec) GS_LDX(SELF, RELU, true); else GS_LDX(SELF, RELU, false); } while (0)
    if (self) { if (relu) GS_LDX_Z(true, true); else GS_LDX_Z(true, false); }
    else { if (relu) GS_LDX_Z(false, true); else GS_LDX_Z(false, false); }
#undef GS_LDX_Z
#undef GS_LDX
    check_launch("gs_sage_linear_bwd_input");
    GS_API_END
}

}  // extern "C"
