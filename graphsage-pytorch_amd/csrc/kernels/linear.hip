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
    lds_barrier();  // (the pair launch's done-flag store, a PCIe write, need not land first)
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
// blocks [0, nb2) sum the layer-2 dW slabs, blocks [nb2, nb2 + nb1) the
// layer-1 ones, both as sum_slabs_split_kernel (64 quads per block, the slabs
// split over its 8 waves: one memory round each; the layer-2 sum on 33 blocks
// of one thread per quad took 3.4 us against 2.3 for the split blocks, the
// launch's critical path) -- each bitwise its standalone kernel (the order of
// sum_slabs_body), partials where those write.
// With spec.S (the trainer's deferred update) the layer-1 sum also writes W1's
// speculative update, and the launch stores the step's done flag (the
// runner's completion signal, otherwise stored by the SGD launch).
__global__ __launch_bounds__(kSlabParts * 64) void sum_slabs_pair_kernel(SlabSum s1, int nb1, SlabSum s2, int nb2,
                                                                         SlabSpec spec, int64_t* done,
                                                                         int64_t done_value, KStamp ks) {
    kstamp_begin(ks);
    signal_done(done, done_value);
    const int bx = blockIdx.x;
    if (bx < nb2)
        sum_slabs_split_body(bx, s2.slabs, s2.S, s2.len, s2.out, s2.part);
    else
        sum_slabs_split_body(bx - nb2, s1.slabs, s1.S, s1.len, s1.out, s1.part, spec);
    kstamp_end(ks);
}

static bool slab_split_on(int64_t len) { return len % 4 == 0; }

static bool fwd_vload(gs_dtype dt, int64_t F, const void* Xs, int64_t ldxs, const void* A, int64_t lda,
                      const void* W) {
    const int EPV = dt == GS_F32 ? 4 : 8;
    return F % EPV == 0 && lda % EPV == 0 && (!Xs || (ldxs % EPV == 0 && aligned16(Xs))) && aligned16(A) &&
           aligned16(W);
}

bool linear_fwd_wide_ok(gs_dtype dt, int64_t F, const void* Xs, int64_t ldxs, const void* A, int64_t lda,
                        const void* W) {
    return (dt == GS_F32 || dt == GS_BF16) && fwd_vload(dt, F, Xs, ldxs, A, lda, W);
}
static int64_t slab_split_blocks(int64_t len) { return (len / 4 + 63) / 64; }

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
    const bool vload = fwd_vload(dt, F, Xs, ldxs, A, lda, Wd);
    hipStream_t st = as_stream(stream);
    const int nn = static_cast<int>(n), ff = static_cast<int>(F), hh = static_cast<int>(H);
    // a pending clip + SGD (the trainer's deferred update): the fp32 wide kernel applies it
    FwdSpec sp = g_fwd_spec;
    g_fwd_spec = {};
    GS_REQUIRE(!sp.on || ((dt == GS_F32 ? (Wd == sp.S && !sp.Wn_lp) : (Wd == sp.S_lp && sp.Wn_lp != nullptr)) &&
                          K % 4 == 0 && self && relu && sp.np0 >= 1 && sp.np0 <= 512 && sp.np1 >= 1 &&
                          sp.np1 <= 512 && sp.up_hi > sp.up_lo),
               GS_EINVAL, "pending update: bad forward");
    if (vload) {
        // W-in-LDS tiles (bitwise the chunked kernel's sums: same MFMA operands
        // in the same order, whatever the row tiling), rows balanced over one
        // workgroup per CU and column tile (FwdRows): each workgroup takes
        // base or base + 1 row tiles of 16, at most 4
        sp.stamp = take_kernel_stamp();  // a timed launch: the kernel stores its own span
        const int64_t tiles = (n + 15) / 16, gy = (H + 63) / 64;
        int64_t groups = std::max<int64_t>(1, device_cus() / gy);
        int64_t per = (tiles + groups - 1) / groups;
        if (per > 4) {  // more than 64 rows per CU: a whole number of workgroups per CU
            groups *= (per + 3) / 4;
            per = (tiles + groups - 1) / groups;
        }
        if (tiles <= groups) {
            per = 1;
            groups = tiles;
        }
        FwdRows rs;
        rs.base = static_cast<int>(tiles / groups);
        rs.extra = static_cast<int>(tiles % groups);
        rs.groups = static_cast<int>(groups);
        // XCD map (a 1-D grid, the kernel derives its tile): the column tiles of
        // a row group share an XCD's L2 (PMC fabric reads 18.8 -> 10.9 MB per launch)
        const dim3 gw = gy == 1 ? dim3(static_cast<unsigned>(groups))
                                : dim3(static_cast<unsigned>((groups + 7) / 8 * 8 * gy));
#define GS_LFWDW(TT, R, SELF, RELU_, PEND)                                                                  \
        launch_k(linear_fwd_wide_kernel<TT, R, SELF, RELU_, PEND>, gw, dim3(R * 16), 0, st, nn, ff, hh, K,   \
                 static_cast<const TT*>(Xs), ldxs, sidx, static_cast<const TT*>(A), lda,                       \
                 static_cast<const TT*>(Wd), out, ldo, rs, sp)
#define GS_LFWDW_R(TT, R)                                                                                \
        do { if (sp.on) GS_LFWDW(TT, R, true, true, true);                                               \
             else if (self) { if (relu) GS_LFWDW(TT, R, true, true, false); else GS_LFWDW(TT, R, true, false, false); } \
             else { if (relu) GS_LFWDW(TT, R, false, true, false); else GS_LFWDW(TT, R, false, false, false); } } while (0)
#define GS_LFWDW_T(TT)                                                                                   \
        do { switch (per) { case 1: GS_LFWDW_R(TT, 16); break; case 2: GS_LFWDW_R(TT, 32); break;        \
                            case 3: GS_LFWDW_R(TT, 48); break; default: GS_LFWDW_R(TT, 64); } } while (0)
        if (dt == GS_F32) GS_LFWDW_T(float);
        else GS_LFWDW_T(bf16_t);
#undef GS_LFWDW_T
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
                    int64_t H_split, int phases) {
    GS_REQUIRE(dt == GS_F32 || dt == GS_BF16, GS_EINVAL, "dtype must be f32 or bf16");
    GS_REQUIRE(phases == 1 || phases == 2, GS_EINVAL, "dW: 1 or 2 row phases");
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
    // phases = 2: two row phases per 512-thread workgroup (linear_dw_body<PH = 2>),
    // half the slabs of the 256-thread form at the same chunk loop per workgroup
    const int S = dw_splits(n, K, Hs, phases);
    const int rps = dw_rows_per_split(n, K, Hs, phases);
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
    const int gx = static_cast<int>(grid.x), tiles = static_cast<int>(grid.x * grid.y);
    // workgroups mapped XCD by XCD: every tile of slab z on XCD z % 8 (PMC HBM
    // bytes 35.2 -> 19.4 MB per launch: dZ no longer fetched by all 8 XCDs)
    const dim3 grid_x(static_cast<unsigned>(kXcds * tiles * ((S + kXcds - 1) / kXcds)));
    const KStamp ks = take_kernel_stamp();  // a timed launch: the kernel stores its own span
#define GS_LDW2(TT, SELF, RELU, VL, ZV, PH)                                                                   \
    launch_k(linear_dw_xcd_kernel<TT, SELF, RELU, VL, ZV, PH>, grid_x, dim3(kThreads * PH), 0, st, nn, ff, hh, kk, \
             rps, gx, tiles, S, static_cast<const TT*>(Xs), ldxs, sidx, static_cast<const TT*>(A), lda, dout, \
             out, ldo, target, H * K, ks)
#define GS_LDW1(TT, SELF, RELU, VL, ZV) \
    do { if (phases == 2) GS_LDW2(TT, SELF, RELU, VL, ZV, 2); else GS_LDW2(TT, SELF, RELU, VL, ZV, 1); } while (0)
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
#undef GS_LDW2
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

bool sum_slabs_pair_ok(int64_t len1, int64_t len2) { return slab_split_on(len1) && slab_split_on(len2); }
int sum_slabs_pair_parts2(int64_t len2) { return static_cast<int>(slab_split_blocks(len2)); }

int sum_slabs_pair_launch(const SlabSum& s1, const SlabSum& s2, hipStream_t st, const float* spec_P, float* spec_S,
                          float lr, uint16_t* spec_S_lp) {
    GS_REQUIRE(slab_split_on(s1.len) && s1.S > 1 && (s2.S <= 1 || slab_split_on(s2.len)), GS_EINVAL,
               "slab pair: sums not split");
    const int nb1 = static_cast<int>(slab_split_blocks(s1.len));
    const int nb2 = s2.S > 1 ? static_cast<int>(slab_split_blocks(s2.len)) : 0;
    SlabSpec spec;
    DoneFlag done;
    if (spec_S) {  // the step's last launch: it carries the done flag
        GS_REQUIRE(spec_P && aligned16(spec_P) && aligned16(spec_S), GS_EINVAL, "slab pair: bad update buffers");
        GS_REQUIRE(!spec_S_lp || reinterpret_cast<uintptr_t>(spec_S_lp) % 8 == 0, GS_EINVAL, "slab pair: bad bf16 buffer");
        spec = SlabSpec{spec_P, spec_S, lr, spec_S_lp};
        done = g_done_flag;
        g_done_flag = {};
    }
    const KStamp ks = take_kernel_stamp();  // a timed launch: the kernel stores its own span
    launch_k(sum_slabs_pair_kernel, dim3(static_cast<unsigned>(nb1 + nb2)), dim3(kSlabParts * 64), 0, st, s1, nb1, s2,
             nb2, spec, done.ptr, done.value, ks);
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
    // two row phases per workgroup from 512 rows (the trainer's layer-1 form), one below
    const int S = linear_dw_slabs(dt, n, F, H, Xs, ldxs, sidx, A, lda, dout, out, ldo, relu, dW, ws, ws_bytes, st,
                                  -1, n >= 512 ? kDw1Phases : 1);
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
