// Horizontally fused backward launches of one SageLayer l >= 2 (see
// internal.hpp).  Each launch runs blocks of independent kernels side by
// side: the role of a block is fixed by its index range, so every role keeps
// the exact code, tiling and summation order of its standalone kernel
// (linear_dev.hpp, agg_dev.hpp, cls_dev.hpp) and the results are bitwise those
// of the unfused sequence.  Only the stream boundaries disappear:
//   A = [dW_l slabs: gx·gy·S blocks][dIn_l: (n/16)·(K/64)][classifier reduce]
//   B = [Σ slabs -> dW_l (+ norm partials)][agg backward -> dH_{l-1}]
// Heavy roles come first in the grid so they are dispatched first.
// After the fused top layer (top.hip wrote dIn_2) a 2-layer step needs one
// launch here, not two: T = [dW_2 slabs][classifier reduce][agg backward ->
// dH_1], and the Σ of the dW_2 slabs moves into the layer-1 slab-sum launch
// (sum_slabs_pair_launch), which runs after the layer-1 dW anyway.
#include "agg_dev.hpp"
#include "cls_dev.hpp"
#include "internal.hpp"
#include "linear_dev.hpp"

namespace gs {

static_assert(kThreads == kBlock && kThreads == kClsRedThreads, "fused roles share one block size");


template <bool HAS_SELF, bool ZVEC, bool CLS>
__global__ __launch_bounds__(kThreads) void layer_bwd_a_kernel(BwdA a) {
    int b = blockIdx.x;
    if (b < a.dw_nb) {
        __shared__ DwSmem<1> sm;
        const int g2 = a.dw_gx * a.dw_gy;
        linear_dw_body<float, HAS_SELF, false, true, ZVEC>(b % a.dw_gx, (b % g2) / a.dw_gx, b / g2, a.n, a.F, a.H,
                                                           a.K, a.rps, a.Xs, a.ldxs, a.sidx, a.A, a.lda, a.dZ,
                                                           nullptr, a.H, a.target,
                                                           static_cast<int64_t>(a.H) * a.K, sm);
        return;
    }
    b -= a.dw_nb;
    if (b < a.dx_nb) {
        linear_dx_body<HAS_SELF, false, ZVEC>(b % a.dx_gx, b / a.dx_gx, a.n, a.F, a.H, a.K, a.dZ, nullptr, a.H,
                                              a.W, a.dSelf, a.dA, a.K);
        return;
    }
    b -= a.dx_nb;
    if constexpr (CLS) cls_reduce_body(b, a.B, a.D, a.C, a.cls_rows, a.cls_slab, a.dWc, a.dbc, a.loss, a.cls_part);
}

struct BwdB {
    const float* slabs;
    int S;
    int64_t len;
    float* dW;
    float* part;
    int sum_nb;
    int n_src, F;
    const int* tptr;
    const int* tidx;
    const int* ptr;
    const float* dA;
    const float* dSelf;
    int64_t ldd;
    const int* argmax;
    const float* Hprev;
    float* dH;
    const int4* rec = nullptr;  // agg_bwd_rec_body's records (layer_bwd_top only)
    int64_t off2 = 0;           // dIn as two partials (the top launch's pair form), the second off2 floats on
};

template <int OP, int G, bool PAIR>
__global__ __launch_bounds__(kThreads) void layer_bwd_b_kernel(BwdB b) {
    const int bx = blockIdx.x;
    if (bx < b.sum_nb) {
        sum_slabs_body(bx, b.sum_nb, b.slabs, b.S, b.len, b.dW, b.part);
        return;
    }
    agg_bwd_body<OP, 4, G, PAIR>(bx - b.sum_nb, b.n_src, b.F, b.tptr, b.tidx, b.ptr, b.dA, b.dSelf, b.ldd, b.argmax,
                           b.Hprev, b.F, b.dH, b.off2);
}

struct BwdT {
    BwdA a;     // dW slabs + classifier reduce roles (dx_nb == 0)
    BwdB b;     // agg backward role (sum_nb == 0)
    int cls_nb;
};

template <int OP, int G, bool PAIR>
__global__ __launch_bounds__(kThreads) void layer_bwd_top_kernel(BwdT t) {
    int b = blockIdx.x;
    if (b < t.a.dw_nb) {
        __shared__ DwSmem<1> sm;
        const int g2 = t.a.dw_gx * t.a.dw_gy;
        linear_dw_body<float, true, false, true, true>(b % t.a.dw_gx, (b % g2) / t.a.dw_gx, b / g2, t.a.n, t.a.F,
                                                       t.a.H, t.a.K, t.a.rps, t.a.Xs, t.a.ldxs, t.a.sidx, t.a.A,
                                                       t.a.lda, t.a.dZ, nullptr, t.a.H, t.a.target,
                                                       static_cast<int64_t>(t.a.H) * t.a.K, sm);
        return;
    }
    b -= t.a.dw_nb;
    if (b < t.cls_nb) {
        cls_reduce_body(b, t.a.B, t.a.D, t.a.C, t.a.cls_rows, t.a.cls_slab, t.a.dWc, t.a.dbc, t.a.loss, t.a.cls_part);
        return;
    }
    b -= t.cls_nb;
    if (t.b.rec)
        agg_bwd_rec_body<OP, 4, G, PAIR>(b, t.b.n_src, t.b.F, t.b.rec, t.b.tidx, t.b.ptr, t.b.dA, t.b.dSelf, t.b.ldd,
                                   t.b.argmax, t.b.Hprev, t.b.F, t.b.dH, t.b.off2);
    else
        agg_bwd_body<OP, 4, G, PAIR>(b, t.b.n_src, t.b.F, t.b.tptr, t.b.tidx, t.b.ptr, t.b.dA, t.b.dSelf, t.b.ldd,
                               t.b.argmax, t.b.Hprev, t.b.F, t.b.dH, t.b.off2);
}

int cls_reduce_grid(int64_t C, int64_t D) { return cls_reduce_blocks(C, D); }

bool layer_bwd_fusable(const LayerBwd& a) {
    const int64_t K = a.Xs ? 2 * a.fin : a.fin;
    const bool al = (a.lda == 0 || (a.lda >= a.fin && a.lda % 4 == 0)) && aligned16(a.A) && aligned16(a.dZ) && aligned16(a.W) && aligned16(a.dW) && aligned16(a.slabs) &&
                    aligned16(a.dIn) && aligned16(a.dH) && aligned16(a.Hprev) && (!a.Xs || aligned16(a.Xs));
    const int G = pick_group(static_cast<int>(a.H), 4);
    return al && a.fin == a.H && a.H % 16 == 0 && a.H <= 256 && K % 4 == 0 && a.ldxs % 4 == 0 && a.n >= 1 &&
           a.n_src >= 1 && (G == 16 || G == 32 || G == 64) && (a.agg == GS_AGG_MEAN || a.argmax) &&
           a.n < (int64_t(1) << 31) && a.n_src < (int64_t(1) << 31);
}

int layer_bwd(const LayerBwd& a, const ClsReduce* cls, float* part, hipStream_t st) {
    GS_REQUIRE(layer_bwd_fusable(a), GS_EINVAL, "layer backward not fusable");
    const bool self = a.Xs != nullptr;
    const int64_t K = self ? 2 * a.fin : a.fin;
    const int S = dw_splits(a.n, K, a.H);
    const int rps = dw_rows_per_split(a.n, K, a.H);
    GS_REQUIRE(S == 1 || a.slab_bytes >= static_cast<int64_t>(S) * K * a.H * 4, GS_EINVAL, "workspace too small");
    BwdA A{};
    A.n = static_cast<int>(a.n);
    A.F = static_cast<int>(a.fin);
    A.H = static_cast<int>(a.H);
    A.K = static_cast<int>(K);
    A.rps = rps;
    A.Xs = a.Xs;
    A.ldxs = a.ldxs;
    A.sidx = a.sidx;
    A.A = a.A;
    A.lda = a.lda > 0 ? a.lda : a.fin;
    A.dZ = a.dZ;
    A.target = S > 1 ? a.slabs : a.dW;
    A.dw_gx = static_cast<int>((K + 63) / 64);
    A.dw_gy = static_cast<int>((a.H + 63) / 64);
    A.dw_nb = A.dw_gx * A.dw_gy * S;
    A.W = a.W;
    A.dSelf = self ? a.dIn : nullptr;
    A.dA = self ? a.dIn + a.fin : a.dIn;
    A.dx_gx = static_cast<int>((a.n + 15) / 16);
    A.dx_nb = a.din_ready ? 0 : A.dx_gx * static_cast<int>((K + 63) / 64);
    int cls_nb = 0;
    if (cls) {
        A.B = static_cast<int>(cls->B);
        A.D = static_cast<int>(cls->D);
        A.C = static_cast<int>(cls->C);
        A.cls_rows = cls->n_row_blocks;
        A.cls_slab = cls->slab;
        A.dWc = cls->dWc;
        A.dbc = cls->dbc;
        A.loss = cls->loss;
        A.cls_part = cls->part;
        cls_nb = cls_reduce_blocks(cls->C, cls->D);
    }
    const dim3 ga(static_cast<unsigned>(A.dw_nb + A.dx_nb + cls_nb));
#define GS_BWDA(SELF, CLS) layer_bwd_a_kernel<SELF, true, CLS><<<ga, kThreads, 0, st>>>(A)
    if (self) {
        if (cls) GS_BWDA(true, true);
        else GS_BWDA(true, false);
    } else {
        if (cls) GS_BWDA(false, true);
        else GS_BWDA(false, false);
    }
#undef GS_BWDA
    check_launch("layer_bwd(A)");

    BwdB Bq{};
    Bq.slabs = a.slabs;
    Bq.S = S;
    Bq.len = a.H * K;
    Bq.dW = a.dW;
    Bq.part = part;
    Bq.sum_nb = S > 1 ? sum_slabs_blocks(Bq.len) : 0;
    Bq.n_src = static_cast<int>(a.n_src);
    Bq.F = static_cast<int>(a.H);
    Bq.tptr = a.tptr;
    Bq.tidx = a.tidx;
    Bq.ptr = a.ptr;
    Bq.dA = A.dA;
    Bq.dSelf = A.dSelf;
    Bq.ldd = K;
    Bq.argmax = a.argmax;
    Bq.Hprev = a.Hprev;
    Bq.dH = a.dH;
    Bq.off2 = a.din_off2;
    const int G = pick_group(static_cast<int>(a.H), 4);
    const int agg_nb = static_cast<int>((a.n_src + (kBlock / G) - 1) / (kBlock / G));
    const dim3 gb(static_cast<unsigned>(Bq.sum_nb + agg_nb));
#define GS_BWDB2(OP, PR)                                                                    \
    do {                                                                                    \
        if (G == 16) layer_bwd_b_kernel<OP, 16, PR><<<gb, kThreads, 0, st>>>(Bq);           \
        else if (G == 32) layer_bwd_b_kernel<OP, 32, PR><<<gb, kThreads, 0, st>>>(Bq);      \
        else layer_bwd_b_kernel<OP, 64, PR><<<gb, kThreads, 0, st>>>(Bq);                   \
    } while (0)
#define GS_BWDB(OP) do { if (Bq.off2) GS_BWDB2(OP, true); else GS_BWDB2(OP, false); } while (0)
    if (a.agg == GS_AGG_MEAN) GS_BWDB(GS_AGG_MEAN);
    else GS_BWDB(GS_AGG_MAX);
#undef GS_BWDB
#undef GS_BWDB2
    check_launch("layer_bwd(B)");
    return Bq.sum_nb;
}

int layer_bwd_top(const LayerBwd& a, const ClsReduce& cls, SlabSum* deferred, hipStream_t st) {
    GS_REQUIRE(layer_bwd_fusable(a) && a.din_ready && a.Xs, GS_EINVAL, "top backward: not the fused top path");
    const int64_t K = 2 * a.fin;
    const int S = dw_splits(a.n, K, a.H);
    const int rps = dw_rows_per_split(a.n, K, a.H);
    GS_REQUIRE(S == 1 || a.slab_bytes >= static_cast<int64_t>(S) * K * a.H * 4, GS_EINVAL, "workspace too small");
    BwdT t{};
    BwdA& A = t.a;
    A.n = static_cast<int>(a.n);
    A.F = static_cast<int>(a.fin);
    A.H = static_cast<int>(a.H);
    A.K = static_cast<int>(K);
    A.rps = rps;
    A.Xs = a.Xs;
    A.ldxs = a.ldxs;
    A.sidx = a.sidx;
    A.A = a.A;
    A.lda = a.lda > 0 ? a.lda : a.fin;
    A.dZ = a.dZ;
    A.target = S > 1 ? a.slabs : a.dW;
    A.dw_gx = static_cast<int>((K + 63) / 64);
    A.dw_gy = static_cast<int>((a.H + 63) / 64);
    A.dw_nb = A.dw_gx * A.dw_gy * S;
    A.B = static_cast<int>(cls.B);
    A.D = static_cast<int>(cls.D);
    A.C = static_cast<int>(cls.C);
    A.cls_rows = cls.n_row_blocks;
    A.cls_slab = cls.slab;
    A.dWc = cls.dWc;
    A.dbc = cls.dbc;
    A.loss = cls.loss;
    A.cls_part = cls.part;
    t.cls_nb = cls_reduce_blocks(cls.C, cls.D);
    BwdB& Bq = t.b;
    Bq.n_src = static_cast<int>(a.n_src);
    Bq.F = static_cast<int>(a.H);
    Bq.tptr = a.tptr;
    Bq.tidx = a.tidx;
    Bq.ptr = a.ptr;
    Bq.dSelf = a.dIn;
    Bq.dA = a.dIn + a.fin;
    Bq.ldd = K;
    Bq.argmax = a.argmax;
    Bq.Hprev = a.Hprev;
    Bq.dH = a.dH;
    Bq.off2 = a.din_off2;
    Bq.rec = a.trec;
    const int G = pick_group(static_cast<int>(a.H), 4);
    const int agg_nb = static_cast<int>((a.n_src + (kBlock / G) - 1) / (kBlock / G));
    const dim3 grid(static_cast<unsigned>(A.dw_nb + t.cls_nb + agg_nb));
#define GS_BWDT2(OP, PR)                                                                \
    do {                                                                                \
        if (G == 16) layer_bwd_top_kernel<OP, 16, PR><<<grid, kThreads, 0, st>>>(t);    \
        else if (G == 32) layer_bwd_top_kernel<OP, 32, PR><<<grid, kThreads, 0, st>>>(t); \
        else layer_bwd_top_kernel<OP, 64, PR><<<grid, kThreads, 0, st>>>(t);            \
    } while (0)
#define GS_BWDT(OP) do { if (t.b.off2) GS_BWDT2(OP, true); else GS_BWDT2(OP, false); } while (0)
    if (a.agg == GS_AGG_MEAN) GS_BWDT(GS_AGG_MEAN);
    else GS_BWDT(GS_AGG_MAX);
#undef GS_BWDT
#undef GS_BWDT2
    check_launch("layer_bwd_top");
    *deferred = SlabSum{a.slabs, S, a.H * K, a.dW, nullptr};
    return S > 1 ? sum_slabs_pair_parts2(a.H * K) : 0;
}

}  // namespace gs
