// C-ABI launchers of the gather-aggregate kernels (kernels/agg_dev.hpp).
#include "agg_dev.hpp"

namespace gs {

template <int OP, typename T, bool EXPAND>
static void launch_fwd(int vec, const T* X, int64_t ldx, int F, int n_dst, const int* ptr,
                       const int* idx, const int64_t* row_ptr, const int* col, const int* dst_ids,
                       int gcn, T* out, int64_t ldo, int* am, hipStream_t st) {
    constexpr int V = sizeof(T) == 4 ? 4 : 8;
    if (vec == 1) {
        const dim3 grid((n_dst + (kBlock / 64) - 1) / (kBlock / 64));
        launch_k(agg_fwd_kernel<OP, T, 1, 64, EXPAND>, grid, dim3(kBlock), 0, st, X, ldx, F, n_dst, ptr, idx, row_ptr,
                 col, dst_ids, gcn, out, ldo, am);
        return;
    }
    const int G = pick_group(F, V);
    const dim3 grid((n_dst + (kBlock / G) - 1) / (kBlock / G));
#define GS_AGG_FWD(GG)                                                                                   \
    launch_k(agg_fwd_kernel<OP, T, V, GG, EXPAND>, grid, dim3(kBlock), 0, st, X, ldx, F, n_dst, ptr, idx, row_ptr, \
             col, dst_ids, gcn, out, ldo, am)
    if (G == 16) GS_AGG_FWD(16);
    else if (G == 32) GS_AGG_FWD(32);
    else GS_AGG_FWD(64);
#undef GS_AGG_FWD
}

template <int OP>
static void launch_bwd(int vec, int n_src, int F, const int* tptr, const int* tidx, const int* ptr,
                       const float* dA, const float* dSelf, int64_t ldd, const int* am,
                       const float* Hprev, int64_t ldh, float* dH, hipStream_t st) {
    if (vec == 1) {
        const dim3 grid((n_src + 3) / 4);
        agg_bwd_kernel<OP, 1, 64><<<grid, kBlock, 0, st>>>(n_src, F, tptr, tidx, ptr, dA, dSelf, ldd, am,
                                                           Hprev, ldh, dH);
        return;
    }
    const int G = pick_group(F, 4);
    const dim3 grid((n_src + (kBlock / G) - 1) / (kBlock / G));
#define GS_AGG_BWD(GG)                                                                          \
    agg_bwd_kernel<OP, 4, GG><<<grid, kBlock, 0, st>>>(n_src, F, tptr, tidx, ptr, dA, dSelf, ldd, am, \
                                                       Hprev, ldh, dH)
    if (G == 16) GS_AGG_BWD(16);
    else if (G == 32) GS_AGG_BWD(32);
    else GS_AGG_BWD(64);
#undef GS_AGG_BWD
}

}  // namespace gs

extern "C" {

int gs_agg_fwd(gs_agg op, gs_dtype xdt, const void* X, int64_t ldx, int64_t F, int64_t n_dst,
               const int32_t* ptr, const int32_t* idx, const int64_t* row_ptr, const int32_t* col,
               const int32_t* dst_ids, int32_t gcn, void* out, gs_dtype odt, int64_t ldo,
               int32_t* argmax, void* stream) {
    GS_API_BEGIN
    using namespace gs;
    GS_REQUIRE(op == GS_AGG_MEAN || op == GS_AGG_MAX, GS_EINVAL, "agg_func must be MEAN or MAX");
    GS_REQUIRE(xdt == odt, GS_EINVAL, "output dtype must equal feature dtype");
    GS_REQUIRE(F >= 1 && F < (1 << 30) && n_dst >= 0 && n_dst < (int64_t(1) << 31), GS_EINVAL, "bad sizes");
    GS_REQUIRE(ldx >= F && ldo >= F, GS_EINVAL, "leading dimension smaller than F");
    if (n_dst == 0) return GS_OK;
    GS_REQUIRE(X && ptr && idx && out, GS_EINVAL, "NULL device pointer");
    const bool expand = col != nullptr;
    GS_REQUIRE(!expand || dst_ids, GS_EINVAL, "expand mode needs dst_ids");
    GS_REQUIRE(!(argmax && expand), GS_EINVAL, "argmax is only produced in explicit mode");
    const int V = xdt == GS_F32 ? 4 : 8;
    const int vec = (F % V == 0 && ldx % V == 0 && ldo % V == 0 && aligned16(X) && aligned16(out)) ? V : 1;
    hipStream_t st = as_stream(stream);
    const int f = static_cast<int>(F), n = static_cast<int>(n_dst);
#define GS_DISPATCH(OPV, TT)                                                                              \
    do {                                                                                                  \
        if (expand)                                                                                       \
            launch_fwd<OPV, TT, true>(vec, static_cast<const TT*>(X), ldx, f, n, ptr, idx, row_ptr, col,  \
                                      dst_ids, gcn, static_cast<TT*>(out), ldo, nullptr, st);             \
        else                                                                                              \
            launch_fwd<OPV, TT, false>(vec, static_cast<const TT*>(X), ldx, f, n, ptr, idx, nullptr,      \
                                       nullptr, nullptr, 0, static_cast<TT*>(out), ldo, argmax, st);      \
    } while (0)
    if (op == GS_AGG_MEAN) {
        if (xdt == GS_F32) GS_DISPATCH(GS_AGG_MEAN, float);
        else GS_DISPATCH(GS_AGG_MEAN, bf16_t);
    } else {
        if (xdt == GS_F32) GS_DISPATCH(GS_AGG_MAX, float);
        else GS_DISPATCH(GS_AGG_MAX, bf16_t);
    }
#undef GS_DISPATCH
    check_launch("gs_agg_fwd");
    GS_API_END
}

int gs_agg_bwd(gs_agg op, int64_t n_src, int64_t F, const int32_t* tptr, const int32_t* tidx,
               const int32_t* ptr, const float* dA, const float* dSelf, int64_t ldd,
               const int32_t* argmax, const float* Hprev, int64_t ldh, float* dH, void* stream) {
    GS_API_BEGIN
    using namespace gs;
    GS_REQUIRE(op == GS_AGG_MEAN || op == GS_AGG_MAX, GS_EINVAL, "agg_func must be MEAN or MAX");
    GS_REQUIRE(F >= 1 && n_src >= 0 && n_src < (int64_t(1) << 31), GS_EINVAL, "bad sizes");
    GS_REQUIRE(ldd >= F && ldh >= F, GS_EINVAL, "leading dimension smaller than F");
    if (n_src == 0) return GS_OK;
    GS_REQUIRE(tptr && tidx && ptr && dA && dH, GS_EINVAL, "NULL device pointer");
    GS_REQUIRE(op != GS_AGG_MAX || argmax, GS_EINVAL, "MAX backward needs argmax");
    const int vec = (F % 4 == 0 && ldd % 4 == 0 && ldh % 4 == 0 && aligned16(dA) && (!dSelf || aligned16(dSelf)) &&
                     aligned16(dH) && (!Hprev || aligned16(Hprev)))
                        ? 4
                        : 1;
    hipStream_t st = as_stream(stream);
    if (op == GS_AGG_MEAN)
        launch_bwd<GS_AGG_MEAN>(vec, static_cast<int>(n_src), static_cast<int>(F), tptr, tidx, ptr, dA, dSelf,
                                ldd, argmax, Hprev, ldh, dH, st);
    else
        launch_bwd<GS_AGG_MAX>(vec, static_cast<int>(n_src), static_cast<int>(F), tptr, tidx, ptr, dA, dSelf,
                               ldd, argmax, Hprev, ldh, dH, st);
    check_launch("gs_agg_bwd");
    GS_API_END
}

}  // extern "C"
