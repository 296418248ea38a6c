// Lab for the layer-1 weight gradient (linear_dev.hpp linear_dw_xcd_kernel,
// two row phases) at the rmat2m step's shape: n 4378 rows of dense
// [self | agg] (2F = 512 floats), dZ [n][128], fp32, the library's slab split.
// Event timing over back-to-back launches (warm caches), a check of the slab
// sum against a host double reference, then one launch's per-workgroup stage
// stamps (100 MHz): 0 start, 1 first chunk stashed, 2 row loop done, 3 stored.
// Developer tool, not part of the library:
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 -I include -I graphsage-pytorch_amd/csrc/kernels \
//         [-DGS_DW_CHUNK=32] tools/lab/dw_lab.hip -o tools/bin/dw_lab
// (The round-5 ablations — no MFMA, MFMAs alone, no barrier, no operand reads,
// no stash, cache-hot loads — compiled hooks into linear_dw_body that have since
// been removed; their results are in DESIGN §14.)
//   tools/bin/dw_lab [n] [rows per slab]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <random>
#include <vector>

__device__ unsigned long long* g_stamps;
// (a global-address-space store: a flat store pending at the row loop would
// make the wait-count pass drain every load in it)
typedef __attribute__((address_space(1))) unsigned long long gstamp_t;
// stamps: [block][phase][8]: 4 s_memrealtime (100 MHz) then 4 s_memtime (shader clock)
#define GS_DW_STAMP(i)                                                                                           \
    do {                                                                                                         \
        if (g_stamps && (threadIdx.x & 255) == 0) {                                                              \
            const unsigned long long rt_ = __builtin_amdgcn_s_memrealtime(), ct_ = __builtin_amdgcn_s_memtime(); \
            ((gstamp_t*)g_stamps)[(blockIdx.x * 2 + (threadIdx.x >> 8)) * 8 + (i)] = rt_;                      \
            ((gstamp_t*)g_stamps)[(blockIdx.x * 2 + (threadIdx.x >> 8)) * 8 + 4 + (i)] = ct_;                  \
        }                                                                                                        \
    } while (0)
#include "../../graphsage-pytorch_amd/csrc/host/errors.cpp"
#include "../../graphsage-pytorch_amd/csrc/kernels/linear_dev.hpp"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); return 2; } } while (0)

int main(int argc, char** argv) {
    const int n = argc > 1 ? std::atoi(argv[1]) : 4378;
    const int F = 256, H = 128, K = 2 * F, PH = 2;
    std::mt19937 rng(5);
    std::uniform_real_distribution<float> U(-1.f, 1.f);
    std::vector<float> hX(size_t(n) * K), hZ(size_t(n) * H);
    for (auto& v : hX) v = U(rng);
    for (auto& v : hZ) v = U(rng);
    // argv[2]: rows per slab (a multiple of 16) instead of the library's split
    const int rps = argc > 2 ? std::atoi(argv[2]) : gs::dw_rows_per_split(n, K, H, PH);
    const int S = argc > 2 ? (n + rps - 1) / rps : gs::dw_splits(n, K, H, PH);
    const int gx = (K + 63) / 64, tiles = gx * ((H + 63) / 64);
    const dim3 grid(gs::kXcds * tiles * ((S + gs::kXcds - 1) / gs::kXcds));
    float *X, *Z, *slabs;
    unsigned long long* stamps;
    CK(hipMalloc(&X, hX.size() * 4));
    CK(hipMalloc(&Z, hZ.size() * 4));
    CK(hipMalloc(&slabs, size_t(S) * H * K * 4));
    CK(hipMalloc(&stamps, size_t(grid.x) * 2 * 8 * 8));
    CK(hipMemcpy(X, hX.data(), hX.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(Z, hZ.data(), hZ.size() * 4, hipMemcpyHostToDevice));
    auto launch = [&]() {
        gs::linear_dw_xcd_kernel<float, true, false, true, true, 2><<<grid, 512>>>(
            n, F, H, K, rps, gx, tiles, S, X, K, nullptr, X + F, K, Z, nullptr, H, slabs, int64_t(H) * K,
            gs::KStamp{});
    };
    unsigned long long* none = nullptr;
    CK(hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), &none, sizeof(none)));
    launch();
    CK(hipDeviceSynchronize());
    std::vector<float> hs(size_t(S) * H * K);
    CK(hipMemcpy(hs.data(), slabs, hs.size() * 4, hipMemcpyDeviceToHost));
    double maxerr = 0, maxref = 0;
    for (int h = 0; h < H; h += 7)
        for (int k = 0; k < K; k += 5) {
            double ref = 0, got = 0;
            for (int i = 0; i < n; ++i) ref += double(hZ[size_t(i) * H + h]) * hX[size_t(i) * K + k];
            for (int z = 0; z < S; ++z) got += hs[(size_t(z) * H + h) * K + k];
            maxerr = std::max(maxerr, std::abs(ref - got));
            maxref = std::max(maxref, std::abs(ref));
        }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    float tot = 0;
    const int reps = 200;
    for (int it = 0; it < reps + 10; ++it) {
        CK(hipEventRecord(e0, 0));
        launch();
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (it >= 10) tot += ms;
    }
    const double flops = 2.0 * n * K * H;
    std::printf("n %d S %d rps %d grid %u chunk %d ahead %d: %.2f us per launch (event), %.1f TFLOP/s, "
                "max|err| %.2e of max|ref| %.2e\n",
                n, S, rps, grid.x, gs::kDwCh, gs::kDwAhead, tot / reps * 1e3, flops / (tot / reps * 1e-3) / 1e12,
                maxerr, maxref);
    CK(hipMemset(stamps, 0, size_t(grid.x) * 2 * 8 * 8));
    CK(hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), &stamps, sizeof(stamps)));
    launch();
    CK(hipDeviceSynchronize());
    CK(hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), &none, sizeof(none)));
    std::vector<unsigned long long> st(size_t(grid.x) * 2 * 8);
    CK(hipMemcpy(st.data(), stamps, st.size() * 8, hipMemcpyDeviceToHost));
    unsigned long long lo = ~0ull, hi = 0;
    double d[4] = {0, 0, 0, 0}, dmax = 0, loop_clk = 0;
    int nb = 0;
    for (unsigned b = 0; b < grid.x; ++b) {
        const unsigned long long* s = &st[size_t(b) * 2 * 8];  // phase 0 (it stores the slab)
        if (!s[0] || !s[3]) continue;
        ++nb;
        lo = std::min(lo, s[0]);
        hi = std::max(hi, s[3]);
        for (int i = 1; i <= 3; ++i) d[i] += double(s[i] - s[i - 1]);
        dmax = std::max(dmax, double(s[3] - s[0]));
        loop_clk += double(s[4 + 2] - s[4 + 1]);
    }
    std::printf("  stamps over %d workgroups: start -> chunk 0 stashed %.2f, row loop %.2f, exchange + store %.2f us; "
                "workgroup max %.2f, span %.2f us; row loop %.0f shader clocks (%.2f GHz)\n",
                nb, d[1] / nb * 1e-2, d[2] / nb * 1e-2, d[3] / nb * 1e-2, dmax * 1e-2, double(hi - lo) * 1e-2,
                loop_clk / nb, loop_clk / (d[2] * 1e-2 * 1e3));
    return 0;
}
