// Lab for the layer-1 SageLayer forward (linear_dev.hpp linear_fwd_wide_kernel)
// at the rmat2m step's shape: n 4400 rows of dense [self | agg] (2F = 512
// floats), W1 [128][512], fp32, relu, no pending update.  Event timing over
// back-to-back launches (warm caches, and with the MALL flushed before each
// launch), then one launch's per-workgroup stage stamps (100 MHz):
//   0 start, 1 first K chunk stashed, 2 K loop done, 3 (PEND fold), 4 stored.
// Row splits: the library's balanced one (one workgroup per CU and column
// tile) and fixed 32-row tiles (the round-4 grid).
// Developer tool, not part of the library:
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 -I include -I graphsage-pytorch_amd/csrc/kernels \
//         tools/lab/fwd_lab.hip -o tools/bin/fwd_lab
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <random>
#include <vector>

__device__ unsigned long long* g_stamps;
// (a global-address-space store: a flat store pending at the K loop would make
// the wait-count pass drain every load in it)
typedef __attribute__((address_space(1))) unsigned long long gstamp_t;
#define GS_FWD_STAMP(i)                                                                                        \
    do {                                                                                                       \
        if (g_stamps && threadIdx.x == 0)                                                                      \
            ((gstamp_t*)g_stamps)[blockIdx.x * 8 + (i)] = __builtin_amdgcn_s_memrealtime();                   \
    } while (0)
#include "../../graphsage-pytorch_amd/csrc/host/errors.cpp"
#include "../../graphsage-pytorch_amd/csrc/kernels/linear_dev.hpp"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); return 2; } } while (0)

__global__ void flush_kernel(float4* p, size_t n4) {
    for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n4; i += size_t(gridDim.x) * blockDim.x)
        p[i] = make_float4(1.f, 2.f, 3.f, 4.f);
}

int main() {
    const int n = 4400, F = 256, H = 128, K = 2 * F;
    std::mt19937 rng(5);
    std::uniform_real_distribution<float> U(-1.f, 1.f);
    std::vector<float> hA(size_t(n) * K), hW(size_t(H) * K);
    for (auto& v : hA) v = U(rng);
    for (auto& v : hW) v = 0.05f * U(rng);
    float *A, *W, *out, *flush;
    unsigned long long* stamps;
    const size_t flush_bytes = size_t(512) << 20;
    CK(hipMalloc(&A, hA.size() * 4));
    CK(hipMalloc(&W, hW.size() * 4));
    CK(hipMalloc(&out, size_t(n) * H * 4));
    CK(hipMalloc(&flush, flush_bytes));
    CK(hipMalloc(&stamps, 4096 * 8 * 8));
    CK(hipMemcpy(A, hA.data(), hA.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(W, hW.data(), hW.size() * 4, hipMemcpyHostToDevice));
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<float> ref;
    auto config = [&](bool balanced, int& rows, gs::FwdRows& rs, dim3& grid) {
        const int tiles = (n + 15) / 16, gy = (H + 63) / 64;
        if (balanced) {
            int groups = std::max(1, cus / gy);
            int per = (tiles + groups - 1) / groups;
            if (per > 4) {
                groups *= (per + 3) / 4;
                per = (tiles + groups - 1) / groups;
            }
            rs.base = tiles / groups;
            rs.extra = tiles % groups;
            rs.groups = groups;
            rows = 16 * per;
        } else {
            rows = 32;
            rs.groups = (n + 31) / 32;
            rs.base = 2;
            rs.extra = 0;
        }
        grid = dim3((rs.groups + 7) / 8 * 8 * gy);
    };
    auto launch = [&](int rows, const gs::FwdRows& rs, dim3 grid) {
        gs::FwdSpec sp{};
        const float* Xs = A;
        const float* Aa = A + F;
        switch (rows) {
            case 16: gs::linear_fwd_wide_kernel<float, 16, true, true, false><<<grid, 16 * 16>>>(n, F, H, K, Xs, K, nullptr, Aa, K, W, out, H, rs, sp); break;
            case 32: gs::linear_fwd_wide_kernel<float, 32, true, true, false><<<grid, 32 * 16>>>(n, F, H, K, Xs, K, nullptr, Aa, K, W, out, H, rs, sp); break;
            case 48: gs::linear_fwd_wide_kernel<float, 48, true, true, false><<<grid, 48 * 16>>>(n, F, H, K, Xs, K, nullptr, Aa, K, W, out, H, rs, sp); break;
            default: gs::linear_fwd_wide_kernel<float, 64, true, true, false><<<grid, 64 * 16>>>(n, F, H, K, Xs, K, nullptr, Aa, K, W, out, H, rs, sp); break;
        }
    };
    const int fl_grid = 4096;
    for (int bal = 1; bal >= 0; --bal) {
        int rows;
        gs::FwdRows rs;
        dim3 grid;
        config(bal == 1, rows, rs, grid);
        // correctness against a host double reference on a few rows
        unsigned long long* none = nullptr;
        CK(hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), &none, sizeof(none)));
        launch(rows, rs, grid);
        CK(hipDeviceSynchronize());
        std::vector<float> ho(size_t(n) * H);
        CK(hipMemcpy(ho.data(), out, ho.size() * 4, hipMemcpyDeviceToHost));
        double maxerr = 0;
        for (int i = 0; i < n; i += 97)
            for (int h = 0; h < H; ++h) {
                double s = 0;
                for (int k = 0; k < K; ++k) s += double(hA[size_t(i) * K + k]) * hW[size_t(h) * K + k];
                s = std::max(0.0, s);
                maxerr = std::max(maxerr, std::abs(s - ho[size_t(i) * H + h]));
            }
        if (ref.empty()) ref = ho;
        const bool same = ho == ref;
        for (int flushed = 0; flushed < 2; ++flushed) {
            float tot = 0;
            const int reps = 100;
            for (int it = 0; it < reps + 10; ++it) {
                if (flushed) flush_kernel<<<fl_grid, 256>>>(reinterpret_cast<float4*>(flush), flush_bytes / 16);
                CK(hipEventRecord(e0, 0));
                launch(rows, rs, grid);
                CK(hipEventRecord(e1, 0));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                if (it >= 10) tot += ms;
            }
            std::printf("%s rows %d grid %u (groups %d base %d extra %d), %s: %.2f us per launch (event), max|err| %.2e, %s\n",
                        bal ? "balanced" : "fixed-32", rows, grid.x, rs.groups, rs.base, rs.extra,
                        flushed ? "MALL flushed" : "warm", tot / reps * 1e3, maxerr,
                        same ? "bitwise = balanced" : "DIFFERS from balanced");
        }
        // stage stamps of one warm launch
        CK(hipMemset(stamps, 0, 4096 * 8 * 8));
        CK(hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), &stamps, sizeof(stamps)));
        launch(rows, rs, grid);
        CK(hipDeviceSynchronize());
        none = nullptr;
        CK(hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), &none, sizeof(none)));
        std::vector<unsigned long long> st(grid.x * 8);
        CK(hipMemcpy(st.data(), stamps, st.size() * 8, hipMemcpyDeviceToHost));
        unsigned long long lo = ~0ull, hi = 0, slo = ~0ull, shi = 0;
        double d[5] = {0, 0, 0, 0, 0}, dmax = 0;
        int nb = 0;
        for (unsigned b = 0; b < grid.x; ++b) {
            const unsigned long long* s = &st[b * 8];
            if (!s[0] || !s[4]) continue;  // spare blocks
            ++nb;
            lo = std::min(lo, s[0]);
            hi = std::max(hi, s[4]);
            slo = std::min(slo, s[0]);
            shi = std::max(shi, s[0]);
            for (int i = 1; i <= 4; ++i) d[i] += double(s[i] - s[i - 1]);
            dmax = std::max(dmax, double(s[4] - s[0]));
        }
        std::printf("  stamps over %d workgroups: start -> chunk 0 in LDS %.2f, K loop %.2f, fold %.2f, store %.2f us; "
                    "workgroup max %.2f, start spread %.2f, span %.2f us\n",
                    nb, d[1] / nb * 1e-2, d[2] / nb * 1e-2, d[3] / nb * 1e-2, d[4] / nb * 1e-2, dmax * 1e-2,
                    double(shi - slo) * 1e-2, double(hi - lo) * 1e-2);
    }
    return 0;
}
