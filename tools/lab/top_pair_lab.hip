// Lab for kernels/top.hip's pair form (sage_top_pair_kernel: two blocks per 4
// roots, each with half of W2, the partial logits exchanged between them)
// against the library's one-block form.  Derived from top_lab.hip: synthetic inputs
// at the rmat2m step's sizes (B 512 roots, n1 4400 layer-1 rows, ~8.4
// neighbours per root, H 128, 16 classes), event timing over repeated
// launches, and per-stage s_memrealtime stamps (100 MHz) of every block.
// Developer tool, not part of the library:
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 -I include -I graphsage-pytorch_amd/csrc/kernels \
//         tools/lab/top_lab.hip -o tools/bin/top_lab
//   tools/bin/top_lab [tids]    (tids: the runner's padded list records, as in the step)
// Runs the library kernel (kernels/top.hip) and the round-4 one (top_v1.hip)
// on the same inputs: time per launch, error against a double-precision CPU
// reference, and the library kernel's stage stamps.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <cstdio>
#include <random>
#include <string>
#include <vector>

__device__ unsigned long long* g_stamps;
#define GS_TOP_STAMP(i)                                                                            \
    do {                                                                                           \
        if (g_stamps && threadIdx.x == 0) g_stamps[blockIdx.x * 16 + (i)] = __builtin_amdgcn_s_memrealtime(); \
    } while (0)
#include "../../graphsage-pytorch_amd/csrc/host/errors.cpp"
#include "../../graphsage-pytorch_amd/csrc/kernels/top.hip"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); return 2; } } while (0)

int main(int argc, char** argv) {
    const int B = 512, n1 = 4400, H = 128, C = 16, K = 256;
    std::mt19937 rng(7);
    std::uniform_real_distribution<float> U(-1.f, 1.f);
    std::vector<float> h1(size_t(n1) * H), W(size_t(H) * K), Wc(C * H), bc(C);
    for (auto& v : h1) v = std::max(0.f, U(rng));
    for (auto& v : W) v = 0.05f * U(rng);
    for (auto& v : Wc) v = 0.1f * U(rng);
    for (auto& v : bc) v = 0.1f * U(rng);
    std::vector<int> ptr(B + 1, 0), nbr, self(B), labels(n1), roots(B);
    for (int r = 0; r < B; ++r) {
        const int d = 1 + rng() % 16;
        std::vector<int> s;
        for (int j = 0; j < d; ++j) s.push_back(rng() % n1);
        std::sort(s.begin(), s.end());
        s.erase(std::unique(s.begin(), s.end()), s.end());
        nbr.insert(nbr.end(), s.begin(), s.end());
        ptr[r + 1] = static_cast<int>(nbr.size());
        self[r] = rng() % n1;
        roots[r] = r;
    }
    for (int i = 0; i < n1; ++i) labels[i] = i % C;
    auto up = [](const auto& v, auto** d) {
        hipMalloc(reinterpret_cast<void**>(d), v.size() * sizeof(v[0]));
        hipMemcpy(*d, v.data(), v.size() * sizeof(v[0]), hipMemcpyHostToDevice);
    };
    float *dh1, *dW, *dWc, *dbc, *agg, *E, *dZ, *dIn, *slab;
    int *dptr, *dnbr, *dself, *dlab, *droots;
    up(h1, &dh1); up(W, &dW); up(Wc, &dWc); up(bc, &dbc);
    up(ptr, &dptr); up(nbr, &dnbr); up(self, &dself); up(labels, &dlab); up(roots, &droots);
    // argv[1] == "tids": the runner's padded records [self | list padded to 25 with -1]
    const bool use_tids = argc > 1 && std::string(argv[1]) == "tids";
    const int tk = 25;
    std::vector<int> tids(size_t(B) * (tk + 1), -1);
    for (int r = 0; r < B; ++r) {
        tids[size_t(r) * (tk + 1)] = self[r];
        for (int e = ptr[r]; e < ptr[r + 1]; ++e) tids[size_t(r) * (tk + 1) + 1 + (e - ptr[r])] = nbr[e];
    }
    int* dtids;
    up(tids, &dtids);
    CK(hipMalloc(&agg, B * K * 4));  // [self | agg] rows (v1 writes the agg half only)
    CK(hipMalloc(&E, B * H * 4)); CK(hipMalloc(&dZ, B * H * 4));
    CK(hipMalloc(&dIn, B * K * 4)); CK(hipMalloc(&slab, (B / 4 + 1) * (C * (H + 1) + 1) * 4));
    float* dIn2;
    CK(hipMalloc(&dIn2, B * K * 4));
    CK(hipMemset(dIn2, 0, B * K * 4));
    unsigned long long* xch;
    unsigned* fail;
    CK(hipMalloc(&xch, size_t(B / 4 + 16) * 2 * 64 * 8));
    CK(hipMemset(xch, 0, size_t(B / 4 + 16) * 2 * 64 * 8));
    CK(hipMalloc(&fail, 4));
    CK(hipMemset(fail, 0, 4));
    unsigned epoch = 0;
    bool pair_mode = false;
    unsigned long long* st;
    const int nb = (B + 3) / 4;
    CK(hipMalloc(&st, size_t(16 * ((nb + 7) / 8)) * 16 * 8));
    if (!gs::top_supported(H, C, false)) { std::printf("top not supported (LDS)\n"); return 3; }
    hipStream_t s;
    CK(hipStreamCreate(&s));
    auto launch = [&] {
        gs::top_fwd_bwd(GS_AGG_MEAN, B, C, dh1, dptr, dnbr, dself, dW, dWc, dbc, dlab, droots, agg, nullptr, E, dZ,
                        dIn, slab, s, use_tids ? dtids : nullptr, use_tids ? tk : 0);
    };
    auto launch_v1 = [&] {  // the pair form
        gs::top_pair_fwd_bwd(GS_AGG_MEAN, B, C, dh1, dptr, dnbr, dself, dW, dWc, dbc, dlab, droots, agg, nullptr, E,
                             dZ, dIn, dIn2, slab, xch, ++epoch, fail, s, use_tids ? dtids : nullptr, use_tids ? tk : 0);
    };
    // double-precision reference of the step's outputs (models.py:209-220, 8-27)
    std::vector<double> rE(size_t(B) * H), rZ(size_t(B) * H), rI(size_t(B) * K), rS(size_t(nb) * (C * (H + 1) + 1), 0.0);
    for (int r = 0; r < B; ++r) {
        std::vector<double> x(K, 0.0);
        for (int f = 0; f < H; ++f) x[f] = h1[size_t(self[r]) * H + f];
        const int cnt = ptr[r + 1] - ptr[r];
        for (int e = ptr[r]; e < ptr[r + 1]; ++e)
            for (int f = 0; f < H; ++f) x[H + f] += h1[size_t(nbr[e]) * H + f] / cnt;
        for (int c = 0; c < H; ++c) {
            double z = 0;
            for (int k = 0; k < K; ++k) z += x[k] * W[size_t(c) * K + k];
            rE[size_t(r) * H + c] = z > 0 ? z : 0;
        }
        std::vector<double> lg(C);
        double mx = -1e300;
        for (int c = 0; c < C; ++c) {
            double z = bc[c];
            for (int d = 0; d < H; ++d) z += rE[size_t(r) * H + d] * Wc[size_t(c) * H + d];
            lg[c] = z;
            mx = std::max(mx, z);
        }
        double se = 0;
        for (int c = 0; c < C; ++c) se += std::exp(lg[c] - mx);
        std::vector<double> dl(C);
        const int y = labels[roots[r]];
        for (int c = 0; c < C; ++c) dl[c] = (std::exp(lg[c] - mx) / se - (c == y ? 1.0 : 0.0)) / B;
        for (int d = 0; d < H; ++d) {
            double z = 0;
            for (int c = 0; c < C; ++c) z += dl[c] * Wc[size_t(c) * H + d];
            rZ[size_t(r) * H + d] = rE[size_t(r) * H + d] > 0 ? z : 0;
        }
        for (int k = 0; k < K; ++k) {
            double z = 0;
            for (int h = 0; h < H; ++h) z += rZ[size_t(r) * H + h] * W[size_t(h) * K + k];
            rI[size_t(r) * K + k] = z;
        }
        const int per = C * (H + 1);
        for (int c = 0; c < C; ++c)
            for (int d = 0; d <= H; ++d) rS[size_t(r / 4) * (per + 1) + c * (H + 1) + d] += dl[c] * (d < H ? rE[size_t(r) * H + d] : 1.0);
        rS[size_t(r / 4) * (per + 1) + per] += -(lg[y] - mx - std::log(se));
    }
    auto check = [&](const char* tag) -> int {
        std::vector<float> hE(B * H), hI(B * K), hZ(B * H), hS(rS.size());
        CK(hipMemcpy(hE.data(), E, B * H * 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(hI.data(), dIn, B * K * 4, hipMemcpyDeviceToHost));
        if (pair_mode) {
            std::vector<float> h2(B * K);
            CK(hipMemcpy(h2.data(), dIn2, B * K * 4, hipMemcpyDeviceToHost));
            for (size_t i = 0; i < hI.size(); ++i) hI[i] += h2[i];
            unsigned f = 0;
            CK(hipMemcpy(&f, fail, 4, hipMemcpyDeviceToHost));
            if (f) std::printf("  PAIR EXCHANGE GAVE UP\n");
        }
        CK(hipMemcpy(hZ.data(), dZ, B * H * 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(hS.data(), slab, hS.size() * 4, hipMemcpyDeviceToHost));
        auto err = [](const std::vector<float>& a, const std::vector<double>& b) {
            double m = 0, s = 0;
            for (size_t i = 0; i < a.size(); ++i) { m = std::max(m, std::fabs(a[i] - b[i])); s = std::max(s, std::fabs(b[i])); }
            return std::make_pair(m, s);
        };
        auto e1 = err(hE, rE), e2 = err(hZ, rZ), e3 = err(hI, rI), e4 = err(hS, rS);
        unsigned long long hsh = 1469598103934665603ull;
        for (auto* v : {&hE, &hZ, &hI})
            for (float x : *v) { uint32_t u; std::memcpy(&u, &x, 4); hsh = (hsh ^ u) * 1099511628211ull; }
        std::printf("  %s: max |err| (max |ref|): E %.2e (%.2e)  dZ %.2e (%.2e)  dIn %.2e (%.2e)  slab %.2e (%.2e)  hash %016llx\n",
                    tag, e1.first, e1.second, e2.first, e2.second, e3.first, e3.second, e4.first, e4.second, hsh);
        return 0;
    };
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    const int reps = 200;
    for (int pass = 0; pass < 2; ++pass) {  // v1 / v2 / v1 / v2: alternating
        for (int v = 0; v < 2; ++v) {
            pair_mode = v == 0;
            for (int i = 0; i < 20; ++i) v ? launch() : launch_v1();
            CK(hipEventRecord(e0, s));
            for (int i = 0; i < reps; ++i) v ? launch() : launch_v1();
            CK(hipEventRecord(e1, s));
            CK(hipEventSynchronize(e1));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            std::printf("%s top kernel: %.2f us per launch (back to back, %d launches)\n", v ? "one-block" : "pair",
                        ms * 1e3 / reps, reps);
            if (pass == 0 && check(v ? "one-block" : "pair")) return 2;
        }
    }
    // stamps of one launch
    CK(hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), &st, sizeof(st)));
    CK(hipMemset(st, 0, size_t(16 * ((nb + 7) / 8)) * 128));
    const int NS = 10;
    const char* names[] = {"", "dma issue + Wc + gather", "wait W2 DMA + barrier", "E (4x4x1 split-K)",
                           "E combine + barrier", "logits + barrier", "softmax + barrier", "dZ + slab + barrier",
                           "dIn MFMA + barrier", "dIn combine + store"};
    for (int rep = 0; rep < 4; ++rep) {  // single launches (warm), stamped: one-block, pair, one-block, pair
        const bool pr = rep & 1;
        const int nbl = pr ? 16 * ((nb + 7) / 8) : nb;
        for (int i = 0; i < 20; ++i) pr ? launch_v1() : launch();
        CK(hipStreamSynchronize(s));
        CK(hipMemset(st, 0, size_t(nbl) * 128));
        CK(hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), &st, sizeof(st)));
        pr ? launch_v1() : launch();
        CK(hipStreamSynchronize(s));
        unsigned long long* nul = nullptr;
        CK(hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), &nul, sizeof(nul)));
        std::vector<unsigned long long> h(nbl * 16);
        CK(hipMemcpy(h.data(), st, size_t(nbl) * 128, hipMemcpyDeviceToHost));
        if (pr) for (int b = 0; b < nbl; ++b) h[b * 16 + 5] = h[b * 16 + 4];  // the pair form has no stage-5 stamp
        unsigned long long t0 = ~0ull;
        for (int b = 0; b < nbl; ++b) if (h[b * 16]) t0 = std::min(t0, h[b * 16]);
        double acc[16] = {0}, mx[16] = {0};
        double last_end = 0, first_start = 1e18;
        int nused = 0;
        for (int b = 0; b < nbl; ++b) {
            if (!h[b * 16]) continue;
            ++nused;
            for (int i = 1; i < NS; ++i) {
                const double d = (h[b * 16 + i] - h[b * 16 + i - 1]) * 0.01;
                acc[i] += d;
                mx[i] = std::max(mx[i], d);
            }
            last_end = std::max(last_end, (h[b * 16 + NS - 1] - t0) * 0.01);
            first_start = std::min(first_start, (h[b * 16] - t0) * 0.01);
        }
        std::printf("stamped launch %d (%s)\n", rep, pr ? "pair" : "one-block");
        for (int i = 1; i < NS; ++i) std::printf("  stage %d %-32s mean %.2f us  max %.2f us\n", i, names[i], acc[i] / nused, mx[i]);
        double spread = 0;
        for (int b = 0; b < nbl; ++b) if (h[b * 16]) spread = std::max(spread, (h[b * 16] - t0) * 0.01);
        std::printf("  block start spread %.2f us; first start -> last end %.2f us\n", spread, last_end - first_start);
    }
    return 0;
}
