// Lab for kernels/top.hip (the fused top layer + loss head): synthetic inputs
// at the rmat2m step's sizes (B 512 roots, n1 4400 layer-1 rows, ~8.4
// neighbours per root, H 128, 16 classes), event timing over repeated
// launches, and per-stage s_memrealtime stamps (100 MHz) of every block.
// Developer tool, not part of the library:
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 -I include tools/lab/top_lab.hip -o tools/bin/top_lab
//   tools/bin/top_lab [tids]    (tids: the runner's padded list records, as in the step)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <random>
#include <string>
#include <vector>

__device__ unsigned long long* g_stamps;
#define GS_TOP_STAMP(i)                                                                            \
    do {                                                                                           \
        if (g_stamps && threadIdx.x == 0) g_stamps[blockIdx.x * 8 + (i)] = __builtin_amdgcn_s_memrealtime(); \
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
    CK(hipMalloc(&agg, B * H * 4)); CK(hipMalloc(&E, B * H * 4)); CK(hipMalloc(&dZ, B * H * 4));
    CK(hipMalloc(&dIn, B * K * 4)); CK(hipMalloc(&slab, (B / 4 + 1) * (C * (H + 1) + 1) * 4));
    unsigned long long* st;
    const int nb = (B + 3) / 4;
    CK(hipMalloc(&st, nb * 8 * 8));
    if (!gs::top_supported(H, C, false)) { std::printf("top not supported (LDS)\n"); return 3; }
    hipStream_t s;
    CK(hipStreamCreate(&s));
    auto launch = [&] {
        gs::top_fwd_bwd(GS_AGG_MEAN, B, C, dh1, dptr, dnbr, dself, dW, dWc, dbc, dlab, droots, agg, nullptr, E, dZ,
                        dIn, slab, s, use_tids ? dtids : nullptr, use_tids ? tk : 0);
    };
    for (int i = 0; i < 20; ++i) launch();
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    const int reps = 200;
    CK(hipEventRecord(e0, s));
    for (int i = 0; i < reps; ++i) launch();
    CK(hipEventRecord(e1, s));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    std::printf("top kernel: %.2f us per launch (back to back, %d launches)\n", ms * 1e3 / reps, reps);
    {  // outputs' bit pattern (variants must agree bit for bit)
        std::vector<uint32_t> hE(B * H), hI(B * K), hZ(B * H);
        CK(hipMemcpy(hE.data(), E, B * H * 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(hI.data(), dIn, B * K * 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(hZ.data(), dZ, B * H * 4, hipMemcpyDeviceToHost));
        unsigned long long hsh = 1469598103934665603ull;
        for (auto* v : {&hE, &hZ, &hI})
            for (uint32_t x : *v) hsh = (hsh ^ x) * 1099511628211ull;
        std::printf("  outputs hash %016llx\n", hsh);
    }
    // stamps of one launch
    CK(hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), &st, sizeof(st)));
    CK(hipMemset(st, 0, nb * 64));
    launch();
    CK(hipStreamSynchronize(s));
    std::vector<unsigned long long> h(nb * 8);
    CK(hipMemcpy(h.data(), st, nb * 64, hipMemcpyDeviceToHost));
    unsigned long long t0 = ~0ull;
    for (int b = 0; b < nb; ++b) t0 = std::min(t0, h[b * 8]);
    double acc[8] = {0};
    double last_end = 0, first_start = 1e18;
    for (int b = 0; b < nb; ++b) {
        for (int i = 1; i <= 6; ++i) acc[i] += (h[b * 8 + i] - h[b * 8 + i - 1]) * 0.01;
        last_end = std::max(last_end, (h[b * 8 + 6] - t0) * 0.01);
        first_start = std::min(first_start, (h[b * 8] - t0) * 0.01);
    }
    const char* names[] = {"", "dma issue + head loads + gather", "wait W2 DMA + barrier", "GEMM (E)", "loss head",
                           "slab", "dIn GEMM"};
    for (int i = 1; i <= 6; ++i) std::printf("  stage %d %-32s mean %.2f us\n", i, names[i], acc[i] / nb);
    double spread = 0;
    for (int b = 0; b < nb; ++b) spread = std::max(spread, (h[b * 8] - t0) * 0.01);
    std::printf("  block start spread %.2f us; first start -> last end %.2f us\n", spread, last_end - first_start);
    return 0;
}
