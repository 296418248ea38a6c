// Probe: can the host write packs straight into device memory (fine-grained
// VRAM through the BAR) and how fast, against pinned host memory that a
// kernel pulls over PCIe?  Developer tool, not part of the library:
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/lab/vram_probe.hip -o tools/bin/vram_probe
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); return 2; } } while (0)

__global__ void sum_kernel(const unsigned* p, size_t n, unsigned long long* out) {
    unsigned long long s = 0;
    for (size_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x) s += p[i];
    atomicAdd(out, s);
}

int main() {
    const size_t bytes = 256 << 10, n = bytes / 4;
    std::vector<unsigned> src(n);
    unsigned long long want = 0;
    for (size_t i = 0; i < n; ++i) {
        src[i] = static_cast<unsigned>(i * 2654435761u);
        want += src[i];
    }
    unsigned long long* dsum;
    CK(hipMalloc(&dsum, 8));
    const struct { const char* name; unsigned flags; } kinds[] = {{"finegrained", hipDeviceMallocFinegrained},
                                                                {"uncached", hipDeviceMallocUncached}};
    for (const auto& k : kinds) {
        void* p = nullptr;
        hipError_t e = hipExtMallocWithFlags(&p, bytes, k.flags);
        if (e != hipSuccess) {
            std::printf("%s: alloc failed: %s\n", k.name, hipGetErrorString(e));
            continue;
        }
        hipPointerAttribute_t attr;
        CK(hipPointerGetAttributes(&attr, p));
        std::printf("%s: device %p, host view %p\n", k.name, attr.devicePointer, attr.hostPointer);
        std::fflush(stdout);
        if (!attr.hostPointer) continue;
        // host writes (this is the part that may not be mapped)
        const int reps = 50;
        const auto t0 = std::chrono::steady_clock::now();
        for (int r = 0; r < reps; ++r) std::memcpy(attr.hostPointer, src.data(), bytes);
        __atomic_thread_fence(__ATOMIC_SEQ_CST);
        const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / reps;
        CK(hipMemset(dsum, 0, 8));
        sum_kernel<<<64, 256>>>(static_cast<const unsigned*>(p), n, dsum);
        unsigned long long got = 0;
        CK(hipMemcpy(&got, dsum, 8, hipMemcpyDeviceToHost));
        std::printf("%s: host memcpy %.1f us per 256 KiB (%.1f GB/s); device sum %s\n", k.name, us, bytes / us / 1e3,
                    got == want ? "matches" : "MISMATCH");
        CK(hipFree(p));
    }
    // the current path: pinned host memory read by a kernel
    void* h = nullptr;
    CK(hipHostMalloc(&h, bytes, hipHostMallocDefault));
    const auto t0 = std::chrono::steady_clock::now();
    for (int r = 0; r < 50; ++r) std::memcpy(h, src.data(), bytes);
    const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / 50;
    std::printf("pinned host: host memcpy %.1f us per 256 KiB\n", us);
    CK(hipHostFree(h));
    return 0;
}
