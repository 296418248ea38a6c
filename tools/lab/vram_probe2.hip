// Probe 2: fine-grained VRAM made host-accessible through HSA
// (hsa_amd_agents_allow_access for the CPU agent), then host memcpy into it
// and a device checksum.  Developer tool, not part of the library:
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/lab/vram_probe2.hip -lhsa-runtime64 -o tools/bin/vram_probe2
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

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

static hsa_status_t find_cpu(hsa_agent_t a, void* data) {
    hsa_device_type_t t;
    if (hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t) == HSA_STATUS_SUCCESS && t == HSA_DEVICE_TYPE_CPU) {
        *static_cast<hsa_agent_t*>(data) = a;
        return HSA_STATUS_INFO_BREAK;
    }
    return HSA_STATUS_SUCCESS;
}

static void info(const char* what, void* p) {
    hsa_amd_pointer_info_t pi{};
    pi.size = sizeof(pi);
    uint32_t na = 0;
    hsa_agent_t* ag = nullptr;
    const hsa_status_t s = hsa_amd_pointer_info(p, &pi, malloc, &na, &ag);
    std::printf("%s: pointer_info status %d type %d agentBase %p hostBase %p size %zu accessible agents %u\n", what,
                int(s), int(pi.type), pi.agentBaseAddress, pi.hostBaseAddress, pi.sizeInBytes, na);
    free(ag);
}

int main() {
    const size_t bytes = 256 << 10, n = bytes / 4;
    CK(hipSetDevice(0));
    std::vector<unsigned> src(n);
    unsigned long long want = 0;
    for (size_t i = 0; i < n; ++i) {
        src[i] = static_cast<unsigned>(i * 2654435761u);
        want += src[i];
    }
    unsigned long long* dsum;
    CK(hipMalloc(&dsum, 8));
    hsa_agent_t cpu{};
    hsa_status_t hs = hsa_iterate_agents(find_cpu, &cpu);
    std::printf("iterate agents: %d, cpu handle %llu\n", int(hs), (unsigned long long)cpu.handle);
    if (!cpu.handle) return 3;
    void* p = nullptr;
    CK(hipExtMallocWithFlags(&p, 2 << 20, hipDeviceMallocFinegrained));
    info("before allow", p);
    hs = hsa_amd_agents_allow_access(1, &cpu, nullptr, p);
    std::printf("allow_access: %d\n", int(hs));
    info("after allow", p);
    std::fflush(stdout);
    hsa_amd_pointer_info_t pi{};
    pi.size = sizeof(pi);
    if (hs != HSA_STATUS_SUCCESS || hsa_amd_pointer_info(p, &pi, nullptr, nullptr, nullptr) != HSA_STATUS_SUCCESS ||
        !pi.hostBaseAddress) {
        std::printf("no host mapping: stop\n");
        return 0;
    }
    void* hp = pi.hostBaseAddress;
    const int reps = 50;
    const auto t0 = std::chrono::steady_clock::now();
    for (int r = 0; r < reps; ++r) std::memcpy(hp, src.data(), bytes);
    __atomic_thread_fence(__ATOMIC_SEQ_CST);
    const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / reps;
    CK(hipMemset(dsum, 0, 8));
    sum_kernel<<<64, 256>>>(static_cast<const unsigned*>(p), n, dsum);
    unsigned long long got = 0;
    CK(hipMemcpy(&got, dsum, 8, hipMemcpyDeviceToHost));
    std::printf("host memcpy into VRAM: %.1f us per 256 KiB (%.2f GB/s); device sum %s\n", us, bytes / us / 1e3,
                got == want ? "matches" : "MISMATCH");
    CK(hipFree(p));
    return 0;
}
