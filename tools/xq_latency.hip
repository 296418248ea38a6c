// Probe: GPU-side latency of a cross-stream dependency (hipStreamWaitEvent)
// versus back-to-back kernels on one stream.  Each kernel stamps
// s_memrealtime (100 MHz) at entry of block 0 and at exit of its last block;
// the gap = consumer entry - producer exit.
//   hipcc -O3 --offload-arch=gfx950 tools/xq_latency.hip -o /tmp/xq && /tmp/xq
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

#define CK(x)                                                                    \
    do {                                                                         \
        hipError_t e_ = (x);                                                     \
        if (e_ != hipSuccess) {                                                  \
            std::printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            return 1;                                                            \
        }                                                                        \
    } while (0)

__global__ void stamp_kernel(unsigned long long* t, int slot, int spin_ticks) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    if (blockIdx.x == 0 && threadIdx.x == 0) t[2 * slot] = t0;
    if (spin_ticks > 0)
        while (__builtin_amdgcn_s_memrealtime() - t0 < static_cast<unsigned long long>(spin_ticks)) {
        }
    __syncthreads();
    if (threadIdx.x == 0) atomicMax(&t[2 * slot + 1], __builtin_amdgcn_s_memrealtime());
}

int main() {
    constexpr int kReps = 64;
    unsigned long long* t;
    CK(hipMalloc(&t, sizeof(unsigned long long) * 2 * 8 * kReps));
    CK(hipMemset(t, 0, sizeof(unsigned long long) * 2 * 8 * kReps));
    hipStream_t a, b;
    CK(hipStreamCreateWithFlags(&a, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&b, hipStreamNonBlocking));
    hipEvent_t ev_nt, ev_t;
    CK(hipEventCreateWithFlags(&ev_nt, hipEventDisableTiming));
    CK(hipEventCreate(&ev_t));
    // warm both streams
    stamp_kernel<<<64, 64, 0, a>>>(t, 0, 0);
    stamp_kernel<<<64, 64, 0, b>>>(t, 0, 0);
    CK(hipDeviceSynchronize());
    CK(hipMemset(t, 0, sizeof(unsigned long long) * 2 * 8 * kReps));
    for (int r = 0; r < kReps; ++r) {
        // (0) same stream: producer (2000 ticks = 20 us, so the consumer is queued) -> consumer
        stamp_kernel<<<64, 64, 0, a>>>(t, 8 * r + 0, 2000);
        stamp_kernel<<<64, 64, 0, a>>>(t, 8 * r + 1, 0);
        // (1) cross stream, event without timing
        stamp_kernel<<<64, 64, 0, a>>>(t, 8 * r + 2, 2000);
        CK(hipEventRecord(ev_nt, a));
        CK(hipStreamWaitEvent(b, ev_nt, 0));
        stamp_kernel<<<64, 64, 0, b>>>(t, 8 * r + 3, 0);
        CK(hipStreamSynchronize(b));
        // (2) cross stream, timing event
        stamp_kernel<<<64, 64, 0, a>>>(t, 8 * r + 4, 2000);
        CK(hipEventRecord(ev_t, a));
        CK(hipStreamWaitEvent(b, ev_t, 0));
        stamp_kernel<<<64, 64, 0, b>>>(t, 8 * r + 5, 0);
        CK(hipStreamSynchronize(b));
        // (3) same stream, timing event recorded between the two kernels
        stamp_kernel<<<64, 64, 0, a>>>(t, 8 * r + 6, 2000);
        CK(hipEventRecord(ev_t, a));
        stamp_kernel<<<64, 64, 0, a>>>(t, 8 * r + 7, 0);
        CK(hipStreamSynchronize(a));
    }
    CK(hipDeviceSynchronize());
    std::vector<unsigned long long> h(2 * 8 * kReps);
    CK(hipMemcpy(h.data(), t, h.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost));
    const char* names[4] = {"same stream", "cross stream (event, no timing)", "cross stream (timing event)",
                            "same stream + timing event between"};
    for (int v = 0; v < 4; ++v) {
        std::vector<double> gap;
        for (int r = 4; r < kReps; ++r) {
            const unsigned long long prod_end = h[2 * (8 * r + 2 * v) + 1];
            const unsigned long long cons_beg = h[2 * (8 * r + 2 * v + 1)];
            gap.push_back((static_cast<double>(cons_beg) - static_cast<double>(prod_end)) * 0.01);  // us
        }
        std::sort(gap.begin(), gap.end());
        std::printf("%-40s gap us: min %.2f  median %.2f  p90 %.2f\n", names[v], gap.front(), gap[gap.size() / 2],
                    gap[gap.size() * 9 / 10]);
    }
    return 0;
}
