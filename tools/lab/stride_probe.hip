// Does the row stride of the layer-1 operands matter?  The wide forward's
// workgroups all read chunk c (256 B) of every row of W (64 rows, shared by
// every workgroup) and of their own 32 A rows at the same time; with 2 KiB
// rows those addresses share their low 11 bits.  This probe times the same
// read pattern (no LDS, no MFMA: loads summed into a register) with the row
// pitch at 512 floats (the library's) and padded pitches.
// Developer tool, not part of the library:
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/lab/stride_probe.hip -o tools/bin/stride_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); return 2; } } while (0)

// Block b: rows [32 b', 32 b' + 32) of A (b' = b / 2) and the 64-row half (b & 1)
// of W, K = 512 floats in chunks of 64 (16 lanes x 16 B per row), the
// forward's thread map; AHEAD chunks of loads in flight.
template <int AHEAD, int MODE>
__global__ __launch_bounds__(512) void probe_kernel(const float4* __restrict__ A, const float4* __restrict__ W,
                                                   int pitch4, int n_rows, float* __restrict__ out) {
    const int tid = threadIdx.x, lr = tid >> 4, ls = tid & 15;
    // MODE bit 2: the two column halves of a row tile 8 blocks apart (one XCD)
    const int rt = (MODE & 4) ? (blockIdx.x / 16) * 8 + (blockIdx.x & 7) : blockIdx.x >> 1;
    const int half = (MODE & 4) ? (blockIdx.x >> 3) & 1 : blockIdx.x & 1;
    const int arow = min(rt * 32 + lr, n_rows - 1);
    const float4* a = A + static_cast<int64_t>(arow) * pitch4 + ls;
    const float4* w0 = W + static_cast<int64_t>(half * 64 + lr) * pitch4 + ls;
    const float4* w1 = W + static_cast<int64_t>(half * 64 + lr + 32) * pitch4 + ls;
    float4 ra[AHEAD], rw0[AHEAD], rw1[AHEAD];
    float s = 0.f;
#pragma unroll
    for (int u = 0; u < AHEAD; ++u) {
        ra[u] = (MODE & 1) ? a[16 * u] : make_float4(0, 0, 0, 0);
        rw0[u] = (MODE & 2) ? w0[16 * u] : make_float4(0, 0, 0, 0);
        rw1[u] = (MODE & 2) ? w1[16 * u] : make_float4(0, 0, 0, 0);
    }
    for (int cb = 0; cb < 8; cb += AHEAD) {
#pragma unroll
        for (int u = 0; u < AHEAD; ++u) {
            const int c = cb + u, cn = min(c + AHEAD, 7);
            s += ra[u].x + ra[u].w + rw0[u].y + rw1[u].z;
            if (MODE & 1) ra[u] = a[16 * cn];
            if (MODE & 2) {
                rw0[u] = w0[16 * cn];
                rw1[u] = w1[16 * cn];
            }
        }
    }
#pragma unroll
    for (int u = 0; u < AHEAD; ++u) s += ra[u].x + rw0[u].y + rw1[u].z;
    if (s == 12345.f) out[blockIdx.x * 512 + tid] = s;  // keeps the loads
}

int main() {
    const int n_rows = 4400, n_w = 128;
    float* out;
    CK(hipMalloc(&out, 1 << 22));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int pitch : {512}) {
        float *A, *W;
        CK(hipMalloc(&A, size_t(n_rows) * pitch * 4));
        CK(hipMalloc(&W, size_t(n_w) * pitch * 4));
        CK(hipMemset(A, 0, size_t(n_rows) * pitch * 4));
        CK(hipMemset(W, 0, size_t(n_w) * pitch * 4));
        auto run = [&](const char* what, int grid, auto kern) -> int {
            float best = 1e9f, sum = 0.f;
            for (int it = 0; it < 60; ++it) {
                CK(hipEventRecord(e0, 0));
                kern<<<grid, 512>>>(reinterpret_cast<float4*>(A), reinterpret_cast<float4*>(W), pitch / 4, n_rows, out);
                CK(hipEventRecord(e1, 0));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                if (it >= 10) {
                    best = std::min(best, ms);
                    sum += ms;
                }
            }
            std::printf("%-40s grid %d: mean %.2f us  best %.2f us\n", what, grid, sum / 50 * 1e3, best * 1e3);
            return 0;
        };
        const int g276 = ((n_rows + 31) / 32) * 2, g16 = ((n_rows + 31) / 32 + 7) / 8 * 16;
        run("A + W, ahead 2", g276, probe_kernel<2, 3>);
        run("A only, ahead 2", g276, probe_kernel<2, 1>);
        run("W only, ahead 2", g276, probe_kernel<2, 2>);
        run("A + W, ahead 2, halves on one XCD", g16, probe_kernel<2, 7>);
        run("A only, ahead 2, halves on one XCD", g16, probe_kernel<2, 5>);
        run("A + W, ahead 4, halves on one XCD", g16, probe_kernel<4, 7>);
        run("A + W, ahead 2, 256 blocks", 256, probe_kernel<2, 3>);
        run("W only, ahead 2, 256 blocks", 256, probe_kernel<2, 2>);
        run("W only, ahead 4, 256 blocks", 256, probe_kernel<4, 2>);
        run("A + W, ahead 2, 128 blocks", 128, probe_kernel<2, 3>);
        CK(hipFree(A));
        CK(hipFree(W));
    }
    return 0;
}
