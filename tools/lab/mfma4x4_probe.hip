// Lane layout of v_mfma_f32_4x4x1_16b_f32 (16 blocks of 4x4x1): which A lane and
// which B lane feed output (lane, reg).  Developer probe, not part of the library.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f32x4 __attribute__((ext_vector_type(4)));
__global__ void probe(float* out) {
    const int l = threadIdx.x;
    f32x4 z = {0.f, 0.f, 0.f, 0.f};
    f32x4 a = __builtin_amdgcn_mfma_f32_4x4x1f32(static_cast<float>(l + 1), 1.0f, z, 0, 0, 0);
    f32x4 b = __builtin_amdgcn_mfma_f32_4x4x1f32(1.0f, static_cast<float>(l + 1), z, 0, 0, 0);
    for (int r = 0; r < 4; ++r) {
        out[l * 8 + r] = a[r];
        out[l * 8 + 4 + r] = b[r];
    }
}
int main() {
    float* d;
    hipMalloc(&d, 64 * 8 * 4);
    probe<<<1, 64>>>(d);
    float h[512];
    hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    for (int l = 0; l < 64; ++l) {
        std::printf("lane %2d A-lane", l);
        for (int r = 0; r < 4; ++r) std::printf(" %3d", static_cast<int>(h[l * 8 + r]) - 1);
        std::printf("  B-lane");
        for (int r = 0; r < 4; ++r) std::printf(" %3d", static_cast<int>(h[l * 8 + 4 + r]) - 1);
        std::printf("\n");
    }
    return 0;
}
