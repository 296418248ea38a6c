// Device-side helpers shared by the gfx950 kernels: bf16 bit conversions,
// 16-byte vector loads/stores for fp32 and bf16 rows, MFMA fragment types and
// the launch-status check used by every C-ABI launcher.
#pragma once

#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>

#include "../host/common.hpp"

namespace gs {

using bf16_t = uint16_t;  // raw bf16 bits in HBM
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ float bf2f(bf16_t h) { return __uint_as_float(static_cast<uint32_t>(h) << 16); }

// Round-to-nearest-even f32 -> bf16, NaN kept a NaN.
__device__ __host__ __forceinline__ bf16_t f2bf(float f) {
    uint32_t u;
    __builtin_memcpy(&u, &f, 4);
    if ((u & 0x7f800000u) == 0x7f800000u && (u & 0x007fffffu)) return static_cast<bf16_t>((u >> 16) | 0x40);
    u += 0x7fffu + ((u >> 16) & 1u);
    return static_cast<bf16_t>(u >> 16);
}

// Load VEC consecutive elements of a row as floats.
template <typename T, int VEC>
struct RowIO;

template <>
struct RowIO<float, 4> {
    static __device__ __forceinline__ void load(const float* p, float (&v)[4]) {
        const float4 t = *reinterpret_cast<const float4*>(p);
        v[0] = t.x; v[1] = t.y; v[2] = t.z; v[3] = t.w;
    }
    static __device__ __forceinline__ void store(float* p, const float (&v)[4]) {
        *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
    }
};

template <>
struct RowIO<float, 1> {
    static __device__ __forceinline__ void load(const float* p, float (&v)[1]) { v[0] = *p; }
    static __device__ __forceinline__ void store(float* p, const float (&v)[1]) { *p = v[0]; }
};

template <>
struct RowIO<bf16_t, 8> {
    static __device__ __forceinline__ void load(const bf16_t* p, float (&v)[8]) {
        const uint4 t = *reinterpret_cast<const uint4*>(p);
        const uint32_t w[4] = {t.x, t.y, t.z, t.w};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            v[2 * i] = __uint_as_float(w[i] << 16);
            v[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
        }
    }
    static __device__ __forceinline__ void store(bf16_t* p, const float (&v)[8]) {
        uint32_t w[4];
#pragma unroll
        for (int i = 0; i < 4; ++i)
            w[i] = static_cast<uint32_t>(f2bf(v[2 * i])) | (static_cast<uint32_t>(f2bf(v[2 * i + 1])) << 16);
        *reinterpret_cast<uint4*>(p) = make_uint4(w[0], w[1], w[2], w[3]);
    }
};

template <>
struct RowIO<bf16_t, 1> {
    static __device__ __forceinline__ void load(const bf16_t* p, float (&v)[1]) { v[0] = bf2f(*p); }
    static __device__ __forceinline__ void store(bf16_t* p, const float (&v)[1]) { *p = f2bf(v[0]); }
};

// Lane exchanges inside a row of 16 lanes by DPP (a VALU operand modifier,
// no LDS round trip like __shfl's ds_bpermute): xor 1 and xor 2 as quad
// permutes, then the half-row and row mirrors (lane i <-> 7 - i, 15 - i).
// After dpp_sum8 every lane of an 8-lane group holds the group's sum, after
// dpp_sum16 / dpp_max16 every lane of a 16-lane row the row's; each lane
// adds the same two operands (a + b == b + a), so the lanes agree bitwise.
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xf, 0xf, false));
}
__device__ __forceinline__ float dpp_sum8(float v) {
    v += dpp_f<0xB1>(v);   // quad_perm [1,0,3,2]
    v += dpp_f<0x4E>(v);   // quad_perm [2,3,0,1]
    return v + dpp_f<0x141>(v);  // row_half_mirror
}
__device__ __forceinline__ float dpp_sum16(float v) { v = dpp_sum8(v); return v + dpp_f<0x140>(v); }  // row_mirror
__device__ __forceinline__ float dpp_max16(float v) {
    v = fmaxf(v, dpp_f<0xB1>(v));
    v = fmaxf(v, dpp_f<0x4E>(v));
    v = fmaxf(v, dpp_f<0x141>(v));
    return fmaxf(v, dpp_f<0x140>(v));
}

// Sum over the 64 lanes of a wave, every lane active; every lane gets the
// total.  DPP only (no ds_bpermute round trips): the 16-lane rows by
// dpp_sum16, then row 1 += row 0 and row 3 += row 2 (row_bcast15), rows 2-3
// += lane 31 (row_bcast31); lane 63 then holds (r2 + r3) + (r0 + r1).
__device__ __forceinline__ float wave_sum(float v) {
    v = dpp_sum16(v);
    v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x142, 0xa, 0xf, false));  // row_bcast15
    v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x143, 0xc, 0xf, false));  // row_bcast31
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63));
}

// Max over the 64 lanes of a wave (every lane active), the wave_sum scheme.
__device__ __forceinline__ float wave_max(float v) {
    v = dpp_max16(v);
    v = fmaxf(v, __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(-INFINITY), __float_as_int(v), 0x142, 0xa,
                                                            0xf, false)));
    v = fmaxf(v, __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(-INFINITY), __float_as_int(v), 0x143, 0xc,
                                                            0xf, false)));
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63));
}

// A workgroup barrier for a hand-off through LDS alone: the LDS ops done
// (lgkmcnt), not the global stores in flight, which __syncthreads() waits for
// (its fence drains vmcnt: a store round trip).  The memory clobber keeps the
// compiler from moving memory accesses across it.  Not for a kernel with an
// LDS-DMA in flight (the DMA is a vmcnt op writing LDS).
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// Sum of v over the (<= 1024-thread) block, written by thread 0 to *dst.
// Every thread of the block must call it.
__device__ __forceinline__ void block_sum_to(float v, float* dst) {
    __shared__ float red[16];
    v = wave_sum(v);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    lds_barrier();  // the caller's output stores need not land first
    if (threadIdx.x == 0) {
        float t = 0.f;
        for (int w = 0; w < static_cast<int>(blockDim.x + 63) / 64; ++w) t += red[w];
        *dst = t;
    }
}

inline bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

// Compute units of the current device (256 on MI355X), cached per thread.
inline int device_cus() {
    thread_local int dev = -1, cus = 256;
    int d = 0;
    if (hipGetDevice(&d) != hipSuccess) return cus;
    if (d != dev) {
        int c = 0;
        if (hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, d) == hipSuccess && c > 0) cus = c;
        dev = d;
    }
    return cus;
}

inline void check_launch(const char* what) {
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) fail(GS_EHIP, std::string(what) + ": " + hipGetErrorString(e));
}

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

// Kernel-bound timing: when armed (by the trainer's roofline timer), the next
// launch through launch_k binds the two events to its own dispatch packet
// (hipExtLaunchKernel), so their elapsed time is the kernel's begin-to-end
// span, the quantity rocprofv3's kernel trace reports, without the marker
// packets' dispatch overhead.  Cleared by that launch.
struct LaunchEvents {
    hipEvent_t start = nullptr, stop = nullptr;
};
inline thread_local LaunchEvents g_launch_events;
// The (mangled) symbol of the last kernel launch_k bound to timing events, so
// a timer site reports which kernel variant it actually timed.
inline thread_local const char* g_launch_name = nullptr;

// In-kernel span of a timed launch (the bench's roofline timers, step.hip):
// when set, the next launch of a kernel that supports it (the layer-1 wide
// forward, the top launch) stores the 100 MHz s_memrealtime clock at each
// workgroup's start and end (plain stores, one slot per workgroup: no
// atomics on a shared word, which serialise across the chip), and the host
// takes min(start) .. max(end): the first-wave-to-last-wave span rocprofv3's
// kernel trace reports.  The launcher takes it (and drops g_launch_events: an
// event pair's start marker is processed before the dispatch, so its span
// also covers the wait for the previous launch of a full queue).
constexpr int kStampBlocks = 1024;  // workgroups per timed launch with a slot (more: not timed)
struct KStamp {
    unsigned long long* start = nullptr;  // [kStampBlocks], zeroed
    unsigned long long* end = nullptr;
};
inline thread_local KStamp g_kernel_stamp;

// Host-visible step-completion flag (runtime/runner.hip): when set, the next
// SGD launch of this thread stores `value` into `ptr` (fine-grained pinned
// memory, system scope) from its first thread at kernel start -- by stream
// order every earlier launch of the step has completed then -- and clears it.
// This replaces an event record between steps (a marker packet that idled
// the queue ~4.4 us, rocprofv3 trace).
struct DoneFlag {
    int64_t* ptr = nullptr;
    int64_t value = 0;
};
inline thread_local DoneFlag g_done_flag;

// bf16 copy of a parameter range the next SGD launch of this thread writes
// beside the fp32 update (gs_trainer's W1 shadow for bf16 features: the next
// forward reads it instead of casting W1 again), then clears.
struct LowpShadow {
    uint16_t* p = nullptr;  // element i of [lo, hi) goes to p[i - lo]
    int64_t lo = 0, hi = 0;
};
inline thread_local LowpShadow g_lowp_shadow;

// A clip + SGD left pending by the previous step (gs_trainer in deferred-update
// mode, step.hip), applied by the next layer-1 forward launch of this thread
// (the fp32 wide kernel), then cleared.  The step's last slab sum wrote
// S = W1 - lr·G1, W1's update when the clip coefficient of its group is 1;
// every workgroup of the forward folds the norm partials itself and reads S
// as W1 when it is, else writes W1 - lr·(coef·G1) into S's buffer first.  The
// forward's grid also applies the pending update to the flat parameters
// [up_lo, up_hi) (W2, Wc, bc: read only after the forward).
struct FwdSpec {
    int on = 0;
    const float* S = nullptr;    // W1 - lr·G1 (clip coefficient 1)
    const float* P = nullptr;    // W1 before the update
    float* Wn = nullptr;         // S's buffer: the updated W1 when the coefficient is not 1
    const uint16_t* S_lp = nullptr;  // bf16 features: S in bf16 (the forward's W1), and its buffer
    uint16_t* Wn_lp = nullptr;       //   for the recomputed W1 (nullptr: fp32 features)
    const float* G1 = nullptr;   // W1's gradient
    const float* part0 = nullptr;  // norm partials, group 0 (the sage weights) and 1 (the classifier)
    const float* part1 = nullptr;
    int np0 = 0, np1 = 0;
    float lr = 0.f, max_norm = 0.f;
    float scale = 1.f;           // gradient scale (1 / world after an all-reduce): S used m = scale
    float* p = nullptr;          // flat params / grads
    float* g = nullptr;
    int64_t up_lo = 0, up_hi = 0, grp1_lo = 0;  // the other parameters; group 1 from grp1_lo
    KStamp stamp;                // a timed launch's span (g_kernel_stamp), independent of `on`
};
inline thread_local FwdSpec g_fwd_spec;

__device__ __forceinline__ int kstamp_block() { return blockIdx.x + blockIdx.y * gridDim.x; }
__device__ __forceinline__ void kstamp_begin(const KStamp& k) {
    if (k.start && threadIdx.x == 0 && kstamp_block() < kStampBlocks)
        k.start[kstamp_block()] = __builtin_amdgcn_s_memrealtime();
}
// At the workgroup's end; every thread of the workgroup calls it (a barrier).
__device__ __forceinline__ void kstamp_end(const KStamp& k) {
    if (!k.end) return;
    __syncthreads();
    if (threadIdx.x == 0 && kstamp_block() < kStampBlocks) k.end[kstamp_block()] = __builtin_amdgcn_s_memrealtime();
}

// A launcher whose kernel stores its span: take the armed stamp, if any (the
// next launch_k then records the kernel's name, as an event-bound one does).
inline thread_local bool g_name_next = false;
inline KStamp take_kernel_stamp() {
    const KStamp k = g_kernel_stamp;
    g_kernel_stamp = {};
    if (k.start) {
        g_launch_events = {};
        g_name_next = true;
    }
    return k;
}

template <typename... KArgs, typename... Args>
inline void launch_k(void (*kernel)(KArgs...), dim3 grid, dim3 block, uint32_t smem, hipStream_t st, Args... args) {
    LaunchEvents ev = g_launch_events;
    if (g_name_next) {
        g_name_next = false;
        g_launch_name = hipKernelNameRefByPtr(reinterpret_cast<const void*>(kernel), st);
    }
    if (ev.start) {
        g_launch_events = {};
        g_launch_name = hipKernelNameRefByPtr(reinterpret_cast<const void*>(kernel), st);
        hipExtLaunchKernelGGL(kernel, grid, block, smem, st, ev.start, ev.stop, 0, static_cast<KArgs>(args)...);
    } else {
        kernel<<<grid, block, smem, st>>>(static_cast<KArgs>(args)...);
    }
}

}  // namespace gs
