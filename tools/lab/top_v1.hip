// The top SageLayer and the loss head of a training step in one launch.
//
// In a 2-layer GraphSage the top layer's rows are the batch's roots, and
// everything from its aggregate to the classifier's gradient is row-local:
//   agg_r  = mean / max of h1 over r's sampled neighbours   (models.py:291-330)
//   E_r    = relu([h1[self_r] | agg_r] · W2ᵀ)               (models.py:216-219)
//   logits, log_softmax, NLL, dlogits = (softmax - onehot)/B  (models.py:8-27,
//            utils.py:159-164), dZ_r = (dlogits · Wc) ⊙ (E_r > 0)
//   dIn_r  = dZ_r · W2 = [dSelf_r | dA_r]                   (autograd of :219)
// One block of 4 waves owns 4 rows (the loss head's row block, so its
// classifier partial slab is the one cls_rows_kernel writes) and runs the
// four stages back to back with the rows in LDS: the three launches this
// replaces (layer-2 aggregate, layer-2 linear, loss head) and the dIn role of
// the layer backward each paid a kernel boundary and a global round trip of
// their inputs.
//
// Numerics are those of the launches it replaces, bit for bit: the aggregate
// adds neighbours in list order as agg_fwd_kernel does; every product chain
// is the fmaf chain the f32 MFMA kernels form (within each 16-wide k block
// the order 0,4,8,12, 1,5,9,13, ... of four v_mfma_f32_16x16x4_f32 over the
// four k-lane groups; blocks ascending); the head is cls_rows_kernel's code.
// The two GEMMs run on the matrix cores in the linear kernels' k order, from a
// copy of W2 in LDS that an LDS-DMA fills under the gather: E on 16x16x4 tiles
// (the 4 rows padded to 16; two accumulators alternate to hide the 40-cycle
// dependent latency), dIn on 4x4x1 multi-block MFMAs (the 4 rows are one
// block's rows, 16 blocks = 64 columns per instruction).  Measured (tools/lab/
// top_lab.hip, per launch): dIn 4.09 -> 2.49 us on 4x4x1; E on 4x4x1 took
// 5.0 us (4.15 with its operands one k block ahead) against 3.3 — one
// accumulator per output chain (the k order is fixed) leaves its dependent
// latency exposed at 32 columns per wave.  Measured alternatives: W2
// streamed from L2 through registers took the kernel to 31 us (latency-bound
// at ~25 GB/s per CU); VALU fmaf chains from LDS spent 3.4 + 3.7 us in the
// two GEMMs, bound by the LDS broadcast reads of the rows.
// round-4 top launch, kept for the lab A/B only (tools/lab/top_lab.hip)
#include "cls_dev.hpp"
#include "internal.hpp"
#include "linear_dev.hpp"

#ifndef GS_TOP_STAMP  // stage stamps for tools/lab/top_lab.hip; no-ops in the library
#define GS_TOP_STAMP(i)
#endif

namespace gs { namespace v1 {

constexpr int kTopRows = 4;
// Threads per block: 512 (8 waves) by default.  The extra waves issue the W2
// DMA (six waves instead of two) and take one 16-column E tile each (two
// waves per SIMD interleave the dependent MFMA chains instead of two
// accumulators per wave); the gather, head, slab and dIn stages keep waves
// 0-3.  Lab, per launch: 15.3 -> 14.0 us, outputs bitwise equal
// (profiles/r04e_top_lab_e8_ab.txt; 16 waves, fourteen of them DMA: 14.6 us,
// profiles/r04f_top_lab_e16_ab.txt).  -DGS_TOP_E8=0 (tools/lab/top_lab.hip)
// builds the 4-wave kernel.
#ifndef GS_TOP_E8
#define GS_TOP_E8 1
#endif
constexpr int kTopThreads = GS_TOP_E8 ? 512 : 256;
constexpr int kTopH = 128;
constexpr int kTopK = 2 * kTopH;
constexpr int kTopMaxC = 32;

struct TopArgs {
    int B, C;
    const float* Hprev;  // h1 [n1][H]
    const int* ptr;      // hop-1 neighbour lists (GS_PK_NBR_PTR / NBR), union-local, ascending
    const int* nbr;
    const int* self;     // GS_PK_SELF
    const float* W;      // W2 [H][2H]
    const float* Wc;     // [C][H]
    const float* bc;
    const int* labels;
    const int* roots;
    float* agg;          // [B][H]
    int* argmax;         // [B][H] (MAX)
    float* E;            // h2 [B][H]
    float* dZ;           // [B][H], masked by relu'(E)
    float* dIn;          // [B][2H]
    float* slab;         // classifier partials, one [C][H+1] + 1 slab per block
    const int* tids;     // optional: per root [self | list padded to tk with -1] (resolve_top_launch)
    int tk;
    KStamp stamp;        // a timed launch's span (g_kernel_stamp)
};

// k offset of step i (0..15) inside a 16-wide block: the MFMA kernels' order.
__device__ __forceinline__ constexpr int mfma_k(int i) { return 4 * (i & 3) + (i >> 2); }

template <int OP, int NT>
__global__ __launch_bounds__(NT) void sage_top_kernel(TopArgs a) {
    constexpr int H = kTopH, K = kTopK, D = kTopH;
    // dynamic LDS: W2 (whole, quad-swizzled rows), [self | agg], E, dZ, Wc, dlogits, loss
    extern __shared__ __attribute__((aligned(16))) float smem[];
    float* sW2 = smem;                                        // [H][K]
    float (*sX)[K] = reinterpret_cast<float (*)[K]>(sW2 + H * K);
    float (*sE)[H] = reinterpret_cast<float (*)[H]>(sX[kTopRows]);
    float (*sZ)[H] = reinterpret_cast<float (*)[H]>(sE[kTopRows]);
    float* sW = &sZ[kTopRows][0];                             // [C][D + 1]
    float* sdl = sW + a.C * (D + 1);                          // [rows][C]
    float* sloss = sdl + kTopRows * a.C;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int C = a.C;
    const int r0 = blockIdx.x * kTopRows;
    const int nr = min(kTopRows, a.B - r0);

    GS_TOP_STAMP(0);
    kstamp_begin(a.stamp);
    // ---- W2 -> LDS by DMA (no registers), issued before anything else so its
    // latency hides under the gather.  Row c is one wave instruction of 64
    // 16-byte quads; quad q of the row lands in slot q ^ (c & 15), which keeps
    // both later access patterns free of bank conflicts: a column read by
    // lanes = rows (ds_read_b128, 16 rows per quarter-wave on 16 distinct
    // slots) and a row read by lanes = k.
    // Waves 2 and 3 issue it: the gather below runs on waves 0 and 1, whose
    // dependent load rounds would otherwise queue behind the DMA (vmcnt
    // retires in order).
    if (w >= 2)
        for (int c = w - 2; c < H; c += NT / 64 - 2)
            __builtin_amdgcn_global_load_lds(a.W + static_cast<int64_t>(c) * K + 4 * (lane ^ (c & 15)), sW2 + c * K, 16,
                                             0, 0);

    // ---- stage 0: loss-head operands (independent of the rest, issued first)
    const int cl = lane & 15, dq = lane >> 4;
    const int wr_ = min(w, nr - 1);
    const int root = a.roots[r0 + wr_];
    const float b_lane = a.bc[min(cl, C - 1)];
    {
        const int nW4 = C * D / 4;
        for (int q = tid; q < nW4; q += NT) {
            const float4 v = reinterpret_cast<const float4*>(a.Wc)[q];
            const int t = 4 * q;
            float* d = sW + t + t / D;  // row pitch D + 1 (D % 4 == 0: a quad stays in one row)
            d[0] = v.x;
            d[1] = v.y;
            d[2] = v.z;
            d[3] = v.w;
        }
    }
    const int y_w = a.labels[root];

    // ---- stage 1: the aggregate (agg_fwd_kernel<OP, float, 4, 32, explicit>)
    // and the self row, one 32-lane group per row.  With the padded records
    // (a.tids) the root's self index and whole list arrive in one load round
    // (lane gl holds list entry gl, as the pack path's lanes do).
    {
        constexpr int G = 32, NR = 32;
        const int g = tid / G, gl = tid % G;
        if (g < nr) {
            const int r = r0 + g;
            const int f0 = gl * 4;
            int srow, beg, end, pre = -1;
            if (a.tids) {
                const int* rec = a.tids + static_cast<int64_t>(r) * (a.tk + 1);
                const int v = gl <= a.tk ? rec[gl] : -1;
                srow = __shfl(v, 0, G);
                pre = __shfl(v, min(gl + 1, G - 1), G);  // lane gl: list entry gl
                if (gl + 1 > a.tk) pre = -1;
                const unsigned long long have = __ballot(pre >= 0);
                const int sh = (tid & 63) & ~(G - 1);  // this group's lanes in the wave's ballot
                beg = 0;
                end = __popcll((have >> sh) & ((G == 64) ? ~0ull : ((1ull << G) - 1)));
            } else {
                srow = a.self[r];
                beg = a.ptr[r];
                end = a.ptr[r + 1];
            }
            const float4 xs = *reinterpret_cast<const float4*>(a.Hprev + static_cast<int64_t>(srow) * H + f0);
            float acc[4];
            int am[4];
#pragma unroll
            for (int v = 0; v < 4; ++v) {
                acc[v] = (OP == GS_AGG_MAX) ? -INFINITY : 0.f;
                am[v] = -1;
            }
            int cnt = 0;
            for (int base = beg; base < end; base += G) {
                const int m = min(G, end - base);
                const bool mine = gl < m;
                const int e = a.tids ? pre : a.nbr[mine ? base + gl : base];
                const int my = mine ? e : -1;
                for (int j = 0; j < m; j += NR) {
                    int rows[NR];
                    bool ok[NR];
#pragma unroll
                    for (int u = 0; u < NR; ++u) {
                        rows[u] = __shfl(my, j + u < m ? j + u : j, G);
                        ok[u] = (j + u < m) && rows[u] >= 0;
                    }
                    const int fallback = rows[0] >= 0 ? rows[0] : 0;
                    float x[NR][4];
#pragma unroll
                    for (int u = 0; u < NR; ++u)
                        RowIO<float, 4>::load(a.Hprev + static_cast<int64_t>(ok[u] ? rows[u] : fallback) * H + f0,
                                              x[u]);
#pragma unroll
                    for (int u = 0; u < NR; ++u) {
                        cnt += ok[u];
#pragma unroll
                        for (int v = 0; v < 4; ++v) {
                            if (OP == GS_AGG_MEAN) {
                                acc[v] += ok[u] ? x[u][v] : 0.f;
                            } else {
                                const bool take = ok[u] && x[u][v] > acc[v];  // strict: first index wins ties
                                acc[v] = take ? x[u][v] : acc[v];
                                am[v] = take ? rows[u] : am[v];
                            }
                        }
                    }
                }
            }
            if (OP == GS_AGG_MEAN) {
                const float inv = 1.0f / static_cast<float>(cnt);  // cnt == 0 -> NaN row, as 0/0 in :313
#pragma unroll
                for (int v = 0; v < 4; ++v) acc[v] *= inv;
            }
            *reinterpret_cast<float4*>(&sX[g][f0]) = xs;
            const float4 av = make_float4(acc[0], acc[1], acc[2], acc[3]);
            *reinterpret_cast<float4*>(&sX[g][H + f0]) = av;
            *reinterpret_cast<float4*>(a.agg + static_cast<int64_t>(r) * H + f0) = av;
            if (OP == GS_AGG_MAX)
                *reinterpret_cast<int4*>(a.argmax + static_cast<int64_t>(r) * H + f0) = make_int4(am[0], am[1], am[2],
                                                                                                   am[3]);
        }
    }
    GS_TOP_STAMP(1);
    __builtin_amdgcn_s_waitcnt(0);  // this wave's W2 DMA has landed (vmcnt); the barrier covers the others'
    __syncthreads();
    GS_TOP_STAMP(2);

    if constexpr (NT >= 512) {
    // ---- stage 2 (8 waves): E = relu([self | agg] · W2ᵀ), wave w owns the
    // 16 columns 16w .. 16w+15 (one tile, the same MFMA chain per tile)
    if (w < 8) {
        const int r = lane & 15, kq = lane >> 4;
        const bool rowok = r < nr;
        const uint4* xr = reinterpret_cast<const uint4*>(sX[min(r, nr - 1)]);
        const uint4* wq = reinterpret_cast<const uint4*>(sW2);
        const int c0 = 16 * w + r;
        f32x4 acc0 = f32x4{0.f, 0.f, 0.f, 0.f};
        auto ld = [&](int k0, uint4& av, uint4& b0) {
            const int q = (k0 >> 2) + kq;
            av = xr[q];
            b0 = wq[c0 * (K / 4) + (q ^ (c0 & 15))];
        };
        uint4 an, bn0;
        ld(0, an, bn0);
#pragma unroll 2
        for (int k0 = 0; k0 < K; k0 += 16) {
            uint4 av = an;
            const uint4 b0 = bn0;
            ld(min(k0 + 16, K - 16), an, bn0);
            if (!rowok) av = make_uint4(0, 0, 0, 0);
            const float a4[4] = {__uint_as_float(av.x), __uint_as_float(av.y), __uint_as_float(av.z),
                                 __uint_as_float(av.w)};
            const float w0[4] = {__uint_as_float(b0.x), __uint_as_float(b0.y), __uint_as_float(b0.z),
                                 __uint_as_float(b0.w)};
#pragma unroll
            for (int j = 0; j < 4; ++j) acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a4[j], w0[j], acc0, 0, 0, 0);
        }
        if (kq == 0) {
#pragma unroll
            for (int j = 0; j < kTopRows; ++j) {
                if (j >= nr) break;
                const float v0 = (!(acc0[j] > 0.f) && acc0[j] == acc0[j]) ? 0.f : acc0[j];  // relu (NaN kept)
                sE[j][c0] = v0;
                a.E[static_cast<int64_t>(r0 + j) * H + c0] = v0;
            }
        }
    }
    } else
    // ---- stage 2: E = relu([self | agg] · W2ᵀ) on the matrix cores, as the
    // linear kernel's tiles: wave w owns columns 32w .. 32w+31 (two 16x16
    // tiles); the 4 rows ride in a 16-row A tile (rows >= nr are zero).
    {
        const int r = lane & 15, kq = lane >> 4;
        const bool rowok = r < nr;
        const uint4* xr = reinterpret_cast<const uint4*>(sX[min(r, nr - 1)]);
        const uint4* wq = reinterpret_cast<const uint4*>(sW2);
        const int c0 = 32 * w + r, c1 = c0 + 16;
        f32x4 acc0 = f32x4{0.f, 0.f, 0.f, 0.f}, acc1 = acc0;
        // operands one k block ahead; the two tiles' MFMAs alternate so each
        // accumulator's dependent latency (40 cycles) hides under the other's issue
        auto ld = [&](int k0, uint4& av, uint4& b0, uint4& b1) {
            const int q = (k0 >> 2) + kq;  // this lane's 4-k slot
            av = xr[q];
            b0 = wq[c0 * (K / 4) + (q ^ (c0 & 15))];
            b1 = wq[c1 * (K / 4) + (q ^ (c1 & 15))];
        };
        uint4 an, bn0, bn1;
        ld(0, an, bn0, bn1);
#pragma unroll 2
        for (int k0 = 0; k0 < K; k0 += 16) {
            uint4 av = an;
            const uint4 b0 = bn0, b1 = bn1;
            ld(min(k0 + 16, K - 16), an, bn0, bn1);
            if (!rowok) av = make_uint4(0, 0, 0, 0);
            const float a4[4] = {__uint_as_float(av.x), __uint_as_float(av.y), __uint_as_float(av.z),
                                 __uint_as_float(av.w)};
            const float w0[4] = {__uint_as_float(b0.x), __uint_as_float(b0.y), __uint_as_float(b0.z),
                                 __uint_as_float(b0.w)};
            const float w1[4] = {__uint_as_float(b1.x), __uint_as_float(b1.y), __uint_as_float(b1.z),
                                 __uint_as_float(b1.w)};
#pragma unroll
            for (int j = 0; j < 4; ++j) {  // = mfma_slot's order on each tile
                acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a4[j], w0[j], acc0, 0, 0, 0);
                acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a4[j], w1[j], acc1, 0, 0, 0);
            }
        }
        if (kq == 0) {  // lanes 0..15 hold rows 0..3 of their column
#pragma unroll
            for (int j = 0; j < kTopRows; ++j) {
                if (j >= nr) break;
                const float v0 = (!(acc0[j] > 0.f) && acc0[j] == acc0[j]) ? 0.f : acc0[j];  // relu (NaN kept)
                const float v1 = (!(acc1[j] > 0.f) && acc1[j] == acc1[j]) ? 0.f : acc1[j];
                sE[j][c0] = v0;
                sE[j][c1] = v1;
                a.E[static_cast<int64_t>(r0 + j) * H + c0] = v0;
                a.E[static_cast<int64_t>(r0 + j) * H + c1] = v1;
            }
        }
    }
    __syncthreads();
    GS_TOP_STAMP(3);

    // ---- stage 3: the loss head, one wave per row (cls_rows_kernel's code)
    const float invB = 1.0f / static_cast<float>(a.B);
    const int wp = D + 1;
    if (w < nr) {
        const int ii = w;
        const float* e = sE[ii];
        const int y = y_w;
        static_assert(D % 4 == 0, "whole D quarters");
        constexpr int DQ = D / 4;  // whole quarters: a straight-line chain
        const int d_lo = dq * DQ;
        float mx = -INFINITY;
        for (int c0 = 0; c0 < C; c0 += 16) {
            const int c = c0 + cl;
            const float* wr = sW + static_cast<int64_t>(min(c, C - 1)) * wp;
            float pz = 0.f;
#pragma unroll
            for (int t = 0; t < DQ; ++t) pz = fmaf(e[d_lo + t], wr[d_lo + t], pz);
            pz += __shfl_xor(pz, 16, 64);
            pz += __shfl_xor(pz, 32, 64);
            const float z = pz + (c0 == 0 ? b_lane : a.bc[min(c, C - 1)]);
            if (dq == 0 && c < C) sdl[ii * C + c] = z;
            if (c < C) mx = fmaxf(mx, z);
        }
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 64));
        __builtin_amdgcn_wave_barrier();
        float se = 0.f;
        for (int c = lane; c < C; c += 64) se += expf(sdl[ii * C + c] - mx);
        const float lse = logf(wave_sum(se));
        for (int c = lane; c < C; c += 64) {
            const float lp = sdl[ii * C + c] - mx - lse;
            if (c == y) sloss[ii] = -lp;
            sdl[ii * C + c] = (expf(lp) - (c == y ? 1.f : 0.f)) * invB;
        }
        __builtin_amdgcn_wave_barrier();
        for (int d = lane; d < D; d += 64) {
            float s = 0.f;
            int c = 0;
            for (; c + 8 <= C; c += 8) {  // eight classes' operands read ahead of their chain
                float g[8], v[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    g[u] = sdl[ii * C + c + u];
                    v[u] = sW[static_cast<int64_t>(c + u) * wp + d];
                }
#pragma unroll
                for (int u = 0; u < 8; ++u) s = fmaf(g[u], v[u], s);
            }
            for (; c < C; ++c) s = fmaf(sdl[ii * C + c], sW[static_cast<int64_t>(c) * wp + d], s);
            if (!(e[d] > 0.f)) s = 0.f;
            sZ[ii][d] = s;
            a.dZ[static_cast<int64_t>(r0 + ii) * D + d] = s;
        }
    }
    __syncthreads();
    GS_TOP_STAMP(4);

    // ---- stage 4: this block's classifier partial slab (cls_rows_kernel's
    // sums): out[c][d] = Σ_rows dlogits[row][c] · [E[row] | 1][d].  Thread t
    // owns class t / 16 (its 4 dlogits in registers) and columns t % 16 + 16 j;
    // the E reads are LDS broadcasts across the class groups (per launch
    // 15.4-15.6 us against 16.3 for one thread per flat slab element, the
    // fallback above 16 classes; same sums).
#ifndef GS_TOP_SLAB_FLAT
    if (C * 16 <= NT) {
        const int per = C * (D + 1);
        float* out = a.slab + static_cast<int64_t>(blockIdx.x) * (per + 1);
        const int c = tid >> 4;
        if (c < C) {
            float dl[kTopRows];
#pragma unroll
            for (int ii = 0; ii < kTopRows; ++ii) dl[ii] = ii < nr ? sdl[ii * C + c] : 0.f;
            if (nr == kTopRows) {  // every block but a ragged last one: straight-line, same sums
                float s[D / 16];
#pragma unroll
                for (int j = 0; j < D / 16; ++j) {
                    const int d = (tid & 15) + 16 * j;
                    s[j] = 0.f;
#pragma unroll
                    for (int ii = 0; ii < kTopRows; ++ii) s[j] = fmaf(dl[ii], sE[ii][d], s[j]);
                }
#pragma unroll
                for (int j = 0; j < D / 16; ++j) out[c * (D + 1) + (tid & 15) + 16 * j] = s[j];
                if ((tid & 15) == 0) {
                    float sb = 0.f;
#pragma unroll
                    for (int ii = 0; ii < kTopRows; ++ii) sb = fmaf(dl[ii], 1.f, sb);
                    out[c * (D + 1) + D] = sb;
                }
            } else {
                for (int d = tid & 15; d <= D; d += 16) {
                    float s = 0.f;
#pragma unroll
                    for (int ii = 0; ii < kTopRows; ++ii)
                        if (ii < nr) s = fmaf(dl[ii], d < D ? sE[ii][d] : 1.f, s);
                    out[c * (D + 1) + d] = s;
                }
            }
        }
        if (tid >= NT - 64) {
            float s = 0.f;
            for (int ii = tid - (NT - 64); ii < nr; ii += 64) s += sloss[ii];
            s = wave_sum(s);
            if (tid == NT - 64) out[per] = s;
        }
    } else
#endif
    // ---- stage 4: this block's classifier partial slab (cls_rows_kernel's)
    {
        const int per = C * (D + 1);
        float* out = a.slab + static_cast<int64_t>(blockIdx.x) * (per + 1);
        int c = tid / (D + 1), d = tid - c * (D + 1);  // advanced by NT per step, no divides
        constexpr int dc = NT / (D + 1), dd = NT % (D + 1);
        for (int t = tid; t < per; t += NT) {
            float s = 0.f;
#pragma unroll
            for (int ii = 0; ii < kTopRows; ++ii)
                if (ii < nr) s = fmaf(sdl[ii * C + c], d < D ? sE[ii][d] : 1.f, s);
            out[t] = s;
            c += dc;
            d += dd;
            if (d > D) {
                d -= D + 1;
                ++c;
            }
        }
        if (tid < 64) {
            float s = 0.f;
            for (int ii = tid; ii < nr; ii += 64) s += sloss[ii];
            s = wave_sum(s);
            if (tid == 0) out[per] = s;
        }
    }

    GS_TOP_STAMP(5);
    // ---- stage 5: dIn = dZ · W2 on the matrix cores, 4x4x1 multi-block as
    // stage 2: wave w owns input columns 64w .. 64w+63, the 16 blocks x 4
    // columns of one instruction (lane l: column 64w + l), one h per
    // instruction in linear_dx_body's order (0,4,8,12, 1,5,9,13, ... per
    // 16-wide h block): the same fmaf chains, bit for bit.
    if (w < 4) {  // (waves >= 4 under GS_TOP_E8: no dIn role)
        const int arow = lane & 3, kc = 64 * w + lane;
        const bool rowok = arow < nr;
        const float4* zr = reinterpret_cast<const float4*>(sZ[min(arow, nr - 1)]);
        f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 2
        for (int g = 0; g < H / 16; ++g) {
            float zv[16], wv[16];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                float4 z = zr[4 * g + q];
                if (!rowok) z = make_float4(0.f, 0.f, 0.f, 0.f);
                zv[4 * q] = z.x;
                zv[4 * q + 1] = z.y;
                zv[4 * q + 2] = z.z;
                zv[4 * q + 3] = z.w;
            }
#pragma unroll
            for (int t = 0; t < 16; ++t) {
                const int h = 16 * g + t;
                wv[t] = sW2[h * K + 4 * ((kc >> 2) ^ (h & 15)) + (kc & 3)];
            }
#pragma unroll
            for (int j = 0; j < 4; ++j)
#pragma unroll
                for (int kq = 0; kq < 4; ++kq)
                    acc = __builtin_amdgcn_mfma_f32_4x4x1f32(zv[4 * kq + j], wv[4 * kq + j], acc, 0, 0, 0);
        }
#pragma unroll
        for (int j = 0; j < kTopRows; ++j)
            if (j < nr) a.dIn[static_cast<int64_t>(r0 + j) * K + kc] = acc[j];
    }
    GS_TOP_STAMP(6);
    kstamp_end(a.stamp);
}

static size_t top_smem_bytes(int64_t C) {
    return sizeof(float) * (static_cast<size_t>(kTopH) * kTopK + kTopRows * (kTopK + 2 * kTopH) + C * (kTopH + 1) +
                            kTopRows * C + kTopRows);
}

// The kernel keeps W2 in LDS (~146 KiB at 16 classes): raise the launch limit
// once; where the runtime refuses, the caller keeps the separate launches.
static bool top_lds_ready(int64_t C) {
    static int ok_bytes = -1;
    const size_t need = top_smem_bytes(C);
    if (ok_bytes < 0) {
        const size_t want = top_smem_bytes(kTopMaxC);
        auto raise = [&](const void* f) {
            return hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(want)) ==
                   hipSuccess;
        };
        const bool a = raise(reinterpret_cast<const void*>(sage_top_kernel<GS_AGG_MEAN, kTopThreads>)) &&
                       raise(reinterpret_cast<const void*>(sage_top_kernel<GS_AGG_MAX, kTopThreads>));
        (void)hipGetLastError();
        ok_bytes = a ? static_cast<int>(want) : 0;
    }
    return need <= static_cast<size_t>(ok_bytes);
}

bool top_supported(int64_t H, int64_t C, bool gcn) {
    return H == kTopH && C >= 1 && C <= kTopMaxC && !gcn && top_lds_ready(C);
}

int top_fwd_bwd(int agg, int64_t B, int64_t C, const float* Hprev, const int32_t* ptr, const int32_t* nbr,
                const int32_t* self, const float* W, const float* Wc, const float* bc, const int32_t* labels,
                const int32_t* roots, float* aggo, int32_t* argmax, float* E, float* dZ, float* dIn, float* slab,
                hipStream_t st, const int32_t* tids, int tk) {
    GS_REQUIRE(B >= 1 && B < (int64_t(1) << 30) && C >= 1 && C <= kTopMaxC, GS_EINVAL, "top: bad sizes");
    GS_REQUIRE(!tids || (tk >= 1 && tk <= 31), GS_EINVAL, "top: padded lists need 1 <= tk <= 31");
    GS_REQUIRE(aligned16(Hprev) && aligned16(W) && aligned16(Wc) && aligned16(aggo) && aligned16(E) && aligned16(dZ) &&
                   aligned16(dIn) && (agg == GS_AGG_MEAN || (argmax && aligned16(argmax))),
               GS_EINVAL, "top: unaligned operand");
    TopArgs a{static_cast<int>(B), static_cast<int>(C), Hprev, ptr, nbr, self, W, Wc, bc, labels, roots,
              aggo, argmax, E, dZ, dIn, slab, tids, tids ? tk : 0, take_kernel_stamp()};
    const dim3 grid(static_cast<unsigned>((B + kTopRows - 1) / kTopRows));
    const size_t smem = top_smem_bytes(C);
    if (agg == GS_AGG_MEAN) launch_k(sage_top_kernel<GS_AGG_MEAN, kTopThreads>, grid, dim3(kTopThreads), smem, st, a);
    else launch_k(sage_top_kernel<GS_AGG_MAX, kTopThreads>, grid, dim3(kTopThreads), smem, st, a);
    check_launch("sage_top");
    return static_cast<int>(grid.x);
}

} }  // namespace gs::v1
