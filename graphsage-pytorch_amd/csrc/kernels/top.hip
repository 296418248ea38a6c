// The top SageLayer and the loss head of a training step in one launch.
//
// In a 2-layer GraphSage the top layer's rows are the batch's roots, and
// everything from its aggregate to the classifier's gradient is row-local:
//   agg_r  = mean / max of h1 over r's sampled neighbours   (models.py:291-330)
//   E_r    = relu([h1[self_r] | agg_r] · W2ᵀ)               (models.py:216-219)
//   logits, log_softmax, NLL, dlogits = (softmax - onehot)/B  (models.py:8-27,
//            utils.py:159-164), dZ_r = (dlogits · Wc) ⊙ (E_r > 0)
//   dIn_r  = dZ_r · W2 = [dSelf_r | dA_r]                   (autograd of :219)
// One block of 8 waves owns 4 rows (the loss head's row block, so its
// classifier partial slab is the one cls_rows_kernel writes) and runs the
// stages back to back with the rows in LDS: the three launches this replaces
// (layer-2 aggregate, layer-2 linear, loss head) and the dIn role of the layer
// backward each paid a kernel boundary and a global round trip of their inputs.
//
// The two GEMMs run on v_mfma_f32_4x4x1_16b_f32: one instruction is 16 blocks
// of a 4-row x 4-column outer product, i.e. the block's 4 rows x 64 columns
// for one k, with no padding of the 4 rows (a 16x16x4 tile would carry 12
// zero rows: 4x the matrix-pipe cycles, which bound the round-4 kernel's E
// stage at two waves per SIMD).  The K range is split over the waves (E: 4
// quarters of 64 k for each half of the 128 columns; dIn: 2 halves of 64 h
// for each of the 4 column groups of 64), each wave's chain runs on two
// accumulators (even / odd k), and the partial sums are added in a fixed
// order through LDS: deterministic, within fp32 rounding of the separate
// launches' single k-ordered chains (tests/test_gpu_model.py compares them at
// tolerance).  The loss head's logits are 8-way split dot products (16 d each,
// an xor-butterfly sum), its softmax one wave, dZ one output per thread.
// W2 arrives in LDS by DMA under the gather (quad-swizzled rows: conflict-free
// for both the row reads of E and the column reads of dIn).
#include "cls_dev.hpp"
#include "internal.hpp"
#include "linear_dev.hpp"

#ifndef GS_TOP_STAMP  // stage stamps for tools/lab/top_lab.hip; no-ops in the library
#define GS_TOP_STAMP(i)
#endif

namespace gs {

constexpr int kTopRows = 4;
constexpr int kTopThreads = 512;  // 8 waves
constexpr int kTopH = 128;
constexpr int kTopK = 2 * kTopH;
constexpr int kTopMaxC = 32;
constexpr int kTopPart = 4 * kTopRows * kTopH;  // floats of the partial-sum area (= 2 * kTopRows * kTopK)
static_assert(kTopPart == 2 * kTopRows * kTopK, "E and dIn partials share one area");

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
    float* agg;          // [B][2H]: each root's [self | agg] row (layer 2's dense GEMM input)
    int* argmax;         // [B][H] (MAX)
    float* E;            // h2 [B][H]
    float* dZ;           // [B][H], masked by relu'(E)
    float* dIn;          // [B][2H]
    float* slab;         // classifier partials, one [C][H+1] + 1 slab per block
    const int* tids;     // optional: per root [self | list padded to tk with -1] (resolve_top_launch)
    int tk;
    KStamp stamp;        // a timed launch's span (g_kernel_stamp)
};

// The stages hand each other LDS only: lds_barrier() (kcommon.hpp), not
// __syncthreads(), which would wait for the stage's global stores (E, dZ,
// the slabs, the [self | agg] rows).  The W2 DMA is waited for explicitly.

__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c, 0, 0, 0);
}
// The same MFMA with block ABID's A operand broadcast to all 16 blocks
// (CBSZ = 4): lanes 4·ABID .. 4·ABID + 3 supply the four rows' A values, the
// other lanes' A registers are not read.  So one 16-byte LDS read per lane,
// lane l = X[l & 3][k0 + 4 (l >> 2) .. + 3], holds the A operands of 64 k
// steps (step k0 + 4 b + r: component r, ABID b) instead of one broadcast
// read per 4 steps.
template <int ABID>
__device__ __forceinline__ f32x4 mfma4b(float a, float b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c, 4, ABID, 0);
}

template <int OP, bool SMALLC>
__global__ __launch_bounds__(kTopThreads) void sage_top_kernel(TopArgs a) {
    constexpr int H = kTopH, K = kTopK, D = kTopH, NT = kTopThreads;
    // Wc's LDS row pitch: D + 4 keeps its rows 16-byte aligned for the small-C
    // logits' quad reads (class c's quads then start at bank 4c: conflict-free);
    // D + 1 for the general path (its 8-part row reads)
    constexpr int WP = SMALLC ? D + 4 : D + 1;
    // dynamic LDS: W2 (whole, quad-swizzled rows), [self | agg], E, dZ, the
    // GEMMs' partial sums, Wc, logits / dlogits, loss
    extern __shared__ __attribute__((aligned(16))) float smem[];
    float* sW2 = smem;                                        // [H][K]
    float (*sX)[K] = reinterpret_cast<float (*)[K]>(sW2 + H * K);
    float (*sE)[H] = reinterpret_cast<float (*)[H]>(sX[kTopRows]);
    float (*sZ)[H] = reinterpret_cast<float (*)[H]>(sE[kTopRows]);
    // the GEMMs' partial sums: E [4 k quarters][rows][H], dIn [2 h halves][rows][K]
    float* sP = &sZ[kTopRows][0];
    float* sW = sP + kTopPart;                                // [C][WP]
    float* sdl = sW + a.C * WP;                               // [rows][C]
    float* sloss = sdl + kTopRows * a.C;
    float* sb = sloss + kTopRows;                             // [C] classifier bias
    int* sy = reinterpret_cast<int*>(sb + a.C);               // [rows] labels
    // C <= 16: dIn's four h-quarter partials [rows][K]: the E input rows (free
    // after stage 2), the partial area, and one more area behind the labels
    float* const dinq[4] = {&sX[0][0], sP, sP + kTopRows * K,
                            smem + ((reinterpret_cast<float*>(sy) + kTopRows - smem + 3) & ~3)};
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int C = a.C;
    const int r0 = blockIdx.x * kTopRows;
    const int nr = min(kTopRows, a.B - r0);

    GS_TOP_STAMP(0);
    kstamp_begin(a.stamp);
    // the fused layer-1 dW launch that follows waits on these (stream order
    // makes the stores visible to it)
    // ---- W2 -> LDS by DMA (no registers), issued first so its latency hides
    // under the gather.  Row c is one wave instruction of 64 16-byte quads;
    // quad q of the row lands in slot q ^ (c & 15).  Waves 2..7 issue it (the
    // gather's dependent load rounds run on waves 0 and 1; vmcnt retires in
    // order, so those would otherwise queue behind the DMA).
    // (Measured and not kept: each block starting the DMA at its own row, so
    // the blocks sharing an XCD's L2 request different lines at a time: the
    // launch 11.15 -> 11.5 us in tools/lab/top_lab.hip; a quarter of the rows
    // on the two gather waves, issued behind their row loads: 9.27 -> 9.6 us,
    // their adds then start after those issues.)
    if (w >= 2)
        for (int c = w - 2; c < H; c += NT / 64 - 2)
            __builtin_amdgcn_global_load_lds(a.W + static_cast<int64_t>(c) * K + 4 * (lane ^ (c & 15)), sW2 + c * K, 16,
                                             0, 0);

    // ---- loss-head operands (independent of the rest), on the DMA waves:
    // their loads queue behind the DMA (vmcnt retires in order), and these
    // waves wait for all of it before the first barrier anyway.  Waves 0 and 1
    // go straight to the gather (its record -> rows chain is the stage's
    // critical path; a labels[roots[]] chain or the Wc quads in front of it had
    // put two dependent global round trips ahead of the record load).
    if (w >= 2) {
        const int t2 = tid - 128;  // 0 .. 383
        if (t2 < kTopRows) sy[t2] = t2 < nr ? a.labels[a.roots[r0 + t2]] : 0;
        else if (t2 >= 64 && t2 < 64 + C) sb[t2 - 64] = a.bc[t2 - 64];
        const int nW4 = C * D / 4;
        for (int q = t2; q < nW4; q += NT - 128) {
            const float4 v = reinterpret_cast<const float4*>(a.Wc)[q];
            const int t = 4 * q;
            float* d = sW + t + (WP - D) * (t / D);  // row pitch WP (D % 4 == 0: a quad stays in one row)
            d[0] = v.x;
            d[1] = v.y;
            d[2] = v.z;
            d[3] = v.w;
        }
    }

    // ---- stage 1: the aggregate (agg_fwd_kernel<OP, float, 4, 32, explicit>:
    // neighbours added in list order) and the self row, one 32-lane group per
    // row.  With the padded records (a.tids) the root's self index and whole
    // list arrive in one load round (lane gl holds list entry gl).
    // this thread's [self | agg] quads and MAX argmax, stored to global after
    // the stage's barrier (a store in flight would hold the compiler's vmcnt(0)
    // that follows the W2 DMA's barrier)
    float4 st_xs{}, st_av{};
    int4 st_am{};
    const int st_g = tid / 32, st_f0 = (tid % 32) * 4;
    {
        constexpr int G = 32, NR = 32;
        const int g = tid / G, gl = tid % G;
        if (g < nr) {
            const int r = r0 + g;
            const int f0 = gl * 4;
            float acc[4];
            int am[4];
#pragma unroll
            for (int v = 0; v < 4; ++v) {
                acc[v] = (OP == GS_AGG_MAX) ? -INFINITY : 0.f;
                am[v] = -1;
            }
            int cnt = 0;
            // one neighbour row (ok: a real one), added in list order
            auto add_row = [&](int row, bool ok, const float (&x)[4]) {
                cnt += ok;
#pragma unroll
                for (int v = 0; v < 4; ++v) {
                    if (OP == GS_AGG_MEAN) {
                        acc[v] += ok ? x[v] : 0.f;
                    } else {
                        const bool take = ok && x[v] > acc[v];  // strict: first index wins ties
                        acc[v] = take ? x[v] : acc[v];
                        am[v] = take ? row : am[v];
                    }
                }
            };
            auto add_rows = [&](const int (&rows)[NR], const bool (&ok)[NR], const float (&x)[NR][4]) {
#pragma unroll
                for (int u = 0; u < NR; ++u) add_row(rows[u], ok[u], x[u]);
            };
            float4 xs;
            if (a.tids) {
                // one record load, then the self row and every neighbour row in
                // ONE load round, straight-line (a loop here had the compiler wait
                // for the self row before issuing the neighbour rows); the list
                // reaches the group's lanes through LDS (sP, unused until stage 2:
                // one 16-byte read per 4 entries instead of a ds_bpermute each)
                const int* rec = a.tids + static_cast<int64_t>(r) * (a.tk + 1);
                const int v = gl <= a.tk ? rec[gl] : -1;
                int* srec = reinterpret_cast<int*>(sP) + g * G;
                srec[gl == 0 ? G - 1 : gl - 1] = gl <= a.tk ? v : -1;  // list entry j at j, self at G - 1
                const unsigned long long have = __ballot(gl >= 1 && gl <= a.tk && v >= 0);
                const int sh = (tid & 63) & ~(G - 1);  // this group's lanes in the wave's ballot
                const int m = __popcll((have >> sh) & ((1ull << G) - 1));  // <= tk <= 31
                int rows[NR];
                bool ok[NR];
#pragma unroll
                for (int q = 0; q < NR / 4; ++q) {
                    const int4 r4 = reinterpret_cast<const int4*>(srec)[q];
                    rows[4 * q] = r4.x; rows[4 * q + 1] = r4.y; rows[4 * q + 2] = r4.z; rows[4 * q + 3] = r4.w;
                }
                const int srow = rows[NR - 1];
#pragma unroll
                for (int u = 0; u < NR; ++u) ok[u] = u < m && rows[u] >= 0;
                xs = *reinterpret_cast<const float4*>(a.Hprev + static_cast<int64_t>(srow) * H + f0);
                // rows in chunks of 8, a chunk only while the longer list of the
                // wave's two groups reaches it (wave-uniform: the ballot): the
                // lists average ~8 of the 25 slots, and rows past a list add
                // nothing (+0 / never the max), so the sums are the same
                const int mw = max(__popcll(have & 0xffffffffull), __popcll(have >> 32));
                float x[NR][4];
#pragma unroll
                for (int q = 0; q < NR / 8; ++q)
                    if (8 * q < mw) {
#pragma unroll
                        for (int u = 8 * q; u < 8 * q + 8; ++u)  // past the list: the self row's line again
                            RowIO<float, 4>::load(a.Hprev + static_cast<int64_t>(ok[u] ? rows[u] : srow) * H + f0,
                                                  x[u]);
                    }
                __builtin_amdgcn_sched_barrier(0);  // every row load issued before the first add waits
                // the same bound through an opaque copy: with one condition the
                // compiler merges each chunk's adds into its load block, and the
                // next chunk's loads then wait for this one's data
                int mwa = mw;
                asm volatile("" : "+s"(mwa));
#pragma unroll
                for (int q = 0; q < NR / 8; ++q)
                    if (8 * q < mwa) {
#pragma unroll
                        for (int u = 8 * q; u < 8 * q + 8; ++u) add_row(rows[u], ok[u], x[u]);
                    }
            } else {
                const int srow = a.self[r];
                const int beg = a.ptr[r], end = a.ptr[r + 1];
                xs = *reinterpret_cast<const float4*>(a.Hprev + static_cast<int64_t>(srow) * H + f0);
                for (int base = beg; base < end; base += G) {
                    const int m = min(G, end - base);
                    const bool mine = gl < m;
                    const int my = mine ? a.nbr[base + gl] : -1;
                    int rows[NR];
                    bool ok[NR];
#pragma unroll
                    for (int u = 0; u < NR; ++u) {
                        rows[u] = __shfl(my, u < m ? u : 0, G);
                        ok[u] = u < m && rows[u] >= 0;
                    }
                    const int fallback = rows[0] >= 0 ? rows[0] : 0;
                    float x[NR][4];
#pragma unroll
                    for (int u = 0; u < NR; ++u)
                        RowIO<float, 4>::load(a.Hprev + static_cast<int64_t>(ok[u] ? rows[u] : fallback) * H + f0,
                                              x[u]);
                    add_rows(rows, ok, x);
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
            st_xs = xs;
            st_av = av;
            if (OP == GS_AGG_MAX) st_am = make_int4(am[0], am[1], am[2], am[3]);
        } else if (g < kTopRows) {  // a ragged last block: zero rows (never stored)
            *reinterpret_cast<float4*>(&sX[g][gl * 4]) = make_float4(0.f, 0.f, 0.f, 0.f);
            *reinterpret_cast<float4*>(&sX[g][H + gl * 4]) = make_float4(0.f, 0.f, 0.f, 0.f);
        }
    }
    GS_TOP_STAMP(1);
    // the W2 DMA has landed: waves 2..7 issued it (vmcnt); waves 0 and 1 ran
    // the gather, whose row stores need not complete before the barrier
    if (w >= 2) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    lds_barrier();
    GS_TOP_STAMP(2);

    // ---- stage 2: E = relu([self | agg] · W2ᵀ), 4x4x1 multi-block MFMAs.
    // Wave w: columns 64 (w & 1) + lane, k quarter w >> 1 (64 k).  Lane l
    // supplies column l of B; the A operand (row l & 3) comes by ABID
    // broadcast from one 16-byte read per lane; acc[j] = row j, column l.
    {
        const int col = 64 * (w & 1) + lane, kb = 64 * (w >> 1);
        const float4 xa = *reinterpret_cast<const float4*>(sX[lane & 3] + kb + 4 * (lane >> 2));
        const float* wrow = sW2 + col * K;
        float bv[64];
#pragma unroll
        for (int m = 0; m < 16; ++m) {
            const int q = (kb >> 2) + m;
            const float4 w4 = *reinterpret_cast<const float4*>(wrow + 4 * (q ^ (col & 15)));
            bv[4 * m] = w4.x; bv[4 * m + 1] = w4.y; bv[4 * m + 2] = w4.z; bv[4 * m + 3] = w4.w;
        }
        // stage 1's global stores, behind the first LDS reads (the compiler
        // waits vmcnt(0) before those, for the DMA: stores issued before
        // would be waited for there)
        if (st_g < nr) {
            const int64_t r = r0 + st_g;
            *reinterpret_cast<float4*>(a.agg + r * K + st_f0) = st_xs;
            *reinterpret_cast<float4*>(a.agg + r * K + H + st_f0) = st_av;
            if (OP == GS_AGG_MAX) *reinterpret_cast<int4*>(a.argmax + r * H + st_f0) = st_am;
        }
        // k = 4 b + r: even k on c0, odd on c1, each in k order (the order of
        // the round-5 kernel's chains)
        f32x4 c0 = f32x4{0.f, 0.f, 0.f, 0.f}, c1 = c0;
#define GS_E_STEP(b)                                     \
        c0 = mfma4b<b>(xa.x, bv[4 * (b)], c0);           \
        c1 = mfma4b<b>(xa.y, bv[4 * (b) + 1], c1);       \
        c0 = mfma4b<b>(xa.z, bv[4 * (b) + 2], c0);       \
        c1 = mfma4b<b>(xa.w, bv[4 * (b) + 3], c1);
        GS_E_STEP(0) GS_E_STEP(1) GS_E_STEP(2) GS_E_STEP(3) GS_E_STEP(4) GS_E_STEP(5) GS_E_STEP(6) GS_E_STEP(7)
        GS_E_STEP(8) GS_E_STEP(9) GS_E_STEP(10) GS_E_STEP(11) GS_E_STEP(12) GS_E_STEP(13) GS_E_STEP(14) GS_E_STEP(15)
#undef GS_E_STEP
        float* pp = sP + (w >> 1) * (kTopRows * H);  // partial of quarter w >> 1: [row][col]
#pragma unroll
        for (int j = 0; j < kTopRows; ++j) pp[j * H + col] = c0[j] + c1[j];
    }
    lds_barrier();
    GS_TOP_STAMP(3);
    // the quarters added in order, relu (NaN kept), E to LDS and global
    {
        const int row = tid >> 7, col = tid & (H - 1);  // 512 threads = 4 rows x 128 columns
        float e = sP[row * H + col];
#pragma unroll
        for (int q = 1; q < 4; ++q) e += sP[q * (kTopRows * H) + row * H + col];
        e = (!(e > 0.f) && e == e) ? 0.f : e;
        sE[row][col] = e;
        if (row < nr) a.E[static_cast<int64_t>(r0 + row) * H + col] = e;
    }
    lds_barrier();
    GS_TOP_STAMP(4);

    // ---- stage 3: the loss head (models.py:8-27, utils.py:159-164).
    const float invB = 1.0f / static_cast<float>(a.B);
    const int wp = WP;
    if constexpr (SMALLC) {
        // C <= 16: logits, softmax, NLL and dlogits of row w on wave w, in one
        // stage: lane = (class lane >> 2, part lane & 3 of 32 d); the parts
        // added by DPP within the quad, the row's max and exp-sum by DPP over
        // the wave (each class counted once: the sum takes part 0 only).
        // (Measured and not kept: the whole dot product per lane in wave 0
        // after an 8-wave logits stage; 1.36 -> 1.54 us.)
        if (w < kTopRows) {
            const int row = w, c = lane >> 2, part = lane & 3;
            const bool cv = c < C;
            const float* e = sE[row] + 32 * part;
            const float* wr = sW + min(c, C - 1) * wp + 32 * part;
            float z = 0.f;
#pragma unroll
            for (int t = 0; t < 32; t += 4) {
                const float4 e4 = *reinterpret_cast<const float4*>(e + t);
                const float4 w4 = *reinterpret_cast<const float4*>(wr + t);
                z = fmaf(e4.x, w4.x, z);
                z = fmaf(e4.y, w4.y, z);
                z = fmaf(e4.z, w4.z, z);
                z = fmaf(e4.w, w4.w, z);
            }
            z += dpp_f<0xB1>(z);  // quad_perm [1,0,3,2]
            z += dpp_f<0x4E>(z);  // quad_perm [2,3,0,1]: (p0 + p1) + (p2 + p3) in every lane of the quad
            const float zl = cv ? z + sb[min(c, C - 1)] : -INFINITY;
            const float mx = wave_max(zl);
            const float lse = logf(wave_sum(cv && part == 0 ? expf(zl - mx) : 0.f));
            if (part == 0 && cv) {
                if (row < nr) {
                    const int y = sy[row];
                    const float lp = zl - mx - lse;
                    if (c == y) sloss[row] = -lp;
                    sdl[row * C + c] = (expf(lp) - (c == y ? 1.f : 0.f)) * invB;
                } else {
                    sdl[row * C + c] = 0.f;  // ragged block: no gradient from the missing rows
                }
            }
        }
        GS_TOP_STAMP(5);
    } else {
        // logits: thread t owns (row, class) (t >> 3) and the 16 d of part t & 7;
        // the eight parts are added by an xor butterfly.
        for (int base = 0; base < kTopRows * C; base += NT / 8) {
            const int rc = base + (tid >> 3), part = tid & 7;
            const int row = min(rc / C, kTopRows - 1), c = rc % C;
            const float* e = sE[row] + 16 * part;
            const float* wr = sW + static_cast<int64_t>(c) * wp + 16 * part;
            float z = 0.f;
#pragma unroll
            for (int t = 0; t < 16; ++t) z = fmaf(e[t], wr[t], z);
            z += __shfl_xor(z, 1, 64);
            z += __shfl_xor(z, 2, 64);
            z += __shfl_xor(z, 4, 64);
            if (part == 0 && rc < kTopRows * C) sdl[row * C + c] = z + sb[c];
        }
        lds_barrier();
        GS_TOP_STAMP(5);
        // softmax / NLL / dlogits: wave w < rows, lane = class (C <= 32 <= 64)
        if (w < nr) {
            const int ii = w;
            const int y = sy[ii];
            const float z = lane < C ? sdl[ii * C + lane] : -INFINITY;
            float mx = z;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 64));
            const float lse = logf(wave_sum(lane < C ? expf(z - mx) : 0.f));
            if (lane < C) {
                const float lp = z - mx - lse;
                if (lane == y) sloss[ii] = -lp;
                sdl[ii * C + lane] = (expf(lp) - (lane == y ? 1.f : 0.f)) * invB;
            }
        } else if (w < kTopRows && lane < C) {
            sdl[w * C + lane] = 0.f;  // ragged block: no gradient from the missing rows
        }
    }
    lds_barrier();
    GS_TOP_STAMP(6);
    // dZ = (dlogits · Wc) ⊙ (E > 0) for one (row, d), classes in order
    auto dz_one = [&](int row, int d) {
        float s = 0.f;
        if constexpr (SMALLC) {
            // every operand read unconditionally (clamped class), then the
            // chain with selects: guarded reads became one branch and one LDS
            // wait per class
            float g[16], v[16];
#pragma unroll
            for (int u = 0; u < 16; ++u) {
                const int uc = min(u, C - 1);
                g[u] = sdl[row * C + uc];
                v[u] = sW[uc * wp + d];
            }
#pragma unroll
            for (int u = 0; u < 16; ++u) s = u < C ? fmaf(g[u], v[u], s) : s;
        } else {
            int c = 0;
            for (; c + 8 <= C; c += 8) {
                float g[8], v[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    g[u] = sdl[row * C + c + u];
                    v[u] = sW[static_cast<int64_t>(c + u) * wp + d];
                }
#pragma unroll
                for (int u = 0; u < 8; ++u) s = fmaf(g[u], v[u], s);
            }
            for (; c < C; ++c) s = fmaf(sdl[row * C + c], sW[static_cast<int64_t>(c) * wp + d], s);
        }
        if (!(sE[row][d] > 0.f)) s = 0.f;
        sZ[row][d] = s;
        if (row < nr) a.dZ[static_cast<int64_t>(r0 + row) * D + d] = s;
    };
    // ---- this block's classifier partial slab (cls_rows_kernel's sums):
    // out[c][d] = Σ_rows dlogits[row][c] · [E[row] | 1][d], rows in order.
    // Thread t owns class t / 16 (its 4 dlogits in registers) and columns
    // t % 16 + 16 j; the E reads are LDS broadcasts across the class groups.
    // `t0`: the first thread of the role (C <= 16: waves 4..7, beside dIn).
    auto slab_role = [&](int t0) {
        const int tt = tid - t0;
        const int per = C * (D + 1);
        float* out = a.slab + static_cast<int64_t>(blockIdx.x) * (per + 1);
        if (C * 16 <= NT - t0) {
            const int c = tt >> 4;
            if (c < C) {
                // all operands read first, unconditionally (rows past nr are
                // zeros in sE), then the chains with selects: guarded reads had
                // the compiler branch and wait on LDS once per (row, column)
                float dl[kTopRows], ev[kTopRows][D / 16];
#pragma unroll
                for (int ii = 0; ii < kTopRows; ++ii) {
                    dl[ii] = sdl[ii * C + c];
#pragma unroll
                    for (int j = 0; j < D / 16; ++j) ev[ii][j] = sE[ii][(tt & 15) + 16 * j];
                }
                float sv[D / 16];
#pragma unroll
                for (int j = 0; j < D / 16; ++j) {
                    sv[j] = 0.f;
#pragma unroll
                    for (int ii = 0; ii < kTopRows; ++ii) sv[j] = ii < nr ? fmaf(dl[ii], ev[ii][j], sv[j]) : sv[j];
                }
#pragma unroll
                for (int j = 0; j < D / 16; ++j) out[c * (D + 1) + (tt & 15) + 16 * j] = sv[j];
                if ((tt & 15) == 0) {
                    float sbias = 0.f;
#pragma unroll
                    for (int ii = 0; ii < kTopRows; ++ii) sbias = ii < nr ? fmaf(dl[ii], 1.f, sbias) : sbias;
                    out[c * (D + 1) + D] = sbias;
                }
            }
        } else {
            for (int t = tt; t < per; t += NT - t0) {
                const int c = t / (D + 1), d = t - c * (D + 1);
                float sv = 0.f;
#pragma unroll
                for (int ii = 0; ii < kTopRows; ++ii)
                    if (ii < nr) sv = fmaf(sdl[ii * C + c], d < D ? sE[ii][d] : 1.f, sv);
                out[t] = sv;
            }
        }
        if (tid == NT - 64) {  // the block's loss, rows in order
            float sl = 0.f;
            for (int ii = 0; ii < nr; ++ii) sl += sloss[ii];
            out[per] = sl;
        }
    };
    if constexpr (SMALLC) {
        // dZ on waves 0..3 (two outputs per thread), the classifier slab beside
        // it on waves 4..7: the stage takes the longer of the two, not the sum
        if (w < 4) {
            dz_one(tid >> 6, tid & 63);
            dz_one(tid >> 6, (tid & 63) + 64);
        } else {
            slab_role(256);
        }
    } else {
        dz_one(tid >> 7, tid & (D - 1));
        slab_role(0);
    }
    lds_barrier();
    GS_TOP_STAMP(7);

    // ---- stage 4: dIn = dZ · W2 (4x4x1 multi-block)
    if constexpr (SMALLC) {
        // Wave w: input columns 128 (w & 1) + 2 lane and + 1 (one 8-byte read
        // of the swizzled W2 row per h: both columns sit in one quad), h quarter
        // w >> 1 (32 h); one MFMA chain per column; the dZ operand by ABID
        // broadcast (blocks 0..7 of the read hold the quarter's 32 h)
        const int k0 = 128 * (w & 1) + 2 * lane, hb = 32 * (w >> 1);
        const float4 za = *reinterpret_cast<const float4*>(sZ[lane & 3] + min(hb + 4 * (lane >> 2), H - 4));
        float2 wv[32];
#pragma unroll
        for (int t = 0; t < 32; ++t) {
            const int h = hb + t;
            wv[t] = *reinterpret_cast<const float2*>(sW2 + h * K + 4 * ((k0 >> 2) ^ (h & 15)) + (k0 & 3));
        }
        f32x4 c0 = f32x4{0.f, 0.f, 0.f, 0.f}, c1 = c0;
#define GS_DIN_STEP(b)                                   \
        c0 = mfma4b<b>(za.x, wv[4 * (b)].x, c0);         \
        c1 = mfma4b<b>(za.x, wv[4 * (b)].y, c1);         \
        c0 = mfma4b<b>(za.y, wv[4 * (b) + 1].x, c0);     \
        c1 = mfma4b<b>(za.y, wv[4 * (b) + 1].y, c1);     \
        c0 = mfma4b<b>(za.z, wv[4 * (b) + 2].x, c0);     \
        c1 = mfma4b<b>(za.z, wv[4 * (b) + 2].y, c1);     \
        c0 = mfma4b<b>(za.w, wv[4 * (b) + 3].x, c0);     \
        c1 = mfma4b<b>(za.w, wv[4 * (b) + 3].y, c1);
        GS_DIN_STEP(0) GS_DIN_STEP(1) GS_DIN_STEP(2) GS_DIN_STEP(3)
        GS_DIN_STEP(4) GS_DIN_STEP(5) GS_DIN_STEP(6) GS_DIN_STEP(7)
#undef GS_DIN_STEP
        float* pp = dinq[w >> 1];
#pragma unroll
        for (int j = 0; j < kTopRows; ++j)
            *reinterpret_cast<float2*>(pp + j * K + k0) = make_float2(c0[j], c1[j]);
    } else {
        // Wave w: input columns 64 (w & 3) + lane, h half w >> 2 (64 h); W2[h][kc]
        // read down a column of the swizzled copy.
        const int kc = 64 * (w & 3) + lane, hb = 64 * (w >> 2);
        const float* zr = sZ[lane & 3] + hb;
        float zv[64], wv[64];
#pragma unroll
        for (int m = 0; m < 16; ++m) {
            const float4 z4 = *reinterpret_cast<const float4*>(zr + 4 * m);
            zv[4 * m] = z4.x; zv[4 * m + 1] = z4.y; zv[4 * m + 2] = z4.z; zv[4 * m + 3] = z4.w;
        }
#pragma unroll
        for (int t = 0; t < 64; ++t) {
            const int h = hb + t;
            wv[t] = sW2[h * K + 4 * ((kc >> 2) ^ (h & 15)) + (kc & 3)];
        }
        f32x4 c0 = f32x4{0.f, 0.f, 0.f, 0.f}, c1 = c0;
#pragma unroll
        for (int t = 0; t < 64; t += 2) {
            c0 = mfma4(zv[t], wv[t], c0);
            c1 = mfma4(zv[t + 1], wv[t + 1], c1);
        }
        float* pp = sP + (w >> 2) * (kTopRows * K);
#pragma unroll
        for (int j = 0; j < kTopRows; ++j) pp[j * K + kc] = c0[j] + c1[j];
    }
    lds_barrier();
    GS_TOP_STAMP(8);
    // the h parts added in order, dIn to global: thread t = (row, 2 columns)
#pragma unroll
    for (int u = 0; u < 2; ++u) {
        const int o = tid + u * NT, row = o >> 8, kc = o & (K - 1);
        float v;
        if constexpr (SMALLC)
            v = ((dinq[0][row * K + kc] + dinq[1][row * K + kc]) + dinq[2][row * K + kc]) + dinq[3][row * K + kc];
        else
            v = sP[row * K + kc] + sP[kTopRows * K + row * K + kc];
        if (row < nr) a.dIn[static_cast<int64_t>(r0 + row) * K + kc] = v;
    }
    GS_TOP_STAMP(9);
    kstamp_end(a.stamp);
}

// ---------------------------------------------------------------- pair form
// The same step on 2 blocks per 4 roots (lab form, C <= 16): block half hh
// holds W2's rows 64·hh .. 64·hh + 63 (64 KB instead of 128), computes E's
// columns of those rows, the logits' partial sums over them, dZ of those
// columns and dIn's partial sum over those h; the two blocks of a pair (same
// XCD: blocks b and b ^ 8) exchange the 4 x 16 partial logits as tagged
// 8-byte granules (one write-through store each, relaxed agent-scope polls),
// add them in a fixed order (half 0's + half 1's), and write dIn's two
// partials to dIn (half 0) and dIn2 (half 1) for the consumer to add.
struct TopPairArgs {
    TopArgs a;
    float* dIn2;                  // [B][2H]: half 1's dIn partial
    unsigned long long* xch;      // granules [quads][2][64], zeroed once
    unsigned epoch;               // this launch's tag (never 0, never repeated)
    unsigned* fail;               // set when a poll gives up (the outputs are then wrong)
};
constexpr int kPairW = kTopH / 2;  // W2 rows / E columns per block

template <int OP>
__global__ __launch_bounds__(kTopThreads) void sage_top_pair_kernel(TopPairArgs pa) {
    const TopArgs& a = pa.a;
    constexpr int H = kTopH, K = kTopK, NT = kTopThreads, HW = kPairW, WP = kPairW + 4;
    extern __shared__ __attribute__((aligned(16))) float smem[];
    float* sW2 = smem;                                               // [HW][K]
    float (*sX)[K] = reinterpret_cast<float (*)[K]>(sW2 + HW * K);  // [rows][K]
    float (*sE)[HW] = reinterpret_cast<float (*)[HW]>(sX[kTopRows]);
    float (*sZ)[HW] = reinterpret_cast<float (*)[HW]>(sE[kTopRows]);
    float* sP = &sZ[kTopRows][0];                                    // E: [8][rows][HW]; dIn: [4][rows][K]
    float* sW = sP + 4 * kTopRows * K;                               // [C][WP] (this half's Wc columns)
    float* sdl = sW + 16 * WP;                                       // [rows][C]
    float* sloss = sdl + kTopRows * 16;
    float* sb = sloss + kTopRows;
    int* sy = reinterpret_cast<int*>(sb + 16);
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int C = a.C;
    const int bq = blockIdx.x, hh = (bq >> 3) & 1, q = (bq >> 4) * 8 + (bq & 7);
    const int r0 = q * kTopRows;
    if (r0 >= a.B) return;  // both halves of a quad past the batch leave together
    const int nr = min(kTopRows, a.B - r0);
    GS_TOP_STAMP(0);
    kstamp_begin(a.stamp);
    if (w >= 2)
        for (int c = w - 2; c < HW; c += NT / 64 - 2)
            __builtin_amdgcn_global_load_lds(a.W + static_cast<int64_t>(HW * hh + c) * K + 4 * (lane ^ (c & 15)),
                                             sW2 + c * K, 16, 0, 0);
    if (w >= 2) {
        const int t2 = tid - 128;
        if (t2 < kTopRows) sy[t2] = t2 < nr ? a.labels[a.roots[r0 + t2]] : 0;
        else if (t2 >= 64 && t2 < 64 + C) sb[t2 - 64] = a.bc[t2 - 64];
        for (int i = t2; i < C * (HW / 4); i += NT - 128) {  // this half's Wc quads
            const int c = i / (HW / 4), j = 4 * (i % (HW / 4));
            const float4 v = *reinterpret_cast<const float4*>(a.Wc + static_cast<int64_t>(c) * H + HW * hh + j);
            *reinterpret_cast<float4*>(sW + c * WP + j) = v;
        }
    }
    // ---- stage 1: sage_top_kernel's gather (padded records: one round)
    float4 st_xs{}, st_av{};
    int4 st_am{};
    const int st_g = tid / 32, st_f0 = (tid % 32) * 4;
    {
        constexpr int G = 32, NR = 32;
        const int g = tid / G, gl = tid % G;
        if (g < nr) {
            const int r = r0 + g;
            const int f0 = gl * 4;
            float acc[4];
            int am[4];
#pragma unroll
            for (int v = 0; v < 4; ++v) {
                acc[v] = (OP == GS_AGG_MAX) ? -INFINITY : 0.f;
                am[v] = -1;
            }
            int cnt = 0;
            auto add_row = [&](int row, bool ok, const float (&x)[4]) {
                cnt += ok;
#pragma unroll
                for (int v = 0; v < 4; ++v) {
                    if (OP == GS_AGG_MEAN) {
                        acc[v] += ok ? x[v] : 0.f;
                    } else {
                        const bool take = ok && x[v] > acc[v];
                        acc[v] = take ? x[v] : acc[v];
                        am[v] = take ? row : am[v];
                    }
                }
            };
            float4 xs;
            if (a.tids) {
                const int* rec = a.tids + static_cast<int64_t>(r) * (a.tk + 1);
                const int v = gl <= a.tk ? rec[gl] : -1;
                int* srec = reinterpret_cast<int*>(sP) + g * G;
                srec[gl == 0 ? G - 1 : gl - 1] = gl <= a.tk ? v : -1;
                const unsigned long long have = __ballot(gl >= 1 && gl <= a.tk && v >= 0);
                const int sh = (tid & 63) & ~(G - 1);
                const int m = __popcll((have >> sh) & ((1ull << G) - 1));
                int rows[NR];
                bool ok[NR];
#pragma unroll
                for (int qq = 0; qq < NR / 4; ++qq) {
                    const int4 r4 = reinterpret_cast<const int4*>(srec)[qq];
                    rows[4 * qq] = r4.x; rows[4 * qq + 1] = r4.y; rows[4 * qq + 2] = r4.z; rows[4 * qq + 3] = r4.w;
                }
                const int srow = rows[NR - 1];
#pragma unroll
                for (int u = 0; u < NR; ++u) ok[u] = u < m && rows[u] >= 0;
                xs = *reinterpret_cast<const float4*>(a.Hprev + static_cast<int64_t>(srow) * H + f0);
                const int mw = max(__popcll(have & 0xffffffffull), __popcll(have >> 32));
                float x[NR][4];
#pragma unroll
                for (int qq = 0; qq < NR / 8; ++qq)
                    if (8 * qq < mw) {
#pragma unroll
                        for (int u = 8 * qq; u < 8 * qq + 8; ++u)
                            RowIO<float, 4>::load(a.Hprev + static_cast<int64_t>(ok[u] ? rows[u] : srow) * H + f0, x[u]);
                    }
                __builtin_amdgcn_sched_barrier(0);
                int mwa = mw;
                asm volatile("" : "+s"(mwa));
#pragma unroll
                for (int qq = 0; qq < NR / 8; ++qq)
                    if (8 * qq < mwa) {
#pragma unroll
                        for (int u = 8 * qq; u < 8 * qq + 8; ++u) add_row(rows[u], ok[u], x[u]);
                    }
            } else {
                const int srow = a.self[r];
                const int beg = a.ptr[r], end = a.ptr[r + 1];
                xs = *reinterpret_cast<const float4*>(a.Hprev + static_cast<int64_t>(srow) * H + f0);
                for (int base = beg; base < end; base += G) {
                    const int mm = min(G, end - base);
                    const int my = gl < mm ? a.nbr[base + gl] : -1;
                    int rows[NR];
                    bool ok[NR];
#pragma unroll
                    for (int u = 0; u < NR; ++u) {
                        rows[u] = __shfl(my, u < mm ? u : 0, G);
                        ok[u] = u < mm && rows[u] >= 0;
                    }
                    const int fallback = rows[0] >= 0 ? rows[0] : 0;
                    float x[NR][4];
#pragma unroll
                    for (int u = 0; u < NR; ++u)
                        RowIO<float, 4>::load(a.Hprev + static_cast<int64_t>(ok[u] ? rows[u] : fallback) * H + f0, x[u]);
#pragma unroll
                    for (int u = 0; u < NR; ++u) add_row(rows[u], ok[u], x[u]);
                }
            }
            if (OP == GS_AGG_MEAN) {
                const float inv = 1.0f / static_cast<float>(cnt);
#pragma unroll
                for (int v = 0; v < 4; ++v) acc[v] *= inv;
            }
            *reinterpret_cast<float4*>(&sX[g][f0]) = xs;
            const float4 av = make_float4(acc[0], acc[1], acc[2], acc[3]);
            *reinterpret_cast<float4*>(&sX[g][H + f0]) = av;
            st_xs = xs;
            st_av = av;
            if (OP == GS_AGG_MAX) st_am = make_int4(am[0], am[1], am[2], am[3]);
        } else if (g < kTopRows) {
            *reinterpret_cast<float4*>(&sX[g][gl * 4]) = make_float4(0.f, 0.f, 0.f, 0.f);
            *reinterpret_cast<float4*>(&sX[g][H + gl * 4]) = make_float4(0.f, 0.f, 0.f, 0.f);
        }
    }
    GS_TOP_STAMP(1);
    if (w >= 2) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    lds_barrier();
    GS_TOP_STAMP(2);
    // ---- stage 2: E's 64 columns of this half; wave w: k eighth w (32 k)
    {
        const int kb = 32 * w;
        const float4 xa = *reinterpret_cast<const float4*>(sX[lane & 3] + min(kb + 4 * (lane >> 2), K - 4));
        const float* wrow = sW2 + lane * K;
        float bv[32];
#pragma unroll
        for (int m = 0; m < 8; ++m) {
            const int qd = (kb >> 2) + m;
            const float4 w4 = *reinterpret_cast<const float4*>(wrow + 4 * (qd ^ (lane & 15)));
            bv[4 * m] = w4.x; bv[4 * m + 1] = w4.y; bv[4 * m + 2] = w4.z; bv[4 * m + 3] = w4.w;
        }
        if (hh == 0 && st_g < nr) {  // stage 1's global stores (half 0 owns them)
            const int64_t r = r0 + st_g;
            *reinterpret_cast<float4*>(a.agg + r * K + st_f0) = st_xs;
            *reinterpret_cast<float4*>(a.agg + r * K + H + st_f0) = st_av;
            if (OP == GS_AGG_MAX) *reinterpret_cast<int4*>(a.argmax + r * H + st_f0) = st_am;
        }
        f32x4 c0 = f32x4{0.f, 0.f, 0.f, 0.f}, c1 = c0;
#define GS_PE_STEP(b)                                    \
        c0 = mfma4b<b>(xa.x, bv[4 * (b)], c0);           \
        c1 = mfma4b<b>(xa.y, bv[4 * (b) + 1], c1);       \
        c0 = mfma4b<b>(xa.z, bv[4 * (b) + 2], c0);       \
        c1 = mfma4b<b>(xa.w, bv[4 * (b) + 3], c1);
        GS_PE_STEP(0) GS_PE_STEP(1) GS_PE_STEP(2) GS_PE_STEP(3) GS_PE_STEP(4) GS_PE_STEP(5) GS_PE_STEP(6) GS_PE_STEP(7)
#undef GS_PE_STEP
        float* pp = sP + w * (kTopRows * HW);
#pragma unroll
        for (int j = 0; j < kTopRows; ++j) pp[j * HW + lane] = c0[j] + c1[j];
    }
    lds_barrier();
    GS_TOP_STAMP(3);
    if (tid < kTopRows * HW) {
        const int row = tid >> 6, col = tid & (HW - 1);
        float e = sP[row * HW + col];
#pragma unroll
        for (int qq = 1; qq < 8; ++qq) e += sP[qq * (kTopRows * HW) + row * HW + col];
        e = (!(e > 0.f) && e == e) ? 0.f : e;
        sE[row][col] = e;
        if (row < nr) a.E[static_cast<int64_t>(r0 + row) * H + HW * hh + col] = e;
    }
    lds_barrier();
    GS_TOP_STAMP(4);
    // ---- stage 3: partial logits over this half's 64 d, exchanged with the
    // pair's other block, then the loss head on the sums (half 0's + half 1's)
    const float invB = 1.0f / static_cast<float>(a.B);
    if (w < kTopRows) {
        const int row = w, c = lane >> 2, part = lane & 3;
        const bool cv = c < C;
        const float* e = sE[row] + 16 * part;
        const float* wr = sW + min(c, C - 1) * WP + 16 * part;
        float z = 0.f;
#pragma unroll
        for (int t = 0; t < 16; t += 4) {
            const float4 e4 = *reinterpret_cast<const float4*>(e + t);
            const float4 w4 = *reinterpret_cast<const float4*>(wr + t);
            z = fmaf(e4.x, w4.x, z);
            z = fmaf(e4.y, w4.y, z);
            z = fmaf(e4.z, w4.z, z);
            z = fmaf(e4.w, w4.w, z);
        }
        z += dpp_f<0xB1>(z);
        z += dpp_f<0x4E>(z);
        typedef __attribute__((address_space(1))) unsigned long long gu64;
        gu64* mine = (gu64*)(pa.xch + (static_cast<int64_t>(q) * 2 + hh) * 64 + row * 16 + c);
        gu64* theirs = (gu64*)(pa.xch + (static_cast<int64_t>(q) * 2 + (hh ^ 1)) * 64 + row * 16 + c);
        if (part == 0)
            __hip_atomic_store(mine, (static_cast<unsigned long long>(pa.epoch) << 32) | __float_as_uint(z),
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        unsigned long long x = 0;
        for (unsigned spins = 0;; ++spins) {
            x = __hip_atomic_load(theirs, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (__all(static_cast<unsigned>(x >> 32) == pa.epoch)) break;
            if (spins > (1u << 18)) {  // the partner never came: flag it, poison the outputs (bounded wait)
                if (lane == 0) atomicOr(pa.fail, 1u);
                x = 0x7fc00000ull;  // NaN: the loss, dZ and dIn turn NaN
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
        const float zo = __uint_as_float(static_cast<unsigned>(x));
        const float zs = hh == 0 ? z + zo : zo + z;  // half 0's partial first in both blocks
        const float zl = cv ? zs + sb[min(c, C - 1)] : -INFINITY;
        const float mx = wave_max(zl);
        const float lse = logf(wave_sum(cv && part == 0 ? expf(zl - mx) : 0.f));
        if (part == 0 && cv) {
            if (row < nr) {
                const int y = sy[row];
                const float lp = zl - mx - lse;
                if (c == y) sloss[row] = -lp;
                sdl[row * C + c] = (expf(lp) - (c == y ? 1.f : 0.f)) * invB;
            } else {
                sdl[row * C + c] = 0.f;
            }
        }
    }
    lds_barrier();
    GS_TOP_STAMP(6);
    // ---- dZ of this half's 64 columns (waves 0..3) beside its slab columns (waves 4..7)
    if (w < 4) {
        const int row = w, d = lane;
        float g[16], v[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) {
            const int uc = min(u, C - 1);
            g[u] = sdl[row * C + uc];
            v[u] = sW[uc * WP + d];
        }
        float s = 0.f;
#pragma unroll
        for (int u = 0; u < 16; ++u) s = u < C ? fmaf(g[u], v[u], s) : s;
        if (!(sE[row][d] > 0.f)) s = 0.f;
        sZ[row][d] = s;
        if (row < nr) a.dZ[static_cast<int64_t>(r0 + row) * H + HW * hh + d] = s;
    } else {
        const int tt = tid - 256, c = tt >> 4;
        const int per = C * (H + 1);
        float* out = a.slab + static_cast<int64_t>(q) * (per + 1);
        if (c < C) {
            float dl[kTopRows], ev[kTopRows][HW / 16];
#pragma unroll
            for (int ii = 0; ii < kTopRows; ++ii) {
                dl[ii] = sdl[ii * C + c];
#pragma unroll
                for (int j = 0; j < HW / 16; ++j) ev[ii][j] = sE[ii][(tt & 15) + 16 * j];
            }
#pragma unroll
            for (int j = 0; j < HW / 16; ++j) {
                float sv = 0.f;
#pragma unroll
                for (int ii = 0; ii < kTopRows; ++ii) sv = ii < nr ? fmaf(dl[ii], ev[ii][j], sv) : sv;
                out[c * (H + 1) + HW * hh + (tt & 15) + 16 * j] = sv;
            }
            if (hh == 0 && (tt & 15) == 0) {
                float sbias = 0.f;
#pragma unroll
                for (int ii = 0; ii < kTopRows; ++ii) sbias = ii < nr ? fmaf(dl[ii], 1.f, sbias) : sbias;
                out[c * (H + 1) + H] = sbias;
            }
        }
        if (hh == 0 && tid == NT - 64) {
            float sl = 0.f;
            for (int ii = 0; ii < nr; ++ii) sl += sloss[ii];
            out[per] = sl;
        }
    }
    lds_barrier();
    GS_TOP_STAMP(7);
    // ---- dIn's partial over this half's 64 h: wave w: input columns
    // 128 (w & 1) + 2 lane, + 1; h quarter w >> 1 (16 h); dZ by ABID broadcast
    {
        const int k0 = 128 * (w & 1) + 2 * lane, hb = 16 * (w >> 1);
        const float4 za = *reinterpret_cast<const float4*>(sZ[lane & 3] + min(hb + 4 * (lane >> 2), HW - 4));
        float2 wv[16];
#pragma unroll
        for (int t = 0; t < 16; ++t) {
            const int h = hb + t;
            wv[t] = *reinterpret_cast<const float2*>(sW2 + h * K + 4 * ((k0 >> 2) ^ (h & 15)) + (k0 & 3));
        }
        f32x4 c0 = f32x4{0.f, 0.f, 0.f, 0.f}, c1 = c0;
#define GS_PD_STEP(b)                                    \
        c0 = mfma4b<b>(za.x, wv[4 * (b)].x, c0);         \
        c1 = mfma4b<b>(za.x, wv[4 * (b)].y, c1);         \
        c0 = mfma4b<b>(za.y, wv[4 * (b) + 1].x, c0);     \
        c1 = mfma4b<b>(za.y, wv[4 * (b) + 1].y, c1);     \
        c0 = mfma4b<b>(za.z, wv[4 * (b) + 2].x, c0);     \
        c1 = mfma4b<b>(za.z, wv[4 * (b) + 2].y, c1);     \
        c0 = mfma4b<b>(za.w, wv[4 * (b) + 3].x, c0);     \
        c1 = mfma4b<b>(za.w, wv[4 * (b) + 3].y, c1);
        GS_PD_STEP(0) GS_PD_STEP(1) GS_PD_STEP(2) GS_PD_STEP(3)
#undef GS_PD_STEP
        float* pp = sP + (w >> 1) * (kTopRows * K);
#pragma unroll
        for (int j = 0; j < kTopRows; ++j) *reinterpret_cast<float2*>(pp + j * K + k0) = make_float2(c0[j], c1[j]);
    }
    lds_barrier();
    GS_TOP_STAMP(8);
    float* dst = hh == 0 ? a.dIn : pa.dIn2;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
        const int o = tid + u * NT, row = o >> 8, kc = o & (K - 1);
        const float v = ((sP[row * K + kc] + sP[kTopRows * K + row * K + kc]) + sP[2 * kTopRows * K + row * K + kc]) +
                        sP[3 * kTopRows * K + row * K + kc];
        if (row < nr) dst[static_cast<int64_t>(r0 + row) * K + kc] = v;
    }
    GS_TOP_STAMP(9);
    kstamp_end(a.stamp);
}

static size_t top_pair_smem_bytes() {
    return sizeof(float) * (static_cast<size_t>(kPairW) * kTopK + kTopRows * kTopK + 2 * kTopRows * kPairW +
                            4 * kTopRows * kTopK + 16 * (kPairW + 4) + kTopRows * 16 + kTopRows + 16 + kTopRows);
}

static bool top_pair_lds_ready() {
    static int ok = -1;
    if (ok < 0) {
        const int smem = static_cast<int>(top_pair_smem_bytes());
        ok = hipFuncSetAttribute(reinterpret_cast<const void*>(sage_top_pair_kernel<GS_AGG_MEAN>),
                                 hipFuncAttributeMaxDynamicSharedMemorySize, smem) == hipSuccess &&
             hipFuncSetAttribute(reinterpret_cast<const void*>(sage_top_pair_kernel<GS_AGG_MAX>),
                                 hipFuncAttributeMaxDynamicSharedMemorySize, smem) == hipSuccess;
        (void)hipGetLastError();
    }
    return ok == 1;
}

bool top_pair_supported(int64_t H, int64_t C, bool gcn) {
    return H == kTopH && C >= 1 && C <= 16 && !gcn && top_pair_lds_ready();
}

int top_pair_fwd_bwd(int agg, int64_t B, int64_t C, const float* Hprev, const int32_t* ptr, const int32_t* nbr,
                     const int32_t* self, const float* W, const float* Wc, const float* bc, const int32_t* labels,
                     const int32_t* roots, float* aggo, int32_t* argmax, float* E, float* dZ, float* dIn, float* dIn2,
                     float* slab, unsigned long long* xch, unsigned epoch, unsigned* fail, hipStream_t st,
                     const int32_t* tids, int tk) {
    GS_REQUIRE(B >= 1 && B < (int64_t(1) << 30) && C >= 1 && C <= 16 && epoch != 0 && xch && fail, GS_EINVAL,
               "top pair: bad arguments");
    GS_REQUIRE(!tids || (tk >= 1 && tk <= 31), GS_EINVAL, "top: padded lists need 1 <= tk <= 31");
    GS_REQUIRE(aligned16(Hprev) && aligned16(W) && aligned16(Wc) && aligned16(aggo) && aligned16(E) && aligned16(dZ) &&
                   aligned16(dIn) && aligned16(dIn2) && (agg == GS_AGG_MEAN || (argmax && aligned16(argmax))),
               GS_EINVAL, "top pair: unaligned operand");
    GS_REQUIRE(top_pair_lds_ready(), GS_EHIP, "top pair: LDS limit refused");
    const size_t smem = top_pair_smem_bytes();
    TopPairArgs pa{TopArgs{static_cast<int>(B), static_cast<int>(C), Hprev, ptr, nbr, self, W, Wc, bc, labels, roots,
                           aggo, argmax, E, dZ, dIn, slab, tids, tids ? tk : 0, take_kernel_stamp()},
                   dIn2, xch, epoch, fail};
    const int64_t quads = (B + kTopRows - 1) / kTopRows;
    const dim3 grid(static_cast<unsigned>(16 * ((quads + 7) / 8)));
    if (agg == GS_AGG_MEAN) launch_k(sage_top_pair_kernel<GS_AGG_MEAN>, grid, dim3(kTopThreads), smem, st, pa);
    else launch_k(sage_top_pair_kernel<GS_AGG_MAX>, grid, dim3(kTopThreads), smem, st, pa);
    check_launch("sage_top_pair");
    return static_cast<int>(quads);
}

static size_t top_smem_bytes(int64_t C) {
    const int64_t wp = C <= 16 ? kTopH + 4 : kTopH + 1;  // sage_top_kernel's WP
    const int64_t q3 = C <= 16 ? kTopRows + 3 + kTopRows * kTopK : 0;  // its fourth dIn partial (16-B aligned)
    return sizeof(float) * (static_cast<size_t>(kTopH) * kTopK + kTopRows * (kTopK + 2 * kTopH) + kTopPart +
                            C * wp + kTopRows * C + kTopRows + C + (q3 ? q3 : kTopRows));
}

// The kernel keeps W2 in LDS (~146 KiB at 16 classes): raise the launch limit
// once; where the runtime refuses, the caller keeps the separate launches.
static bool top_lds_ready(int64_t C) {
    static int ok_bytes = -1;
    const size_t need = top_smem_bytes(C);
    if (ok_bytes < 0) {
        // the whole 160 KiB of a CU: W2 alone is 128 KiB; classes beyond what
        // fits (C > 20) keep the separate launches
        const size_t want = std::min<size_t>(top_smem_bytes(kTopMaxC), 160 * 1024);
        auto raise = [&](const void* f) {
            return hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(want)) ==
                   hipSuccess;
        };
        const bool a = raise(reinterpret_cast<const void*>(sage_top_kernel<GS_AGG_MEAN, true>)) &&
                       raise(reinterpret_cast<const void*>(sage_top_kernel<GS_AGG_MAX, true>)) &&
                       raise(reinterpret_cast<const void*>(sage_top_kernel<GS_AGG_MEAN, false>)) &&
                       raise(reinterpret_cast<const void*>(sage_top_kernel<GS_AGG_MAX, false>));
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
    const bool small = C <= 16;
    if (agg == GS_AGG_MEAN) {
        if (small) launch_k(sage_top_kernel<GS_AGG_MEAN, true>, grid, dim3(kTopThreads), smem, st, a);
        else launch_k(sage_top_kernel<GS_AGG_MEAN, false>, grid, dim3(kTopThreads), smem, st, a);
    } else {
        if (small) launch_k(sage_top_kernel<GS_AGG_MAX, true>, grid, dim3(kTopThreads), smem, st, a);
        else launch_k(sage_top_kernel<GS_AGG_MAX, false>, grid, dim3(kTopThreads), smem, st, a);
    }
    check_launch("sage_top");
    return static_cast<int>(grid.x);
}

}  // namespace gs
