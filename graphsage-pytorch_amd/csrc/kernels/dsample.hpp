// Device sampler internals shared by dsample.hip (stream, draws, C-ABI) and
// dsample_union.hip (per-node sets, the frontier union and the lists).
#pragma once

#include "kcommon.hpp"

namespace gs {
namespace ds {

constexpr int64_t kRing = int64_t(1) << 20;  // words kept per stream ring (tempered and raw)
constexpr int64_t kRingMask = kRing - 1;
constexpr int kWMax = 4096;                  // widest rejection-count window per block
constexpr int kComposeEntries = 30720;       // G * W entries a compose block stages in LDS (60 KiB)
constexpr int kMinG = kComposeEntries / kWMax;
constexpr int kChainEntries = 30720;         // group exits the chain block stages in LDS (uint16)
constexpr int kMaxGroups = 1024;
constexpr int kMEntries = 256;               // window entries per table-kernel workgroup
constexpr int kResSlots = 4;                 // runs whose results are kept (gs_dsampler_result_of)

// status bits (Ctl::status)
constexpr int kStWindow = 1;   // a true entry fell outside its block window
constexpr int kStWords = 2;    // a walk ran past the words loaded for it
constexpr int kStTable = 4;    // a frontier union outgrew the device table
constexpr int kStEmpty = 8;    // empty neighbourhood with GS_SAMPLE_FAIL_EMPTY
constexpr int kStSize = 16;    // a frontier outgrew its preallocated bound
constexpr int kStOrder = 32;   // block states lost their order (never expected)
constexpr int kStSpin = 64;    // a table insert exceeded its probe / displacement bound (never expected)
// Statuses after which the run's later kernels have nothing valid to read
// (unwritten sample entries, a frontier never built, stale hop sizes): every
// kernel after begin_kernel returns at once once one is set (GS_DS_BAIL), so a
// failed run reports its status instead of reading garbage indices.
constexpr int kStFail = kStWindow | kStWords | kStTable | kStSize | kStOrder | kStSpin;
// Block-uniform early return on a failed run: thread 0 reads the status once
// (another block of the same launch may set it meanwhile) and the block
// follows that one reading.
#define GS_DS_BAIL(c)                                               \
    do {                                                            \
        __shared__ int s_bail_;                                     \
        if (threadIdx.x == 0) s_bail_ = (c)->status & kStFail;      \
        __syncthreads();                                            \
        if (s_bail_) return;                                        \
    } while (0)

// Probe steps one key may take in a table of mask + 1 slots before the insert
// gives up (kStSpin): CPython's probe sequence (10 linear slots, then
// i = 5 i + 1 + perturb, full period once perturb is 0) reaches every slot
// within (mask + 1) + 7 * 10 steps, so a table that is at most 3/5 full never
// gets near this; only a broken invariant (more keys than free slots) does,
// and it then fails loudly instead of spinning the kernel forever.
__host__ __device__ constexpr uint32_t probe_cap(uint32_t mask) { return 2u * (mask + 1u) + 256u; }

struct DevGraph {
    const int64_t* row_ptr;
    const int32_t* col;
    const uint32_t* slot;      // slot of each entry in its row's set table
    const uint8_t* log2size;   // row table size = 1 << log2size
    const uint8_t* dirty;      // row set has dummies (nullptr: none)
    int64_t n_nodes;
};

struct HopCtl {
    int32_t n_dst, n_pos, n_draws;
    int32_t n_blocks, W, G, n_groups;
    int32_t j_end;
    int32_t n_empty;
    int32_t n_src, n_nbr;      // hops before the last (union, lists)
    int32_t big;               // the union's table outgrew LDS uint32 slots: ubig_kernel builds it
    int32_t n_wg;              // table-kernel work items (HopBufs::wg)
    int64_t P0;                // absolute stream position at the hop's first draw
    int64_t need_end;          // words the hop may read (exclusive)
    int32_t off[GS_PK_NFIELDS];
};

struct Ctl {
    int64_t gen_end;           // raw/tempered words valid below this absolute index
    int64_t gen_spec;          // words the aux stream generated ahead (valid below it once joined)
    int64_t pos_cur;           // next word of the stream
    int64_t pos_batch;         // stream position at the start of the last run
    int32_t status;
    int32_t epoch;
    int32_t total;             // pack elements before the roots
    int32_t used;
    HopCtl hop[GS_MAX_HOPS];
    int64_t dbg[64];           // diagnostics of the last run (gs_dsampler_debug)
};

struct HopBufs {
    int32_t* dst;              // frontier F(j-1) (ids), [nd_max]
    int32_t* deg;              // [nd_max]
    float2* mv;                // rejection moments per node
    int32_t* pos_ptr;          // [nd_max + 1]
    int32_t* blo;              // block windows' first entry, [nb_max + 1]
    int32_t* bw;               // block windows' widths (multiples of 64, <= W), [nb_max + 1]
    int32_t* dbase;            // draws before each block, [nb_max + 1]
    uint16_t* tab;             // block maps [nb_max][kWMax]
    int32_t* path;             // group paths [nb_max][kWMax]
    uint16_t* gexit;           // group exits relative to the next group's window [ng_max][kWMax]
    int32_t* gexit_last;       // the last group's absolute exits [kWMax]
    int32_t* entry;            // true entry per block [nb_max]
    int32_t* ent;              // absolute CSR entries of the hop's samples (hops before the last)
    uint8_t* rej;              // rejections of sampled node m of block b from entry e: [(b * R + m) * kWMax + e]
    int32_t* wg;               // table-kernel work items b | part << 16, blocks ascending, [nb_max * kWMax / kMEntries]
};

struct UnionBufs {
    int32_t* set_cnt;          // |samp_neighs[r]| per frontier node, [nd_max]
    int32_t* set_items;        // their items in iteration order at [pos_ptr[r] + r], [npos_max + nd_max]
    int32_t* first_tab;        // samp_neighs[0]'s table, [kSmallSet]
    int32_t* first_meta;       // its (mask, used)
    uint64_t* mark;            // [n_nodes]: epoch << 32 | ~t, the first occurrence of a key in the union
    int32_t* tpre;             // items of runs 1..r-1 (union order), [nd_max + 1]
    int32_t* ubef;             // union size before run r, [nd_max]
    int32_t* fresh;            // keys new to the union, in insertion order, [npos_max + nd_max]
    int32_t* tcnt;             // transposed counts / cursors, [nd_next_max + 1]
    uint64_t* fmask;           // per run: bit q = item q is new to the union, [nd_max]
    int32_t* sched;            // resize schedule (run, mask) of a big union, [2 * (kMaxStages + 1)]
    int32_t* skeys;            // a big union's stage keys by priority, two stages, [2 * kBigKeys]
    int32_t* lid;              // [n_nodes]: a union key's position in the next frontier (this hop's keys only)
    int32_t* longs;            // [0] count, then the sources whose transposed list tsort_kernel leaves
                               // to tlong_kernel, [nd_next_max + 1]
};

constexpr int kSmallSet = 128;      // table slots of one samp_neighs set (k <= 32)
constexpr int kUnionMax = 16384;    // table slots of a frontier union in LDS (uint32 priorities)
constexpr int kUnionBig = 65536;    // ... with uint16 priorities, keys in global memory (ubig_kernel)
constexpr int kBigKeys = kUnionBig * 3 / 5 + 1024;  // a big stage's keys (its table <= 3/5 full)
constexpr int kMaxStages = 24;


__device__ __forceinline__ int warp_incl_scan(int v) {
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int t = __shfl_up(v, o, 64);
        if ((threadIdx.x & 63) >= o) v += t;
    }
    return v;
}
__device__ __forceinline__ float warp_incl_scan(float v) {
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const float t = __shfl_up(v, o, 64);
        if ((threadIdx.x & 63) >= o) v += t;
    }
    return v;
}

// Exclusive scan over a 1024-thread block of one value per thread; returns
// the thread's exclusive prefix, *total the block total.
template <typename T>
__device__ __forceinline__ T block_excl_scan(T v, T* sh /* >= 17 */, T* total) {
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const T inc = warp_incl_scan(v);
    if (lane == 63) sh[w] = inc;
    __syncthreads();
    if (threadIdx.x == 0) {
        T run = T(0);
        for (int q = 0; q < 16; ++q) {
            const T t = sh[q];
            sh[q] = run;
            run += t;
        }
        sh[16] = run;
    }
    __syncthreads();
    const T out = sh[w] + inc - v;
    *total = sh[16];
    __syncthreads();
    return out;
}

__device__ __forceinline__ int32_t al4(int32_t n) { return (n + 3) & ~3; }

}  // namespace ds
}  // namespace gs

namespace gs {
namespace ds {
// dsample_union.hip: for hop `hop` (not the last): per-node sets, the frontier
// union (next.dst, n_src), the neighbour / self / transposed lists into the
// pack.  Buffers in `ub` are allocated on first use.
// with_lists = false: the caller launches the lists (launch_hop_lists) itself
// later, e.g. on another stream beside the next hop's draws (nothing of the
// next hop reads them; it needs next.dst only).
void launch_hop_union(const DevGraph& g, Ctl* c, const HopBufs& hb, UnionBufs& ub, const HopBufs& next, int hop,
                      int k, int64_t nd_max, int64_t nd_next_max, int flags, int32_t* pack, hipStream_t st,
                      bool with_lists);
// The neighbour / self / transposed lists of hop `hop` into the pack (reads
// the union's lid, so before any later union).
void launch_hop_lists(Ctl* c, const HopBufs& hb, UnionBufs& ub, int hop, int64_t nd_max, int64_t nd_next_max,
                      int flags, int32_t* pack, hipStream_t st);
}  // namespace ds
}  // namespace gs
