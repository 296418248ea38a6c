// extend_nodes' negatives on the device (models.py:152-164):
// the N_WALK_LEN-hop balls of a batch's nodes as a bit-parallel multi-source
// BFS (bit b of word w = node 64w+b, 64 balls per 64-bit word, word-major
// [w][node]), and the far-list elements the host's draws pick.
//
// The far list of a node is set(train) - ball in CPython iteration order
// (host/unsup.cpp, file header): either the train set's copy order with the
// ball's members skipped, or — when the ball is large — a fresh set filled in
// train order, whose iteration order is ascending ids whenever its final table
// has a slot per id (mask + 1 >= n_nodes: every key at home).  Both are a
// fixed order of the train nodes filtered by "not in this ball", so the j-th
// element is a select query: per (ball word, 64 consecutive order entries) one
// ballot per ball gives the 64-bit mask of far entries, a per-ball prefix over
// the chunk counts finds the chunk, and the rank inside the chunk the entry.
// The host keeps the sequential part (the draws, models.py:164, on the one
// random stream) and reads back only the counts and the picked ids.
#include <algorithm>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "../host/graph.hpp"
#include "../host/unsup_dev.hpp"
#include "kcommon.hpp"

namespace gs {
namespace {

void hip_ok(hipError_t e, const char* what) {
    if (e != hipSuccess) fail(GS_EHIP, std::string(what) + ": " + hipGetErrorString(e));
}

__global__ void ball_seed_kernel(const int32_t* __restrict__ roots, int n_roots, int64_t n_nodes,
                                 unsigned long long* __restrict__ S, unsigned long long* __restrict__ E) {
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n_roots) return;
    const int64_t at = static_cast<int64_t>(r >> 6) * n_nodes + roots[r];
    const unsigned long long bit = 1ull << (r & 63);
    atomicOr(&S[at], bit);
    atomicOr(&E[at], bit);
}

// One BFS level (models.py:156-161: current |= adj[outer] for outer in
// frontier; frontier = current - neighbors; neighbors |= current), pulled:
// node v of word w ORs the frontier bits of its in-neighbours (the transposed
// CSR, t_ptr/t_col: u -> v in adj[u] is v <- u) and keeps the new ones.  No
// atomics and no scratch to clear; the frontier is double-buffered (Ecur is
// read by every in-neighbour's lanes while Enext is written).  kPullLanes
// lanes per (word, node) stride over the in-row and xor-shuffle their ORs, so
// a hub's row is spread (OR is order-free).  Pushing with 64-bit atomicOr
// took 57 us per level on Pubmed (8 words x 19.7k nodes).
constexpr int kPullLanes = 8;
__global__ __launch_bounds__(256) void ball_pull_kernel(const int64_t* __restrict__ t_ptr,
                                                        const int32_t* __restrict__ t_col, int64_t n_nodes,
                                                        int64_t total, const unsigned long long* __restrict__ Ecur,
                                                        unsigned long long* __restrict__ S,
                                                        unsigned long long* __restrict__ Enext) {
    const int64_t t = blockIdx.x * int64_t(blockDim.x) + threadIdx.x;
    const int64_t i = min(t / kPullLanes, total - 1);  // clamped: every lane reaches the shuffles
    const int sub = static_cast<int>(t % kPullLanes);
    const int64_t w = i / n_nodes, v = i - w * n_nodes;
    const unsigned long long* Ew = Ecur + w * n_nodes;
    unsigned long long acc = 0;
    const int64_t end = t_ptr[v + 1];
    for (int64_t e = t_ptr[v] + sub; e < end; e += kPullLanes) acc |= Ew[t_col[e]];
#pragma unroll
    for (int o = 1; o < kPullLanes; o <<= 1) acc |= __shfl_xor(acc, o, 64);
    if (sub == 0 && t / kPullLanes < total) {
        const unsigned long long s = S[i], nw = acc & ~s;
        Enext[i] = nw;
        S[i] = s | nw;
    }
}

// Per ball (blockIdx.x = word, lane b of every wave counting ball 64w+b;
// blockIdx.y = one of gridDim.y slices of the node and train ranges, so a
// batch of a few words still fills the chip): len(neighbors) over all nodes
// and |train ∩ ball| over the train ids.  Slices add into zeroed counters
// with integer atomics (order-free, so the counts are exact).
__global__ __launch_bounds__(256) void ball_count_kernel(const unsigned long long* __restrict__ S, int64_t n_nodes,
                                                          const int32_t* __restrict__ train, int n_train,
                                                          int n_roots, int64_t* __restrict__ size,
                                                          int64_t* __restrict__ in_train) {
    __shared__ int64_t acc[2][4][64];
    const int w = blockIdx.x, lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int64_t P = gridDim.y, p = blockIdx.y;
    const unsigned long long* Sw = S + static_cast<int64_t>(w) * n_nodes;
    int64_t cs = 0, ct = 0;
    const int64_t ns = (n_nodes + 255) / 256, ne = min(n_nodes, (ns * (p + 1) / P) * 256);
    for (int64_t base = (ns * p / P) * 256 + 64 * wave; base < ne; base += 256) {
        const int64_t u = base + lane;
        const unsigned long long x = u < ne ? Sw[u] : 0ull;
        for (int b = 0; b < 64; ++b) {
            const int c = __popcll(__ballot((x >> b) & 1ull));
            if (lane == b) cs += c;
        }
    }
    const int64_t ts = (static_cast<int64_t>(n_train) + 255) / 256;
    const int64_t te = min(static_cast<int64_t>(n_train), (ts * (p + 1) / P) * 256);
    for (int64_t base = (ts * p / P) * 256 + 64 * wave; base < te; base += 256) {
        const int64_t t = base + lane;
        const unsigned long long x = t < te ? Sw[train[t]] : 0ull;
        for (int b = 0; b < 64; ++b) {
            const int c = __popcll(__ballot((x >> b) & 1ull));
            if (lane == b) ct += c;
        }
    }
    acc[0][wave][lane] = cs;
    acc[1][wave][lane] = ct;
    __syncthreads();
    if (wave == 0) {
        const int r = 64 * w + lane;
        if (r < n_roots) {
            const int64_t a = acc[0][0][lane] + acc[0][1][lane] + acc[0][2][lane] + acc[0][3][lane];
            const int64_t b = acc[1][0][lane] + acc[1][1][lane] + acc[1][2][lane] + acc[1][3][lane];
            if (a) atomicAdd(reinterpret_cast<unsigned long long*>(size + r), static_cast<unsigned long long>(a));
            if (b) atomicAdd(reinterpret_cast<unsigned long long*>(in_train + r), static_cast<unsigned long long>(b));
        }
    }
}

// Far masks: for order entries 64c .. 64c+63 and the 64 balls of word w,
// M[r][c] = entries NOT in ball r (one ballot per ball); cnt in pre[r][c].
__global__ __launch_bounds__(64) void far_mask_kernel(const unsigned long long* __restrict__ S, int64_t n_nodes,
                                                       const int32_t* __restrict__ order, int n_order, int n_chunks,
                                                       int n_roots, unsigned long long* __restrict__ M,
                                                       int32_t* __restrict__ cnt) {
    const int c = blockIdx.x, w = blockIdx.y, lane = threadIdx.x;
    const int t = 64 * c + lane;
    const bool ok = t < n_order;
    const unsigned long long x = ok ? S[static_cast<int64_t>(w) * n_nodes + order[t]] : ~0ull;
    unsigned long long mine = 0;
    for (int b = 0; b < 64; ++b) {
        const unsigned long long m = __ballot(ok && !((x >> b) & 1ull));
        if (lane == b) mine = m;
    }
    const int r = 64 * w + lane;
    if (r < n_roots) {
        M[static_cast<int64_t>(r) * n_chunks + c] = mine;
        cnt[static_cast<int64_t>(r) * (n_chunks + 1) + c] = __popcll(mine);
    }
}

// Exclusive prefix of the chunk counts, one wave per ball.
__global__ __launch_bounds__(64) void far_prefix_kernel(int32_t* __restrict__ pre, int n_chunks) {
    int32_t* p = pre + static_cast<int64_t>(blockIdx.x) * (n_chunks + 1);
    const int lane = threadIdx.x;
    int run = 0;
    for (int base = 0; base < n_chunks; base += 64) {
        const int c = base + lane;
        const int v = c < n_chunks ? p[c] : 0;
        int inc = v;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int t = __shfl_up(inc, o, 64);
            if (lane >= o) inc += t;
        }
        if (c < n_chunks) p[c] = run + inc - v;
        run += __shfl(inc, 63, 64);
    }
    if (lane == 0) p[n_chunks] = run;
}

// The three far orders: set(train).copy(), ascending ids, set(train) itself.
struct FarOrders {
    const unsigned long long* M[3];
    const int32_t* pre[3];
    const int32_t* order[3];
};

// The picks: request q = (ball r, order kind, position j) -> order[entry].
__global__ void far_select_kernel(const int32_t* __restrict__ req_r, const int32_t* __restrict__ req_j,
                                  const uint8_t* __restrict__ req_kind, int n_req, int n_chunks,
                                  FarOrders o, int32_t* __restrict__ out) {
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= n_req) return;
    const int r = req_r[q], j = req_j[q];
    const int kd = req_kind[q];
    const int32_t* p = o.pre[kd] + static_cast<int64_t>(r) * (n_chunks + 1);
    int lo = 0, hi = n_chunks - 1;  // last chunk with p[c] <= j
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (p[mid] <= j) lo = mid;
        else hi = mid - 1;
    }
    unsigned long long m = o.M[kd][static_cast<int64_t>(r) * n_chunks + lo];
    for (int t = j - p[lo]; t > 0; --t) m &= m - 1;
    out[q] = o.order[kd][64 * lo + __ffsll(m) - 1];
}

// Whole far lists in set(train) order (order kind 2) for the listed balls:
// one wave per ball walks its chunk masks and writes every entry at its rank.
__global__ __launch_bounds__(64) void far_list_kernel(const int32_t* __restrict__ balls, const int64_t* __restrict__ base,
                                                      int n_chunks, FarOrders o, int32_t* __restrict__ out) {
    const int q = blockIdx.x, lane = threadIdx.x;
    const int r = balls[q];
    const unsigned long long* M = o.M[2] + static_cast<int64_t>(r) * n_chunks;
    const int32_t* p = o.pre[2] + static_cast<int64_t>(r) * (n_chunks + 1);
    int32_t* dst = out + base[q];
    for (int c = 0; c < n_chunks; ++c) {
        const unsigned long long m = M[c];
        if ((m >> lane) & 1ull) dst[p[c] + __popcll(m & ((1ull << lane) - 1ull))] = o.order[2][64 * c + lane];
    }
}

}  // namespace

struct UnsupDev {
    int64_t n_nodes = 0;
    int n_order = 0, n_chunks = 0;
    std::vector<void*> owned;
    const int64_t* t_ptr = nullptr;  // transposed CSR (in-neighbours) for the pulls
    const int32_t* t_col = nullptr;
    int32_t* copy_order = nullptr;  // list(set(train).copy())
    int32_t* asc_order = nullptr;   // sorted(set(train))
    int32_t* set_order = nullptr;   // list(set(train))
    int cap_roots = 0;
    unsigned long long *S = nullptr, *E = nullptr, *X = nullptr;
    int32_t* roots = nullptr;
    int64_t* counts = nullptr;  // [2][cap_roots]
    unsigned long long* M[3] = {};
    int32_t* pre[3] = {};
    int cap_req = 0;
    int32_t *req_r = nullptr, *req_j = nullptr, *picks = nullptr;
    int cap_lists = 0;
    int64_t cap_list_out = 0;
    int32_t* list_balls = nullptr;
    int64_t* list_base = nullptr;
    int32_t* list_out = nullptr;
    uint8_t* req_kind = nullptr;
    hipStream_t st = nullptr;

    template <typename T>
    T* alloc(int64_t n) {
        void* p = nullptr;
        hip_ok(hipMalloc(&p, std::max<int64_t>(n, 1) * sizeof(T)), "hipMalloc(unsup dev)");
        owned.push_back(p);
        return static_cast<T*>(p);
    }
    // A grown buffer replaces the old one, which is freed at once: every call
    // ends with a stream synchronise, so no launch still reads it.
    template <typename T>
    void regrow(T*& p, int64_t n) {
        if (p) {
            owned.erase(std::remove(owned.begin(), owned.end(), static_cast<void*>(p)), owned.end());
            hip_ok(hipFree(p), "hipFree(unsup dev)");
        }
        p = alloc<T>(n);
    }
    void free_all() {
        if (st) (void)hipStreamSynchronize(st);
        for (void* p : owned) (void)hipFree(p);
        owned.clear();
        if (st) (void)hipStreamDestroy(st);
        st = nullptr;
    }
    ~UnsupDev() { free_all(); }
};

// The device half owns a non-blocking stream on the current device: its calls
// synchronise only their own work (not the caller's queued model launches, so
// the host can draw while the previous step's backward runs) and never depend
// on a caller stream's lifetime.  It reads no caller tensors.
UnsupDev* unsup_dev_create(const Graph& g, const std::vector<int32_t>& copy_order,
                           const std::vector<int32_t>& set_order, void* /*stream: unused*/) {
    auto d = std::make_unique<UnsupDev>();
    hip_ok(hipStreamCreateWithFlags(&d->st, hipStreamNonBlocking), "hipStreamCreate(unsup dev)");
    d->n_nodes = g.n_nodes;
    d->n_order = static_cast<int>(copy_order.size());
    d->n_chunks = std::max(1, (d->n_order + 63) / 64);
    auto up = [&](const void* src, size_t bytes) {
        void* p = d->alloc<uint8_t>(static_cast<int64_t>(bytes));
        if (bytes) hip_ok(hipMemcpy(p, src, bytes, hipMemcpyHostToDevice), "hipMemcpy(unsup dev)");
        return p;
    };
    {  // in-neighbour CSR by a counting sort over col (order within a row is irrelevant to OR)
        const int64_t n = g.n_nodes, m = g.row_ptr[n];
        std::vector<int64_t> tp(n + 1, 0);
        for (int64_t e = 0; e < m; ++e) ++tp[g.col[e] + 1];
        for (int64_t v = 0; v < n; ++v) tp[v + 1] += tp[v];
        std::vector<int64_t> at(tp.begin(), tp.end() - 1);
        std::vector<int32_t> tc(static_cast<size_t>(m));
        for (int64_t u = 0; u < n; ++u)
            for (int64_t e = g.row_ptr[u]; e < g.row_ptr[u + 1]; ++e) tc[at[g.col[e]]++] = static_cast<int32_t>(u);
        d->t_ptr = static_cast<const int64_t*>(up(tp.data(), tp.size() * sizeof(int64_t)));
        d->t_col = static_cast<const int32_t*>(up(tc.data(), tc.size() * sizeof(int32_t)));
    }
    std::vector<int32_t> asc(copy_order);
    std::sort(asc.begin(), asc.end());
    d->copy_order = static_cast<int32_t*>(up(copy_order.data(), copy_order.size() * sizeof(int32_t)));
    d->asc_order = static_cast<int32_t*>(up(asc.data(), asc.size() * sizeof(int32_t)));
    d->set_order = static_cast<int32_t*>(up(set_order.data(), set_order.size() * sizeof(int32_t)));
    return d.release();
}

void unsup_dev_destroy(UnsupDev* d) { delete d; }

static void reserve_roots(UnsupDev* d, int n) {
    if (n <= d->cap_roots) return;
    const int cap = std::max(n, 64);
    const int64_t words = (cap + 63) / 64;
    d->regrow(d->S, words * d->n_nodes);
    d->regrow(d->E, words * d->n_nodes);
    d->regrow(d->X, words * d->n_nodes);
    d->regrow(d->roots, cap);
    d->regrow(d->counts, 2 * cap);
    for (int o = 0; o < 3; ++o) {
        d->regrow(d->M[o], static_cast<int64_t>(cap) * d->n_chunks);
        d->regrow(d->pre[o], static_cast<int64_t>(cap) * (d->n_chunks + 1));
    }
    d->cap_roots = cap;
}

void unsup_dev_balls(UnsupDev* d, const int64_t* nodes, int n, int hops, int64_t* ball_size, int64_t* train_in_ball) {
    if (n <= 0) return;  // no balls: no launch (a zero-block grid is an error)
    reserve_roots(d, n);
    const int n_words = (n + 63) / 64;
    const int64_t total = static_cast<int64_t>(n_words) * d->n_nodes;
    std::vector<int32_t> r32(nodes, nodes + n);
    hipStream_t st = d->st;
    hip_ok(hipMemcpyAsync(d->roots, r32.data(), n * sizeof(int32_t), hipMemcpyHostToDevice, st), "hipMemcpyAsync");
    hip_ok(hipMemsetAsync(d->S, 0, total * 8, st), "hipMemsetAsync");
    hip_ok(hipMemsetAsync(d->E, 0, total * 8, st), "hipMemsetAsync");
    ball_seed_kernel<<<(n + 255) / 256, 256, 0, st>>>(d->roots, n, d->n_nodes, d->S, d->E);
    check_launch("ball_seed_kernel");
    const unsigned nb_pull = static_cast<unsigned>((total * kPullLanes + 255) / 256);
    unsigned long long *cur = d->E, *next = d->X;
    for (int h = 0; h < hops; ++h) {
        ball_pull_kernel<<<nb_pull, 256, 0, st>>>(d->t_ptr, d->t_col, d->n_nodes, total, cur, d->S, next);
        check_launch("ball_pull_kernel");
        std::swap(cur, next);
    }
    // >= ~512 blocks however few words the batch has
    const unsigned slices = static_cast<unsigned>(std::min(64, std::max(1, (512 + n_words - 1) / n_words)));
    hip_ok(hipMemsetAsync(d->counts, 0, 2 * static_cast<size_t>(d->cap_roots) * sizeof(int64_t), st), "hipMemsetAsync");
    ball_count_kernel<<<dim3(static_cast<unsigned>(n_words), slices), 256, 0, st>>>(
        d->S, d->n_nodes, d->asc_order, d->n_order, n, d->counts, d->counts + d->cap_roots);
    check_launch("ball_count_kernel");
    // far masks and their prefixes for the three orders (needed by the picks)
    const dim3 mg(static_cast<unsigned>(d->n_chunks), static_cast<unsigned>(n_words));
    const int32_t* orders[3] = {d->copy_order, d->asc_order, d->set_order};
    for (int o = 0; o < 3; ++o) {
        far_mask_kernel<<<mg, 64, 0, st>>>(d->S, d->n_nodes, orders[o], d->n_order, d->n_chunks, n, d->M[o], d->pre[o]);
        check_launch("far_mask_kernel");
        far_prefix_kernel<<<n, 64, 0, st>>>(d->pre[o], d->n_chunks);
        check_launch("far_prefix_kernel");
    }
    hip_ok(hipMemcpyAsync(ball_size, d->counts, n * sizeof(int64_t), hipMemcpyDeviceToHost, st), "hipMemcpyAsync");
    hip_ok(hipMemcpyAsync(train_in_ball, d->counts + d->cap_roots, n * sizeof(int64_t), hipMemcpyDeviceToHost, st),
           "hipMemcpyAsync");
    hip_ok(hipStreamSynchronize(st), "hipStreamSynchronize");
}

void unsup_dev_select(UnsupDev* d, const std::vector<int32_t>& req_r, const std::vector<int32_t>& req_j,
                      const std::vector<uint8_t>& req_kind, std::vector<int32_t>& out) {
    const int n = static_cast<int>(req_r.size());
    out.resize(n);
    if (!n) return;
    if (n > d->cap_req) {
        const int cap = std::max(n, 1024);
        d->regrow(d->req_r, cap);
        d->regrow(d->req_j, cap);
        d->regrow(d->picks, cap);
        d->regrow(d->req_kind, cap);
        d->cap_req = cap;
    }
    hipStream_t st = d->st;
    hip_ok(hipMemcpyAsync(d->req_r, req_r.data(), n * sizeof(int32_t), hipMemcpyHostToDevice, st), "hipMemcpyAsync");
    hip_ok(hipMemcpyAsync(d->req_j, req_j.data(), n * sizeof(int32_t), hipMemcpyHostToDevice, st), "hipMemcpyAsync");
    hip_ok(hipMemcpyAsync(d->req_kind, req_kind.data(), n, hipMemcpyHostToDevice, st), "hipMemcpyAsync");
    const FarOrders fo{{d->M[0], d->M[1], d->M[2]}, {d->pre[0], d->pre[1], d->pre[2]},
                       {d->copy_order, d->asc_order, d->set_order}};
    far_select_kernel<<<(n + 255) / 256, 256, 0, st>>>(d->req_r, d->req_j, d->req_kind, n, d->n_chunks, fo, d->picks);
    check_launch("far_select_kernel");
    hip_ok(hipMemcpyAsync(out.data(), d->picks, n * sizeof(int32_t), hipMemcpyDeviceToHost, st), "hipMemcpyAsync");
    hip_ok(hipStreamSynchronize(st), "hipStreamSynchronize");
}

}  // namespace gs

namespace gs {

void unsup_dev_far_lists(UnsupDev* d, const std::vector<int32_t>& balls, const std::vector<int64_t>& base,
                         std::vector<int32_t>& out) {
    const int n = static_cast<int>(balls.size());
    const int64_t total = n ? base[n] : 0;
    out.resize(static_cast<size_t>(total));
    if (!n || !total) return;
    if (n > d->cap_lists) {  // geometric growth: a long run settles after a few batches
        const int cap = std::max(n, d->cap_lists + d->cap_lists / 2);
        d->regrow(d->list_balls, cap);
        d->regrow(d->list_base, static_cast<int64_t>(cap) + 1);
        d->cap_lists = cap;
    }
    if (total > d->cap_list_out) {
        const int64_t cap = std::max(total, d->cap_list_out + d->cap_list_out / 2);
        d->regrow(d->list_out, cap);
        d->cap_list_out = cap;
    }
    hipStream_t st = d->st;
    hip_ok(hipMemcpyAsync(d->list_balls, balls.data(), n * sizeof(int32_t), hipMemcpyHostToDevice, st), "hipMemcpyAsync");
    hip_ok(hipMemcpyAsync(d->list_base, base.data(), (n + 1) * sizeof(int64_t), hipMemcpyHostToDevice, st),
           "hipMemcpyAsync");
    const FarOrders fo{{d->M[0], d->M[1], d->M[2]}, {d->pre[0], d->pre[1], d->pre[2]},
                       {d->copy_order, d->asc_order, d->set_order}};
    far_list_kernel<<<n, 64, 0, st>>>(d->list_balls, d->list_base, d->n_chunks, fo, d->list_out);
    check_launch("far_list_kernel");
    hip_ok(hipMemcpyAsync(out.data(), d->list_out, total * sizeof(int32_t), hipMemcpyDeviceToHost, st), "hipMemcpyAsync");
    hip_ok(hipStreamSynchronize(st), "hipStreamSynchronize");
}

}  // namespace gs
