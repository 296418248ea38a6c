// Native pipeline runner: the reference's per-epoch batch loop
// (utils.py:144-191) with its two halves overlapped instead of alternating —
// host neighbour sampling on S threads and the device step on one stream —
// so that no Python code runs per step.
//
//   sampler thread w : batches w, w+S, ... in order, each into a free pinned
//                      slot of its ring (gs_sample_pack_run, its own rng)
//   gs_runner_run    : batch i from stream i % S, in order: device pull of
//                      its pack (ring entry i % 3) and its layer-1 gather on
//                      a side stream, issued one batch ahead when sampled so
//                      they run under step i-1; then forward/backward from
//                      the gathered slot, all-reduce (with a communicator) and update
//                      on the caller's stream.
// A pinned slot returns to its sampler once the copy that read it has
// completed.  Only the driver thread makes HIP calls: it polls the copy events
// of consumed slots (hipEventQuery) and hands finished slots back, and waits
// on the oldest copy only when a stream has no slot left to sample into.
#include <rccl/rccl.h>
#include <sys/mman.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <sched.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../kernels/internal.hpp"

namespace gs {

using Clock = std::chrono::steady_clock;

static double secs(Clock::time_point a, Clock::time_point b) {
    return std::chrono::duration<double>(b - a).count();
}

static void hip_ok(hipError_t e, const char* what) {
    if (e != hipSuccess) fail(GS_EHIP, std::string(what) + ": " + hipGetErrorString(e));
}

// The runner's events only order work: the host never reads device memory
// through them (it waits on them before reusing a pinned slot the device has
// read, or a device buffer whose readers have finished), and cross-stream
// consumers are ordered by them on one device.  So they skip the system-scope
// release that a default event performs (a cache writeback + invalidate at
// every step boundary).
static unsigned sync_event_flags() {
    return hipEventDisableTiming | static_cast<unsigned>(hipEventDisableSystemFence);
}

// Device-side pull of a pinned host pack (hipHostMalloc memory is mapped into
// the device address space): the host pays one kernel launch instead of
// hipMemcpyAsync's host-side cost (measured ~50 us per 0.3 MB pack).
__global__ __launch_bounds__(256) void pull_pack_kernel(const int4* __restrict__ src, int4* __restrict__ dst,
                                                        int64_t n16, const int32_t* __restrict__ src_tail,
                                                        int32_t* __restrict__ dst_tail, int n_tail) {
    // grid-stride, four 16-B loads in flight per lane before their stores
    const int64_t stride = gridDim.x * int64_t(256);
    for (int64_t i = blockIdx.x * int64_t(256) + threadIdx.x; i < n16; i += 4 * stride) {
        int4 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u)
            if (i + u * stride < n16) v[u] = src[i + u * stride];
#pragma unroll
        for (int u = 0; u < 4; ++u)
            if (i + u * stride < n16) dst[i + u * stride] = v[u];
    }
    const int64_t t = blockIdx.x * int64_t(256) + threadIdx.x;
    if (t < n_tail) dst_tail[t] = src_tail[t];
}

struct PackSlot {
    int32_t* host = nullptr;  // pinned
    int32_t* dptr = nullptr;  // its device address (the pull kernel's source)
    size_t thp_bytes = 0;     // a 2 MiB-aligned registered mapping of this size
    hipEvent_t copied = nullptr;
    int64_t batch = -1;
    int64_t hop_sizes[4 * GS_MAX_HOPS];
    int64_t offsets[GS_MAX_HOPS * GS_PK_NFIELDS];
    int64_t used = 0;
    double sample_s = 0;
    int status = GS_OK;
    std::string error;
};

struct SamplerStream {
    gs_rng* rng = nullptr;
    gs_team* team = nullptr;       // cfg.helpers threads (owned), or none
    std::vector<int64_t> batches;  // global batch indices, in order
    std::vector<PackSlot> slots;
    std::deque<int> free, ready;  // guarded by mu
    std::deque<int> copying;      // driver-only: consumed, H2D copy in flight
    std::mutex mu;
    std::condition_variable cv;
    std::thread th;
};

}  // namespace gs

namespace gs {
struct Inflight {
    int stream = -1, slot = -1;
};
}  // namespace gs

struct gs_runner {
    gs_runner_config cfg{};
    std::vector<int32_t> fanouts;
    std::vector<int64_t> roots;  // n_batches x batch
    int64_t cap = 0;             // int32 words per pack slot (pack bound + roots)
    int64_t merge = 1;           // reference batches per step (inference only)
    int64_t n_units = 0;         // steps: ceil(n_batches / merge)
    std::vector<std::unique_ptr<gs::SamplerStream>> streams;
    std::atomic<bool> stop{false};
    // cfg.hold: sampler threads start no batch >= mark until gs_runner_release
    std::atomic<int64_t> release_mark{INT64_MAX};
    std::atomic<int64_t> sampled{0};      // batches whose sampling completed
    std::mutex warm_mu;                   // cfg.warm: threads done warming
    std::condition_variable warm_cv;
    int warmed = 0;
    int64_t next_batch = 0;
    // cfg.ar_buckets == 2: the upper gradients' all-reduce on its own stream
    hipStream_t comm_stream = nullptr;
    hipEvent_t upper_ready = nullptr, upper_reduced = nullptr;
    // GS_AR_W1_CHUNKS (default 2): W1's gradient all-reduced in row chunks as
    // the trainer's chunked dW1 produces them (trainer_set_w1_chunk_hook);
    // w1_issued counts the chunks the current step handed over (0: the
    // trainer took the one-piece path, so the runner reduces W1 itself)
    hipEvent_t w1_ready = nullptr;
    int w1_issued = 0;
    // Ring of 3 per batch in flight (b % 3): device pack buffer, trainer
    // gather slot, events.  The side stream pulls batch b's pack and gathers
    // its layer 1 (reads only X and the pack) while the main stream runs
    // batch b-1.  No stream ever waits on another's event (a cross-queue wait
    // measured ~17 us of idle GPU here): the host checks instead that the step
    // three batches back released the ring entry, and that the gather of the
    // batch it is about to issue has completed.
    static constexpr int kDev = 3;
    // Device pack buffers: one per gather-ring entry (b % kDev); entry k's
    // previous user, step b-3, is the one wait_entry(k) waits for.
    static constexpr int kPack = kDev;
    int32_t* dev[kPack] = {};
    gs::Inflight pulled_slot[kPack];       // sampler stream + slot of the pack in entry p
    hipEvent_t dev_done[kDev] = {};        // main: step of the batch in entry k finished
    bool dev_busy[kDev] = {};
    // Step completion without an event between steps: the step's SGD launch
    // (with a deferred update: its last slab sum) stores its batch index into done_host (fine-grained pinned memory) when
    // it starts, i.e. once every launch that reads the step's ring entry has
    // completed (stream order); the host polls it.  dev_done events remain for
    // the last step of each gs_runner_run call (teardown) and for inference.
    bool use_flag = false;
    int64_t* done_host = nullptr;          // hipHostMalloc, coherent
    int64_t* done_dev = nullptr;
    int64_t flag_step[kDev] = {-1, -1, -1};  // batch whose SGD signals entry k free (-1: none pending)
    void wait_entry(int k) {
        if (flag_step[k] >= 0) {
            const int64_t want = flag_step[k];
            const auto t0 = std::chrono::steady_clock::now();
            for (uint64_t spin = 0; __atomic_load_n(done_host, __ATOMIC_ACQUIRE) < want; ++spin) {
                __builtin_ia32_pause();
                // offer the core to runnable sampler threads every 64 polls
                // while the step runs (the runner is two steps ahead, so a few
                // microseconds of reaction cost nothing; profiles/r04f_runner_yield_ab.txt)
                if ((spin & 63) == 63) sched_yield();
                if ((spin & 0xfffff) == 0xfffff &&
                    std::chrono::steady_clock::now() - t0 > std::chrono::seconds(5)) {
                    // no progress for 5 s: let the runtime report a device error, then give up
                    gs::hip_ok(hipDeviceSynchronize(), "hipDeviceSynchronize");
                    if (__atomic_load_n(done_host, __ATOMIC_ACQUIRE) < want)
                        gs::fail(GS_EHIP, "runner: step completion flag never arrived");
                }
            }
            flag_step[k] = -1;
        }
        if (dev_busy[k]) gs::hip_ok(hipEventSynchronize(dev_done[k]), "hipEventSynchronize");
    }
    hipEvent_t gathered[kDev] = {};        // side: pull + gather of the batch in entry k
    hipStream_t side = nullptr;
    gs::Inflight inflight[kDev];
    int64_t issued = 0;                    // batches whose pull + gather are issued
    void* ws = nullptr;
    int64_t ws_bytes = 0;
    float* clip_ws = nullptr;
    int device = 0;
    gs_runner_stats stats{};

    // cfg.device_sampler: one gs_dsampler per stream, each on its own HIP
    // stream, up to dev_depth runs queued per stream (the sampler keeps each
    // run's result: gs_dsampler_result_of), so a stream's next run is already
    // on the GPU when its current one finishes; packs are written straight into
    // a device ring of dev_depth * S + 3 entries (batch b's entry was last read
    // by step b - dev_depth * S - 3, which issue() has waited for before
    // enqueuing b).
    static constexpr int kDevDepthMax = 2;
    struct DevStream {
        gs_dsampler* ds = nullptr;
        hipStream_t st = nullptr;
        // queued runs, oldest first: batch, sampler run number, events around
        // the run (its device time), already counted in `sampled`
        int nq = 0;
        int64_t qb[kDevDepthMax] = {}, qrun[kDevDepthMax] = {};
        hipEvent_t t0[kDevDepthMax] = {}, t1[kDevDepthMax] = {};
        bool counted[kDevDepthMax] = {};
        int64_t next = 0;                       // next batch to enqueue (w, w + S, ...)
    };
    int dev_depth = kDevDepthMax;
    struct DevResult {
        int64_t hop_sizes[4 * GS_MAX_HOPS];
        int64_t offsets[GS_MAX_HOPS * GS_PK_NFIELDS];
        int64_t used = 0;
        double sample_s = 0;
    };
    bool devmode = false;
    // guards dstreams' queues (nq, qb, next, counted): gs_runner_release and
    // gs_runner_progress may be called from another thread than gs_runner_run
    std::recursive_mutex dev_mu;
    std::vector<DevStream> dstreams;
    int32_t* roots_dev = nullptr;
    int64_t n_dpack = 0, dcap = 0;
    std::vector<int32_t*> dpack;
    std::vector<DevResult> dres;
    void dev_enqueue(int w);
    bool dev_take(int64_t b, bool block);
    void dev_poll();
    void dev_sync_rngs();

    ~gs_runner();
    void sampler_loop(gs::SamplerStream& s);
    void recycle(gs::SamplerStream& s, bool block);
    bool issue(int64_t b, bool block);
    int take_slot(int64_t b, bool block);
    void pull(int64_t b, int slot_id);
};

// Hand the slots whose copy has completed back to their sampler; with
// `block`, wait for the oldest one when none is free yet.
void gs_runner::recycle(gs::SamplerStream& s, bool block) {
    int n_back = 0;
    while (!s.copying.empty()) {
        const int q = s.copying.front();
        const hipError_t e = (block && n_back == 0) ? hipEventSynchronize(s.slots[q].copied)
                                                     : hipEventQuery(s.slots[q].copied);
        if (e == hipErrorNotReady) break;
        gs::hip_ok(e, "copy event");
        s.copying.pop_front();
        {
            std::lock_guard<std::mutex> lk(s.mu);
            s.free.push_back(q);
        }
        ++n_back;
    }
    if (n_back) s.cv.notify_all();
}

void gs_runner::sampler_loop(gs::SamplerStream& s) {
    if (cfg.warm) {
        // one throwaway batch from a copy of the stream's rng into a free
        // slot: the context's buffers grow and fault in here, not inside a
        // measured step; the stream itself does not advance
        gs_rng* tmp = nullptr;
        uint32_t mt[624];
        int64_t pos = 0;
        if (!s.batches.empty() && !s.free.empty() && gs_rng_create(&tmp) == GS_OK &&
            gs_rng_get_state(s.rng, mt, &pos) == GS_OK && gs_rng_set_state(tmp, mt, pos) == GS_OK) {
            gs::PackSlot& slot = s.slots[s.free.front()];
            const int64_t b = s.batches.back();
            const int64_t nb = std::min(merge, cfg.n_batches - b * merge);
            (void)gs_sample_pack_run_multi_team(cfg.graph, tmp, roots.data() + b * merge * cfg.batch, nb * cfg.batch,
                                                cfg.batch, fanouts.data(), cfg.n_hops, cfg.flags, slot.host, cap,
                                                slot.hop_sizes, slot.offsets, &slot.used, s.team);
        }
        if (tmp) gs_rng_destroy(tmp);
        {
            std::lock_guard<std::mutex> lk(warm_mu);
            ++warmed;
        }
        warm_cv.notify_all();
    }
    for (int64_t b : s.batches) {
        int slot_id;
        {
            std::unique_lock<std::mutex> lk(s.mu);
            s.cv.wait(lk, [&] { return stop.load() || (!s.free.empty() && b < release_mark.load()); });
            if (stop) return;
            slot_id = s.free.front();
            s.free.pop_front();
        }
        gs::PackSlot& slot = s.slots[slot_id];
        const auto t0 = gs::Clock::now();
        slot.batch = b;
        const int64_t nb = std::min(merge, cfg.n_batches - b * merge);  // reference batches of step b
        slot.status = gs_sample_pack_run_multi_team(cfg.graph, s.rng, roots.data() + b * merge * cfg.batch,
                                                    nb * cfg.batch, cfg.batch, fanouts.data(), cfg.n_hops, cfg.flags,
                                                    slot.host, cap, slot.hop_sizes, slot.offsets, &slot.used, s.team);
        if (slot.status != GS_OK) slot.error = gs_last_error();
        slot.sample_s = gs::secs(t0, gs::Clock::now());
        {
            std::lock_guard<std::mutex> lk(s.mu);
            s.ready.push_back(slot_id);
        }
        sampled.fetch_add(1);
        s.cv.notify_all();
        if (slot.status != GS_OK) return;  // the driver reports it when it reaches this batch
    }
}

// Take batch b's sampled slot off its stream's ready queue (-1: not sampled
// yet and !block).
int gs_runner::take_slot(int64_t b, bool block) {
    using namespace gs;
    SamplerStream& s = *streams[b % cfg.n_streams];
    int slot_id;
    const auto tw = Clock::now();
    for (;;) {
        std::unique_lock<std::mutex> lk(s.mu);
        if (!s.ready.empty()) {
            slot_id = s.ready.front();
            s.ready.pop_front();
            break;
        }
        if (!block) return -1;
        // wait for a sampled batch, or free a slot for a starved sampler
        s.cv.wait(lk, [&] { return !s.ready.empty() || (s.free.empty() && !s.copying.empty()); });
        if (!s.ready.empty()) continue;
        lk.unlock();
        recycle(s, true);
    }
    stats.wait_sample_s += secs(tw, Clock::now());
    PackSlot& slot = s.slots[slot_id];
    GS_REQUIRE(slot.batch == b, GS_EINVAL, "sampler ring out of order");
    if (slot.status != GS_OK) fail(slot.status, slot.error);
    return slot_id;
}

// Batch b's pack: pinned slot -> device pack entry b % kPack on the side
// stream (a kernel reading the mapped slot; the copy engine measured no
// faster).  The entry's previous user, step b - kPack, must have completed.
void gs_runner::pull(int64_t b, int slot_id) {
    using namespace gs;
    PackSlot& slot = streams[b % cfg.n_streams]->slots[slot_id];
    int32_t* d = dev[b % kPack];
    const int64_t n16 = slot.used / 4, tail = slot.used - 4 * n16;
    const int64_t blocks = std::max<int64_t>(1, (n16 + 255) / 256);
    pull_pack_kernel<<<dim3(static_cast<unsigned>(blocks)), 256, 0, side>>>(
        reinterpret_cast<const int4*>(slot.dptr), reinterpret_cast<int4*>(d), n16, slot.dptr + 4 * n16, d + 4 * n16,
        static_cast<int>(tail));
    hip_ok(hipGetLastError(), "pull_pack_kernel");
    hip_ok(hipEventRecord(slot.copied, side), "hipEventRecord");
    pulled_slot[b % kPack] = {static_cast<int>(b % cfg.n_streams), slot_id};
}

// Device sampler: enqueue stream w's next batches, up to dev_depth queued.
void gs_runner::dev_enqueue(int w) {
    using namespace gs;
    std::lock_guard<std::recursive_mutex> lk(dev_mu);
    DevStream& d = dstreams[w];
    while (d.nq < dev_depth) {
        const int64_t b = d.next;
        if (b >= n_units || b >= release_mark.load()) return;
        const int q = d.nq;
        hip_ok(hipEventRecord(d.t0[q], d.st), "hipEventRecord");
        const int rc = gs_dsampler_run(d.ds, roots_dev + b * cfg.batch, cfg.batch, dpack[b % n_dpack], dcap, d.st);
        if (rc != GS_OK) fail(rc, gs_last_error());
        hip_ok(hipEventRecord(d.t1[q], d.st), "hipEventRecord");
        d.qb[q] = b;
        d.qrun[q] = gs_dsampler_runs(d.ds) - 1;
        d.counted[q] = false;
        d.nq = q + 1;
        d.next = b + cfg.n_streams;
    }
}

// Device sampler: batch b's result (hop sizes, layout) into dres[b % ring];
// block == false: false while its sampling is still running.
bool gs_runner::dev_take(int64_t b, bool block) {
    using namespace gs;
    std::lock_guard<std::recursive_mutex> lk(dev_mu);
    DevStream& d = dstreams[b % cfg.n_streams];
    const bool queued = d.nq > 0 && d.qb[0] == b;
    if (!block && (!queued || !dsampler_run_ready(d.ds, d.qrun[0]))) return false;  // not enqueued yet (held) or running
    GS_REQUIRE(queued, GS_EINVAL, "device sampler: batch not enqueued (past the release mark?)");
    const auto tw = Clock::now();
    DevResult& R = dres[b % n_dpack];
    const int rc = gs_dsampler_result_of(d.ds, d.qrun[0], R.hop_sizes, R.offsets, &R.used);
    if (rc != GS_OK) fail(rc, gs_last_error());
    hip_ok(hipEventSynchronize(d.t1[0]), "hipEventSynchronize");
    float ms = 0.f;
    hip_ok(hipEventElapsedTime(&ms, d.t0[0], d.t1[0]), "hipEventElapsedTime");
    R.sample_s = 1e-3 * ms;
    stats.wait_sample_s += secs(tw, Clock::now());
    if (!d.counted[0]) sampled.fetch_add(1);
    // pop the front: every slot moves up one, the freed events to the back
    const hipEvent_t e0 = d.t0[0], e1 = d.t1[0];
    for (int q = 1; q < kDevDepthMax; ++q) {
        d.qb[q - 1] = d.qb[q];
        d.qrun[q - 1] = d.qrun[q];
        d.t0[q - 1] = d.t0[q];
        d.t1[q - 1] = d.t1[q];
        d.counted[q - 1] = d.counted[q];
    }
    d.t0[kDevDepthMax - 1] = e0;
    d.t1[kDevDepthMax - 1] = e1;
    --d.nq;
    return true;
}

// Device sampler: count finished sampling runs (progress()).
void gs_runner::dev_poll() {
    std::lock_guard<std::recursive_mutex> lk(dev_mu);
    for (auto& d : dstreams)
        for (int q = 0; q < d.nq; ++q)
            if (!d.counted[q] && gs::dsampler_run_ready(d.ds, d.qrun[q])) {
                d.counted[q] = true;
                sampled.fetch_add(1);
            }
}

// Device sampler: every stream's state back into its rng (waits for the
// stream's run in flight).
void gs_runner::dev_sync_rngs() {
    using namespace gs;
    for (int w = 0; w < static_cast<int>(dstreams.size()); ++w) {
        DevStream& d = dstreams[w];
        if (!d.ds) continue;
        uint32_t mt[624];
        int64_t pos = 0;
        int rc = gs_dsampler_get_rng(d.ds, mt, &pos, d.st);
        if (rc != GS_OK) fail(rc, gs_last_error());
        rc = gs_rng_set_state(cfg.rngs[w], mt, pos);
        if (rc != GS_OK) fail(rc, gs_last_error());
    }
}

// Pull batch b's pack to the device and gather its layer 1, both on the side
// stream.  block == false: return false if b is not sampled yet.
bool gs_runner::issue(int64_t b, bool block) {
    using namespace gs;
    int slot_id = -1;
    if (devmode) {
        if (!dev_take(b, block)) return false;
    } else {
        slot_id = take_slot(b, block);
        if (slot_id < 0) return false;
    }
    const auto tr = Clock::now();
    const int k = static_cast<int>(b % kDev);
    wait_entry(k);  // batch b-3 done
    stats.wait_ring_s += secs(tr, Clock::now());
    if (devmode) {
        const DevResult& R = dres[b % n_dpack];
        const int rc = gs_trainer_gather(cfg.trainer, dpack[b % n_dpack], R.hop_sizes, R.offsets, k, side);
        if (rc != GS_OK) fail(rc, gs_last_error());
        hip_ok(hipEventRecord(gathered[k], side), "hipEventRecord");
        inflight[k] = {-1, static_cast<int>(b % n_dpack)};
        issued = b + 1;
        // this stream's next batch, b + S, into the ring entry step b - 3 read
        // (wait_entry above saw it complete)
        dev_enqueue(static_cast<int>(b % cfg.n_streams));
        return true;
    }
    pull(b, slot_id);
    const Inflight f = pulled_slot[b % kPack];
    PackSlot& slot = streams[f.stream]->slots[f.slot];
    const int rc = gs_trainer_gather(cfg.trainer, dev[b % kPack], slot.hop_sizes, slot.offsets, k, side);
    if (rc != GS_OK) fail(rc, gs_last_error());
    hip_ok(hipEventRecord(gathered[k], side), "hipEventRecord");
    inflight[k] = f;
    issued = b + 1;
    return true;
}

gs_runner::~gs_runner() {
    if (devmode) {
        for (auto& d : dstreams)
            if (d.st) (void)hipStreamSynchronize(d.st);
        try {
            dev_sync_rngs();
        } catch (...) {
        }
        for (auto& d : dstreams) {
            if (d.ds) gs_dsampler_destroy(d.ds);
            for (int q = 0; q < kDevDepthMax; ++q) {
                if (d.t0[q]) (void)hipEventDestroy(d.t0[q]);
                if (d.t1[q]) (void)hipEventDestroy(d.t1[q]);
            }
            if (d.st) (void)hipStreamDestroy(d.st);
        }
    }
    stop = true;
    for (auto& s : streams) {
        { std::lock_guard<std::mutex> lk(s->mu); }  // a sampler between its predicate check and its wait sees stop
        s->cv.notify_all();
    }
    for (auto& s : streams)
        if (s->th.joinable()) s->th.join();
    for (auto& s : streams) gs_team_destroy(s->team);
    // Device work that may still read the pinned slots or the device rings:
    // the side stream (pull kernels of consumed and of issued-but-unconsumed
    // lookahead batches), the steps in flight and the comm stream.  Drain all
    // of it before any buffer is freed.
    if (side) (void)hipStreamSynchronize(side);
    if (comm_stream) (void)hipStreamSynchronize(comm_stream);
    for (int d = 0; d < kDev; ++d)
        if (dev_busy[d]) (void)hipEventSynchronize(dev_done[d]);
    if (done_host) (void)hipHostFree(done_host);
    for (auto& s : streams)
        for (auto& slot : s->slots) {
            if (slot.copied) {
                (void)hipEventSynchronize(slot.copied);
                (void)hipEventDestroy(slot.copied);
            }
            if (slot.host && slot.thp_bytes) {
                (void)hipHostUnregister(slot.host);
                munmap(slot.host, slot.thp_bytes);
            } else if (slot.host) {
                (void)hipHostFree(slot.host);
            }
        }
    for (int d = 0; d < kPack; ++d)
        if (dev[d]) (void)hipFree(dev[d]);
    for (int32_t* p : dpack)
        if (p) (void)hipFree(p);
    if (roots_dev) (void)hipFree(roots_dev);
    for (int d = 0; d < kDev; ++d) {
        if (dev_done[d]) (void)hipEventDestroy(dev_done[d]);
        if (gathered[d]) (void)hipEventDestroy(gathered[d]);
    }
    if (cfg.trainer && comm_stream) {
        gs::trainer_set_upper_hook(cfg.trainer, {});
        gs::trainer_set_w1_chunk_hook(cfg.trainer, 1, {});
    }
    if (w1_ready) (void)hipEventDestroy(w1_ready);
    if (upper_ready) (void)hipEventDestroy(upper_ready);
    if (upper_reduced) (void)hipEventDestroy(upper_reduced);
    if (comm_stream) (void)hipStreamDestroy(comm_stream);
    if (side) (void)hipStreamDestroy(side);
    if (ws) (void)hipFree(ws);
    if (clip_ws) (void)hipFree(clip_ws);
}

extern "C" {

int gs_comm_unique_id(uint8_t id[128]) {
    GS_API_BEGIN
    GS_REQUIRE(id, GS_EINVAL, "NULL argument");
    static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId size");
    ncclUniqueId u;
    GS_REQUIRE(ncclGetUniqueId(&u) == ncclSuccess, GS_EHIP, "ncclGetUniqueId failed");
    std::memcpy(id, &u, 128);
    GS_API_END
}

int gs_comm_create(const uint8_t id[128], int32_t n_ranks, int32_t rank, void** comm) {
    GS_API_BEGIN
    GS_REQUIRE(id && comm && n_ranks >= 1 && rank >= 0 && rank < n_ranks, GS_EINVAL, "bad arguments");
    ncclUniqueId u;
    std::memcpy(&u, id, 128);
    ncclComm_t c = nullptr;
    const ncclResult_t r = ncclCommInitRank(&c, n_ranks, u, rank);
    GS_REQUIRE(r == ncclSuccess, GS_EHIP, std::string("ncclCommInitRank: ") + ncclGetErrorString(r));
    *comm = c;
    GS_API_END
}

void gs_comm_destroy(void* comm) {
    if (comm) (void)ncclCommDestroy(static_cast<ncclComm_t>(comm));
}

int gs_comm_allreduce_sum(void* comm, float* buf, int64_t n, void* stream) {
    GS_API_BEGIN
    GS_REQUIRE(comm && buf && n >= 0, GS_EINVAL, "bad arguments");
    const ncclResult_t r = ncclAllReduce(buf, buf, static_cast<size_t>(n), ncclFloat32, ncclSum,
                                         static_cast<ncclComm_t>(comm), gs::as_stream(stream));
    GS_REQUIRE(r == ncclSuccess, GS_EHIP, std::string("ncclAllReduce: ") + ncclGetErrorString(r));
    GS_API_END
}

int gs_runner_create(const gs_runner_config* cfg, gs_runner** out) {
    GS_API_BEGIN
    using namespace gs;
    GS_REQUIRE(cfg && out, GS_EINVAL, "NULL argument");
    GS_REQUIRE(cfg->graph && cfg->trainer && cfg->batches && cfg->rngs, GS_EINVAL, "NULL pointer in config");
    GS_REQUIRE(cfg->n_batches >= 1 && cfg->batch >= 1 && cfg->batch < (int64_t(1) << 30), GS_EINVAL,
               "bad batch shape");
    GS_REQUIRE(cfg->n_hops >= 1 && cfg->n_hops <= GS_MAX_HOPS, GS_EINVAL, "n_hops out of [1, 8]");
    GS_REQUIRE(cfg->n_streams >= 1 && cfg->n_streams <= 64 && cfg->depth >= 1 && cfg->depth <= 64, GS_EINVAL,
               "n_streams / depth out of range");
    GS_REQUIRE(cfg->world >= 1 && (cfg->world == 1 || cfg->comm), GS_EINVAL, "world > 1 needs a communicator");
    GS_REQUIRE(!cfg->embed_out || (cfg->embed_ld >= 1 && !cfg->comm), GS_EINVAL,
               "embed_out needs embed_ld >= 1 and no communicator");
    GS_REQUIRE(cfg->merge <= 1 || cfg->embed_out, GS_EINVAL, "merge > 1 is inference only (embed_out)");
    GS_REQUIRE(cfg->helpers >= 0 && cfg->helpers <= 64, GS_EINVAL, "helpers out of [0, 64]");
    for (int32_t w = 0; w < cfg->n_streams; ++w) GS_REQUIRE(cfg->rngs[w], GS_EINVAL, "NULL rng");
    std::unique_ptr<gs_runner> r(new gs_runner());
    r->cfg = *cfg;
    r->fanouts.assign(cfg->fanouts ? cfg->fanouts : nullptr, cfg->fanouts ? cfg->fanouts + cfg->n_hops : nullptr);
    if (r->fanouts.empty()) r->fanouts.assign(cfg->n_hops, 10);
    r->cfg.fanouts = r->fanouts.data();
    r->roots.assign(cfg->batches, cfg->batches + cfg->n_batches * cfg->batch);
    r->cfg.batches = r->roots.data();
    r->merge = std::max<int64_t>(1, std::min<int64_t>(cfg->merge, cfg->n_batches));
    r->n_units = (cfg->n_batches + r->merge - 1) / r->merge;
    const int64_t mb = r->merge * cfg->batch;  // roots per step
    const int64_t bound = gs_sample_pack_bound_multi(cfg->graph, mb, cfg->batch, r->fanouts.data(), cfg->n_hops);
    GS_REQUIRE(bound > 0, GS_EINVAL, "pack bound failed");
    r->cap = bound + mb;
    hip_ok(hipGetDevice(&r->device), "hipGetDevice");
    {  // high priority: the side stream's pull + gather dispatch ahead of the step they overlap
        int lo = 0, hi = 0;
        hip_ok(hipDeviceGetStreamPriorityRange(&lo, &hi), "hipDeviceGetStreamPriorityRange");
        hip_ok(hipStreamCreateWithPriority(&r->side, hipStreamNonBlocking, hi), "hipStreamCreateWithPriority");
    }
    for (int d = 0; d < gs_runner::kDev; ++d) {
        hip_ok(hipEventCreateWithFlags(&r->dev_done[d], sync_event_flags()), "hipEventCreate");
        hip_ok(hipEventCreateWithFlags(&r->gathered[d], sync_event_flags()), "hipEventCreate");
    }
    for (int d = 0; d < gs_runner::kPack; ++d)
        hip_ok(hipMalloc(&r->dev[d], r->cap * sizeof(int32_t)), "hipMalloc(pack)");
    hip_ok(hipMalloc(&r->clip_ws, 64 * 8 * sizeof(float)), "hipMalloc(clip ws)");
    r->use_flag = !cfg->embed_out;
    if (r->use_flag) {
        void* hp = nullptr;
        hip_ok(hipHostMalloc(&hp, 64, hipHostMallocCoherent | hipHostMallocMapped), "hipHostMalloc(done flag)");
        r->done_host = static_cast<int64_t*>(hp);
        *r->done_host = -1;
        void* dp = nullptr;
        hip_ok(hipHostGetDevicePointer(&dp, hp, 0), "hipHostGetDevicePointer");
        r->done_dev = static_cast<int64_t*>(dp);
    }
    {  // layer-1 destinations bound (the last hop's frontier), for the gather slots
        int64_t nn = 0, ne = 0, md = 0;
        GS_REQUIRE(gs_graph_dims(cfg->graph, &nn, &ne, &md) == GS_OK, GS_EINVAL, "gs_graph_dims");
        int64_t nd = cfg->batch;
        for (int32_t j = 0; j + 1 < cfg->n_hops; ++j) {
            const int64_t k = r->fanouts[j];
            const int64_t per = k > 0 ? std::min<int64_t>(k, md) : md;
            nd = std::min<int64_t>(nn, nd + nd * per);
        }
        const int32_t k_last = r->fanouts[cfg->n_hops - 1];  // bounds every last-hop neighbourhood
        const int rc = gs_trainer_gather_reserve(cfg->trainer, nd * r->merge, k_last > 0 ? k_last : 0);
        if (rc != GS_OK) fail(rc, gs_last_error());
        // the fused top launch's padded hop-1 records (2-layer training, fanout <= 31)
        if (!cfg->embed_out && cfg->n_hops == 2 && !(cfg->flags & GS_SAMPLE_GCN) && r->fanouts[0] > 0)
            trainer_reserve_top(cfg->trainer, cfg->batch, r->fanouts[0]);
        // The step workspace at the sampler's worst-case sizes, allocated once:
        // growing it on the first large batch synchronised the stream and
        // stalled that step by ~3 ms inside a measured window.
        int64_t hs[4 * GS_MAX_HOPS] = {};
        int64_t d = cfg->batch * r->merge;
        for (int32_t j = 0; j < cfg->n_hops; ++j) {
            const int64_t k = r->fanouts[j];
            const int64_t per = k > 0 ? std::min<int64_t>(k, md) : md;
            const int64_t np = d * per, ns = std::min<int64_t>(nn, d + np);
            hs[4 * j] = d;
            hs[4 * j + 1] = np;
            hs[4 * j + 2] = ns;
            hs[4 * j + 3] = np;
            d = ns;
        }
        const int64_t need = gs_trainer_ws_bytes(cfg->trainer, hs);
        GS_REQUIRE(need >= 0, GS_EINVAL, gs_last_error());
        r->ws_bytes = need + (1 << 20);
        hip_ok(hipMalloc(&r->ws, r->ws_bytes), "hipMalloc(ws)");
    }
    const int32_t S = cfg->n_streams;
    r->devmode = cfg->device_sampler != 0;
    if (r->devmode) {
        GS_REQUIRE(r->merge == 1, GS_EINVAL, "device_sampler: merge must be 1");
        GS_REQUIRE(!(cfg->flags & GS_SAMPLE_FULL), GS_EINVAL, "device_sampler: no GS_SAMPLE_FULL");
        std::vector<int32_t> r32(r->roots.size());
        for (size_t i = 0; i < r32.size(); ++i) {
            GS_REQUIRE(r->roots[i] >= 0 && r->roots[i] < (int64_t(1) << 31), GS_ERANGE, "root id out of range");
            r32[i] = static_cast<int32_t>(r->roots[i]);
        }
        hip_ok(hipMalloc(&r->roots_dev, r32.size() * sizeof(int32_t)), "hipMalloc(roots)");
        hip_ok(hipMemcpy(r->roots_dev, r32.data(), r32.size() * sizeof(int32_t), hipMemcpyHostToDevice), "hipMemcpy");
        r->dstreams.resize(S);
        for (int32_t w = 0; w < S; ++w) {
            gs_runner::DevStream& d = r->dstreams[w];
            hip_ok(hipStreamCreateWithFlags(&d.st, hipStreamNonBlocking), "hipStreamCreate(dsampler)");
            for (int q = 0; q < gs_runner::kDevDepthMax; ++q) {
                hip_ok(hipEventCreate(&d.t0[q]), "hipEventCreate");
                hip_ok(hipEventCreate(&d.t1[q]), "hipEventCreate");
            }
            int rc = gs_dsampler_create(cfg->graph, r->fanouts.data(), cfg->n_hops, cfg->batch,
                                        (cfg->flags & (GS_SAMPLE_GCN | GS_SAMPLE_FAIL_EMPTY)) |
                                            (S > 1 ? GS_DSAMPLER_NO_AUX : 0),
                                        &d.ds);
            if (rc != GS_OK) fail(rc, gs_last_error());
            uint32_t mt[624];
            int64_t pos = 0;
            rc = gs_rng_get_state(cfg->rngs[w], mt, &pos);
            if (rc != GS_OK) fail(rc, gs_last_error());
            rc = gs_dsampler_set_rng(d.ds, mt, pos, d.st);
            if (rc != GS_OK) fail(rc, gs_last_error());
            d.next = w;
        }
        r->dcap = std::max<int64_t>(r->cap, gs_dsampler_pack_bound(r->dstreams[0].ds, cfg->batch));
        r->dev_depth = gs_runner::kDevDepthMax;
        r->n_dpack = r->dev_depth * S + 3;
        r->dpack.assign(r->n_dpack, nullptr);
        for (auto& p : r->dpack) hip_ok(hipMalloc(&p, r->dcap * sizeof(int32_t)), "hipMalloc(pack)");
        r->dres.resize(r->n_dpack);
    }
    // GS_SHARED_HELPERS=1: one pool of S x helpers threads behind all the
    // streams' teams (a stream's set builds take the helpers the others leave
    // idle) instead of helpers private to each stream.
    const char* shared_env = std::getenv("GS_SHARED_HELPERS");
    const bool shared_helpers = shared_env && std::atoi(shared_env) == 1;
    // pack slots on transparent huge pages: the pull kernel's host reads then
    // need one translation per 2 MiB instead of per 4 KiB page (pull kernel
    // 13.26 -> 12.63 us)
    for (int32_t w = 0; w < S && !r->devmode; ++w) {
        auto s = std::make_unique<SamplerStream>();
        s->rng = cfg->rngs[w];
        if (cfg->helpers > 0) {
            const int rc = shared_helpers && w > 0 ? gs_team_create_shared(r->streams[0]->team, &s->team)
                                                   : gs_team_create(shared_helpers ? cfg->helpers * S : cfg->helpers,
                                                                    &s->team);
            if (rc != GS_OK) fail(GS_EINVAL, gs_last_error());
        }
        for (int64_t b = w; b < r->n_units; b += S) s->batches.push_back(b);
        s->slots.resize(cfg->depth);
        for (int32_t q = 0; q < cfg->depth; ++q) {
            PackSlot& sl = s->slots[q];
            {  // the slot on transparent huge pages (madvise), registered
                constexpr size_t kHuge = size_t(2) << 20;
                const size_t bytes = (r->cap * sizeof(int32_t) + kHuge - 1) / kHuge * kHuge;
                void* p = mmap(nullptr, bytes + kHuge, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
                if (p == MAP_FAILED) fail(GS_ENOMEM, "mmap(pack slot)");
                // a 2 MiB-aligned window of the mapping; the rest goes back
                const uintptr_t a = (reinterpret_cast<uintptr_t>(p) + kHuge - 1) / kHuge * kHuge;
                const size_t head = a - reinterpret_cast<uintptr_t>(p);
                if (head) munmap(p, head);
                if (kHuge - head) munmap(reinterpret_cast<char*>(a) + bytes, kHuge - head);
                (void)madvise(reinterpret_cast<void*>(a), bytes, MADV_HUGEPAGE);
                std::memset(reinterpret_cast<void*>(a), 0, bytes);
                sl.host = reinterpret_cast<int32_t*>(a);
                sl.thp_bytes = bytes;
                hip_ok(hipHostRegister(sl.host, bytes, hipHostRegisterMapped), "hipHostRegister(pack slot)");
                void* dp = nullptr;
                hip_ok(hipHostGetDevicePointer(&dp, sl.host, 0), "hipHostGetDevicePointer");
                sl.dptr = static_cast<int32_t*>(dp);
            }
            hip_ok(hipEventCreateWithFlags(&s->slots[q].copied, sync_event_flags()), "hipEventCreate");
            s->free.push_back(q);
        }
        r->streams.push_back(std::move(s));
    }
    r->release_mark = cfg->hold ? 0 : INT64_MAX;
    for (int32_t w = 0; w < S && r->devmode; ++w) r->dev_enqueue(w);
    if (cfg->comm && cfg->ar_buckets == 2 && !cfg->embed_out && cfg->n_hops >= 2) {
        hip_ok(hipStreamCreateWithFlags(&r->comm_stream, hipStreamNonBlocking), "hipStreamCreate(comm)");
        hip_ok(hipEventCreateWithFlags(&r->upper_ready, hipEventDisableTiming), "hipEventCreate");
        hip_ok(hipEventCreateWithFlags(&r->upper_reduced, hipEventDisableTiming), "hipEventCreate");
        gs_runner* rp = r.get();
        trainer_set_upper_hook(cfg->trainer, [rp](hipStream_t st) {
            const int64_t w1 = trainer_w1_floats(rp->cfg.trainer);
            const int64_t n = gs_trainer_n_params(rp->cfg.trainer);
            hip_ok(hipEventRecord(rp->upper_ready, st), "hipEventRecord");
            hip_ok(hipStreamWaitEvent(rp->comm_stream, rp->upper_ready, 0), "hipStreamWaitEvent");
            const int rc = gs_comm_allreduce_sum(rp->cfg.comm, gs_trainer_grads(rp->cfg.trainer) + w1, n - w1,
                                                 rp->comm_stream);
            if (rc != GS_OK) fail(rc, gs_last_error());
        });
        const char* ch_env = std::getenv("GS_AR_W1_CHUNKS");
        const int chunks = ch_env ? std::atoi(ch_env) : 2;
        if (chunks > 1) {
            hip_ok(hipEventCreateWithFlags(&r->w1_ready, hipEventDisableTiming), "hipEventCreate");
            trainer_set_w1_chunk_hook(cfg->trainer, chunks, [rp](hipStream_t st, int64_t off, int64_t n) {
                // same comm stream, after the upper bucket: every rank issues
                // the collectives on one communicator in one stream order
                hip_ok(hipEventRecord(rp->w1_ready, st), "hipEventRecord");
                hip_ok(hipStreamWaitEvent(rp->comm_stream, rp->w1_ready, 0), "hipStreamWaitEvent");
                const int rc = gs_comm_allreduce_sum(rp->cfg.comm, gs_trainer_grads(rp->cfg.trainer) + off, n,
                                                     rp->comm_stream);
                if (rc != GS_OK) fail(rc, gs_last_error());
                ++rp->w1_issued;
            });
        }
    }
    for (auto& s : r->streams) {
        SamplerStream* sp = s.get();
        gs_runner* rp = r.get();
        s->th = std::thread([rp, sp] { rp->sampler_loop(*sp); });
    }
    if (cfg->warm && !r->devmode) {
        std::unique_lock<std::mutex> lk(r->warm_mu);
        r->warm_cv.wait(lk, [&] { return r->warmed == static_cast<int>(r->streams.size()); });
    }
    *out = r.release();
    GS_API_END
}

int gs_runner_run(gs_runner* r, int64_t n_steps, float* loss, void* stream) {
    GS_API_BEGIN
    using namespace gs;
    GS_REQUIRE(r && (loss || r->cfg.embed_out) && n_steps >= 0, GS_EINVAL, "bad arguments");
    GS_REQUIRE(r->next_batch + n_steps <= r->n_units, GS_ERANGE, "runner has fewer batches left");
    GS_REQUIRE(r->next_batch + n_steps <= r->release_mark, GS_EINVAL,
               "steps past the release mark (gs_runner_release) would wait forever");
    hipStream_t st = as_stream(stream);
    const int64_t n_params = gs_trainer_n_params(r->cfg.trainer);
    float* grads = gs_trainer_grads(r->cfg.trainer);
    // If a step throws (e.g. MAX over an empty neighbourhood in take_slot),
    // the steps issued before it signal completion only through the pinned
    // flag: record an event on the step stream for every ring entry still
    // pending, so the destructor drains them before freeing what they read.
    struct Unwind {
        gs_runner* r;
        hipStream_t st;
        bool armed = true;
        ~Unwind() {
            gs::g_done_flag = {};  // never left for a later SGD launch of this thread
            if (!armed) return;
            for (int k = 0; k < gs_runner::kDev; ++k)
                if (r->flag_step[k] >= 0 && hipEventRecord(r->dev_done[k], st) == hipSuccess) {
                    r->flag_step[k] = -1;
                    r->dev_busy[k] = true;
                }
        }
    } unwind{r, st};
    struct KeepLowp {  // the SGD keeps the bf16 W1 current for this loop's steps only
        gs_trainer* t;
        explicit KeepLowp(gs_trainer* t_) : t(t_) {
            if (t) gs::trainer_keep_lowp(t, true);
        }
        ~KeepLowp() {
            if (t) gs::trainer_keep_lowp(t, false);
        }
    } keep_lowp{r->cfg.trainer};
    // Each step's clip + SGD is deferred into the next step's launches (W1's
    // update for clip coefficient 1 written by the last slab sum, or with a
    // communicator by the norm launch after the all-reduce; the next layer-1
    // forward applies the update) instead of a launch between the steps; the
    // loop's end applies the last one (trainer option GS_TOPT_DEFER_UPDATE = 0: off).
    struct DeferUpdate {
        gs_trainer* t;
        hipStream_t st;
        bool on = false;
        DeferUpdate(gs_trainer* t_, hipStream_t s, bool comm) : t(t_), st(s) {
            if (t) on = gs::trainer_defer_update(t, true, st, comm);
        }
        ~DeferUpdate() {
            if (!on) return;
            try {
                gs::trainer_defer_update(t, false, st);
            } catch (const gs::Error& e) {
                std::fprintf(stderr, "graphsage_amd: runner: applying the last deferred update failed: %s\n", e.what());
            }
        }
    } defer_update{r->cfg.trainer && !r->cfg.embed_out ? r->cfg.trainer : nullptr, st, r->cfg.comm != nullptr};
    for (int64_t step = 0; step < n_steps; ++step) {
        const int64_t b = r->next_batch;
        const auto t0 = Clock::now();
        for (auto& o : r->streams) r->recycle(*o, false);
        if (r->issued <= b) {
            ++r->stats.lookahead_misses;
            r->issue(b, true);
        }
        // look ahead: batch b+1's pull + gather run on the side stream under
        // this step (never block here: with a slow sampler that would idle the GPU)
        if (b + 1 < r->n_units && r->issued == b + 1) r->issue(b + 1, false);
        const int k = static_cast<int>(b % gs_runner::kDev);
        const auto tg = Clock::now();
        hip_ok(hipEventSynchronize(r->gathered[k]), "hipEventSynchronize");  // normally long done
        const auto t1 = Clock::now();
        r->stats.wait_gather_s += secs(tg, t1);
        const gs::Inflight f = r->inflight[k];
        const int64_t* hop_sizes;
        const int64_t* offsets;
        int64_t used;
        double sample_s;
        if (r->devmode) {
            const gs_runner::DevResult& R = r->dres[f.slot];
            hop_sizes = R.hop_sizes;
            offsets = R.offsets;
            used = R.used;
            sample_s = R.sample_s;
        } else {
            const PackSlot& slot = r->streams[f.stream]->slots[f.slot];
            hop_sizes = slot.hop_sizes;
            offsets = slot.offsets;
            used = slot.used;
            sample_s = slot.sample_s;
        }
        const auto t2 = t1;
        const int64_t need = gs_trainer_ws_bytes(r->cfg.trainer, hop_sizes);
        GS_REQUIRE(need >= 0, GS_EINVAL, gs_last_error());
        if (need > r->ws_bytes) {
            hip_ok(hipStreamSynchronize(st), "hipStreamSynchronize");
            if (r->ws) hip_ok(hipFree(r->ws), "hipFree");
            r->ws = nullptr;
            r->ws_bytes = need + need / 4 + (1 << 20);
            hip_ok(hipMalloc(&r->ws, r->ws_bytes), "hipMalloc(ws)");
        }
        const int64_t pack_total = used - r->cfg.batch;
        bool consumed_flag = false;
        int32_t* pk = r->devmode ? r->dpack[f.slot] : r->dev[b % gs_runner::kPack];
        auto t3 = Clock::now();
        if (r->cfg.embed_out) {  // inference: the forward into this batch's output rows
            const int rc = gs_trainer_forward_gathered(r->cfg.trainer, pk, hop_sizes, offsets, k, r->ws,
                                                       r->ws_bytes,
                                                       r->cfg.embed_out + b * r->merge * r->cfg.batch * r->cfg.embed_ld,
                                                       st);
            if (rc != GS_OK) fail(rc, gs_last_error());
            t3 = Clock::now();
        } else {
            // the done flag goes to the step's SGD launch: the fused slab sum
            // inside the step, or gs_trainer_update* below
            if (r->use_flag) g_done_flag = {r->done_dev, b};
            r->w1_issued = 0;
            int rc = gs_trainer_forward_backward_gathered(r->cfg.trainer, pk, hop_sizes, offsets,
                                                          pk + pack_total, r->cfg.batch, k, r->ws, r->ws_bytes, loss,
                                                          st);
            if (rc != GS_OK) fail(rc, gs_last_error());
            t3 = Clock::now();
            // with a communicator (any world size, so one rank exercises the same
            // path): sum the gradients, then clip the averaged sum; without one
            // the clip uses the norm partials of the step's own reductions
            if (r->cfg.comm && r->comm_stream) {
                // bucketed: the upper gradients went out on comm_stream under the
                // layer-1 dW GEMM; W1's collective follows them on the SAME stream,
                // so every rank issues the two collectives on one communicator in
                // one stream order (not by host issue order across two streams)
                if (r->w1_issued == 0) {  // W1 in one piece (the trainer's unchunked path)
                    hip_ok(hipEventRecord(r->upper_ready, st), "hipEventRecord");  // dW1 final
                    hip_ok(hipStreamWaitEvent(r->comm_stream, r->upper_ready, 0), "hipStreamWaitEvent");
                    rc = gs_comm_allreduce_sum(r->cfg.comm, grads, trainer_w1_floats(r->cfg.trainer), r->comm_stream);
                    if (rc != GS_OK) fail(rc, gs_last_error());
                }
                hip_ok(hipEventRecord(r->upper_reduced, r->comm_stream), "hipEventRecord");
                hip_ok(hipStreamWaitEvent(st, r->upper_reduced, 0), "hipStreamWaitEvent");
            } else if (r->cfg.comm) {
                rc = gs_comm_allreduce_sum(r->cfg.comm, grads, n_params, st);
                if (rc != GS_OK) fail(rc, gs_last_error());
            }
            rc = r->cfg.comm
                     ? gs_trainer_update(r->cfg.trainer, 1.0f / static_cast<float>(r->cfg.world), r->clip_ws, st)
                     : gs_trainer_update_local(r->cfg.trainer, st);
            consumed_flag = r->use_flag && g_done_flag.ptr == nullptr;
            g_done_flag = {};
            if (rc != GS_OK) fail(rc, gs_last_error());
        }
        if (consumed_flag) {
            r->flag_step[k] = b;  // its SGD signals the entry free
            r->dev_busy[k] = false;
        }
        if (!consumed_flag || step + 1 == n_steps) {
            hip_ok(hipEventRecord(r->dev_done[k], st), "hipEventRecord");  // ring entry k free again
            r->dev_busy[k] = true;
        }
        for (int q = 0; q < 4 * GS_MAX_HOPS; ++q) r->stats.hop_sizes[q] += static_cast<double>(hop_sizes[q]);
        r->stats.sample_s += sample_s;
        if (!r->devmode) r->streams[f.stream]->copying.push_back(f.slot);
        ++r->next_batch;
        ++r->stats.steps;
        const auto t4 = Clock::now();
        r->stats.wait_s += secs(t0, t1);
        r->stats.issue_s += secs(t1, t4);
        r->stats.fwd_bwd_s += secs(t2, t3);
        r->stats.update_s += secs(t3, t4);
        r->stats.max_step_s = std::max(r->stats.max_step_s, secs(t0, t4));
    }
    if (defer_update.on) {  // the last step's update, errors reported here (the destructor covers unwinding)
        defer_update.on = false;
        gs::trainer_defer_update(defer_update.t, false, st);
    }
    unwind.armed = false;
    GS_API_END
}

int gs_runner_stats_get(const gs_runner* r, gs_runner_stats* out) {
    GS_API_BEGIN
    GS_REQUIRE(r && out, GS_EINVAL, "NULL argument");
    *out = r->stats;
    GS_API_END
}

void gs_runner_stats_reset(gs_runner* r) {
    if (r) r->stats = gs_runner_stats{};
}

int gs_runner_release(gs_runner* r, int64_t mark) {
    GS_API_BEGIN
    GS_REQUIRE(r && mark >= r->release_mark.load(), GS_EINVAL, "release mark may only grow");
    r->release_mark = mark;
    for (auto& s : r->streams) {
        { std::lock_guard<std::mutex> lk(s->mu); }
        s->cv.notify_all();
    }
    for (int w = 0; w < static_cast<int>(r->dstreams.size()); ++w) r->dev_enqueue(w);
    GS_API_END
}

int gs_runner_sync_rngs(gs_runner* r) {
    GS_API_BEGIN
    GS_REQUIRE(r, GS_EINVAL, "NULL argument");
    if (r->devmode) r->dev_sync_rngs();
    GS_API_END
}

int gs_runner_progress(const gs_runner* r, int64_t* sampled, int64_t* consumed) {
    GS_API_BEGIN
    GS_REQUIRE(r && sampled && consumed, GS_EINVAL, "NULL argument");
    if (r->devmode) const_cast<gs_runner*>(r)->dev_poll();
    *sampled = r->sampled.load();
    *consumed = r->next_batch;
    GS_API_END
}

void gs_runner_destroy(gs_runner* r) { delete r; }

}  // extern "C"
