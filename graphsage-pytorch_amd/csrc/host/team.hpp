// Helper threads of one sampler stream.  A batch's sampling is sequential
// where the reference's RNG stream and set-iteration order make it so (the
// draws, the frontier union), but its per-node set builds and the
// neighbour-list / transpose construction of a hop are independent of the
// RNG: those run on the helpers, the latter concurrently with the next hop's
// draws.  Only the owning sampler thread submits work.
//
// A job is a handful of coarse tasks, taken under the mutex (so a helper that
// wakes late finds either the finished job or the next one fully set up).
// Helpers spin briefly on a generation counter (a batch submits several jobs
// tens of microseconds apart), then sleep on the condition variable.
#pragma once

#include <immintrin.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <exception>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace gs {

class Team {
  public:
    // spin_us: how long a helper polls for the next job before sleeping on
    // the condition variable, in microseconds of wall time (a pause count
    // spans 4-10x different times on different CPUs).  A sampler stream's
    // jobs come every ~0.1-0.3 ms, so its helpers stay awake between them
    // (a futex wake-up at each batch's set builds cost tens of microseconds);
    // 0 for a caller whose jobs come once per step: idle helpers then leave
    // the cores to the other host threads at once.
    explicit Team(int helpers, int spin_us = 500) : spin_us_(spin_us) {
        for (int i = 0; i < helpers; ++i) th_.emplace_back([this] { loop(); });
    }
    ~Team() {
        {
            std::lock_guard<std::mutex> lk(mu_);
            stop_ = true;
            gen_.fetch_add(1);
        }
        cv_.notify_all();
        for (auto& t : th_) t.join();
    }
    Team(const Team&) = delete;
    Team& operator=(const Team&) = delete;

    int helpers() const { return static_cast<int>(th_.size()); }

    // Tasks 0..n-1 of fn start on the helpers; the caller continues.  At most
    // one job is outstanding: wait() before the next start().
    void start(int n, std::function<void(int)> fn) {
        {
            std::lock_guard<std::mutex> lk(mu_);
            fn_ = std::move(fn);
            n_ = n;
            next_ = 0;
            done_.store(0, std::memory_order_relaxed);
            gen_.fetch_add(1, std::memory_order_release);
        }
        cv_.notify_all();
    }

    // The caller takes the job's remaining tasks too, then waits for the rest
    // (all of them have returned when this does).  A task that threw counts
    // as returned; the first such exception is rethrown here, once every task
    // is done (nothing of the job is still running when the caller unwinds).
    // A job whose tasks make no progress for kStallSeconds is a bug (a task
    // that never returns): it is reported on stderr and the process aborts,
    // rather than hanging silently or unwinding while helpers still run.
    static constexpr int kStallSeconds = 120;
    void wait() {
        work();
        int seen = done_.load(std::memory_order_acquire);
        auto t_seen = std::chrono::steady_clock::now();
        for (uint64_t spin = 0; seen < n_; ++spin) {
            _mm_pause();
            const int now = done_.load(std::memory_order_acquire);
            if (now != seen) {
                seen = now;
                t_seen = std::chrono::steady_clock::now();
            } else if ((spin & 0xFFFFF) == 0xFFFFF &&
                       std::chrono::steady_clock::now() - t_seen > std::chrono::seconds(kStallSeconds)) {
                std::fprintf(stderr, "graphsage_amd: sampler helper team stalled: %d of %d tasks done, no progress "
                                     "for %d s; aborting\n", seen, n_, kStallSeconds);
                std::abort();
            }
        }
        std::exception_ptr e;
        {
            std::lock_guard<std::mutex> lk(mu_);
            std::swap(e, err_);
        }
        if (e) std::rethrow_exception(e);
    }

    // start() + wait(): the caller is one more worker.
    void parallel_for(int n, std::function<void(int)> fn) {
        start(n, std::move(fn));
        wait();
    }

  private:
    void work() {
        for (;;) {
            int i;
            {
                std::lock_guard<std::mutex> lk(mu_);
                if (next_ >= n_) return;
                i = next_++;
            }
            try {
                fn_(i);  // fn_ is replaced only after every task has returned
            } catch (...) {
                std::lock_guard<std::mutex> lk(mu_);
                if (!err_) err_ = std::current_exception();
            }
            done_.fetch_add(1, std::memory_order_release);
        }
    }

    void loop() {
        uint64_t seen = gen_.load();
        for (;;) {
            uint64_t g = gen_.load(std::memory_order_acquire);
            if (g == seen && spin_us_ > 0) {
                const auto until = std::chrono::steady_clock::now() + std::chrono::microseconds(spin_us_);
                for (uint32_t spin = 1; g == seen; ++spin) {
                    _mm_pause();
                    g = gen_.load(std::memory_order_acquire);
                    if ((spin & 255) == 0 && std::chrono::steady_clock::now() > until) break;
                }
            }
            if (g == seen) {
                std::unique_lock<std::mutex> lk(mu_);
                cv_.wait(lk, [&] { return gen_.load() != seen; });
                g = gen_.load();
            }
            seen = g;
            {
                std::lock_guard<std::mutex> lk(mu_);
                if (stop_) return;
            }
            work();
        }
    }

    std::vector<std::thread> th_;
    std::function<void(int)> fn_;
    std::exception_ptr err_;  // the job's first task exception (guarded by mu_)
    int n_ = 0, next_ = 0;  // guarded by mu_
    std::atomic<int> done_{0};
    std::atomic<uint64_t> gen_{0};
    std::mutex mu_;
    std::condition_variable cv_;
    bool stop_ = false;
    int spin_us_;
};

}  // namespace gs
