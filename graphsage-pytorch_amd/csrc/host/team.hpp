// Helper threads of the host sampler.  A batch's sampling is sequential
// where the reference's RNG stream and set-iteration order make it so (the
// draws, the frontier union), but its per-node set builds and the
// neighbour-list / transpose construction of a hop are independent of the
// RNG: those run on helpers, the latter concurrently with the next hop's
// draws.
//
// A Pool owns the helper threads; a Team is one submitter's handle on a pool
// (its own private pool, or one pool shared by all the sampler streams of a
// runner, so a stream's set builds can take the helpers its neighbours leave
// idle).  A job is a handful of coarse tasks, claimed under the pool mutex (a
// helper that wakes late finds either a finished job or a fully set-up one).
// Helpers take the first posted job with unclaimed tasks, spin a while on a
// generation counter when there is none (a stream submits a job every
// ~0.1 ms), then sleep on the condition variable.
#pragma once

#include <immintrin.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <exception>
#include <functional>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

namespace gs {

class Pool {
  public:
    struct Job {
        std::function<void(int)> fn;
        int n = 0, next = 0;     // guarded by the pool mutex
        std::atomic<int> done{0};
        std::exception_ptr err;  // the job's first task exception (guarded by the pool mutex)
    };

    // spin_us: how long an idle helper polls for the next job before sleeping,
    // in microseconds of wall time (a pause count spans 4-10x different times
    // on different CPUs); 0 for callers whose jobs come once per step (idle
    // helpers then leave the cores to the other host threads at once).
    Pool(int threads, int spin_us) : spin_us_(spin_us) {
        for (int i = 0; i < threads; ++i) th_.emplace_back([this] { loop(); });
    }
    ~Pool() {
        {
            std::lock_guard<std::mutex> lk(mu_);
            stop_ = true;
            gen_.fetch_add(1);
        }
        cv_.notify_all();
        for (auto& t : th_) t.join();
    }
    Pool(const Pool&) = delete;
    Pool& operator=(const Pool&) = delete;

    int threads() const { return static_cast<int>(th_.size()); }

    void post(Job* j, int n, std::function<void(int)> fn) {
        {
            std::lock_guard<std::mutex> lk(mu_);
            j->fn = std::move(fn);
            j->n = n;
            j->next = 0;
            j->err = nullptr;
            j->done.store(0, std::memory_order_relaxed);
            jobs_.push_back(j);
            gen_.fetch_add(1, std::memory_order_release);
        }
        cv_.notify_all();
    }

    // Run j's unclaimed tasks on the calling thread.
    void run_own(Job* j) {
        for (;;) {
            int i;
            {
                std::lock_guard<std::mutex> lk(mu_);
                if (j->next >= j->n) return;
                i = j->next++;
            }
            run(j, i);
        }
    }

    // j has completed (done == n): no helper touches it again.
    std::exception_ptr retire(Job* j) {
        std::lock_guard<std::mutex> lk(mu_);
        for (size_t q = 0; q < jobs_.size(); ++q)
            if (jobs_[q] == j) {
                jobs_.erase(jobs_.begin() + static_cast<std::ptrdiff_t>(q));
                break;
            }
        std::exception_ptr e;
        std::swap(e, j->err);
        return e;
    }

  private:
    void run(Job* j, int i) {
        try {
            j->fn(i);  // fn is replaced only after the job is retired
        } catch (...) {
            std::lock_guard<std::mutex> lk(mu_);
            if (!j->err) j->err = std::current_exception();
        }
        j->done.fetch_add(1, std::memory_order_release);
    }

    // A task of the oldest posted job that has one left (under the mutex).
    bool take(Job*& j, int& i) {
        for (Job* c : jobs_)
            if (c->next < c->n) {
                j = c;
                i = c->next++;
                return true;
            }
        return false;
    }

    void loop() {
        uint64_t seen = gen_.load();
        for (;;) {
            Job* j = nullptr;
            int i = 0;
            bool got;
            {
                std::lock_guard<std::mutex> lk(mu_);
                if (stop_) return;
                got = take(j, i);
                if (!got) seen = gen_.load();
            }
            if (got) {
                run(j, i);
                continue;
            }
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
                cv_.wait(lk, [&] { return stop_ || gen_.load() != seen; });
            }
        }
    }

    std::vector<std::thread> th_;
    std::vector<Job*> jobs_;  // posted, not yet retired (guarded by mu_)
    std::atomic<uint64_t> gen_{0};
    std::mutex mu_;
    std::condition_variable cv_;
    bool stop_ = false;
    int spin_us_;
};

class Team {
  public:
    // A private pool of `helpers` threads.  Sampler jobs come every
    // ~0.1-0.3 ms, so its helpers stay awake between them by default (a futex
    // wake-up at each batch's set builds cost tens of microseconds).
    explicit Team(int helpers, int spin_us = 500)
        : pool_(helpers > 0 ? std::make_shared<Pool>(helpers, spin_us) : nullptr) {}
    // A handle on a pool shared with other submitters (the runner's streams).
    explicit Team(std::shared_ptr<Pool> pool) : pool_(std::move(pool)) {}
    Team(const Team&) = delete;
    Team& operator=(const Team&) = delete;

    int helpers() const { return pool_ ? pool_->threads() : 0; }
    const std::shared_ptr<Pool>& pool() const { return pool_; }

    // Tasks 0..n-1 of fn start on the helpers; the caller continues.  At most
    // one job of this handle is outstanding: wait() before the next start().
    void start(int n, std::function<void(int)> fn) { pool_->post(&job_, n, std::move(fn)); }

    // The caller takes the job's unclaimed tasks too, then waits for the rest
    // (all of them have returned when this does).  A task that threw counts
    // as returned; the first such exception is rethrown here, once every task
    // is done (nothing of the job is still running when the caller unwinds).
    // A job whose tasks make no progress for kStallSeconds is a bug (a task
    // that never returns): it is reported on stderr and the process aborts,
    // rather than hanging silently or unwinding while helpers still run.
    static constexpr int kStallSeconds = 120;
    void wait() {
        pool_->run_own(&job_);
        const int n = job_.n;  // set by this thread's start()
        int seen = job_.done.load(std::memory_order_acquire);
        auto t_seen = std::chrono::steady_clock::now();
        for (uint64_t spin = 0; seen < n; ++spin) {
            _mm_pause();
            const int now = job_.done.load(std::memory_order_acquire);
            if (now != seen) {
                seen = now;
                t_seen = std::chrono::steady_clock::now();
            } else if ((spin & 0xFFFFF) == 0xFFFFF &&
                       std::chrono::steady_clock::now() - t_seen > std::chrono::seconds(kStallSeconds)) {
                std::fprintf(stderr, "graphsage_amd: sampler helper team stalled: %d of %d tasks done, no progress "
                                     "for %d s; aborting\n", seen, n, kStallSeconds);
                std::abort();
            }
        }
        if (std::exception_ptr e = pool_->retire(&job_)) std::rethrow_exception(e);
    }

    // start() + wait(): the caller is one more worker.
    void parallel_for(int n, std::function<void(int)> fn) {
        start(n, std::move(fn));
        wait();
    }

  private:
    std::shared_ptr<Pool> pool_;
    Pool::Job job_;
};

}  // namespace gs
