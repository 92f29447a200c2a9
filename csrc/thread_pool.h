// Persistent host worker pool for the block codec and the other data-parallel host passes.
//
// Spawning std::threads per call (the first version) made the 8,300-tx block decode SLOWER with more
// threads: every fresh thread gets a fresh malloc arena, and first-touch page faults of those arenas
// serialise on the process's mmap lock. The workers here live for the whole process (arenas stay
// warm), rows are handed out in contiguous chunks from one atomic counter (no false sharing between
// neighbouring outputs, dynamic balance across uneven txs), and the calling thread works too.
#pragma once

#include <string>
#include <pthread.h>
#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <exception>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

#include <unistd.h>

namespace upow {

class HostPool {
public:
    static HostPool& get() {
        static HostPool pool;
        return pool;
    }

    // f(i) for i in [0, n) on up to `threads` threads (caller included). Not re-entrant.
    template <typename F>
    void parallel_for(int64_t n, int threads, F&& f) {
        threads = int(std::max<int64_t>(1, std::min<int64_t>({int64_t(threads), n, int64_t(kMaxThreads)})));
        if (threads == 1 || n < 64) {
            for (int64_t i = 0; i < n; ++i) f(i);
            return;
        }
        std::lock_guard<std::mutex> serial(call_mu_);  // one parallel region at a time
        ensure_workers(threads - 1);
        const int64_t chunk = std::max<int64_t>(16, n / (int64_t(threads) * 8));
        std::function<void(int64_t)> body = [&f](int64_t i) { f(i); };
        {
            std::lock_guard<std::mutex> g(mu_);
            body_ = &body;
            n_ = n;
            chunk_ = chunk;
            next_.store(0, std::memory_order_relaxed);
            active_ = threads - 1;
            wanted_ = threads - 1;
            ++generation_;
        }
        cv_.notify_all();
        drain();
        std::unique_lock<std::mutex> lk(mu_);
        done_cv_.notify_all();
        done_cv_.wait(lk, [&] { return active_ == 0; });
        body_ = nullptr;
        if (error_) {  // first exception of any participant, rethrown on the calling thread
            std::exception_ptr e = error_;
            error_ = nullptr;
            std::rethrow_exception(e);
        }
    }

    ~HostPool() {
        {
            std::lock_guard<std::mutex> g(mu_);
            stop_ = true;
            ++generation_;
        }
        cv_.notify_all();
        for (auto& t : workers_) t.join();
    }

private:
    static constexpr int kMaxThreads = 32;

    void drain() {
        try {
            for (;;) {
                const int64_t b = next_.fetch_add(chunk_, std::memory_order_relaxed);
                if (b >= n_) return;
                const int64_t e = std::min(n_, b + chunk_);
                for (int64_t i = b; i < e; ++i) (*body_)(i);
            }
        } catch (...) {
            std::lock_guard<std::mutex> g(mu_);
            if (!error_) error_ = std::current_exception();
            next_.store(n_, std::memory_order_relaxed);  // the others stop at their next chunk
        }
    }

    void ensure_workers(int k) {
        if (pid_ != getpid()) {  // forked child: the parent's workers do not exist here
            new std::vector<std::thread>(std::move(workers_));  // deliberately leaked, never joined
            workers_.clear();
            pid_ = getpid();
        }
        while (int(workers_.size()) < k) {
            const int id = int(workers_.size());
            uint64_t gen;
            {
                std::lock_guard<std::mutex> g(mu_);
                gen = generation_;  // start from the current region: never replay an old one
            }
            workers_.emplace_back([this, id, gen] { loop(id, gen); });
        }
    }

    void loop(int id, uint64_t seen) {
        pthread_setname_np(pthread_self(), ("upow-pool-" + std::to_string(id)).c_str());
        for (;;) {
            {
                std::unique_lock<std::mutex> lk(mu_);
                cv_.wait(lk, [&] { return stop_ || generation_ != seen; });
                if (stop_) return;
                seen = generation_;
                if (id >= wanted_) continue;  // this region uses fewer threads
            }
            drain();
            std::lock_guard<std::mutex> g(mu_);
            if (--active_ == 0) done_cv_.notify_all();
        }
    }

    std::mutex call_mu_, mu_;
    std::condition_variable cv_, done_cv_;
    std::vector<std::thread> workers_;
    std::function<void(int64_t)>* body_ = nullptr;
    int64_t n_ = 0, chunk_ = 1;
    std::atomic<int64_t> next_{0};
    int active_ = 0, wanted_ = 0;
    uint64_t generation_ = 0;
    bool stop_ = false;
    std::exception_ptr error_;
    pid_t pid_ = getpid();
};

}  // namespace upow
