// workers.hpp — the host mirror's worker pool (aeron_cluster_amd.cpp), in a header of its own so
// that tests/cpp/test_workers.cpp can stress it on the CPU.
//
// A fixed set of threads (AERON_AMD_HOST_THREADS, default min(16, cores)) runs the tasks of one
// parallel_for at a time; the calling thread takes tasks too.  A second caller arriving while a loop
// runs executes its own loop inline (the mirror's entry points are reentrant across threads, like
// the reference's static codec functions).
//
// Small loops are cheaper: a loop of T tasks wakes at most T - 1 workers (the others sleep on), and
// the caller waits for the tasks it did not run by watching a counter.  A worker that finished a
// loop can watch for the next one for AERON_AMD_SPIN_US microseconds before it sleeps (default 0:
// on a GPU box whose process gets 16 cores, 15 spinning helpers took the cores the HIP runtime's
// own threads needed, and 1 K-record calls got slower, profiles/r04_host_latency_pool.log against
// r04_host_latency_pool_nospin.log).
#pragma once

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstdlib>
#include <exception>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace aeron_cluster {
namespace detail {

inline void cpu_relax() {
#if defined(__x86_64__) || defined(__i386__)
    __builtin_ia32_pause();
#else
    std::this_thread::yield();
#endif
}

class Workers {
public:
    static Workers& get() {
        static Workers* w = new Workers(default_threads());  // never destroyed: the threads outlive static teardown
        return *w;
    }
    static unsigned default_threads() {
        unsigned n = std::min(16u, std::max(1u, std::thread::hardware_concurrency()));
        if (const char* e = std::getenv("AERON_AMD_HOST_THREADS")) n = (unsigned)std::max(1, std::atoi(e));
        return n;
    }
    // a pool of `n` threads in all (n - 1 workers and the caller); tests make their own
    explicit Workers(unsigned n, int spin_us = -1) {
        if (spin_us < 0) {
            spin_us = 0;
            if (const char* e = std::getenv("AERON_AMD_SPIN_US")) spin_us = std::max(0, std::atoi(e));
        }
        spin_ = std::chrono::microseconds(spin_us);
        for (unsigned i = 1; i < n; ++i) threads_.emplace_back([this] { loop(); });
        for (auto& t : threads_) t.detach();
    }
    Workers(const Workers&) = delete;
    Workers& operator=(const Workers&) = delete;
    unsigned size() const { return (unsigned)threads_.size() + 1; }

    // fn(t) for every t in [0, ntasks), on the caller and up to ntasks - 1 workers; rethrows the
    // first exception a task threw once every task has finished
    template <class F>
    void parallel_for(size_t ntasks, F&& fn) {
        if (ntasks == 0) return;
        std::unique_lock<std::mutex> call(call_m_, std::try_to_lock);
        if (ntasks == 1 || threads_.empty() || !call.owns_lock()) {
            for (size_t t = 0; t < ntasks; ++t) fn(t);
            return;
        }
        std::function<void(size_t)> job(std::forward<F>(fn));
        const unsigned helpers = (unsigned)std::min<size_t>(ntasks - 1, threads_.size());
        unsigned wake = 0;
        {
            std::lock_guard<std::mutex> g(m_);
            job_ = &job;
            ntasks_ = ntasks;
            next_.store(0, std::memory_order_relaxed);
            finished_.store(0, std::memory_order_relaxed);
            seats_ = helpers;
            gen_.fetch_add(1, std::memory_order_release);  // spinning workers see this without a wake
            wake = std::min(helpers, sleeping_);
        }
        for (unsigned i = 0; i < wake; ++i) cv_.notify_one();
        run_tasks(job, ntasks);
        // the tasks the workers took: they are running, so the wait is short
        while (finished_.load(std::memory_order_acquire) < ntasks) cpu_relax();
        std::unique_lock<std::mutex> g(m_);
        job_ = nullptr;
        seats_ = 0;
        // a worker that took a seat may still be on its way out of run_tasks (it holds `job`)
        done_cv_.wait(g, [&] { return seated_ == 0; });
        if (err_) {
            std::exception_ptr e = err_;
            err_ = nullptr;
            std::rethrow_exception(e);
        }
    }

private:
    void run_tasks(const std::function<void(size_t)>& job, size_t ntasks) {
        for (size_t t; (t = next_.fetch_add(1, std::memory_order_relaxed)) < ntasks;) {
            try {
                job(t);
            } catch (...) {
                std::lock_guard<std::mutex> g(m_);
                if (!err_) err_ = std::current_exception();
            }
            finished_.fetch_add(1, std::memory_order_release);
        }
    }
    void loop() {
        uint64_t seen = gen_.load(std::memory_order_acquire);
        for (;;) {
            // watch for the next loop for spin_, then sleep until one is posted
            const auto t0 = std::chrono::steady_clock::now();
            uint32_t k = 0;
            while (gen_.load(std::memory_order_acquire) == seen) {
                cpu_relax();
                if ((++k & 63) == 0 && std::chrono::steady_clock::now() - t0 > spin_) break;
            }
            const std::function<void(size_t)>* job = nullptr;
            size_t ntasks = 0;
            {
                std::unique_lock<std::mutex> g(m_);
                if (gen_.load(std::memory_order_relaxed) == seen) {
                    ++sleeping_;
                    cv_.wait(g, [&] { return gen_.load(std::memory_order_relaxed) != seen; });
                    --sleeping_;
                }
                seen = gen_.load(std::memory_order_relaxed);
                if (!job_ || seats_ == 0) continue;  // finished already, or enough helpers joined
                --seats_;
                ++seated_;
                job = job_;
                ntasks = ntasks_;
            }
            run_tasks(*job, ntasks);
            std::lock_guard<std::mutex> g(m_);
            if (--seated_ == 0) done_cv_.notify_all();
        }
    }
    std::vector<std::thread> threads_;
    std::chrono::microseconds spin_{50};
    std::mutex call_m_, m_;
    std::condition_variable cv_, done_cv_;
    const std::function<void(size_t)>* job_ = nullptr;  // guarded by m_
    size_t ntasks_ = 0;                                 // guarded by m_
    unsigned seats_ = 0, seated_ = 0, sleeping_ = 0;     // guarded by m_
    // each on a cache line of its own: the spinning workers read gen_ while the tasks count
    alignas(64) std::atomic<uint64_t> gen_{0};
    alignas(64) std::atomic<size_t> next_{0};
    alignas(64) std::atomic<size_t> finished_{0};
    std::exception_ptr err_;                            // guarded by m_
};

}  // namespace detail
}  // namespace aeron_cluster
