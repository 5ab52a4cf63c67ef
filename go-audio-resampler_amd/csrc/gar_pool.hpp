// gar_pool.hpp -- the host worker pool of the large host C-ABI calls (gar_engine.cpp forSlices).
// Header-only so the TSan stress test (tools/pool_tsan.cpp) builds it without the HIP runtime.
#pragma once
#include <immintrin.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace gar {

// Host worker pool for packing / unpacking large host C-ABI calls (one job split over
// min(15, cores - 1) workers + the caller); small calls run inline.  Workers spin for ~100 us
// after a job before sleeping (a streaming host call hands the pool two jobs, pack and unpack, a few
// hundred microseconds apart; a futex wake per job and worker cost tens of microseconds), and job
// completion is an atomic count.
class Pool {
   public:
    static Pool& get() {
        static Pool p;
        return p;
    }
    void run(int n, const std::function<void(int)>& f) {
        // one job at a time: handles are independent, so a second thread's call must not
        // overwrite a running job; when the pool is busy that caller runs its job inline
        std::unique_lock<std::mutex> owner(runMu_, std::try_to_lock);
        if (n <= 1 || n > kMaxJobs || th_.empty() || !owner.owns_lock()) {
            for (int i = 0; i < n; ++i) f(i);
            return;
        }
        uint64_t g;
        {
            std::lock_guard<std::mutex> lk(mu_);
            job_.store(&f);
            pending_.store(n);
            g = (genOf(ticket_.load()) + 1) & kGenMask;
            // publishes the job: generation g, its job count and next index 0 in ONE word, so a
            // worker's CAS checks all three together (with the count in a separate
            // atomic, a worker holding the previous generation's ticket could read the new count)
            ticket_.store(g << 40 | static_cast<uint64_t>(n) << 20);
            cv_.notify_all();
        }
        work(g);
        if (!spinUntil([&] { return pending_.load() == 0; })) {
            std::unique_lock<std::mutex> lk(mu_);
            done_.wait(lk, [&] { return pending_.load() == 0; });
        }
    }
    int workers() const { return static_cast<int>(th_.size()) + 1; }

   private:
    Pool() {
        const unsigned hw = std::thread::hardware_concurrency();
        const int n = std::max(0, std::min<int>(15, static_cast<int>(hw) - 1));
        for (int i = 0; i < n; ++i) th_.emplace_back([this] { loop(); });
    }
    ~Pool() {
        {
            std::lock_guard<std::mutex> lk(mu_);
            stop_.store(true);
        }
        cv_.notify_all();
        for (auto& t : th_) t.join();
    }
    template <class P>
    static bool spinUntil(P pred) {  // up to ~100 us
        const auto t0 = std::chrono::steady_clock::now();
        for (int k = 0;; ++k) {
            if (pred()) return true;
            _mm_pause();
            if ((k & 255) == 255 && std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(100)) return false;
        }
    }
    // Ticket word: generation (24 bits) << 40 | job count (20 bits) << 20 | next index (20 bits).
    static constexpr int kMaxJobs = (1 << 20) - 1;
    static constexpr uint64_t kGenMask = (uint64_t(1) << 24) - 1;
    static uint64_t genOf(uint64_t t) { return t >> 40; }
    // Claims indices of generation g only (a worker that woke late for a finished job must not
    // take an index of the next one): the CAS succeeds only on a ticket of generation g whose
    // index is below that generation's own job count, and job_ is read only after it.
    void work(uint64_t g) {
        for (;;) {
            uint64_t t = ticket_.load();
            for (;;) {
                if (genOf(t) != g || (t & 0xfffffu) >= ((t >> 20) & 0xfffffu)) return;
                if (ticket_.compare_exchange_weak(t, t + 1)) break;
            }
            (*job_.load())(static_cast<int>(t & 0xfffffu));
            if (pending_.fetch_sub(1) == 1) {
                std::lock_guard<std::mutex> lk(mu_);
                done_.notify_all();
            }
        }
    }
    void loop() {
        uint64_t seen = 0;
        for (;;) {
            if (!spinUntil([&] { return stop_.load() || genOf(ticket_.load()) != seen; })) {
                std::unique_lock<std::mutex> lk(mu_);
                cv_.wait(lk, [&] { return stop_.load() || genOf(ticket_.load()) != seen; });
            }
            if (stop_.load()) return;
            seen = genOf(ticket_.load());
            work(seen);
        }
    }
    std::vector<std::thread> th_;
    std::mutex runMu_;  // held by the caller whose job the workers run
    std::mutex mu_;
    std::condition_variable cv_, done_;
    std::atomic<const std::function<void(int)>*> job_{nullptr};
    std::atomic<int> pending_{0};
    std::atomic<uint64_t> ticket_{0};  // generation << 40 | job count << 20 | next job index
    std::atomic<bool> stop_{false};
};

}  // namespace gar
