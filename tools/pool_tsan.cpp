// pool_tsan.cpp -- ThreadSanitizer stress test of the host worker pool (csrc/gar_pool.hpp).
// Several caller threads run jobs back to back with different job counts (the ADVICE r05 case: a
// worker holding a stale ticket of the previous job must not claim an index of the next one), and
// every job checks that each index ran exactly once and that nothing runs after run() returns.
//   make -C go-audio-resampler_amd tsan   (builds and runs it; exit status 0 = clean)
#include <cstdio>
#include <vector>

#include "gar_pool.hpp"

int main() {
    gar::Pool& pool = gar::Pool::get();
    std::atomic<long> bad{0};
    auto caller = [&](int t) {
        for (int it = 0; it < 400; ++it) {
            // alternate small and large job counts per caller, different per thread
            const int n = 2 + ((it * 7 + t * 13) % (it & 1 ? 40 : 5));
            std::vector<int> hits(static_cast<size_t>(n), 0);  // plain ints: TSan flags any race on them
            std::atomic<int> live{0};
            pool.run(n, [&](int i) {
                live.fetch_add(1);
                if (i < 0 || i >= n) { bad.fetch_add(1); return; }
                hits[static_cast<size_t>(i)] += 1;
                live.fetch_sub(1);
            });
            if (live.load() != 0) bad.fetch_add(1);  // a job index still running after run() returned
            for (int i = 0; i < n; ++i) bad.fetch_add(hits[static_cast<size_t>(i)] != 1);
        }
    };
    std::vector<std::thread> th;
    for (int t = 1; t < 4; ++t) th.emplace_back(caller, t);
    caller(0);
    for (auto& x : th) x.join();
    std::printf("pool_tsan: %ld bad\n", bad.load());
    return bad.load() == 0 ? 0 : 1;
}
