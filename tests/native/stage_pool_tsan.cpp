// ThreadSanitizer driver for the staging slot-set pool (TEST INFRASTRUCTURE ONLY;
// tests/test_sanitizers.py).  spark-timeseries_amd/csrc/sts_stage_pool.hpp is compiled for
// the host with fake sets (no HIP) and hammered by many threads the way Spark's executor
// task threads call the `_host` entry points (S/TimeSeriesRDD.scala:417-421):
//   * a borrowed set is never held by two threads at once (owner word per set);
//   * at most `cap` sets are alive per device, whatever the thread count, also while the cap
//     is lowered and raised and idle sets are trimmed concurrently;
//   * failed creations and forgotten sets keep the count right;
//   * every created set is destroyed exactly once by the end (trim), none twice.
// Prints "ok" and exits 0 on success.
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <thread>
#include <vector>

#include "sts_stage_pool.hpp"

namespace {

struct FakeSet {
    int dev;
    std::atomic<int> owner{-1};
    long long payload = 0;   // written by the borrower only: TSan flags any unsynchronised sharing
};

std::atomic<int> g_alive[4];
std::atomic<int> g_created{0}, g_destroyed{0}, g_fail_next{0};
std::atomic<int> g_failures{0};
std::atomic<int> g_cap_now{3};

int create(int dev, FakeSet** out) {
    if (g_fail_next.fetch_sub(1) > 0) return 7;   // an injected creation failure
    auto* s = new FakeSet;
    s->dev = dev;
    g_alive[dev]++;
    g_created++;
    *out = s;
    return 0;
}

void destroy(FakeSet* s) {
    if (s->owner.load() != -1) {
        std::printf("FAIL destroyed while borrowed\n");
        g_failures++;
    }
    g_alive[s->dev]--;
    g_destroyed++;
    delete s;
}

}  // namespace

int main(int argc, char** argv) {
    const int nthreads = argc > 1 ? std::atoi(argv[1]) : 16;
    const int iters = argc > 2 ? std::atoi(argv[2]) : 400;
    sts::StagePool<FakeSet> pool(create, destroy, 3);
    std::atomic<int> forgotten{0};
    std::vector<std::thread> th;
    for (int t = 0; t < nthreads; t++) {
        th.emplace_back([&, t] {
            std::mt19937 rng(1234 + t);
            for (int i = 0; i < iters; i++) {
                const int dev = (int)(rng() % 2);
                if (t == 0 && i % 50 == 25) {   // one thread moves the limit and trims meanwhile
                    const int cap = 1 + (int)(rng() % 4);
                    pool.set_cap(cap);
                    g_cap_now = cap;
                    pool.trim();
                    continue;
                }
                if (rng() % 97 == 0) g_fail_next = 1;
                FakeSet* s = nullptr;
                const int r = pool.acquire(dev, &s);
                if (r != 0) {
                    if (r != 7) {
                        std::printf("FAIL acquire status %d\n", r);
                        g_failures++;
                    }
                    continue;
                }
                int expect = -1;
                if (!s->owner.compare_exchange_strong(expect, t)) {
                    std::printf("FAIL set shared by threads %d and %d\n", expect, t);
                    g_failures++;
                }
                s->payload += t;   // exclusive use
                if (rng() % 3 == 0) std::this_thread::sleep_for(std::chrono::microseconds(rng() % 50));
                // the pool's own view never exceeds the largest limit in use
                const auto in = pool.info(dev);
                if (in.live > 4 || in.borrowed > in.live + 0) {
                    std::printf("FAIL live %d borrowed %d\n", in.live, in.borrowed);
                    g_failures++;
                }
                s->owner = -1;
                if (rng() % 211 == 0) {   // a device error: the set is abandoned, not reused
                    forgotten++;
                    pool.forget(dev);
                    destroy(s);   // (the real pool leaks it; the harness frees it to count it)
                    continue;
                }
                pool.give_back(dev, s);
            }
        });
    }
    for (auto& x : th) x.join();
    for (int d = 0; d < 2; d++) {
        const auto in = pool.info(d);
        if (in.borrowed != 0 || in.live != in.idle || in.high > 4 || in.lost < 0) {
            std::printf("FAIL dev %d end state live %d idle %d borrowed %d high %d\n", d, in.live, in.idle, in.borrowed,
                        in.high);
            g_failures++;
        }
    }
    pool.trim();
    for (int d = 0; d < 2; d++) {
        if (pool.info(d).live != 0 || g_alive[d].load() != 0) {
            std::printf("FAIL dev %d: %d sets alive after trim (pool says %d)\n", d, g_alive[d].load(),
                        pool.info(d).live);
            g_failures++;
        }
    }
    if (g_created.load() != g_destroyed.load()) {
        std::printf("FAIL created %d destroyed %d\n", g_created.load(), g_destroyed.load());
        g_failures++;
    }
    if (g_failures.load()) return 1;
    std::printf("ok created=%d forgotten=%d\n", g_created.load(), forgotten.load());
    return 0;
}
