// sts_stage_pool.hpp -- a bounded, process-wide pool of staging slot sets (sts_host.cpp).
//
// Spark runs N executor task threads in one JVM, each calling the `_host` entry points
// (S/TimeSeriesRDD.scala:417-421: compute() per partition, one task thread each; SURVEY.md
// §5 "the JNI layer must be reentrant").  Executors recycle their task threads, so staging
// state owned by a thread (round 2: a thread_local slot set of 5 x 64 MB HBM + 5 x 64 MB
// pinned memory, freed only by an explicit sts_staging_release) grew with the number of
// threads that ever called and leaked with every retired thread.  Here a call BORROWS a
// whole slot set for its duration and returns it afterwards:
//   * at most `cap` sets exist per device (sts_staging_set_limit; default kDefaultSets), so
//     staging memory is bounded whatever the thread count; a call that finds every set
//     borrowed waits for one (PCIe is shared anyway: more concurrent pipelines than sets
//     would not move more bytes);
//   * idle sets stay allocated for the next call (no hipMalloc / hipHostMalloc per call);
//     trim() (sts_staging_release) frees the idle ones;
//   * nothing is thread-local, so a retired thread leaves nothing behind.
// The pool is generic over the set type and its create / destroy functions so that the CPU
// harness (tests/native/stage_pool_tsan.cpp) can drive it under ThreadSanitizer with fake
// sets; sts_host.cpp instantiates it with HIP streams, events and buffers.
#pragma once

#include <condition_variable>
#include <mutex>
#include <vector>

namespace sts {

template <class Set>
class StagePool {
  public:
    using Create = int (*)(int dev, Set** out);   // 0 = ok, else a status (set is not created)
    using Destroy = void (*)(Set* s);
    static constexpr int kMaxDevices = 64;

    StagePool(Create c, Destroy d, int cap) : create_(c), destroy_(d), cap_(cap < 1 ? 1 : cap) {}
    StagePool(const StagePool&) = delete;
    StagePool& operator=(const StagePool&) = delete;

    // Borrow a set for device `dev`: an idle one, else a new one while fewer than cap
    // exist, else wait until one is given back.  Returns create()'s status on failure.
    int acquire(int dev, Set** out) {
        *out = nullptr;
        if (dev < 0 || dev >= kMaxDevices) return -1;
        std::unique_lock<std::mutex> lk(m_);
        Dev& d = dev_[dev];
        for (;;) {
            if (!d.idle.empty()) {
                *out = d.idle.back();
                d.idle.pop_back();
                d.borrowed++;
                return 0;
            }
            if (d.live < cap_) break;
            d.waits++;
            cv_.wait(lk);
        }
        d.live++;   // reserve the slot in the count, create outside the lock
        d.borrowed++;
        if (d.live > d.high) d.high = d.live;
        lk.unlock();
        Set* s = nullptr;
        const int r = create_(dev, &s);
        if (r != 0) {
            lk.lock();
            d.live--;
            d.borrowed--;
            lk.unlock();
            cv_.notify_all();
            return r;
        }
        *out = s;
        return 0;
    }

    // Return a borrowed set (every transfer on it complete).
    void give_back(int dev, Set* s) {
        {
            std::lock_guard<std::mutex> lk(m_);
            Dev& d = dev_[dev];
            d.borrowed--;
            if (d.live > cap_) {   // the limit was lowered while it was out
                d.live--;
                d.dying.push_back(s);
            } else {
                d.idle.push_back(s);
            }
        }
        cv_.notify_all();
        reap_dying(dev);
    }

    // A borrowed set whose transfers could not be confirmed complete (device error): it is
    // neither reused nor freed (freeing memory a DMA may still target is worse than leaking it).
    void forget(int dev) {
        {
            std::lock_guard<std::mutex> lk(m_);
            Dev& d = dev_[dev];
            d.borrowed--;
            d.live--;
            d.lost++;
        }
        cv_.notify_all();
    }

    // Free every idle set of every device; returns how many were freed.
    int trim() {
        std::vector<Set*> v;
        {
            std::lock_guard<std::mutex> lk(m_);
            for (Dev& d : dev_) {
                d.live -= (int)d.idle.size();
                v.insert(v.end(), d.idle.begin(), d.idle.end());
                d.idle.clear();
            }
        }
        for (Set* s : v) destroy_(s);
        cv_.notify_all();
        return (int)v.size();
    }

    // Change the per-device limit (>= 1).  Idle sets beyond it are freed now, borrowed ones
    // when they come back.
    int set_cap(int cap) {
        if (cap < 1) return -1;
        std::vector<Set*> v;
        {
            std::lock_guard<std::mutex> lk(m_);
            cap_ = cap;
            for (Dev& d : dev_)
                while (d.live > cap_ && !d.idle.empty()) {
                    v.push_back(d.idle.back());
                    d.idle.pop_back();
                    d.live--;
                }
        }
        for (Set* s : v) destroy_(s);
        cv_.notify_all();
        return 0;
    }

    struct Info {
        int live, idle, borrowed, cap, high, lost;
        long long waits;
    };
    Info info(int dev) {
        std::lock_guard<std::mutex> lk(m_);
        if (dev < 0 || dev >= kMaxDevices) return Info{0, 0, 0, cap_, 0, 0, 0};
        const Dev& d = dev_[dev];
        return Info{d.live, (int)d.idle.size(), d.borrowed, cap_, d.high, d.lost, d.waits};
    }

  private:
    struct Dev {
        std::vector<Set*> idle, dying;
        int live = 0, borrowed = 0, high = 0, lost = 0;
        long long waits = 0;
    };
    void reap_dying(int dev) {
        std::vector<Set*> v;
        {
            std::lock_guard<std::mutex> lk(m_);
            v.swap(dev_[dev].dying);
        }
        for (Set* s : v) destroy_(s);
    }

    Create create_;
    Destroy destroy_;
    std::mutex m_;
    std::condition_variable cv_;
    Dev dev_[kMaxDevices];
    int cap_;
};

}  // namespace sts
