// sts_host.cpp -- host-buffer entry points (the JNI path): a PINNED
// STAGING PIPELINE in front of the device entry points.
//
// A `_host` call is split by series into chunks of ~kChunkBytes of device traffic.  Each
// chunk runs H2D -> kernel(s) -> D2H on one of kSlots slots, each slot owning a HIP stream,
// a device buffer and pinned bounce buffers, all reused across calls.  While chunk i's
// kernel runs, later chunks upload and earlier ones download (one stream per slot), and the calling
// thread fills the next slot's bounce buffer: copy, compute and the CPU side overlap.
//
// Host memory that is already pinned (hipHostMalloc'd, e.g. by sts_host_alloc -- the JNI
// shim copies a Java array straight into such a buffer with GetDoubleArrayRegion) is moved
// by DMA directly, with no bounce copy; pageable memory goes through the slot's pinned
// buffer (one CPU copy, the same one hipMemcpy would make internally, but overlapped).
//
// Every device entry point runs on the slot's stream; per-series statuses always go to a
// device array and come back with the chunk, so a NULL err_per_series keeps the reference's
// exception semantics (the first failing series becomes the return status after all
// chunks) without a synchronisation per chunk.
//
// Reentrancy and memory (round 3).  A call BORROWS a whole slot set from a process-wide pool
// (sts_stage_pool.hpp) for its duration: at most sts_staging_set_limit() sets per device
// (default kDefaultSets = 4, i.e. at most 4 x 5 x 64 MB of HBM and as much pinned memory
// however many executor threads call), a call finding every set borrowed waits for one, and
// nothing is owned by a thread, so retired threads leak nothing.  A call never returns while
// a transfer of its own is in flight: every exit path (success, a HIP error in the middle of
// the pipeline, a failing kernel) drains the set's busy slots first, and a slot whose kernel
// or copy-out did not run is never copied to the caller.  sts_staging_release frees the idle
// sets.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <functional>
#include <vector>

#include "sts_internal.hpp"
#include "sts_stage_pool.hpp"

namespace {

// Pipeline shape (A/B on C2 from pinned host memory, profiles/r02_v6_ab_staging.jsonl): 2-D
// copies on 5 slots 78 ms per call, 3 slots 87 ms, 4 slots 94 ms; linear copies for
// contiguous rows were bimodal run to run (56-112 ms), so the 2-D form stays.
#ifndef STS_STAGE_LINEAR
#define STS_STAGE_LINEAR 0
#endif
#ifndef STS_STAGE_SLOTS
#define STS_STAGE_SLOTS 5
#define STS_STAGE_MB 64
#endif
constexpr int kSlots = STS_STAGE_SLOTS;
constexpr size_t kChunkBytes = size_t(STS_STAGE_MB) << 20;   // device bytes (in + out) per chunk
constexpr size_t kAlign = 256;
constexpr int kDefaultSets = 4;                                // slot sets per device (sts_staging_set_limit)
// what a slot keeps between calls: one chunk plus the per-argument alignment; a call whose single
// series is larger than a chunk grows its slots for that call only (Borrow trims them again)
constexpr size_t kSlotKeep = kChunkBytes + 16 * kAlign;

size_t align_up(size_t b) { return (b + kAlign - 1) / kAlign * kAlign; }

struct Slot {
    hipStream_t st = nullptr;
    hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};   // before H2D, after H2D, after kernel, after D2H
    void* dev = nullptr;
    size_t dev_cap = 0;
    void* pin = nullptr;
    size_t pin_cap = 0;
    bool busy = false;       // ev[3] recorded for a chunk not yet reaped
    bool copy_out = false;   // its kernel and D2H copies were enqueued: pageable outputs may be copied
    int64_t s0 = 0, ns = 0;
};

struct SlotSet {
    int device = -1;
    Slot slot[kSlots];
};

// statistics of this thread's last _host call (sts_staging_stats)
struct Stats {
    double h2d_ms = 0, kernel_ms = 0, d2h_ms = 0, wall_ms = 0;
    double bytes_h2d = 0, bytes_d2h = 0, chunks = 0, direct = 0;   // bytes moved by direct DMA
};
thread_local Stats g_stats;

int hip_status(hipError_t e, const char* where) {
    char buf[256];
    snprintf(buf, sizeof buf, "%s: %s", where, hipGetErrorString(e));
    return sts::set_error(STS_ERR_HIP, buf);
}

void destroy_set(SlotSet* g) {
    int cur = -1;
    const bool switch_dev = hipGetDevice(&cur) == hipSuccess && cur != g->device;
    if (switch_dev) (void)hipSetDevice(g->device);
    for (Slot& s : g->slot) {
        if (s.st) (void)hipStreamSynchronize(s.st);
        if (s.dev) (void)hipFree(s.dev);
        if (s.pin) (void)hipHostFree(s.pin);
        for (hipEvent_t& e : s.ev)
            if (e) (void)hipEventDestroy(e);
        if (s.st) (void)hipStreamDestroy(s.st);
    }
    if (switch_dev) (void)hipSetDevice(cur);
    delete g;
}

int create_set(int dev, SlotSet** out) {
    SlotSet* g = new SlotSet;
    g->device = dev;
    hipError_t e = hipSuccess;
    for (Slot& s : g->slot) {
        if ((e = hipStreamCreateWithFlags(&s.st, hipStreamNonBlocking)) != hipSuccess) break;
        for (hipEvent_t& ev : s.ev)
            if ((e = hipEventCreate(&ev)) != hipSuccess) break;
        if (e != hipSuccess) break;
    }
    if (e != hipSuccess) {
        const int r = hip_status(e, "staging: stream / event");
        destroy_set(g);
        return r;
    }
    *out = g;
    return STS_OK;
}

// never destroyed: at process exit the HIP runtime may already be gone, and the OS reclaims
sts::StagePool<SlotSet>& pool() {
    static sts::StagePool<SlotSet>* p = new sts::StagePool<SlotSet>(create_set, destroy_set, kDefaultSets);
    return *p;
}

// A borrowed set; on destruction (every exit path of staged()) all its busy slots are
// drained WITHOUT copying to the caller, then it goes back to the pool -- or, when a drain
// fails (device error), it is forgotten rather than reused or freed under a live DMA.
struct Borrow {
    SlotSet* set = nullptr;
    int dev = -1;
    ~Borrow() {
        if (!set) return;
        bool ok = true;
        for (Slot& sl : set->slot) {
            if (sl.busy && hipEventSynchronize(sl.ev[3]) != hipSuccess) ok = false;
            if (sl.st && hipStreamSynchronize(sl.st) != hipSuccess) ok = false;   // a partly enqueued chunk
            sl.busy = false;
            sl.copy_out = false;
        }
        // a set goes back to the pool at its bound (kSlots x kSlotKeep of HBM and of pinned
        // memory): buffers a one-series-larger-than-a-chunk call grew are freed here (drained above)
        if (ok)
            for (Slot& sl : set->slot) {
                if (sl.dev_cap > kSlotKeep) {
                    (void)hipFree(sl.dev);
                    sl.dev = nullptr;
                    sl.dev_cap = 0;
                }
                if (sl.pin_cap > kSlotKeep) {
                    (void)hipHostFree(sl.pin);
                    sl.pin = nullptr;
                    sl.pin_cap = 0;
                }
            }
        if (ok) pool().give_back(dev, set);
        else pool().forget(dev);
    }
};

bool is_pinned(const void* p) {
    if (!p) return false;
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();   // pageable memory: clear the sticky lookup error
        return false;
    }
    return a.type == hipMemoryTypeHost;
}

// One per-series array of a _host call.  On the device, chunk rows are contiguous (`row`
// bytes per series); on the host, series s starts at s * hstride.
struct Arg {
    const void* src = nullptr;   // host input (copied in), or nullptr
    void* dst = nullptr;         // host output (copied out), or nullptr; == src for in place
    size_t row = 0;              // device bytes per series
    size_t hstride = 0;          // host bytes between series
    bool pinned_src = false, pinned_dst = false;
    size_t dev_off = 0, pin_off = 0;   // per-slot layout (set per chunk size)
};

Arg in_arg(const void* p, size_t row, size_t hstride) {
    Arg a;
    a.src = p;
    a.row = row;
    a.hstride = hstride;
    return a;
}
Arg out_arg(void* p, size_t row, size_t hstride) {
    Arg a;
    a.dst = p;
    a.row = row;
    a.hstride = hstride;
    return a;
}
Arg inout_arg(void* p, size_t row, size_t hstride) {
    Arg a;
    a.src = p;
    a.dst = p;
    a.row = row;
    a.hstride = hstride;
    return a;
}

// kernel(device pointers per arg (chunk-local, row-contiguous), first series, series, stream)
using Kernel = std::function<int(void* const* dev, int64_t s0, int64_t ns, hipStream_t st)>;

void copy_rows(void* dst, size_t dstride, const void* src, size_t sstride, size_t row, int64_t n) {
    if (dstride == row && sstride == row) {
        std::memcpy(dst, src, row * (size_t)n);
        return;
    }
    for (int64_t i = 0; i < n; i++)
        std::memcpy(static_cast<char*>(dst) + (size_t)i * dstride, static_cast<const char*>(src) + (size_t)i * sstride,
                    row);
}

// Wait for a slot's chunk, account its time, copy its pageable outputs to the caller (only
// when its kernel and copy-out were enqueued).
int reap(Slot& sl, std::vector<Arg>& args) {
    if (!sl.busy) return STS_OK;
    hipError_t e = hipEventSynchronize(sl.ev[3]);
    if (e != hipSuccess) return hip_status(e, "staging: chunk");   // stays busy: Borrow drains it
    sl.busy = false;
    Stats& g = g_stats;
    float a = 0, b = 0, c = 0;
    if (hipEventElapsedTime(&a, sl.ev[0], sl.ev[1]) == hipSuccess) g.h2d_ms += a;
    if (hipEventElapsedTime(&b, sl.ev[1], sl.ev[2]) == hipSuccess) g.kernel_ms += b;
    if (hipEventElapsedTime(&c, sl.ev[2], sl.ev[3]) == hipSuccess) g.d2h_ms += c;
    if (!sl.copy_out) return STS_OK;
    sl.copy_out = false;
    for (Arg& x : args)
        if (x.dst && !x.pinned_dst)
            copy_rows(static_cast<char*>(x.dst) + (size_t)sl.s0 * x.hstride, x.hstride,
                      static_cast<char*>(sl.pin) + x.pin_off, x.row, x.row, sl.ns);
    return STS_OK;
}

// Run `kern` over S series in chunks through a borrowed slot set.
int staged(int64_t S, std::vector<Arg> args, const Kernel& kern) {
    const auto t_start = std::chrono::steady_clock::now();
    Stats& g = g_stats;
    g = Stats();
    int r;
    // the device entry point's own argument checks first, on the caller's shapes and host
    // pointers (never dereferenced in validate-only mode): no staging on bad input
    {
        void* hp[16];
        for (size_t k = 0; k < args.size() && k < 16; k++)
            hp[k] = const_cast<void*>(args[k].src ? args[k].src : static_cast<const void*>(args[k].dst));
        if ((r = sts::validate([&] { return kern(hp, 0, S, nullptr); }))) return r;
    }
    if (S <= 0) return STS_OK;
    Borrow bw;
    {
        hipError_t e = hipGetDevice(&bw.dev);
        if (e != hipSuccess) return hip_status(e, "hipGetDevice");
        if ((r = pool().acquire(bw.dev, &bw.set))) return r > 0 ? r : sts::set_error(STS_ERR_BAD_ARG, "staging: device id");
    }
    Slot* slots = bw.set->slot;
    size_t per_series = 0;
    for (Arg& x : args) {
        x.pinned_src = is_pinned(x.src);
        x.pinned_dst = (x.dst == x.src) ? x.pinned_src : is_pinned(x.dst);
        per_series += x.row;
    }
    int64_t ns = per_series ? (int64_t)(kChunkBytes / per_series) : S;
    ns = std::max<int64_t>(1, std::min<int64_t>(ns, S));
    // per-slot layout: one device region per arg; one pinned region per pageable in / out
    size_t dev_bytes = 0, pin_bytes = 0;
    for (Arg& x : args) {
        x.dev_off = dev_bytes;
        dev_bytes += align_up(x.row * (size_t)ns);
        x.pin_off = pin_bytes;
        if ((x.src && !x.pinned_src) || (x.dst && !x.pinned_dst)) pin_bytes += align_up(x.row * (size_t)ns);
    }
    hipError_t e;
    for (int k = 0; k < kSlots; k++) {
        Slot& sl = slots[k];
        if (sl.dev_cap < dev_bytes) {
            if (sl.dev) (void)hipFree(sl.dev);
            sl.dev = nullptr;
            sl.dev_cap = 0;
            if ((e = hipMalloc(&sl.dev, dev_bytes)) != hipSuccess) return hip_status(e, "staging: hipMalloc");
            sl.dev_cap = dev_bytes;
        }
        if (sl.pin_cap < pin_bytes) {
            if (sl.pin) (void)hipHostFree(sl.pin);
            sl.pin = nullptr;
            sl.pin_cap = 0;
            if ((e = hipHostMalloc(&sl.pin, pin_bytes, hipHostMallocDefault)) != hipSuccess)
                return hip_status(e, "staging: hipHostMalloc");
            sl.pin_cap = pin_bytes;
        }
    }
    const int64_t nchunks = (S + ns - 1) / ns;
    int status = STS_OK;
    for (int64_t i = 0; i < nchunks && status == STS_OK; i++) {
        Slot& sl = slots[i % kSlots];
        if ((r = reap(sl, args))) return r;
        sl.s0 = i * ns;
        sl.ns = std::min<int64_t>(ns, S - sl.s0);
        char* dev = static_cast<char*>(sl.dev);
        char* pin = static_cast<char*>(sl.pin);
        // the calling thread stages pageable inputs while earlier chunks are on the device
        for (Arg& x : args)
            if (x.src && !x.pinned_src)
                copy_rows(pin + x.pin_off, x.row, static_cast<const char*>(x.src) + (size_t)sl.s0 * x.hstride,
                          x.hstride, x.row, sl.ns);
        if ((e = hipEventRecord(sl.ev[0], sl.st)) != hipSuccess) return hip_status(e, "staging: event");
        for (Arg& x : args) {
            if (!x.src) continue;
            const size_t n = x.row * (size_t)sl.ns;
            if (STS_STAGE_LINEAR && x.pinned_src && x.hstride == x.row)   // contiguous rows: one linear copy
                e = hipMemcpyAsync(dev + x.dev_off, static_cast<const char*>(x.src) + (size_t)sl.s0 * x.hstride, n,
                                   hipMemcpyHostToDevice, sl.st);
            else if (x.pinned_src)
                e = hipMemcpy2DAsync(dev + x.dev_off, x.row, static_cast<const char*>(x.src) + (size_t)sl.s0 * x.hstride,
                                     x.hstride, x.row, (size_t)sl.ns, hipMemcpyHostToDevice, sl.st);
            else
                e = hipMemcpyAsync(dev + x.dev_off, pin + x.pin_off, n, hipMemcpyHostToDevice, sl.st);
            if (e != hipSuccess) return hip_status(e, "staging: H2D");
            g.bytes_h2d += (double)n;
            if (x.pinned_src) g.direct += (double)n;
        }
        if ((e = hipEventRecord(sl.ev[1], sl.st)) != hipSuccess) return hip_status(e, "staging: event");
        void* ptrs[16];
        for (size_t k = 0; k < args.size() && k < 16; k++) ptrs[k] = dev + args[k].dev_off;
        status = kern(ptrs, sl.s0, sl.ns, sl.st);
        if ((e = hipEventRecord(sl.ev[2], sl.st)) != hipSuccess) return hip_status(e, "staging: event");
        if (status == STS_OK) {
            for (Arg& x : args) {
                if (!x.dst) continue;
                const size_t n = x.row * (size_t)sl.ns;
                if (STS_STAGE_LINEAR && x.pinned_dst && x.hstride == x.row)
                    e = hipMemcpyAsync(static_cast<char*>(x.dst) + (size_t)sl.s0 * x.hstride, dev + x.dev_off, n,
                                       hipMemcpyDeviceToHost, sl.st);
                else if (x.pinned_dst)
                    e = hipMemcpy2DAsync(static_cast<char*>(x.dst) + (size_t)sl.s0 * x.hstride, x.hstride,
                                         dev + x.dev_off, x.row, x.row, (size_t)sl.ns, hipMemcpyDeviceToHost, sl.st);
                else
                    e = hipMemcpyAsync(pin + x.pin_off, dev + x.dev_off, n, hipMemcpyDeviceToHost, sl.st);
                if (e != hipSuccess) return hip_status(e, "staging: D2H");
                g.bytes_d2h += (double)n;
                if (x.pinned_dst) g.direct += (double)n;
            }
        }
        if ((e = hipEventRecord(sl.ev[3], sl.st)) != hipSuccess) return hip_status(e, "staging: event");
        sl.busy = true;
        sl.copy_out = (status == STS_OK);
        g.chunks += 1;
    }
    for (int64_t i = 0; i < kSlots; i++) {   // drain in issue order
        Slot& sl = slots[(nchunks + i) % kSlots];
        if ((r = reap(sl, args))) return r;
    }
    g.wall_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_start).count();
    return status;
}

size_t panel_stride(int64_t ld) { return (size_t)(ld > 0 ? ld : 0) * sizeof(double); }

// Per-series statuses: the caller's host array, or an internal one whose first failure
// becomes the return status (the reference's exception) once every chunk is back.
struct ErrOut {
    std::vector<int32_t> own;
    int32_t* h;
    explicit ErrOut(int32_t* user, int64_t S) : h(user) {
        if (!h) {
            own.assign((size_t)(S > 0 ? S : 0), 0);
            h = own.data();
        }
    }
    int finish(int st, int64_t S, const char* what) {
        if (st != STS_OK || !own.size()) return st;
        return sts::series_status(h, S, what);
    }
};

}  // namespace

extern "C" {

int sts_host_alloc(size_t bytes, void** out) {
    if (!out) return sts::set_error(STS_ERR_BAD_ARG, "sts_host_alloc: null output");
    *out = nullptr;
    hipError_t e = hipHostMalloc(out, bytes ? bytes : 16, hipHostMallocDefault);
    return e == hipSuccess ? STS_OK : hip_status(e, "hipHostMalloc");
}

int sts_host_free(void* p) {
    if (!p) return STS_OK;
    hipError_t e = hipHostFree(p);
    return e == hipSuccess ? STS_OK : hip_status(e, "hipHostFree");
}

int sts_staging_release(void) {
    (void)pool().trim();
    return STS_OK;
}

int sts_staging_set_limit(int max_sets) {
    if (max_sets < 1) return sts::set_error(STS_ERR_BAD_ARG, "sts_staging_set_limit: max_sets must be >= 1");
    (void)pool().set_cap(max_sets);
    return STS_OK;
}

int sts_staging_pool_info(int64_t* out8) {
    if (!out8) return sts::set_error(STS_ERR_BAD_ARG, "sts_staging_pool_info: null output");
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return hip_status(e, "hipGetDevice");
    const auto in = pool().info(dev);
    const int64_t v[8] = {in.live, in.idle, in.borrowed, in.cap, in.high, in.lost, in.waits,
                          (int64_t)kSlots * (int64_t)kSlotKeep};
    std::memcpy(out8, v, sizeof v);
    return STS_OK;
}

int sts_staging_stats(double* out8) {
    if (!out8) return sts::set_error(STS_ERR_BAD_ARG, "sts_staging_stats: null output");
    const Stats& g = g_stats;
    const double tot = g.bytes_h2d + g.bytes_d2h;
    const double v[8] = {g.wall_ms, g.h2d_ms, g.kernel_ms, g.d2h_ms,
                         g.bytes_h2d, g.bytes_d2h, g.chunks, tot > 0 ? g.direct / tot : 0.0};
    std::memcpy(out8, v, sizeof v);
    return STS_OK;
}

int sts_fill_host(const double* in, double* out, int64_t S, int64_t T, int64_t ld, int method, int32_t* err) {
    const size_t row = (size_t)(T > 0 ? T : 0) * sizeof(double);
    if (S > 0 && T > 0 && (!in || !out)) return sts::set_error(STS_ERR_BAD_ARG, "fill: null panel pointer");
    if (in == out && S * T > 0) return sts::set_error(STS_ERR_BAD_ARG, "fill: out must not alias in (fillts returns a new vector)");
    // validate through the device entry point's own checks first (no staging on bad input)
    if (method < STS_FILL_LINEAR || method > STS_FILL_SPLINE)
        return sts_fill(nullptr, nullptr, 0, 0, 0, 0, method, nullptr, nullptr);
    if (ld < T) return sts_fill(in, out, S, T, ld, ld, method, nullptr, nullptr);
    ErrOut eo(err, S);
    const int st = staged(S, {in_arg(in, row, panel_stride(ld)), out_arg(out, row, panel_stride(ld)),
                              out_arg(eo.h, sizeof(int32_t), sizeof(int32_t))},
                          [&](void* const* d, int64_t, int64_t n, hipStream_t s) {
                              return sts_fill(static_cast<const double*>(d[0]), static_cast<double*>(d[1]), n, T, T, T,
                                              method, static_cast<int32_t*>(d[2]), s);
                          });
    return eo.finish(st, S, "fill");
}

int sts_autocorr_host(const double* in, int64_t S, int64_t T, int64_t ld, int K, double* acf) {
    if (K < 0 || ld < T || (S > 0 && T > 0 && !in) || (S > 0 && K > 0 && !acf))
        return sts_autocorr(in, S, T, ld, K, acf, nullptr);   // the device entry point's error
    const size_t row = (size_t)(T > 0 ? T : 0) * sizeof(double), krow = (size_t)K * sizeof(double);
    // a device err array per chunk (it stays all zero: raw autocorr has no failing series), so
    // the device entry point never synchronises inside the pipeline
    ErrOut eo(nullptr, S);
    const int st = staged(S, {in_arg(in, row, panel_stride(ld)), out_arg(acf, krow, krow),
                              out_arg(eo.h, sizeof(int32_t), sizeof(int32_t))},
                          [&](void* const* d, int64_t, int64_t n, hipStream_t s) {
                              return sts_fill_autocorr(static_cast<const double*>(d[0]), nullptr, n, T, T, T,
                                                       STS_FILL_NONE, K, static_cast<double*>(d[1]),
                                                       static_cast<int32_t*>(d[2]), s);
                          });
    return eo.finish(st, S, "autocorr");
}

int sts_fill_autocorr_host(const double* in, double* filled, int64_t S, int64_t T, int64_t ld, int method, int K,
                           double* acf, int32_t* err) {
    if (method == STS_FILL_NONE) {
        if (filled) return sts::set_error(STS_ERR_BAD_ARG, "fill_autocorr: filled must be NULL for STS_FILL_NONE");
        return sts_autocorr_host(in, S, T, ld, K, acf);
    }
    if (method < STS_FILL_LINEAR || method > STS_FILL_SPLINE || K < 0 || ld < T ||
        (S * T > 0 && (!in || !filled || in == filled)) || (S > 0 && K > 0 && !acf))
        return sts_fill_autocorr(in, filled, S, T, ld, ld, method, K, acf, nullptr, nullptr);
    const size_t row = (size_t)(T > 0 ? T : 0) * sizeof(double), krow = (size_t)K * sizeof(double);
    ErrOut eo(err, S);
    const int st = staged(S, {in_arg(in, row, panel_stride(ld)), out_arg(filled, row, panel_stride(ld)),
                              out_arg(acf, krow, krow), out_arg(eo.h, sizeof(int32_t), sizeof(int32_t))},
                          [&](void* const* d, int64_t, int64_t n, hipStream_t s) {
                              return sts_fill_autocorr(static_cast<const double*>(d[0]), static_cast<double*>(d[1]), n,
                                                       T, T, T, method, K, static_cast<double*>(d[2]),
                                                       static_cast<int32_t*>(d[3]), s);
                          });
    return eo.finish(st, S, "fill_autocorr");
}

int sts_diff_at_lag_host(const double* in, double* out, int64_t S, int64_t T, int64_t ld, int lag, int start) {
    if (!(start >= lag) || lag <= 0 || ld < T || S * T == 0 || !in || !out)   // require(), lag 0: dest untouched
        return sts_diff_at_lag(in, out, S, T, ld, ld, lag, start, nullptr);
    const size_t row = (size_t)T * sizeof(double);
    if (in == out)   // dest eq ts: the reference's in-place recurrence, per series
        return staged(S, {inout_arg(out, row, panel_stride(ld))}, [&](void* const* d, int64_t, int64_t n, hipStream_t s) {
            return sts_diff_at_lag(static_cast<double*>(d[0]), static_cast<double*>(d[0]), n, T, T, T, lag, start, s);
        });
    // out-of-place: dest(i) = ts(i) for i < start (:363-369), so dest is fully written
    return staged(S, {in_arg(in, row, panel_stride(ld)), out_arg(out, row, panel_stride(ld))},
                  [&](void* const* d, int64_t, int64_t n, hipStream_t s) {
                      return sts_diff_at_lag(static_cast<const double*>(d[0]), static_cast<double*>(d[1]), n, T, T, T,
                                             lag, start, s);
                  });
}

int sts_lag_matrix_host(const double* in, double* out, int64_t S, int64_t T, int64_t ld, int max_lag, int inc) {
    if (max_lag < 0 || max_lag > T || ld < T || (S * T > 0 && !in))
        return sts_lag_matrix(in, out, S, T, ld, max_lag, inc, nullptr);
    const int64_t rows = T - max_lag, cols = max_lag + (inc ? 1 : 0);
    const size_t orow = (size_t)(rows * cols) * sizeof(double), row = (size_t)T * sizeof(double);
    if (orow == 0 || S == 0) return STS_OK;
    if (!out) return sts_lag_matrix(in, nullptr, S, T, ld, max_lag, inc, nullptr);
    return staged(S, {in_arg(in, row, panel_stride(ld)), out_arg(out, orow, orow)},
                  [&](void* const* d, int64_t, int64_t n, hipStream_t s) {
                      return sts_lag_matrix(static_cast<const double*>(d[0]), static_cast<double*>(d[1]), n, T, T,
                                            max_lag, inc, s);
                  });
}

static int ewma_host(bool add, const double* in, double* out, int64_t S, int64_t T, int64_t ld, const double* sm) {
    auto dev_call = [&](const double* i, double* o, int64_t n, const double* m, hipStream_t s) {
        return add ? sts_ewma_add(i, o, n, T, T, T, m, s) : sts_ewma_remove(i, o, n, T, T, T, m, s);
    };
    if (!out || ld < T || (S > 0 && !sm) || (S * T > 0 && !in))
        return add ? sts_ewma_add(in, out, S, T, ld, ld, sm, nullptr) : sts_ewma_remove(in, out, S, T, ld, ld, sm, nullptr);
    if (S * T == 0) return STS_OK;
    const size_t row = (size_t)T * sizeof(double);
    if (in == out)   // add: safe; remove: the reference's read-after-overwrite, per series
        return staged(S, {inout_arg(out, row, panel_stride(ld)), in_arg(sm, sizeof(double), sizeof(double))},
                      [&](void* const* d, int64_t, int64_t n, hipStream_t s) {
                          return dev_call(static_cast<double*>(d[0]), static_cast<double*>(d[0]), n,
                                          static_cast<const double*>(d[1]), s);
                      });
    return staged(S, {in_arg(in, row, panel_stride(ld)), out_arg(out, row, panel_stride(ld)),
                      in_arg(sm, sizeof(double), sizeof(double))},
                  [&](void* const* d, int64_t, int64_t n, hipStream_t s) {
                      return dev_call(static_cast<const double*>(d[0]), static_cast<double*>(d[1]), n,
                                      static_cast<const double*>(d[2]), s);
                  });
}

int sts_ewma_add_host(const double* in, double* out, int64_t S, int64_t T, int64_t ld, const double* sm) {
    return ewma_host(true, in, out, S, T, ld, sm);
}

int sts_ewma_remove_host(const double* in, double* out, int64_t S, int64_t T, int64_t ld, const double* sm) {
    return ewma_host(false, in, out, S, T, ld, sm);
}

int sts_fill_diff_ewma_host(const double* in, double* out, int64_t S, int64_t T, int64_t ld, int method, int lag,
                            const double* smoothing, int32_t* err) {
    if (method < STS_FILL_NONE || method > STS_FILL_SPLINE || lag < 0 || ld < T ||
        (S > 0 && !smoothing) || (S * T > 0 && (!in || !out || in == out)))
        return sts_fill_diff_ewma(in, out, S, T, ld, ld, method, lag, smoothing, nullptr, nullptr);
    if (S * T == 0) return STS_OK;
    const size_t row = (size_t)T * sizeof(double);
    ErrOut eo(err, S);
    const int st = staged(S, {in_arg(in, row, panel_stride(ld)), out_arg(out, row, panel_stride(ld)),
                              in_arg(smoothing, sizeof(double), sizeof(double)),
                              out_arg(eo.h, sizeof(int32_t), sizeof(int32_t))},
                          [&](void* const* d, int64_t, int64_t n, hipStream_t s) {
                              return sts_fill_diff_ewma(static_cast<const double*>(d[0]), static_cast<double*>(d[1]), n,
                                                        T, T, T, method, lag, static_cast<const double*>(d[2]),
                                                        static_cast<int32_t*>(d[3]), s);
                          });
    return eo.finish(st, S, "fill_diff_ewma");
}

int sts_ewma_fit_host(const double* in, int64_t S, int64_t T, int64_t ld, double* smoothing, int32_t* err) {
    if (ld < T || (S > 0 && (T < 1 || !smoothing || !in))) return sts_ewma_fit(in, S, T, ld, smoothing, nullptr, nullptr);
    const size_t row = (size_t)T * sizeof(double);
    ErrOut eo(err, S);
    const int st = staged(S, {in_arg(in, row, panel_stride(ld)), out_arg(smoothing, sizeof(double), sizeof(double)),
                              out_arg(eo.h, sizeof(int32_t), sizeof(int32_t))},
                          [&](void* const* d, int64_t, int64_t n, hipStream_t s) {
                              return sts_ewma_fit(static_cast<const double*>(d[0]), n, T, T, static_cast<double*>(d[1]),
                                                  static_cast<int32_t*>(d[2]), s);
                          });
    return eo.finish(st, S, "EWMA.fitModel");
}

int sts_ar_fit_host(const double* in, int64_t S, int64_t T, int64_t ld, int p, int no_intercept, double* c,
                    double* coef, int32_t* err) {
    if (ld < T || p < 1 || p > 31 || T - p < (int64_t)p + 1 || (S > 0 && (!c || !coef || !in)))
        return sts_ar_fit(in, S, T, ld, p, no_intercept, c, coef, nullptr, nullptr);
    const size_t row = (size_t)T * sizeof(double), prow = (size_t)p * sizeof(double);
    ErrOut eo(err, S);
    const int st = staged(S, {in_arg(in, row, panel_stride(ld)), out_arg(c, sizeof(double), sizeof(double)),
                              out_arg(coef, prow, prow), out_arg(eo.h, sizeof(int32_t), sizeof(int32_t))},
                          [&](void* const* d, int64_t, int64_t n, hipStream_t s) {
                              return sts_ar_fit(static_cast<const double*>(d[0]), n, T, T, p, no_intercept,
                                                static_cast<double*>(d[1]), static_cast<double*>(d[2]),
                                                static_cast<int32_t*>(d[3]), s);
                          });
    return eo.finish(st, S, "ar_fit");
}

int sts_ar_fit_remove_host(const double* in, double* out, int64_t S, int64_t T, int64_t ld, int p, int no_intercept,
                           double* c, double* coef, int32_t* err) {
    if (!out || in == out || ld < T || p < 1 || p > 31 || T - p < (int64_t)p + 1 || (S > 0 && (!c || !coef || !in)))
        return sts_ar_fit_remove(in, out, S, T, ld, ld, p, no_intercept, c, coef, nullptr, nullptr);
    const size_t row = (size_t)T * sizeof(double), prow = (size_t)p * sizeof(double);
    ErrOut eo(err, S);
    const int st = staged(S, {in_arg(in, row, panel_stride(ld)), out_arg(out, row, panel_stride(ld)),
                              out_arg(c, sizeof(double), sizeof(double)), out_arg(coef, prow, prow),
                              out_arg(eo.h, sizeof(int32_t), sizeof(int32_t))},
                          [&](void* const* d, int64_t, int64_t n, hipStream_t s) {
                              return sts_ar_fit_remove(static_cast<const double*>(d[0]), static_cast<double*>(d[1]), n,
                                                       T, T, T, p, no_intercept, static_cast<double*>(d[2]),
                                                       static_cast<double*>(d[3]), static_cast<int32_t*>(d[4]), s);
                          });
    return eo.finish(st, S, "ar_fit_remove");
}

int sts_garch_fit_host(const double* in, int64_t S, int64_t T, int64_t ld, double* params, int32_t* err) {
    if (ld < T || (S > 0 && (!params || (T > 0 && !in)))) return sts_garch_fit(in, S, T, ld, params, nullptr, nullptr);
    const size_t row = (size_t)(T > 0 ? T : 0) * sizeof(double);
    ErrOut eo(err, S);
    const int st = staged(S, {in_arg(in, row, panel_stride(ld)), out_arg(params, 3 * sizeof(double), 3 * sizeof(double)),
                              out_arg(eo.h, sizeof(int32_t), sizeof(int32_t))},
                          [&](void* const* d, int64_t, int64_t n, hipStream_t s) {
                              return sts_garch_fit(static_cast<const double*>(d[0]), n, T, T, static_cast<double*>(d[1]),
                                                   static_cast<int32_t*>(d[2]), s);
                          });
    return eo.finish(st, S, "GARCH.fitModel");
}

int sts_argarch_fit_host(const double* in, int64_t S, int64_t T, int64_t ld, double* c, double* phi, double* params,
                         int32_t* err) {
    if (ld < T || T - 1 < 2 || (S > 0 && (!c || !phi || !params || !in)))
        return sts_argarch_fit(in, S, T, ld, c, phi, params, nullptr, nullptr);
    const size_t row = (size_t)T * sizeof(double);
    ErrOut eo(err, S);
    const int st = staged(S, {in_arg(in, row, panel_stride(ld)), out_arg(c, sizeof(double), sizeof(double)),
                              out_arg(phi, sizeof(double), sizeof(double)),
                              out_arg(params, 3 * sizeof(double), 3 * sizeof(double)),
                              out_arg(eo.h, sizeof(int32_t), sizeof(int32_t))},
                          [&](void* const* d, int64_t, int64_t n, hipStream_t s) {
                              return sts_argarch_fit(static_cast<const double*>(d[0]), n, T, T,
                                                     static_cast<double*>(d[1]), static_cast<double*>(d[2]),
                                                     static_cast<double*>(d[3]), static_cast<int32_t*>(d[4]), s);
                          });
    return eo.finish(st, S, "ARGARCH.fitModel");
}

static int ar_host(bool add, const double* in, double* out, int64_t S, int64_t T, int64_t ld, const double* c,
                   const double* coef, int p) {
    auto dev_call = [&](const double* i, double* o, int64_t n, const double* cc, const double* k, hipStream_t s) {
        return add ? sts_ar_add(i, o, n, T, T, T, cc, k, p, s) : sts_ar_remove(i, o, n, T, T, T, cc, k, p, s);
    };
    if (!out || ld < T || p < 0 || (S > 0 && (!c || (p > 0 && !coef))) || (S * T > 0 && !in))
        return add ? sts_ar_add(in, out, S, T, ld, ld, c, coef, p, nullptr)
                   : sts_ar_remove(in, out, S, T, ld, ld, c, coef, p, nullptr);
    if (S * T == 0) return STS_OK;
    const size_t row = (size_t)T * sizeof(double), prow = (size_t)(p > 0 ? p : 1) * sizeof(double);
    const double zero = 0.0;
    const double* k = p > 0 ? coef : &zero;
    const size_t kst = p > 0 ? prow : 0;   // (p = 0: no coefficients; a dummy row)
    if (in == out)
        return staged(S, {inout_arg(out, row, panel_stride(ld)), in_arg(c, sizeof(double), sizeof(double)),
                          in_arg(k, prow, kst)},
                      [&](void* const* d, int64_t, int64_t n, hipStream_t s) {
                          return dev_call(static_cast<double*>(d[0]), static_cast<double*>(d[0]), n,
                                          static_cast<const double*>(d[1]), static_cast<const double*>(d[2]), s);
                      });
    return staged(S, {in_arg(in, row, panel_stride(ld)), out_arg(out, row, panel_stride(ld)),
                      in_arg(c, sizeof(double), sizeof(double)), in_arg(k, prow, kst)},
                  [&](void* const* d, int64_t, int64_t n, hipStream_t s) {
                      return dev_call(static_cast<const double*>(d[0]), static_cast<double*>(d[1]), n,
                                      static_cast<const double*>(d[2]), static_cast<const double*>(d[3]), s);
                  });
}

int sts_ar_remove_host(const double* in, double* out, int64_t S, int64_t T, int64_t ld, const double* c,
                       const double* coef, int p) {
    return ar_host(false, in, out, S, T, ld, c, coef, p);
}

int sts_ar_add_host(const double* in, double* out, int64_t S, int64_t T, int64_t ld, const double* c,
                    const double* coef, int p) {
    return ar_host(true, in, out, S, T, ld, c, coef, p);
}

}  // extern "C"
