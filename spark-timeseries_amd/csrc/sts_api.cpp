// sts_api.cpp -- the C ABI (include/sts.h): argument validation with the reference's
// error semantics, stream/workspace handling, kernel dispatch, host-buffer staging.
//
// Reentrancy: no mutable global state after first use except the per-device
// memory-pool setup (guarded by std::call_once); every call runs on the caller's
// stream (NULL -> hipStreamPerThread) and allocates its scratch stream-ordered
// (hipMallocAsync / hipFreeAsync), so Spark's N executor threads can call
// concurrently.  Errors are reported through a thread-local message.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "sts_internal.hpp"

namespace {

thread_local std::string g_err;

int fail(int status, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
    return status;
}

int hip_fail(hipError_t e, const char* where) {
    return fail(STS_ERR_HIP, "%s: %s", where, hipGetErrorString(e));
}

#define HIP_TRY(call, where)                       \
    do {                                           \
        hipError_t e_ = (call);                    \
        if (e_ != hipSuccess) return hip_fail(e_, where); \
    } while (0)

hipStream_t as_stream(void* s) { return s ? reinterpret_cast<hipStream_t>(s) : hipStreamPerThread; }

std::once_flag g_pool_once[64];

// validate-only mode (sts::validate_call): every entry point validates its arguments
// before its first device action, ensure_device(), which then stops the call
thread_local bool g_validate_only = false;
constexpr int kValidated = -1000;

int ensure_device() {
    if (g_validate_only) return kValidated;
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return hip_fail(e, "hipGetDevice");
    int n = 0;
    e = hipGetDeviceCount(&n);
    if (e != hipSuccess || n == 0) return fail(STS_ERR_NO_DEVICE, "no HIP device visible");
    if (dev >= 0 && dev < 64) {
        std::call_once(g_pool_once[dev], [dev] {
            hipMemPool_t pool;
            if (hipDeviceGetDefaultMemPool(&pool, dev) == hipSuccess) {
                uint64_t thr = UINT64_MAX;
                (void)hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &thr);
            }
        });
    }
    return STS_OK;
}

// stream-ordered scratch
struct Scratch {
    void* p = nullptr;
    hipStream_t st;
    explicit Scratch(hipStream_t s) : st(s) {}
    hipError_t alloc(size_t bytes) { return hipMallocAsync(&p, bytes ? bytes : 16, st); }
    ~Scratch() {
        if (p) (void)hipFreeAsync(p, st);
    }
};

int check_panel(const void* in, int64_t S, int64_t T, int64_t ld, const char* name) {
    if (S < 0 || T < 0) return fail(STS_ERR_BAD_ARG, "%s: negative panel shape (S=%lld, T=%lld)", name,
                                    (long long)S, (long long)T);
    if (T > 0x7fffffffLL) return fail(STS_ERR_BAD_ARG, "%s: T=%lld exceeds the reference's Int index range",
                                      name, (long long)T);
    if (ld < T) return fail(STS_ERR_BAD_ARG, "%s: leading dimension %lld < T=%lld", name, (long long)ld,
                            (long long)T);
    if (S * T > 0 && !in) return fail(STS_ERR_BAD_ARG, "%s: null panel pointer", name);
    return STS_OK;
}

// The calling thread's host-mapped status array for calls without a caller err array (round 6):
// the kernels write it over PCIe and the call reads it after its stream synchronize, instead of a
// stream-ordered allocation + memset + D2H copy (a one-series fill: 35 -> ~15 us,
// tools/percall_parts.py).  Grown on demand up to kMappedErrMax entries, freed with the thread.
constexpr int64_t kMappedErrMax = 1 << 16;
struct MappedErr {
    int32_t* host = nullptr;
    int32_t* dev = nullptr;
    int64_t cap = 0;
    int32_t* get(int64_t n, int32_t** devp) {
        if (n > cap) {
            if (host) (void)hipHostFree(host);
            host = dev = nullptr;
            cap = 0;
            void* p = nullptr;
            if (hipHostMalloc(&p, (size_t)n * sizeof(int32_t), hipHostMallocMapped | hipHostMallocPortable) != hipSuccess)
                return nullptr;
            void* d = nullptr;
            if (hipHostGetDevicePointer(&d, p, 0) != hipSuccess) {
                (void)hipHostFree(p);
                return nullptr;
            }
            host = static_cast<int32_t*>(p);
            dev = static_cast<int32_t*>(d);
            cap = n;
        }
        *devp = dev;
        return host;
    }
    ~MappedErr() {
        if (host) (void)hipHostFree(host);
    }
};
thread_local MappedErr t_mapped_err;

// err handling: caller array (async) or internal buffer checked synchronously
struct ErrSink {
    int32_t* dev = nullptr;
    int32_t* mapped = nullptr;   // host view of dev when dev is the thread's mapped array
    bool owned = false;
    Scratch scratch;
    int64_t S;
    ErrSink(int32_t* user, int64_t S_, hipStream_t st) : dev(user), scratch(st), S(S_) {}
    // zero = false: the caller guarantees that the kernel writes every entry, or zeroes it
    // itself (run_tile)
    int prepare(bool zero = true) {
        if (!dev) {
            owned = true;
            if (S > 0 && S <= kMappedErrMax) mapped = t_mapped_err.get(S, &dev);
            if (mapped) {
                std::memset(mapped, 0, (size_t)S * sizeof(int32_t));   // before any launch of this call
                return STS_OK;
            }
            hipError_t e = scratch.alloc((size_t)(S > 0 ? S : 1) * sizeof(int32_t));
            if (e != hipSuccess) return hip_fail(e, "hipMallocAsync(err)");
            dev = static_cast<int32_t*>(scratch.p);
        }
        if (S > 0 && zero) {
            hipError_t e = hipMemsetAsync(dev, 0, (size_t)S * sizeof(int32_t), scratch.st);
            if (e != hipSuccess) return hip_fail(e, "hipMemsetAsync(err)");
        }
        return STS_OK;
    }
    // a call that returns early (a failed launch) may still have kernels in flight that write
    // the thread's mapped array: wait for them before the next call on this thread reuses it
    ~ErrSink() {
        if (mapped && !finished) (void)hipStreamSynchronize(scratch.st);
    }
    bool finished = false;
    // for the internal buffer: wait and turn the first failing series into a status
    int finish(const char* what) {
        finished = true;
        if (!owned || S == 0) return STS_OK;
        if (mapped) {
            const hipError_t e = hipStreamSynchronize(scratch.st);
            if (e != hipSuccess) return hip_fail(e, what);
            return sts::series_status(mapped, S, what);
        }
        std::vector<int32_t> h((size_t)S);
        hipError_t e = hipMemcpyAsync(h.data(), dev, (size_t)S * sizeof(int32_t), hipMemcpyDeviceToHost, scratch.st);
        if (e == hipSuccess) e = hipStreamSynchronize(scratch.st);
        if (e != hipSuccess) return hip_fail(e, what);
        return sts::series_status(h.data(), S, what);
    }
};

int method_ok(int method, bool allow_none, const char* name) {
    if (method < (allow_none ? STS_FILL_NONE : STS_FILL_LINEAR) || method > STS_FILL_SPLINE)
        return fail(STS_ERR_UNSUPPORTED_METHOD, "%s: unsupported fill method %d", name, method);
    return STS_OK;
}

int tile_width(int64_t T) { return T <= 512 ? 512 : 4096; }
constexpr int64_t kTilesPerChunk = 16;  // tiles per workgroup (prefetch pipeline depth 1)
// without the ACF (fill only, fill + lag matrix: C5) one tile per workgroup: the denser sweep
// beats the prefetch pipeline (C5: 1.527-1.534 vs 1.647-1.659 ms same box, and 1.83 vs 2.03-2.07 on
// a box in its slow state, profiles/r04_v11_ab_c5_tpc.jsonl; fill only on the C3 shard 31.2-31.6 vs
// 33.3 ms, r04_v2_ab_tiles_per_chunk.jsonl)
constexpr int64_t kTilesPerChunkFill = 1;

// Measurement hook (bench.py): HIP events recorded on the launch stream around every
// tile-kernel launch of this thread while profiling is on.
struct ProfileState {
    bool on = false;
    std::vector<hipEvent_t> pool;
    size_t used = 0;
};
thread_local ProfileState g_prof;

void prof_mark(hipStream_t st) {
    if (!g_prof.on) return;
    if (g_prof.used == g_prof.pool.size()) {
        hipEvent_t e;
        if (hipEventCreate(&e) != hipSuccess) return;
        g_prof.pool.push_back(e);
    }
    (void)hipEventRecord(g_prof.pool[g_prof.used++], st);
}

// a kernel launch bracketed by profiling events (bench.py's per-kernel timing)
template <typename F>
hipError_t timed(hipStream_t st, F&& launch) {
    prof_mark(st);
    const hipError_t e = launch();
    prof_mark(st);
    return e;
}

// fillts "spline" (sts_spline.hip): its own kernel, not a tile-kernel method.  err (device,
// S entries) is written for every series.
int run_spline(const double* in, double* out, int64_t S, int64_t T, int64_t ld_in, int64_t ld_out, int32_t* err,
               hipStream_t st) {
    if (S == 0) return STS_OK;
    if (T == 0) {
        if (err) HIP_TRY(hipMemsetAsync(err, 0, (size_t)S * sizeof(int32_t), st), "hipMemsetAsync(err)");
        return STS_OK;
    }
    const int64_t batch = sts::spline_batch(S, T);
    Scratch sc(st);
    hipError_t e = sc.alloc((size_t)batch * (size_t)T * 2 * sizeof(double));
    if (e != hipSuccess) return hip_fail(e, "hipMallocAsync(spline scratch)");
    e = timed(st, [&] {
        return sts::launch_spline(in, out, S, T, ld_in, ld_out, err, static_cast<double*>(sc.p), batch, st);
    });
    if (e != hipSuccess) return hip_fail(e, "fill (spline)");
    return STS_OK;
}

// fill (+ optional ACF partials / lag matrix) through the tile kernel
// err: zeroed here unless the chosen kernel writes every entry (the seg kernel with one
// segment per series); callers prepare their ErrSink with zero = false.
int run_tile(const double* in, double* out, double* lagmat, int64_t S, int64_t T, int64_t ld_in, int64_t ld_out,
             int method, int K, double* acf, int max_lag, int inc, int32_t* err, hipStream_t st, const char* name) {
    if (method == STS_FILL_SPLINE) {
        // the spline is not fused: callers compose it (sts_fill_autocorr / _lag_matrix / _diff_ewma)
        if (K > 0 || lagmat) return fail(STS_ERR_BAD_ARG, "%s: spline fill is not fused", name);
        return run_spline(in, out, S, T, ld_in, ld_out, err, st);
    }
    if (S == 0) return STS_OK;
    if (T == 0) {
        if (err) HIP_TRY(hipMemsetAsync(err, 0, (size_t)S * sizeof(int32_t), st), "hipMemsetAsync(err)");
        return STS_OK;
    }
    // short series (T <= 16384: C1, the 10-year daily panels) go to the wave-private
    // segment kernel (2x faster there: one wave per series, no barriers), long ones to the
    // workgroup tile kernel (faster from T = 32768: C3, C5).  The segment kernel needs a
    // 16-B aligned panel, no lag matrix and K <= 60.  In the A/B build STS_TILE_KERNEL=tile|seg
    // forces one (tools/kbench.py, the knob tests).
    const char* force = sts::ab_knob("STS_TILE_KERNEL");
    const bool seg_ok = !lagmat && sts::seg_nt(K) >= 0 && (reinterpret_cast<uintptr_t>(in) & 15) == 0 &&
                        (ld_in % 2) == 0 &&
                        (!out || ((reinterpret_cast<uintptr_t>(out) & 15) == 0 && ld_out % 2 == 0)) &&
                        T < 0x7fff0000LL;
    const bool seg = seg_ok && (force ? !std::strcmp(force, "seg") : T <= 16384);
    // STS_TILE_W=2048: 2-wave workgroups on 2048-step tiles for K <= 60 (A/B build only)
    const char* tw_env = (!seg && K > 0 && K <= 60 && !lagmat) ? sts::ab_knob("STS_TILE_W") : nullptr;
    const int tw = seg ? sts::kSegW : (K > 0) ? (tw_env && std::atoi(tw_env) == 2048 ? 2048 : 4096) : tile_width(T);
    sts::TileArgs a{};
    a.in = in;
    a.out = out;
    a.lagmat = lagmat;
    a.err = err;
    a.S = S;
    a.T = T;
    a.ld_in = ld_in;
    a.ld_out = ld_out;
    a.tiles_per_series = (T + tw - 1) / tw;
    // STS_SEG_TILES: segment length (tiles) of the seg kernel, for A/B runs only
    const char* seg_env = seg ? sts::ab_knob("STS_SEG_TILES") : nullptr;
    // STS_TILES_PER_CHUNK: tiles per tile-kernel workgroup, for A/B runs only
    const char* tpc_env = seg ? nullptr : sts::ab_knob("STS_TILES_PER_CHUNK");
    const int seg_knob = seg_env ? std::atoi(seg_env) : 0, tpc_knob = tpc_env ? std::atoi(tpc_env) : 0;
    const int64_t per_chunk = seg ? (seg_knob > 0 ? seg_knob : sts::kSegTiles)
                                  : (tpc_knob > 0 ? tpc_knob : (K > 0 ? kTilesPerChunk : kTilesPerChunkFill));
    a.tiles_per_chunk = a.tiles_per_series < per_chunk ? a.tiles_per_series : per_chunk;
    a.chunks_per_series = (a.tiles_per_series + a.tiles_per_chunk - 1) / a.tiles_per_chunk;
    a.K = K;
    a.max_lag = max_lag;
    a.include_original = inc;
    if (S * a.chunks_per_series > 0x7fffffffLL) return fail(STS_ERR_BAD_ARG, "%s: panel too large for one launch", name);
    // one segment per series: the seg kernel writes err[s] for every series and, when the
    // finalize's general path applies (T > 2K) and the last tile holds >= 64 steps, the
    // final ACF itself (no partials, no second launch)
    const bool one_seg = seg && a.chunks_per_series == 1;
    const int64_t last_len = T - (a.tiles_per_series - 1) * tw;
    const bool fuse = one_seg && K > 0 && T > 2 * (int64_t)K && T >= 2 * sts::kAcfEdge && last_len >= 64 &&
                      !sts::ab_knob("STS_NO_FUSED_ACF");
    a.err_all = one_seg ? 1 : 0;
    a.acf_fused = fuse ? acf : nullptr;
    // any of the four fills + ACF with K <= 24 on T <= 2560 (C1): one wave holds the whole series
    // (sts_short.hip; its rule-3 fallback re-reads the filled series from out); STS_NO_SHORT keeps
    // the segment kernel (A/B build)
    const bool short_k = fuse && out && sts::short_ok(method, T, K) && !sts::ab_knob("STS_NO_SHORT");
    // two series per workgroup on one LDS block (sts_short.hip short_pair_kernel); STS_SHORT_PAIR=0/1
    // picks the form on the A/B build
    const char* pair_env = sts::ab_knob("STS_SHORT_PAIR");
    const bool short_pair = pair_env ? pair_env[0] == '1' : sts::kShortPairDefault;
    if (err && !one_seg) HIP_TRY(hipMemsetAsync(err, 0, (size_t)S * sizeof(int32_t), st), "hipMemsetAsync(err)");
    Scratch part(st);
    int32_t* exact = nullptr;
    if (K > 0 && !fuse) {
        // chunk partials, then (tile kernel) the per-series shifts, then rule 3's per-series flags
        const size_t np = (size_t)(S * a.chunks_per_series) * sts::kPartStride;
        const size_t nsh = seg ? 0 : (size_t)S;
        hipError_t e = part.alloc((np + nsh + ((size_t)S + 1) / 2) * sizeof(double));
        if (e != hipSuccess) return hip_fail(e, "hipMallocAsync(partials)");
        a.partials = static_cast<double*>(part.p);
        exact = reinterpret_cast<int32_t*>(a.partials + np + nsh);
        HIP_TRY(hipMemsetAsync(exact, 0, (size_t)S * sizeof(int32_t), st), "hipMemsetAsync(rule 3 flags)");
        if (!seg) {
            double* sh = a.partials + np;
            e = sts::launch_acf_shift(in, S, T, ld_in, method, sh, st);
            if (e != hipSuccess) return hip_fail(e, "acf shift");
            a.shift = sh;
        }
    }
    prof_mark(st);
    hipError_t e = short_k ? sts::launch_short(method, a, st, short_pair)
                   : seg   ? sts::launch_segment(method, a, st)
                           : sts::launch_tile(method, tw, a, st);
    prof_mark(st);
    if (e != hipSuccess) return hip_fail(e, name);
    if (K > 0 && !fuse) {
        sts::FinalizeArgs f{};
        f.F = out ? out : in;
        f.partials = a.partials;
        f.acf = acf;
        f.S = S;
        f.T = T;
        f.ldF = out ? ld_out : ld_in;
        f.parts_per_series = a.chunks_per_series;
        f.K = K;
        f.exact = exact;
        e = sts::launch_acf_finalize(f, st);
        if (e != hipSuccess) return hip_fail(e, "acf finalize");
        e = sts::launch_acf_exact(f.F, S, T, f.ldF, K, exact, acf, st);
        if (e != hipSuccess) return hip_fail(e, "acf exact (rule 3)");
    }
    return STS_OK;
}

}  // namespace

namespace sts {

// The first failing series of a host copy of err_per_series -> the reference's exception
// (status + thread-local message); STS_OK when none failed.
int series_status(const int32_t* h, int64_t S, const char* what) {
    for (int64_t s = 0; s < S; s++) {
        if (h[s] == STS_ERR_ALL_NAN) return fail(STS_ERR_ALL_NAN, "Input is all NaNs! (series %lld)", (long long)s);
        if (h[s] == STS_ERR_SINGULAR) return fail(STS_ERR_SINGULAR, "singular AR design matrix (series %lld)", (long long)s);
        if (h[s] == STS_ERR_TOO_FEW_POINTS)
            return fail(STS_ERR_TOO_FEW_POINTS,
                        "NumberIsTooSmallException: number of points: fewer than 3 non-NaN values for a spline (series %lld)",
                        (long long)s);
        if (h[s] == STS_ERR_TOO_MANY_EVALUATIONS)
            return fail(STS_ERR_TOO_MANY_EVALUATIONS,
                        "TooManyEvaluationsException: illegal state: maximal count (10000) exceeded: evaluations (series %lld)",
                        (long long)s);
        if (h[s] != 0) return fail(h[s], "%s failed for series %lld", what, (long long)s);
    }
    return STS_OK;
}

int set_error(int status, const char* msg) { return fail(status, "%s", msg); }

int validate_call(int (*fn)(void*), void* ctx) {
    g_validate_only = true;
    const int r = fn(ctx);
    g_validate_only = false;
    return r == kValidated ? STS_OK : r;
}

}  // namespace sts

extern "C" {

int sts_abi_version(void) { return STS_ABI_VERSION; }

int sts_init(int device) {
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess || n == 0) return fail(STS_ERR_NO_DEVICE, "no HIP device visible");
    if (device < 0 || device >= n) return fail(STS_ERR_BAD_ARG, "device %d out of range (%d devices)", device, n);
    HIP_TRY(hipSetDevice(device), "hipSetDevice");
    hipDeviceProp_t prop;
    HIP_TRY(hipGetDeviceProperties(&prop, device), "hipGetDeviceProperties");
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return fail(STS_ERR_NO_DEVICE, "device %d is %s; this library is built for gfx950 only", device, prop.gcnArchName);
    return ensure_device();
}

const char* sts_last_error(void) { return g_err.c_str(); }

int sts_fill_method_from_name(const char* name) {
    if (!name) return -2;
    if (!std::strcmp(name, "linear")) return STS_FILL_LINEAR;
    if (!std::strcmp(name, "nearest")) return STS_FILL_NEAREST;
    if (!std::strcmp(name, "next")) return STS_FILL_NEXT;
    if (!std::strcmp(name, "previous")) return STS_FILL_PREVIOUS;
    if (!std::strcmp(name, "spline")) return STS_FILL_SPLINE;
    return -2;
}

int sts_profile_begin(void) {
    // create the event pool here, before the caller's timed region: a hipEventCreate inside
    // it costs CPU time per launch and can starve the queue of short kernels (C1: 0.13 ms)
    constexpr size_t kPrealloc = 512;
    while (g_prof.pool.size() < kPrealloc) {
        hipEvent_t e;
        HIP_TRY(hipEventCreate(&e), "hipEventCreate");
        g_prof.pool.push_back(e);
    }
    g_prof.on = true;
    g_prof.used = 0;
    return STS_OK;
}

int sts_profile_end(double* kernel_ms, int64_t* launches) {
    g_prof.on = false;
    double total = 0.0;
    int64_t n = 0;
    for (size_t i = 0; i + 1 < g_prof.used; i += 2) {
        HIP_TRY(hipEventSynchronize(g_prof.pool[i + 1]), "hipEventSynchronize");
        float ms = 0.f;
        HIP_TRY(hipEventElapsedTime(&ms, g_prof.pool[i], g_prof.pool[i + 1]), "hipEventElapsedTime");
        total += ms;
        n++;
    }
    g_prof.used = 0;
    for (hipEvent_t e : g_prof.pool) (void)hipEventDestroy(e);   // recreated by the next begin
    g_prof.pool.clear();
    if (kernel_ms) *kernel_ms = total;
    if (launches) *launches = n;
    return STS_OK;
}

int sts_stream_synchronize(void* stream) {
    HIP_TRY(hipStreamSynchronize(as_stream(stream)), "hipStreamSynchronize");
    return STS_OK;
}

int sts_fill(const double* in, double* out, int64_t S, int64_t T, int64_t ld_in, int64_t ld_out, int method,
             int32_t* err_per_series, void* stream) {
    int r;
    if ((r = method_ok(method, false, "fill"))) return r;
    if ((r = check_panel(in, S, T, ld_in, "fill"))) return r;
    if ((r = check_panel(out, S, T, ld_out, "fill"))) return r;
    if (S * T > 0 && in == out) return fail(STS_ERR_BAD_ARG, "fill: out must not alias in (fillts returns a new vector)");
    if ((r = ensure_device())) return r;
    hipStream_t st = as_stream(stream);
    ErrSink es(err_per_series, S, st);
    if ((r = es.prepare(false))) return r;   // run_tile zeroes err unless its kernel writes all of it
    if ((r = run_tile(in, out, nullptr, S, T, ld_in, ld_out, method, 0, nullptr, 0, 0, es.dev, st, "fill"))) return r;
    return es.finish("fill");
}

int sts_fill_autocorr(const double* in, double* filled, int64_t S, int64_t T, int64_t ld_in, int64_t ld_out,
                      int method, int K, double* acf, int32_t* err_per_series, void* stream) {
    int r;
    if ((r = method_ok(method, true, "fill_autocorr"))) return r;
    if ((r = check_panel(in, S, T, ld_in, "fill_autocorr"))) return r;
    if (method != STS_FILL_NONE) {
        if ((r = check_panel(filled, S, T, ld_out, "fill_autocorr"))) return r;
        if (S * T > 0 && in == filled) return fail(STS_ERR_BAD_ARG, "fill_autocorr: filled must not alias in");
    } else if (filled) {
        return fail(STS_ERR_BAD_ARG, "fill_autocorr: filled must be NULL for STS_FILL_NONE");
    }
    if (K < 0) return fail(STS_ERR_BAD_ARG, "autocorr: negative numLags %d", K);
    if (S > 0 && K > 0 && !acf) return fail(STS_ERR_BAD_ARG, "autocorr: null output");
    if ((r = ensure_device())) return r;
    hipStream_t st = as_stream(stream);
    ErrSink es(err_per_series, S, st);
    if ((r = es.prepare(false))) return r;   // zeroed by run_tile, or below when it does not run
    if (method == STS_FILL_SPLINE) {
        // fillSpline (not fused: sts_spline.hip), then autocorr of the filled panel; the ACF
        // pass reports into a scratch array so the spline's per-series status stands
        if ((r = run_spline(in, filled, S, T, ld_in, ld_out, es.dev, st))) return r;
        if (K > 0 && S > 0) {
            Scratch e2(st);
            HIP_TRY(e2.alloc((size_t)S * sizeof(int32_t)), "hipMallocAsync(err)");
            if ((r = sts_fill_autocorr(filled, nullptr, S, T, ld_out, ld_out, STS_FILL_NONE, K, acf,
                                       static_cast<int32_t*>(e2.p), st))) return r;
        }
        return es.finish("fill_autocorr");
    }
    if (S > 0 && (T == 0 || (K == 0 && method == STS_FILL_NONE)))
        HIP_TRY(hipMemsetAsync(es.dev, 0, (size_t)S * sizeof(int32_t), st), "hipMemsetAsync(err)");
    if (T == 0 && S > 0 && K > 0) {
        std::vector<double> nan((size_t)(S * K), NAN);
        HIP_TRY(hipMemcpyAsync(acf, nan.data(), nan.size() * sizeof(double), hipMemcpyHostToDevice, st), "acf");
        HIP_TRY(hipStreamSynchronize(st), "acf");
        return es.finish("fill_autocorr");
    }
    if (K == 0) {
        if (method != STS_FILL_NONE && (r = run_tile(in, filled, nullptr, S, T, ld_in, ld_out, method, 0, nullptr, 0, 0,
                                                    es.dev, st, "fill"))) return r;
        return es.finish("fill_autocorr");
    }
    if (K > sts::kFusedMaxLags) {
        // any numLags (sts_acf_wide.hip): fill first (no ACF), then lag blocks of 61 on MFMA
        const double* F = in;
        int64_t ldF = ld_in;
        if (method != STS_FILL_NONE) {
            if ((r = run_tile(in, filled, nullptr, S, T, ld_in, ld_out, method, 0, nullptr, 0, 0, es.dev, st, "fill")))
                return r;
            F = filled;
            ldF = ld_out;
        } else {
            HIP_TRY(hipMemsetAsync(es.dev, 0, (size_t)S * sizeof(int32_t), st), "hipMemsetAsync(err)");
        }
        Scratch sc(st);
        const size_t np = sts::acf_wide_partials(S, T, K);
        hipError_t e = sc.alloc(((size_t)S + np + ((size_t)S + 1) / 2) * sizeof(double));
        if (e != hipSuccess) return hip_fail(e, "hipMallocAsync(acf partials)");
        double* shift = static_cast<double*>(sc.p);
        int32_t* exact = reinterpret_cast<int32_t*>(shift + S + np);
        HIP_TRY(hipMemsetAsync(exact, 0, (size_t)S * sizeof(int32_t), st), "hipMemsetAsync(rule 3 flags)");
        HIP_TRY(sts::launch_acf_shift(F, S, T, ldF, STS_FILL_NONE, shift, st), "acf shift");
        HIP_TRY(timed(st, [&] { return sts::launch_acf_wide(F, S, T, ldF, shift, K, shift + S, acf, exact, st); }),
                "autocorr (wide)");
        return es.finish("fill_autocorr");
    }
    if ((r = run_tile(in, method == STS_FILL_NONE ? nullptr : filled, nullptr, S, T, ld_in, ld_out, method, K, acf, 0,
                      0, es.dev, st, "fill_autocorr"))) return r;
    return es.finish("fill_autocorr");
}

int sts_autocorr(const double* in, int64_t S, int64_t T, int64_t ld, int K, double* acf, void* stream) {
    return sts_fill_autocorr(in, nullptr, S, T, ld, ld, STS_FILL_NONE, K, acf, nullptr, stream);
}

int sts_diff_at_lag(const double* in, double* out, int64_t S, int64_t T, int64_t ld_in, int64_t ld_out, int lag,
                    int start, void* stream) {
    int r;
    if (!(start >= lag)) return fail(STS_ERR_REQUIREMENT, "requirement failed: starting index cannot be less than lag");
    if (lag < 0) return fail(STS_ERR_BAD_ARG, "differencesAtLag: negative lag %d", lag);
    if ((r = check_panel(in, S, T, ld_in, "differencesAtLag"))) return r;
    if ((r = check_panel(out, S, T, ld_out, "differencesAtLag"))) return r;
    if (lag == 0 || S * T == 0) return STS_OK;  // dest returned untouched (:363-364)
    if ((r = ensure_device())) return r;
    hipStream_t st = as_stream(stream);
    if (in == out) {
        if (ld_in != ld_out) return fail(STS_ERR_BAD_ARG, "differencesAtLag: in-place call with different ld");
        HIP_TRY(sts::launch_diff_inplace(out, S, T, ld_out, lag, start, st), "differencesAtLag(in place)");
    } else {
        HIP_TRY(sts::launch_diff(in, out, S, T, ld_in, ld_out, lag, start, st), "differencesAtLag");
    }
    return STS_OK;
}

int sts_lag_matrix(const double* in, double* out, int64_t S, int64_t T, int64_t ld_in, int max_lag,
                   int include_original, void* stream) {
    int r;
    if ((r = check_panel(in, S, T, ld_in, "lag"))) return r;
    if (max_lag < 0 || max_lag > T) return fail(STS_ERR_BAD_ARG, "lag: maxLag %d outside [0, T=%lld]", max_lag, (long long)T);
    const int64_t n = S * (T - max_lag) * (max_lag + (include_original ? 1 : 0));
    if (n > 0 && !out) return fail(STS_ERR_BAD_ARG, "lag: null output");
    if (n == 0) return STS_OK;
    if ((r = ensure_device())) return r;
    HIP_TRY(sts::launch_lagmat(in, out, S, T, ld_in, max_lag, include_original, as_stream(stream)), "lag");
    return STS_OK;
}

int sts_fill_lag_matrix(const double* in, double* filled, double* lagmat, int64_t S, int64_t T, int64_t ld_in,
                        int64_t ld_out, int method, int max_lag, int include_original, int32_t* err_per_series,
                        void* stream) {
    int r;
    if ((r = method_ok(method, true, "fill_lag_matrix"))) return r;
    if ((r = check_panel(in, S, T, ld_in, "fill_lag_matrix"))) return r;
    if (filled && (r = check_panel(filled, S, T, ld_out, "fill_lag_matrix"))) return r;
    if (filled && S * T > 0 && filled == in) return fail(STS_ERR_BAD_ARG, "fill_lag_matrix: filled must not alias in");
    if (max_lag < 0 || max_lag > T) return fail(STS_ERR_BAD_ARG, "lag: maxLag %d outside [0, T=%lld]", max_lag, (long long)T);
    const int64_t n = S * (T - max_lag) * (max_lag + (include_original ? 1 : 0));
    if (n > 0 && !lagmat) return fail(STS_ERR_BAD_ARG, "lag: null output");
    if ((r = ensure_device())) return r;
    hipStream_t st = as_stream(stream);
    ErrSink es(err_per_series, S, st);
    if ((r = es.prepare(false))) return r;   // run_tile zeroes err unless its kernel writes all of it
    if (method == STS_FILL_SPLINE) {
        // fillSpline (sts_spline.hip) into `filled` (or a scratch panel), then the lag matrix
        Scratch tmp(st);
        double* F = filled;
        int64_t ldF = ld_out;
        if (!F && S * T > 0) {
            HIP_TRY(tmp.alloc((size_t)(S * T) * sizeof(double)), "hipMallocAsync(filled)");
            F = static_cast<double*>(tmp.p);
            ldF = T;
        }
        if ((r = run_spline(in, F, S, T, ld_in, ldF, es.dev, st))) return r;
        if (n > 0) HIP_TRY(sts::launch_lagmat(F, lagmat, S, T, ldF, max_lag, include_original ? 1 : 0, st), "lag");
        return es.finish("fill_lag_matrix");
    }
    if ((r = run_tile(in, filled, n > 0 ? lagmat : nullptr, S, T, ld_in, ld_out, method, 0, nullptr, max_lag,
                      include_original ? 1 : 0, es.dev, st, "fill_lag_matrix"))) return r;
    return es.finish("fill_lag_matrix");
}

int sts_ewma_add(const double* in, double* out, int64_t S, int64_t T, int64_t ld_in, int64_t ld_out,
                 const double* smoothing, void* stream) {
    int r;
    if (!out) return fail(STS_ERR_NULL_DEST, "EWMAModel.addTimeDependentEffects: dest is null (NullPointerException)");
    if ((r = check_panel(in, S, T, ld_in, "ewma_add"))) return r;
    if ((r = check_panel(out, S, T, ld_out, "ewma_add"))) return r;
    if (S > 0 && !smoothing) return fail(STS_ERR_BAD_ARG, "ewma_add: null smoothing");
    if (S * T == 0) return STS_OK;
    if ((r = ensure_device())) return r;
    sts::RecurArgs a{};
    a.in = in; a.out = out; a.S = S; a.T = T; a.ld_in = ld_in; a.ld_out = ld_out; a.sm = smoothing;
    HIP_TRY(sts::launch_recur(sts::kEwmaAdd, a, as_stream(stream)), "ewma_add");
    return STS_OK;
}

int sts_ewma_remove(const double* in, double* out, int64_t S, int64_t T, int64_t ld_in, int64_t ld_out,
                    const double* smoothing, void* stream) {
    int r;
    if (!out) return fail(STS_ERR_NULL_DEST, "EWMAModel.removeTimeDependentEffects: dest is null (NullPointerException)");
    if ((r = check_panel(in, S, T, ld_in, "ewma_remove"))) return r;
    if ((r = check_panel(out, S, T, ld_out, "ewma_remove"))) return r;
    if (S > 0 && !smoothing) return fail(STS_ERR_BAD_ARG, "ewma_remove: null smoothing");
    if (S * T == 0) return STS_OK;
    if ((r = ensure_device())) return r;
    hipStream_t st = as_stream(stream);
    if (in == out) {
        sts::RecurArgs a{};
        a.in = in; a.out = out; a.S = S; a.T = T; a.ld_in = ld_in; a.ld_out = ld_out; a.sm = smoothing;
        HIP_TRY(sts::launch_recur(sts::kEwmaRemoveInplace, a, st), "ewma_remove(in place)");
    } else {
        HIP_TRY(sts::launch_ewma_remove(in, out, S, T, ld_in, ld_out, smoothing, st), "ewma_remove");
    }
    return STS_OK;
}

int sts_ar_remove(const double* in, double* out, int64_t S, int64_t T, int64_t ld_in, int64_t ld_out,
                  const double* c, const double* coef, int p, void* stream) {
    int r;
    if ((r = check_panel(in, S, T, ld_in, "ar_remove"))) return r;
    if ((r = check_panel(out, S, T, ld_out, "ar_remove"))) return r;
    if (p < 0) return fail(STS_ERR_BAD_ARG, "ar_remove: negative order");
    if (S > 0 && (!c || (p > 0 && !coef))) return fail(STS_ERR_BAD_ARG, "ar_remove: null model");
    if (S * T == 0) return STS_OK;
    if ((r = ensure_device())) return r;
    hipStream_t st = as_stream(stream);
    if (in == out) {
        sts::RecurArgs a{};
        a.in = in; a.out = out; a.S = S; a.T = T; a.ld_in = ld_in; a.ld_out = ld_out; a.c = c; a.coef = coef; a.p = p;
        HIP_TRY(sts::launch_recur(sts::kArRemoveInplace, a, st), "ar_remove(in place)");
    } else {
        HIP_TRY(sts::launch_ar_remove(in, out, S, T, ld_in, ld_out, c, coef, p, st), "ar_remove");
    }
    return STS_OK;
}

int sts_ar_add(const double* in, double* out, int64_t S, int64_t T, int64_t ld_in, int64_t ld_out, const double* c,
               const double* coef, int p, void* stream) {
    int r;
    if ((r = check_panel(in, S, T, ld_in, "ar_add"))) return r;
    if ((r = check_panel(out, S, T, ld_out, "ar_add"))) return r;
    if (p < 0) return fail(STS_ERR_BAD_ARG, "ar_add: negative order");
    if (S > 0 && (!c || (p > 0 && !coef))) return fail(STS_ERR_BAD_ARG, "ar_add: null model");
    if (S * T == 0) return STS_OK;
    if ((r = ensure_device())) return r;
    sts::RecurArgs a{};
    a.in = in; a.out = out; a.S = S; a.T = T; a.ld_in = ld_in; a.ld_out = ld_out; a.c = c; a.coef = coef; a.p = p;
    HIP_TRY(sts::launch_recur(sts::kArAdd, a, as_stream(stream)), "ar_add");
    return STS_OK;
}

static int ar_fit_common(const double* in, double* out, int64_t S, int64_t T, int64_t ld_in, int64_t ld_out, int p,
                         int no_intercept, double* c, double* coef, int32_t* err_per_series, void* stream,
                         const char* name) {
    int r;
    if ((r = check_panel(in, S, T, ld_in, name))) return r;
    if (out && (r = check_panel(out, S, T, ld_out, name))) return r;
    if (p < 1 || p > 31) return fail(STS_ERR_BAD_ARG, "%s: AR order %d outside [1, 31]", name, p);
    if (T - p < (int64_t)p + 1)
        return fail(STS_ERR_NOT_ENOUGH_DATA, "%s: not enough data (%lld rows) for the number of predictors (%d)", name,
                    (long long)(T - p), p);
    if (S > 0 && (!c || !coef)) return fail(STS_ERR_BAD_ARG, "%s: null model output", name);
    if (out && in == out) return fail(STS_ERR_BAD_ARG, "%s: out must not alias in", name);
    if (S == 0) return STS_OK;
    if ((r = ensure_device())) return r;
    hipStream_t st = as_stream(stream);
    ErrSink es(err_per_series, S, st);
    if ((r = es.prepare())) return r;
    sts::ArArgs a{};
    a.in = in; a.out = out; a.c = c; a.coef = coef; a.err = es.dev;
    a.S = S; a.T = T; a.ld_in = ld_in; a.ld_out = ld_out; a.p = p; a.no_intercept = no_intercept ? 1 : 0;
    HIP_TRY(timed(st, [&] { return sts::launch_ar_fit(a, st); }), name);
    return es.finish(name);
}

int sts_ar_fit(const double* in, int64_t S, int64_t T, int64_t ld, int p, int no_intercept, double* c, double* coef,
               int32_t* err_per_series, void* stream) {
    return ar_fit_common(in, nullptr, S, T, ld, ld, p, no_intercept, c, coef, err_per_series, stream, "ar_fit");
}

int sts_ar_rule_count(const double* in, int64_t S, int64_t T, int64_t ld, int p, int no_intercept, int64_t* count,
                      void* stream) {
    int r;
    const char* name = "ar_rule_count";
    if ((r = check_panel(in, S, T, ld, name))) return r;
    if (!count) return fail(STS_ERR_BAD_ARG, "%s: null count", name);
    if (p < 1 || p > 31) return fail(STS_ERR_BAD_ARG, "%s: AR order %d outside [1, 31]", name, p);
    if (T - p < (int64_t)p + 1)
        return fail(STS_ERR_NOT_ENOUGH_DATA, "%s: not enough data (%lld rows) for the number of predictors (%d)", name,
                    (long long)(T - p), p);
    *count = 0;
    if (S == 0) return STS_OK;
    if (no_intercept) {
        *count = S;
        return STS_OK;
    }
    if ((r = ensure_device())) return r;
    hipStream_t st = as_stream(stream);
    Scratch sc(st);
    const size_t S8 = (size_t)S * sizeof(double);
    HIP_TRY(sc.alloc(S8 * (size_t)(p + 1) + S * sizeof(int32_t) + 64), "hipMallocAsync(ar_rule_count)");
    char* base = static_cast<char*>(sc.p);
    sts::ArArgs a{};
    a.in = in; a.out = nullptr; a.c = reinterpret_cast<double*>(base); a.coef = a.c + S;
    a.err = reinterpret_cast<int32_t*>(base + S8 * (size_t)(p + 1));
    a.S = S; a.T = T; a.ld_in = ld; a.ld_out = ld; a.p = p; a.no_intercept = 0;
    uint32_t* dcount = reinterpret_cast<uint32_t*>(base + S8 * (size_t)(p + 1) + S * sizeof(int32_t));
    HIP_TRY(sts::launch_ar_rule_count(a, dcount, st), name);
    uint32_t h = 0;
    HIP_TRY(hipMemcpyAsync(&h, dcount, sizeof(h), hipMemcpyDeviceToHost, st), name);
    HIP_TRY(hipStreamSynchronize(st), name);
    *count = (int64_t)h;
    return STS_OK;
}

int sts_ar_fit_remove(const double* in, double* out, int64_t S, int64_t T, int64_t ld_in, int64_t ld_out, int p,
                      int no_intercept, double* c, double* coef, int32_t* err_per_series, void* stream) {
    if (!out) return fail(STS_ERR_BAD_ARG, "ar_fit_remove: null output");
    return ar_fit_common(in, out, S, T, ld_in, ld_out, p, no_intercept, c, coef, err_per_series, stream,
                         "ar_fit_remove");
}

int sts_ewma_fit(const double* in, int64_t S, int64_t T, int64_t ld, double* smoothing, int32_t* err_per_series,
                 void* stream) {
    int r;
    if ((r = check_panel(in, S, T, ld, "EWMA.fitModel"))) return r;
    if (S > 0 && T < 1) return fail(STS_ERR_BAD_ARG, "EWMA.fitModel: empty series (ts(0) does not exist)");
    if (S > 0 && !smoothing) return fail(STS_ERR_BAD_ARG, "EWMA.fitModel: null output");
    if (S == 0) return STS_OK;
    if ((r = ensure_device())) return r;
    hipStream_t st = as_stream(stream);
    ErrSink es(err_per_series, S, st);
    if ((r = es.prepare())) return r;
    sts::EwmaFitArgs a{};
    a.in = in; a.S = S; a.T = T; a.ld = ld; a.smoothing = smoothing; a.err = es.dev;
    HIP_TRY(timed(st, [&] { return sts::launch_ewma_fit(a, true, st); }), "EWMA.fitModel");
    return es.finish("EWMA.fitModel");
}

int sts_ewma_sse_gradient(const double* in, int64_t S, int64_t T, int64_t ld, const double* smoothing, double* sse,
                          double* gradient, void* stream) {
    int r;
    if ((r = check_panel(in, S, T, ld, "EWMAModel.sse"))) return r;
    if (S > 0 && T < 1) return fail(STS_ERR_BAD_ARG, "EWMAModel.sse: empty series (ts(0) does not exist)");
    if (S > 0 && !smoothing) return fail(STS_ERR_BAD_ARG, "EWMAModel.sse: null smoothing");
    if (S == 0 || (!sse && !gradient)) return STS_OK;
    if ((r = ensure_device())) return r;
    hipStream_t st = as_stream(stream);
    sts::EwmaFitArgs a{};
    a.in = in; a.S = S; a.T = T; a.ld = ld; a.smoothing = const_cast<double*>(smoothing);
    a.sse = sse; a.grad = gradient;
    HIP_TRY(timed(st, [&] { return sts::launch_ewma_fit(a, false, st); }), "EWMAModel.sse/gradient");
    return STS_OK;
}

// ---- GARCH(1,1) / AR(1)+GARCH(1,1): S/models/GARCH.scala ----

int sts_garch_fit(const double* in, int64_t S, int64_t T, int64_t ld, double* params, int32_t* err_per_series,
                  void* stream) {
    int r;
    if ((r = check_panel(in, S, T, ld, "GARCH.fitModel"))) return r;
    if (S > 0 && !params) return fail(STS_ERR_BAD_ARG, "GARCH.fitModel: null output");
    if (S == 0) return STS_OK;
    if ((r = ensure_device())) return r;
    hipStream_t st = as_stream(stream);
    ErrSink es(err_per_series, S, st);
    if ((r = es.prepare())) return r;
    sts::GarchFitArgs a{};
    a.in = in; a.S = S; a.T = T; a.ld = ld; a.params = params; a.err = es.dev;
    HIP_TRY(timed(st, [&] { return sts::launch_garch_fit(a, true, st); }), "GARCH.fitModel");
    return es.finish("GARCH.fitModel");
}

int sts_garch_loglik_gradient(const double* in, int64_t S, int64_t T, int64_t ld, const double* params,
                              double* loglik, double* gradient, void* stream) {
    int r;
    if ((r = check_panel(in, S, T, ld, "GARCHModel.logLikelihood"))) return r;
    if (S > 0 && !params) return fail(STS_ERR_BAD_ARG, "GARCHModel.logLikelihood: null params");
    if (S == 0 || (!loglik && !gradient)) return STS_OK;
    if ((r = ensure_device())) return r;
    hipStream_t st = as_stream(stream);
    sts::GarchFitArgs a{};
    a.in = in; a.S = S; a.T = T; a.ld = ld; a.params = const_cast<double*>(params);
    a.loglik = loglik; a.grad = gradient;
    HIP_TRY(timed(st, [&] { return sts::launch_garch_fit(a, false, st); }), "GARCHModel.logLikelihood/gradient");
    return STS_OK;
}

static int garch_effects(int op, const double* in, double* out, int64_t S, int64_t T, int64_t ld_in, int64_t ld_out,
                         const double* c, const double* phi, const double* omega, const double* alpha,
                         const double* beta, void* stream, const char* name) {
    int r;
    if ((r = check_panel(in, S, T, ld_in, name))) return r;
    if (!out) return fail(STS_ERR_NULL_DEST, "%s: dest is null (the reference writes into dest)", name);
    if ((r = check_panel(out, S, T, ld_out, name))) return r;
    if (S > 0 && (!omega || !alpha || !beta)) return fail(STS_ERR_BAD_ARG, "%s: null model parameters", name);
    const bool ar = op != sts::kGarchRemove && op != sts::kGarchAdd;
    if (S > 0 && ar && (!c || !phi)) return fail(STS_ERR_BAD_ARG, "%s: null model parameters", name);
    if (S * T == 0) return STS_OK;
    if (in == out && ld_in != ld_out) return fail(STS_ERR_BAD_ARG, "%s: in place needs ld_in == ld_out", name);
    if (op == sts::kArgarchRemove && in == out) op = sts::kArgarchRemoveInplace;   // dest eq ts
    if ((r = ensure_device())) return r;
    hipStream_t st = as_stream(stream);
    sts::GarchEffectsArgs a{};
    a.in = in; a.out = out; a.S = S; a.T = T; a.ld_in = ld_in; a.ld_out = ld_out;
    a.c = c; a.phi = phi; a.omega = omega; a.alpha = alpha; a.beta = beta;
    HIP_TRY(timed(st, [&] { return sts::launch_garch_effects(op, a, st); }), name);
    return STS_OK;
}

int sts_garch_remove(const double* in, double* out, int64_t S, int64_t T, int64_t ld_in, int64_t ld_out,
                     const double* omega, const double* alpha, const double* beta, void* stream) {
    return garch_effects(sts::kGarchRemove, in, out, S, T, ld_in, ld_out, nullptr, nullptr, omega, alpha, beta,
                         stream, "GARCHModel.removeTimeDependentEffects");
}

int sts_garch_add(const double* in, double* out, int64_t S, int64_t T, int64_t ld_in, int64_t ld_out,
                  const double* omega, const double* alpha, const double* beta, void* stream) {
    return garch_effects(sts::kGarchAdd, in, out, S, T, ld_in, ld_out, nullptr, nullptr, omega, alpha, beta, stream,
                         "GARCHModel.addTimeDependentEffects");
}

int sts_argarch_remove(const double* in, double* out, int64_t S, int64_t T, int64_t ld_in, int64_t ld_out,
                       const double* c, const double* phi, const double* omega, const double* alpha,
                       const double* beta, void* stream) {
    return garch_effects(sts::kArgarchRemove, in, out, S, T, ld_in, ld_out, c, phi, omega, alpha, beta, stream,
                         "ARGARCHModel.removeTimeDependentEffects");
}

int sts_argarch_add(const double* in, double* out, int64_t S, int64_t T, int64_t ld_in, int64_t ld_out,
                    const double* c, const double* phi, const double* omega, const double* alpha,
                    const double* beta, void* stream) {
    return garch_effects(sts::kArgarchAdd, in, out, S, T, ld_in, ld_out, c, phi, omega, alpha, beta, stream,
                         "ARGARCHModel.addTimeDependentEffects");
}

int sts_argarch_fit(const double* in, int64_t S, int64_t T, int64_t ld, double* c, double* phi, double* params,
                    int32_t* err_per_series, void* stream) {
    int r;
    if ((r = check_panel(in, S, T, ld, "ARGARCH.fitModel"))) return r;
    if (S > 0 && (!c || !phi || !params)) return fail(STS_ERR_BAD_ARG, "ARGARCH.fitModel: null output");
    if (T - 1 < 2)
        return fail(STS_ERR_NOT_ENOUGH_DATA, "ARGARCH.fitModel: not enough data (%lld rows) for the number of predictors (1)",
                    (long long)(T - 1));
    if (S == 0) return STS_OK;
    if ((r = ensure_device())) return r;
    hipStream_t st = as_stream(stream);
    ErrSink es(err_per_series, S, st);
    if ((r = es.prepare())) return r;
    // Autoregression.fitModel(ts) = AR(1) with intercept; residuals into dest = zeros(n)
    Scratch resid(st);
    HIP_TRY(resid.alloc((size_t)(S * T) * sizeof(double)), "hipMallocAsync(argarch)");
    double* rs = static_cast<double*>(resid.p);
    sts::ArArgs ar{};
    ar.in = in; ar.out = rs; ar.c = c; ar.coef = phi; ar.err = es.dev;
    ar.S = S; ar.T = T; ar.ld_in = ld; ar.ld_out = T; ar.p = 1; ar.no_intercept = 0;
    HIP_TRY(timed(st, [&] { return sts::launch_ar_fit(ar, st); }), "ARGARCH.fitModel (AR stage)");
    // GARCH.fitModel(residuals); an AR-stage failure keeps its status
    sts::GarchFitArgs g{};
    g.in = rs; g.S = S; g.T = T; g.ld = T; g.params = params; g.err = es.dev; g.keep_err = 1;
    HIP_TRY(timed(st, [&] { return sts::launch_garch_fit(g, true, st); }), "ARGARCH.fitModel (GARCH stage)");
    return es.finish("ARGARCH.fitModel");
}

int sts_series_stats(const double* in, int64_t S, int64_t T, int64_t ld, double* stats, void* stream) {
    int r;
    if ((r = check_panel(in, S, T, ld, "seriesStats"))) return r;
    if (S > 0 && !stats) return fail(STS_ERR_BAD_ARG, "seriesStats: null output");
    if (S == 0) return STS_OK;
    if ((r = ensure_device())) return r;
    hipStream_t st = as_stream(stream);
    HIP_TRY(timed(st, [&] { return sts::launch_series_stats(in, stats, S, T, ld, st); }), "seriesStats");
    return STS_OK;
}

int sts_nan_instants(const double* in, int64_t S, int64_t T, int64_t ld, uint8_t* flags, void* stream) {
    int r;
    if ((r = check_panel(in, S, T, ld, "removeInstantsWithNaNs"))) return r;
    if (T > 0 && !flags) return fail(STS_ERR_BAD_ARG, "removeInstantsWithNaNs: null flags");
    if (S * T == 0) return STS_OK;
    if ((r = ensure_device())) return r;
    hipStream_t st = as_stream(stream);
    HIP_TRY(timed(st, [&] { return sts::launch_nan_instants(in, flags, S, T, ld, st); }), "nan_instants");
    return STS_OK;
}

int sts_active_instants(const uint8_t* flags, int64_t T, int64_t* active, int64_t* n_active, void* stream) {
    if (T < 0) return fail(STS_ERR_BAD_ARG, "active_instants: negative T");
    if (!n_active || (T > 0 && (!flags || !active))) return fail(STS_ERR_BAD_ARG, "active_instants: null pointer");
    int r;
    if ((r = ensure_device())) return r;
    hipStream_t st = as_stream(stream);
    Scratch sc(st);
    HIP_TRY(sc.alloc((size_t)sts::active_scratch_elems(T) * sizeof(int64_t)), "hipMallocAsync(active scratch)");
    HIP_TRY(sts::launch_active_instants(flags, T, active, n_active, static_cast<int64_t*>(sc.p), st), "active_instants");
    return STS_OK;
}

int sts_gather_instants(const double* in, double* out, int64_t S, int64_t ld_in, int64_t ld_out, const int64_t* active,
                        int64_t n_active, void* stream) {
    if (S < 0 || n_active < 0 || ld_out < n_active) return fail(STS_ERR_BAD_ARG, "gather_instants: bad shape");
    if (S * n_active > 0 && (!in || !out || !active)) return fail(STS_ERR_BAD_ARG, "gather_instants: null pointer");
    if (S * n_active == 0) return STS_OK;
    int r;
    if ((r = ensure_device())) return r;
    hipStream_t st = as_stream(stream);
    HIP_TRY(timed(st, [&] { return sts::launch_gather_instants(in, out, active, n_active, S, ld_in, ld_out, st); }),
            "gather_instants");
    return STS_OK;
}

int sts_to_instants(const double* in, double* out, int64_t S, int64_t T, int64_t ld_in, int64_t ld_out, void* stream) {
    int r;
    if ((r = check_panel(in, S, T, ld_in, "toInstants"))) return r;
    if (ld_out < S) return fail(STS_ERR_BAD_ARG, "toInstants: ld_out %lld < S=%lld", (long long)ld_out, (long long)S);
    if (S * T > 0 && !out) return fail(STS_ERR_BAD_ARG, "toInstants: null output");
    if (S * T == 0) return STS_OK;
    if ((r = ensure_device())) return r;
    hipStream_t st = as_stream(stream);
    HIP_TRY(timed(st, [&] { return sts::launch_transpose(in, out, S, T, ld_in, ld_out, st); }), "toInstants");
    return STS_OK;
}

static inline int64_t be32(const uint8_t* p) {
    return (int64_t)(int32_t)(((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | (uint32_t)p[3]);
}

int sts_wire_scan(const uint8_t* bytes, int64_t nbytes, int64_t max_records, int64_t* n_records, int64_t* T,
                  int64_t* key_off, int32_t* key_len, int64_t* val_off) {
    if (!n_records || !T || nbytes < 0 || (nbytes > 0 && !bytes)) return fail(STS_ERR_BAD_ARG, "wire_scan: bad arguments");
    int64_t pos = 0, n = 0, len = -1;
    while (pos < nbytes) {
        if (pos + 4 > nbytes) return fail(STS_ERR_BAD_ARG, "wire_scan: truncated key length at byte %lld", (long long)pos);
        const int64_t kl = be32(bytes + pos);
        if (kl < 0 || pos + 4 + kl + 4 > nbytes)
            return fail(STS_ERR_BAD_ARG, "wire_scan: bad key length %lld at byte %lld", (long long)kl, (long long)pos);
        const int64_t vn = be32(bytes + pos + 4 + kl);
        if (vn < 0 || pos + 8 + kl + 8 * vn > nbytes)
            return fail(STS_ERR_BAD_ARG, "wire_scan: bad series length %lld at byte %lld", (long long)vn, (long long)pos);
        if (len >= 0 && vn != len)
            return fail(STS_ERR_BAD_ARG, "wire_scan: record %lld holds %lld values, record 0 holds %lld (one shared index)",
                        (long long)n, (long long)vn, (long long)len);
        len = vn;
        if (n < max_records) {
            if (key_off) key_off[n] = pos + 4;
            if (key_len) key_len[n] = (int32_t)kl;
            if (val_off) val_off[n] = pos + 8 + kl;
        }
        n++;
        pos += 8 + kl + 8 * vn;
    }
    *n_records = n;
    *T = len < 0 ? 0 : len;
    return n > max_records ? fail(STS_ERR_BAD_ARG, "wire_scan: %lld records > capacity %lld", (long long)n,
                                  (long long)max_records)
                           : STS_OK;
}

int sts_wire_decode(const uint8_t* bytes, const int64_t* val_off, int64_t S, int64_t T, double* panel, int64_t ld,
                    void* stream) {
    int r;
    if ((r = check_panel(panel, S, T, ld, "wire_decode"))) return r;
    if (S * T > 0 && (!bytes || !val_off)) return fail(STS_ERR_BAD_ARG, "wire_decode: null pointer");
    if (S * T == 0) return STS_OK;
    if ((r = ensure_device())) return r;
    hipStream_t st = as_stream(stream);
    HIP_TRY(timed(st, [&] { return sts::launch_wire_decode(bytes, val_off, panel, S, T, ld, st); }), "wire_decode");
    return STS_OK;
}

int sts_wire_encode(const double* panel, int64_t S, int64_t T, int64_t ld, const int64_t* val_off, uint8_t* bytes,
                    void* stream) {
    int r;
    if ((r = check_panel(panel, S, T, ld, "wire_encode"))) return r;
    if (S * T > 0 && (!bytes || !val_off)) return fail(STS_ERR_BAD_ARG, "wire_encode: null pointer");
    if (S * T == 0) return STS_OK;
    if ((r = ensure_device())) return r;
    hipStream_t st = as_stream(stream);
    HIP_TRY(timed(st, [&] { return sts::launch_wire_encode(panel, S, T, ld, val_off, bytes, st); }), "wire_encode");
    return STS_OK;
}

int sts_observations_to_panel(const int32_t* series_id, const int64_t* loc, const double* value, int64_t n_obs,
                              double* panel, int64_t S, int64_t T, int64_t ld, void* stream) {
    int r;
    if ((r = check_panel(panel, S, T, ld, "timeSeriesRDDFromObservations"))) return r;
    if (n_obs < 0 || (n_obs > 0 && (!series_id || !loc || !value)))
        return fail(STS_ERR_BAD_ARG, "timeSeriesRDDFromObservations: bad observation arrays");
    if (S * T == 0) return STS_OK;
    if ((r = ensure_device())) return r;
    hipStream_t st = as_stream(stream);
    Scratch win(st);
    HIP_TRY(win.alloc((size_t)(n_obs > 0 ? n_obs : 1)), "hipMallocAsync(obs flags)");
    HIP_TRY(timed(st, [&] {
                return sts::launch_observations(series_id, loc, value, n_obs, panel, S, T, ld,
                                                static_cast<unsigned char*>(win.p), st);
            }),
            "timeSeriesRDDFromObservations");
    return STS_OK;
}

// java.lang.Double.parseDouble for the tokens Double.toString writes (decimal, optional
// exponent, NaN, Infinity, -Infinity); surrounding whitespace is trimmed like Java's.
static bool parse_java_double(const char* b, const char* e, double* out) {
    while (b < e && (unsigned char)*b <= ' ') b++;
    while (e > b && (unsigned char)e[-1] <= ' ') e--;
    const size_t n = (size_t)(e - b);
    if (n == 0 || n > 400) return false;
    char buf[401];
    std::memcpy(buf, b, n);
    buf[n] = 0;
    const char* q = buf;
    const bool neg = (*q == '-'), sgn = (neg || *q == '+');
    if (sgn) q++;
    if (!std::strcmp(q, "NaN")) { *out = NAN; return true; }
    if (!std::strcmp(q, "Infinity")) { *out = neg ? -INFINITY : INFINITY; return true; }
    for (const char* c = q; *c; c++)   // decimal digits, '.', exponent (strtod would also take hex / "inf")
        if (!((*c >= '0' && *c <= '9') || *c == '.' || *c == 'e' || *c == 'E' || *c == '+' || *c == '-' ||
              *c == 'd' || *c == 'D' || *c == 'f' || *c == 'F'))
            return false;
    if (n > 0 && (buf[n - 1] == 'd' || buf[n - 1] == 'D' || buf[n - 1] == 'f' || buf[n - 1] == 'F')) buf[n - 1] = 0;
    char* end = nullptr;
    *out = std::strtod(buf, &end);   // correctly rounded (glibc), as parseDouble is
    return end && *end == 0 && end != q;
}

int sts_csv_parse(const char* text, int64_t len, int64_t max_records, int64_t* n_records, int64_t* T,
                  int64_t* key_off, int32_t* key_len, double* values, int64_t values_cap) {
    if (!n_records || !T || len < 0 || (len > 0 && !text)) return fail(STS_ERR_BAD_ARG, "csv_parse: bad arguments");
    int64_t pos = 0, n = 0, width = -1;
    while (pos < len) {
        int64_t eol = pos;
        while (eol < len && text[eol] != '\n') eol++;
        int64_t end = eol;
        if (end > pos && text[end - 1] == '\r') end--;
        if (end > pos) {   // sc.textFile skips nothing, but an empty trailing line is no record
            int64_t c = pos;
            while (c < end && text[c] != ',') c++;
            int64_t cnt = 0;
            int64_t f = c;
            while (f < end) {   // tokens.tail
                const int64_t g0 = f + 1;
                int64_t g = g0;
                while (g < end && text[g] != ',') g++;
                double v;
                if (!parse_java_double(text + g0, text + g, &v))
                    return fail(STS_ERR_BAD_ARG, "csv_parse: NumberFormatException at line %lld: \"%.*s\"", (long long)n,
                                (int)(g - g0 > 64 ? 64 : g - g0), text + g0);
                if (n < max_records && values && width >= 0 && n * width + cnt < values_cap) values[n * width + cnt] = v;
                else if (n < max_records && values && width < 0 && cnt < values_cap) values[cnt] = v;
                cnt++;
                f = g;
            }
            if (width >= 0 && cnt != width)
                return fail(STS_ERR_BAD_ARG, "csv_parse: line %lld holds %lld values, line 0 holds %lld", (long long)n,
                            (long long)cnt, (long long)width);
            width = cnt;
            if ((n + 1) * width > values_cap && values)
                return fail(STS_ERR_BAD_ARG, "csv_parse: values capacity %lld exceeded", (long long)values_cap);
            if (n < max_records) {
                if (key_off) key_off[n] = pos;
                if (key_len) key_len[n] = (int32_t)(c - pos);
            }
            n++;
        }
        pos = eol + 1;
    }
    *n_records = n;
    *T = width < 0 ? 0 : width;
    return n > max_records ? fail(STS_ERR_BAD_ARG, "csv_parse: %lld lines > capacity %lld", (long long)n,
                                  (long long)max_records)
                           : STS_OK;
}

int sts_arima_fit_ar(const double* in, int64_t S, int64_t T, int64_t ld, int p, int d, int include_intercept,
                     double* c, double* coef, int32_t* err_per_series, void* stream) {
    int r;
    if ((r = check_panel(in, S, T, ld, "ARIMA.fitModel"))) return r;
    if (d < 0 || d > T) return fail(STS_ERR_BAD_ARG, "ARIMA.fitModel: differencing order %d outside [0, T]", d);
    if (d == 0) return sts_ar_fit(in, S, T, ld, p, include_intercept ? 0 : 1, c, coef, err_per_series, stream);
    if (p < 1 || p > 31) return fail(STS_ERR_BAD_ARG, "ARIMA.fitModel: AR order %d outside [1, 31]", p);
    const int64_t Tn = T - d;
    if (Tn - p < (int64_t)p + 1)
        return fail(STS_ERR_NOT_ENOUGH_DATA, "ARIMA.fitModel: not enough data (%lld rows) for the number of predictors (%d)",
                    (long long)(Tn - p), p);
    if (S == 0) return STS_OK;
    if ((r = ensure_device())) return r;
    hipStream_t st = as_stream(stream);
    // differencesOfOrderD: level i differences level i-1 at lag 1 from index i (ping-pong)
    Scratch bufA(st), bufB(st);
    HIP_TRY(bufA.alloc((size_t)(S * T) * sizeof(double)), "hipMallocAsync(arima)");
    if (d > 1) HIP_TRY(bufB.alloc((size_t)(S * T) * sizeof(double)), "hipMallocAsync(arima)");
    const double* cur = in;
    int64_t cur_ld = ld;
    double* bufs[2] = {static_cast<double*>(bufA.p), static_cast<double*>(bufB.p)};
    for (int i = 1; i <= d; i++) {
        double* nxt = bufs[(i - 1) & 1];
        HIP_TRY(sts::launch_diff(cur, nxt, S, T, cur_ld, T, 1, i, st), "differencesOfOrderD");
        cur = nxt;
        cur_ld = T;
    }
    // .drop(d), then Autoregression.fitModel(diffed, p, !includeIntercept)
    return sts_ar_fit(cur + d, S, Tn, T, p, include_intercept ? 0 : 1, c, coef, err_per_series, stream);
}

int sts_fill_diff_ewma(const double* in, double* out, int64_t S, int64_t T, int64_t ld_in, int64_t ld_out, int method,
                       int lag, const double* smoothing, int32_t* err_per_series, void* stream) {
    int r;
    if ((r = method_ok(method, true, "fill_diff_ewma"))) return r;
    if ((r = check_panel(in, S, T, ld_in, "fill_diff_ewma"))) return r;
    if ((r = check_panel(out, S, T, ld_out, "fill_diff_ewma"))) return r;
    if (lag < 0) return fail(STS_ERR_BAD_ARG, "fill_diff_ewma: negative lag");
    if (S > 0 && !smoothing) return fail(STS_ERR_BAD_ARG, "fill_diff_ewma: null smoothing");
    if (S * T > 0 && in == out) return fail(STS_ERR_BAD_ARG, "fill_diff_ewma: out must not alias in");
    if (S * T == 0) return STS_OK;
    if ((r = ensure_device())) return r;
    hipStream_t st = as_stream(stream);
    ErrSink es(err_per_series, S, st);
    if ((r = es.prepare())) return r;
    if ((method == STS_FILL_PREVIOUS || method == STS_FILL_NONE) && lag >= 1 && lag <= 32 && method == STS_FILL_PREVIOUS) {
        sts::RecurArgs a{};
        a.in = in; a.out = out; a.S = S; a.T = T; a.ld_in = ld_in; a.ld_out = ld_out; a.sm = smoothing;
        a.lag = lag; a.start = lag; a.method = method;
        HIP_TRY(timed(st, [&] { return sts::launch_recur(sts::kFillDiffEwma, a, st); }), "fill_diff_ewma");
        return es.finish("fill_diff_ewma");
    }
    // general composition: fill (a fresh vector) -> differencesAtLag(filled, lag), which reads
    // the FILLED values (out of place: the reference's (ts, lag) form copies, :384-386) ->
    // EWMA add in place on `out` (dest eq ts is safe for add, S/models/EWMA.scala:135-142)
    const double* F = in;
    int64_t ldF = ld_in;
    Scratch tmp(st);
    if (method != STS_FILL_NONE) {
        double* f = out;
        if (lag > 0) {
            HIP_TRY(tmp.alloc((size_t)(S * T) * sizeof(double)), "hipMallocAsync(filled)");
            f = static_cast<double*>(tmp.p);
        }
        const int64_t ldf = lag > 0 ? T : ld_out;
        if ((r = run_tile(in, f, nullptr, S, T, ld_in, ldf, method, 0, nullptr, 0, 0, es.dev, st, "fill"))) return r;
        F = f;
        ldF = ldf;
    }
    if (lag > 0) {
        HIP_TRY(sts::launch_diff(F, out, S, T, ldF, ld_out, lag, lag, st), "differencesAtLag");
    } else if (F != out) {
        HIP_TRY(hipMemcpy2DAsync(out, ld_out * sizeof(double), F, ldF * sizeof(double), T * sizeof(double), S,
                                 hipMemcpyDeviceToDevice, st), "copy");
    }
    sts::RecurArgs a{};
    a.in = out; a.out = out; a.S = S; a.T = T; a.ld_in = ld_out; a.ld_out = ld_out; a.sm = smoothing;
    HIP_TRY(sts::launch_recur(sts::kEwmaAdd, a, st), "ewma_add");
    return es.finish("fill_diff_ewma");
}

int sts_gen_panel(double* out, int64_t s0, int64_t S, int64_t T, int64_t ld, uint64_t seed, double nan_p,
                  void* stream) {
    int r;
    if ((r = check_panel(out, S, T, ld, "gen_panel"))) return r;
    if ((r = ensure_device())) return r;
    uint32_t thr = 0;
    if (nan_p >= 1.0) thr = 0xFFFFFFFFu;
    else if (nan_p > 0.0) thr = (uint32_t)std::floor(nan_p * 4294967296.0);
    HIP_TRY(sts::launch_gen_panel(out, s0, S, T, ld, seed, thr, as_stream(stream)), "gen_panel");
    return STS_OK;
}

int sts_gen_ar_panel(double* out, double* c, double* phi, int64_t s0, int64_t S, int64_t T, int64_t ld, uint64_t seed,
                     int p, void* stream) {
    int r;
    if ((r = check_panel(out, S, T, ld, "gen_ar_panel"))) return r;
    if (p < 1 || p > 32) return fail(STS_ERR_BAD_ARG, "gen_ar_panel: order %d outside [1, 32]", p);
    if (S > 0 && (!c || !phi)) return fail(STS_ERR_BAD_ARG, "gen_ar_panel: null parameter outputs");
    if ((r = ensure_device())) return r;
    HIP_TRY(sts::launch_gen_ar(out, c, phi, s0, S, T, ld, seed, p, as_stream(stream)), "gen_ar_panel");
    return STS_OK;
}

}  // extern "C"
