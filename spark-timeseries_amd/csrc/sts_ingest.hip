// sts_ingest.hip -- the step before the hot path: staging a
// partition's records into the HBM panel, and the way back out.
//
//   Python wire format  S/PythonConnector.scala:47-90 (BytesToKeyAndSeries /
//                       KeyAndSeriesToBytes), python/sparkts/timeseriesrdd.py:239-290:
//                       record = int32 BE keyLen | keyLen UTF-8 bytes | int32 BE n | n x f64 BE
//   observations        S/TimeSeriesRDD.scala:493-542 (timeSeriesRDDFromObservations): NaN
//                       panel, every (key, timestamp, value) written at locAtDateTime
//   CSV                 S/TimeSeriesRDD.scala:547-561 (timeSeriesRDDFromCsv): "key,v1,...,vn"
//
// Device side: the big-endian value blocks are byte-swapped by a gather kernel straight
// from the staged record bytes into the series-contiguous panel (and back for encoding);
// observations are scattered into a NaN-filled panel with a deterministic last-writer rule.
// The per-record headers (O(S) bytes) are parsed on the host (sts_api.cpp).
#include "sts_internal.hpp"

#include <hip/hip_runtime.h>

#ifndef STS_WIRE_ROWS
#define STS_WIRE_ROWS 1               // one wave per record for short series
#endif

namespace sts {
namespace {

__device__ __forceinline__ unsigned long long bswap64(unsigned long long v) { return __builtin_bswap64(v); }

// panel[s*ld + t] = BE double at bytes[val_off[s] + 8 t]; 8-byte loads when the block is
// aligned (the common case: keys padded by the writer), byte loads otherwise.
__global__ __launch_bounds__(256) void wire_decode_kernel(const unsigned char* __restrict__ bytes,
                                                          const int64_t* __restrict__ val_off, double* __restrict__ panel,
                                                          int64_t T, int64_t ld) {
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int64_t s = blockIdx.y;
    if (t >= T) return;
    const unsigned char* p = bytes + val_off[s] + 8 * t;
    unsigned long long v;
    if ((reinterpret_cast<uintptr_t>(p) & 7) == 0) {
        v = bswap64(*reinterpret_cast<const unsigned long long*>(p));
    } else {
        v = 0;
#pragma unroll
        for (int i = 0; i < 8; i++) v = (v << 8) | p[i];
    }
    panel[s * ld + t] = __longlong_as_double((long long)v);
}

// Short series (T <= kRowT): one wave per record, 4 records per block, so a few-hundred-
// value record does not leave most of a 256-wide block idle.
constexpr int kRowT = 4096;
__global__ __launch_bounds__(256) void wire_decode_rows_kernel(const unsigned char* __restrict__ bytes,
                                                               const int64_t* __restrict__ val_off,
                                                               double* __restrict__ panel, int64_t S, int64_t T,
                                                               int64_t ld) {
    const int64_t s = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (s >= S) return;
    const unsigned char* p = bytes + val_off[s];
    double* o = panel + s * ld;
    if ((reinterpret_cast<uintptr_t>(p) & 7) == 0) {
        const unsigned long long* q = reinterpret_cast<const unsigned long long*>(p);
        for (int64_t t = threadIdx.x & 63; t < T; t += 64) o[t] = __longlong_as_double((long long)bswap64(q[t]));
    } else {
        for (int64_t t = threadIdx.x & 63; t < T; t += 64) {
            unsigned long long v = 0;
#pragma unroll
            for (int i = 0; i < 8; i++) v = (v << 8) | p[8 * t + i];
            o[t] = __longlong_as_double((long long)v);
        }
    }
}

// the reverse: BE doubles of series s into bytes[val_off[s] ...]
__global__ __launch_bounds__(256) void wire_encode_kernel(const double* __restrict__ panel, int64_t T, int64_t ld,
                                                          const int64_t* __restrict__ val_off,
                                                          unsigned char* __restrict__ bytes) {
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int64_t s = blockIdx.y;
    if (t >= T) return;
    const unsigned long long v = (unsigned long long)__double_as_longlong(panel[s * ld + t]);
    unsigned char* p = bytes + val_off[s] + 8 * t;
    if ((reinterpret_cast<uintptr_t>(p) & 7) == 0) {
        *reinterpret_cast<unsigned long long*>(p) = bswap64(v);
    } else {
#pragma unroll
        for (int i = 0; i < 8; i++) p[i] = (unsigned char)(v >> (56 - 8 * i));
    }
}

__global__ __launch_bounds__(256) void wire_encode_rows_kernel(const double* __restrict__ panel, int64_t S, int64_t T,
                                                               int64_t ld, const int64_t* __restrict__ val_off,
                                                               unsigned char* __restrict__ bytes) {
    const int64_t s = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (s >= S) return;
    unsigned char* p = bytes + val_off[s];
    const double* x = panel + s * ld;
    if ((reinterpret_cast<uintptr_t>(p) & 7) == 0) {
        unsigned long long* q = reinterpret_cast<unsigned long long*>(p);
        for (int64_t t = threadIdx.x & 63; t < T; t += 64) q[t] = bswap64((unsigned long long)__double_as_longlong(x[t]));
    } else {
        for (int64_t t = threadIdx.x & 63; t < T; t += 64) {
            const unsigned long long v = (unsigned long long)__double_as_longlong(x[t]);
#pragma unroll
            for (int i = 0; i < 8; i++) p[8 * t + i] = (unsigned char)(v >> (56 - 8 * i));
        }
    }
}

// observations, last writer in input order wins a cell.  The panel itself holds the
// winning observation index (as uint64, zeroed first) until the winners are marked, so the
// only scratch is one byte per observation.
__global__ __launch_bounds__(256) void obs_winner_kernel(const int32_t* __restrict__ sid, const int64_t* __restrict__ loc,
                                                         int64_t n, int64_t S, int64_t T, double* panel, int64_t ld) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const int64_t s = sid[i], t = loc[i];
    if (s < 0 || s >= S || t < 0 || t >= T) return;   // locAtDateTime == -1: dropped (:529-535)
    atomicMax(reinterpret_cast<unsigned long long*>(panel + s * ld + t), (unsigned long long)(i + 1));
}

__global__ __launch_bounds__(256) void obs_mark_kernel(const int32_t* __restrict__ sid, const int64_t* __restrict__ loc,
                                                       int64_t n, int64_t S, int64_t T, const double* panel, int64_t ld,
                                                       unsigned char* __restrict__ win) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const int64_t s = sid[i], t = loc[i];
    bool w = false;
    if (s >= 0 && s < S && t >= 0 && t < T)
        w = *reinterpret_cast<const unsigned long long*>(panel + s * ld + t) == (unsigned long long)(i + 1);
    win[i] = w ? 1 : 0;
}

__global__ __launch_bounds__(256) void obs_scatter_kernel(const int32_t* __restrict__ sid, const int64_t* __restrict__ loc,
                                                          const double* __restrict__ val, int64_t n,
                                                          const unsigned char* __restrict__ win, double* __restrict__ panel,
                                                          int64_t ld) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n && win[i]) panel[(int64_t)sid[i] * ld + loc[i]] = val[i];
}

__global__ __launch_bounds__(256) void fill_nan_kernel(double* panel, int64_t S, int64_t T, int64_t ld) {
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int64_t s = blockIdx.y;
    if (t < T) panel[s * ld + t] = __builtin_nan("");
}

template <typename F>
hipError_t per_series_grid(int64_t S, int64_t T, F&& launch) {
    for (int64_t s = 0; s < S; s += 65535) {
        const int64_t n = (S - s < 65535) ? S - s : 65535;
        launch(s, dim3((unsigned)((T + 255) / 256), (unsigned)n));
    }
    return hipGetLastError();
}

}  // namespace

hipError_t launch_wire_decode(const unsigned char* bytes, const int64_t* val_off, double* panel, int64_t S, int64_t T,
                              int64_t ld, hipStream_t st) {
    if (S <= 0 || T <= 0) return hipSuccess;
    if (STS_WIRE_ROWS && T <= kRowT && (S + 3) / 4 <= 0x7fffffffLL) {
        hipLaunchKernelGGL(wire_decode_rows_kernel, dim3((unsigned)((S + 3) / 4)), dim3(256), 0, st, bytes, val_off,
                           panel, S, T, ld);
        return hipGetLastError();
    }
    return per_series_grid(S, T, [&](int64_t s, dim3 g) {
        hipLaunchKernelGGL(wire_decode_kernel, g, dim3(256), 0, st, bytes, val_off + s, panel + s * ld, T, ld);
    });
}

hipError_t launch_wire_encode(const double* panel, int64_t S, int64_t T, int64_t ld, const int64_t* val_off,
                              unsigned char* bytes, hipStream_t st) {
    if (S <= 0 || T <= 0) return hipSuccess;
    if (STS_WIRE_ROWS && T <= kRowT && (S + 3) / 4 <= 0x7fffffffLL) {
        hipLaunchKernelGGL(wire_encode_rows_kernel, dim3((unsigned)((S + 3) / 4)), dim3(256), 0, st, panel, S, T, ld,
                           val_off, bytes);
        return hipGetLastError();
    }
    return per_series_grid(S, T, [&](int64_t s, dim3 g) {
        hipLaunchKernelGGL(wire_encode_kernel, g, dim3(256), 0, st, panel + s * ld, T, ld, val_off + s, bytes);
    });
}

hipError_t launch_observations(const int32_t* sid, const int64_t* loc, const double* val, int64_t n, double* panel,
                               int64_t S, int64_t T, int64_t ld, unsigned char* win, hipStream_t st) {
    if (S <= 0 || T <= 0) return hipSuccess;
    hipError_t e;
    const unsigned g = (unsigned)((n + 255) / 256);
    if (n > 0) {
        e = hipMemset2DAsync(panel, (size_t)ld * sizeof(double), 0, (size_t)T * sizeof(double), (size_t)S, st);
        if (e != hipSuccess) return e;
        hipLaunchKernelGGL(obs_winner_kernel, dim3(g), dim3(256), 0, st, sid, loc, n, S, T, panel, ld);
        hipLaunchKernelGGL(obs_mark_kernel, dim3(g), dim3(256), 0, st, sid, loc, n, S, T, panel, ld, win);
    }
    e = per_series_grid(S, T, [&](int64_t s, dim3 gg) {
        hipLaunchKernelGGL(fill_nan_kernel, gg, dim3(256), 0, st, panel + s * ld, S, T, ld);
    });
    if (e != hipSuccess || n <= 0) return e;
    hipLaunchKernelGGL(obs_scatter_kernel, dim3(g), dim3(256), 0, st, sid, loc, val, n, win, panel, ld);
    return hipGetLastError();
}

}  // namespace sts
