// sts_stream.hip -- element-parallel streaming operators (no recurrence):
//   differencesAtLag (out of place)  S/UnivariateTimeSeries.scala:356-376
//   EWMAModel.removeTimeDependentEffects (out of place)  S/models/EWMA.scala:125-133
//   ARModel.removeTimeDependentEffects (out of place)    S/models/Autoregression.scala:60-73
//   Lag.lagMatTrimBoth (standalone)                      S/Lag.scala:62-77
// Each output element depends on a few inputs at fixed backward offsets, so threads
// map to consecutive steps (coalesced along time) and the backward re-reads are L1/L2
// hits.  The arithmetic is written in the reference's order and the library is built
// with -ffp-contract=off, so every result is bit-exact.
#include "sts_internal.hpp"

#include <hip/hip_runtime.h>

namespace sts {
namespace {

constexpr int kThreads = 256;
constexpr int kPerThread = 8;
constexpr int64_t kChunk = (int64_t)kThreads * kPerThread;

// split a logical index g in [0, S*T) into (s, t) with a double reciprocal + fix-up
__device__ __forceinline__ void split(int64_t g, int64_t T, double rT, int64_t& s, int64_t& t) {
    s = (int64_t)((double)g * rT);
    int64_t b = s * T;
    if (b > g) { s--; b -= T; }
    else if (b + T <= g) { s++; b += T; }
    t = g - b;
}

__global__ __launch_bounds__(kThreads) void diff_kernel(const double* __restrict__ in, double* __restrict__ out,
                                                        int64_t S, int64_t T, int64_t ld_in, int64_t ld_out,
                                                        double rT, int lag, int start) {
    const int64_t n = S * T;
    const int64_t g0 = (int64_t)blockIdx.x * kChunk + threadIdx.x;
#pragma unroll
    for (int j = 0; j < kPerThread; j++) {
        const int64_t g = g0 + (int64_t)j * kThreads;
        if (g >= n) break;
        int64_t s, t;
        split(g, T, rT, s, t);
        const double* x = in + s * ld_in;
        out[s * ld_out + t] = (t < start) ? x[t] : x[t] - x[t - lag];
    }
}

__global__ __launch_bounds__(kThreads) void ewma_remove_kernel(const double* __restrict__ in, double* __restrict__ out,
                                                               int64_t S, int64_t T, int64_t ld_in, int64_t ld_out,
                                                               double rT, const double* __restrict__ sm) {
    const int64_t n = S * T;
    const int64_t g0 = (int64_t)blockIdx.x * kChunk + threadIdx.x;
#pragma unroll
    for (int j = 0; j < kPerThread; j++) {
        const int64_t g = g0 + (int64_t)j * kThreads;
        if (g >= n) break;
        int64_t s, t;
        split(g, T, rT, s, t);
        const double* x = in + s * ld_in;
        const double sv = sm[s];
        // dest(i) = (ts(i) - (1 - smoothing) * ts(i - 1)) / smoothing,   EWMA.scala:131
        out[s * ld_out + t] = (t == 0) ? x[0] : (x[t] - (1.0 - sv) * x[t - 1]) / sv;
    }
}

__global__ __launch_bounds__(kThreads) void ar_remove_kernel(const double* __restrict__ in, double* __restrict__ out,
                                                             int64_t S, int64_t T, int64_t ld_in, int64_t ld_out,
                                                             double rT, const double* __restrict__ c,
                                                             const double* __restrict__ coef, int p) {
    const int64_t n = S * T;
    const int64_t g0 = (int64_t)blockIdx.x * kChunk + threadIdx.x;
#pragma unroll 2
    for (int j = 0; j < kPerThread; j++) {
        const int64_t g = g0 + (int64_t)j * kThreads;
        if (g >= n) break;
        int64_t s, t;
        split(g, T, rT, s, t);
        const double* x = in + s * ld_in;
        const double* cf = coef + s * p;
        // dest(i) = ts(i) - c; dest(i) -= ts(i - j - 1) * coefficients(j)   Autoregression.scala:64-68
        double d = x[t] - c[s];
        for (int k = 0; k < p && t - k - 1 >= 0; k++) d -= x[t - k - 1] * cf[k];
        out[s * ld_out + t] = d;
    }
}

// out for series s: (T - p) x ncols column-major at out + s * (T - p) * ncols;
// M(r, c - init) = x(r + p - c)
__global__ __launch_bounds__(kThreads) void lagmat_kernel(const double* __restrict__ in, double* __restrict__ out,
                                                          int64_t S, int64_t T, int64_t ld_in, int p, int init,
                                                          int ncols, double rR) {
    const int64_t rows = T - p;
    const int64_t n = S * (int64_t)ncols * rows;
    const int64_t g0 = (int64_t)blockIdx.x * kChunk + threadIdx.x;
#pragma unroll
    for (int j = 0; j < kPerThread; j++) {
        const int64_t g = g0 + (int64_t)j * kThreads;
        if (g >= n) break;
        int64_t col, r;
        split(g, rows, rR, col, r);          // col = s * ncols + k
        const int64_t s = col / ncols;
        const int k = (int)(col - s * ncols);
        const int c = k + init;
        out[g] = in[s * ld_in + r + p - c];
    }
}

inline dim3 grid_for(int64_t n) { return dim3((unsigned)((n + kChunk - 1) / kChunk)); }

}  // namespace

hipError_t launch_diff(const double* in, double* out, int64_t S, int64_t T, int64_t ld_in, int64_t ld_out,
                       int lag, int start, hipStream_t st) {
    if (S * T == 0) return hipSuccess;
    hipLaunchKernelGGL(diff_kernel, grid_for(S * T), dim3(kThreads), 0, st, in, out, S, T, ld_in, ld_out,
                       1.0 / (double)T, lag, start);
    return hipGetLastError();
}

hipError_t launch_ewma_remove(const double* in, double* out, int64_t S, int64_t T, int64_t ld_in,
                              int64_t ld_out, const double* sm, hipStream_t st) {
    if (S * T == 0) return hipSuccess;
    hipLaunchKernelGGL(ewma_remove_kernel, grid_for(S * T), dim3(kThreads), 0, st, in, out, S, T, ld_in,
                       ld_out, 1.0 / (double)T, sm);
    return hipGetLastError();
}

hipError_t launch_ar_remove(const double* in, double* out, int64_t S, int64_t T, int64_t ld_in,
                            int64_t ld_out, const double* c, const double* coef, int p, hipStream_t st) {
    if (S * T == 0) return hipSuccess;
    hipLaunchKernelGGL(ar_remove_kernel, grid_for(S * T), dim3(kThreads), 0, st, in, out, S, T, ld_in, ld_out,
                       1.0 / (double)T, c, coef, p);
    return hipGetLastError();
}

hipError_t launch_lagmat(const double* in, double* out, int64_t S, int64_t T, int64_t ld_in, int max_lag,
                         int include_original, hipStream_t st) {
    const int64_t rows = T - max_lag;
    const int ncols = max_lag + (include_original ? 1 : 0);
    const int64_t n = S * ncols * rows;
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(lagmat_kernel, grid_for(n), dim3(kThreads), 0, st, in, out, S, T, ld_in, max_lag,
                       include_original ? 0 : 1, ncols, 1.0 / (double)rows);
    return hipGetLastError();
}

}  // namespace sts
