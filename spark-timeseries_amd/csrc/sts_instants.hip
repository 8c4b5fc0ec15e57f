// sts_instants.hip -- the callers either side of the hot path:
//
//   seriesStats             S/TimeSeriesRDD.scala:204-206 -> Spark 1.3.1 StatCounter
//                           (org.apache.spark.util.StatCounter.merge, not vendored: restated)
//   removeInstantsWithNaNs  S/TimeSeriesRDD.scala:131-152 (column-wise NaN OR, compaction)
//   toInstants              S/TimeSeriesRDD.scala:215-324 (panel transpose: one record per
//                           instant holding every series' value, series in partition order)
//
// StatCounter.merge is a sequential Welford update with one IEEE division per value, so it
// runs one LANE per series in the reference's order (bit-exact), the series block staged
// through LDS like the recurrence kernels (sts_recur.hip).  The NaN-instant scan reads each
// element once (workgroup = 256 consecutive instants x a group of series, coalesced rows);
// the compaction and the gather are plain streaming kernels; the transpose goes through a
// padded LDS tile.
#include "sts_internal.hpp"

#include <hip/hip_runtime.h>

namespace sts {
namespace {

// java.lang.Math.max / min (what Scala's math.max / min call): NaN propagates, and
// max(-0.0, 0.0) = 0.0, min(0.0, -0.0) = -0.0.
__device__ __forceinline__ double jmax(double a, double b) {
    if (a != a) return a;
    if (a == 0.0 && b == 0.0 && __builtin_signbit(a)) return b;
    return (a >= b) ? a : b;
}
__device__ __forceinline__ double jmin(double a, double b) {
    if (a != a) return a;
    if (a == 0.0 && b == 0.0 && __builtin_signbit(b)) return b;
    return (a <= b) ? a : b;
}

// new StatCounter(series.valuesIterator) per series: out[s] = (mu, m2, max, min), n = T.
template <int SPW, int CH>
__global__ __launch_bounds__(64) void stats_kernel(const double* __restrict__ in, double* __restrict__ out,
                                                   int64_t S, int64_t T, int64_t ld) {
    constexpr int kRow = CH + 1;
    constexpr int NLD = SPW * CH / 64;
    __shared__ double tile[SPW * kRow];
    const int lane = threadIdx.x;
    const int64_t s0 = (int64_t)blockIdx.x * SPW;
    const bool live = lane < SPW && s0 + lane < S;
    const int ns = (S - s0 < SPW) ? (int)(S - s0) : SPW;
    const double* base = in + s0 * ld;
    double mu = 0.0, m2 = 0.0, mx = -__builtin_inf(), mn = __builtin_inf();
    long long n = 0;
    double pre[NLD];
    auto fetch = [&](int64_t tc) {
#pragma unroll
        for (int i = 0; i < NLD; i++) {
            const int row = (i * 64 + lane) / CH, col = (i * 64 + lane) % CH;
            pre[i] = (row < ns && tc + col < T) ? base[row * ld + tc + col] : 0.0;
        }
    };
    fetch(0);
    for (int64_t tc = 0; tc < T; tc += CH) {
        const int len = (T - tc < CH) ? (int)(T - tc) : CH;
#pragma unroll
        for (int i = 0; i < NLD; i++) {
            const int row = (i * 64 + lane) / CH, col = (i * 64 + lane) % CH;
            tile[row * kRow + col] = pre[i];
        }
        if (tc + CH < T) fetch(tc + CH);
        __syncthreads();
        if (live) {
            const double* row = tile + lane * kRow;
            for (int c = 0; c < len; c++) {
                const double v = row[c];
                const double delta = v - mu;         // StatCounter.merge(value)
                n += 1;
                mu += delta / (double)n;
                m2 += delta * (v - mu);
                mx = jmax(mx, v);
                mn = jmin(mn, v);
            }
        }
        __syncthreads();
    }
    if (live) {
        double* o = out + (s0 + lane) * 4;
        o[0] = mu;
        o[1] = m2;
        o[2] = mx;
        o[3] = mn;
    }
}

// flags[t] = 1 if any series of the panel is NaN at instant t (flags are only ever SET,
// so partial panels, other ranks and repeated calls combine by OR / max).
constexpr int kNanT = 256;
constexpr int kNanSeries = 64;
__global__ __launch_bounds__(kNanT) void nan_instants_kernel(const double* __restrict__ in, uint8_t* flags,
                                                             int64_t S, int64_t T, int64_t ld) {
    const int64_t t = (int64_t)blockIdx.x * kNanT + threadIdx.x;
    const int64_t sa = (int64_t)blockIdx.y * kNanSeries;
    const int64_t sb = (sa + kNanSeries < S) ? sa + kNanSeries : S;
    if (t >= T) return;
    bool any = false;
    const double* p = in + sa * ld + t;
#pragma unroll 8
    for (int64_t s = sa; s < sb; s++, p += ld) any |= __builtin_isnan(*p);
    if (any) flags[t] = 1;
}

// active-instant compaction: block b counts the zero flags of its kCompact instants
constexpr int kCompact = 4096;
__global__ __launch_bounds__(256) void count_active_kernel(const uint8_t* flags, int64_t T, int64_t* counts) {
    __shared__ int64_t part[4];
    const int64_t t0 = (int64_t)blockIdx.x * kCompact;
    int64_t c = 0;
    for (int i = threadIdx.x; i < kCompact; i += 256)
        if (t0 + i < T && !flags[t0 + i]) c++;
    for (int d = 32; d >= 1; d >>= 1) c += __shfl_xor(c, d);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) counts[blockIdx.x] = part[0] + part[1] + part[2] + part[3];
}

// exclusive scan of the block counts (one workgroup, sequential over chunks of 256)
__global__ __launch_bounds__(256) void scan_counts_kernel(int64_t* counts, int64_t nb, int64_t* total) {
    __shared__ int64_t buf[256];
    __shared__ int64_t carry;
    if (threadIdx.x == 0) carry = 0;
    __syncthreads();
    for (int64_t b0 = 0; b0 < nb; b0 += 256) {
        const int64_t i = b0 + threadIdx.x;
        const int64_t v = (i < nb) ? counts[i] : 0;
        buf[threadIdx.x] = v;
        __syncthreads();
        for (int d = 1; d < 256; d <<= 1) {
            const int64_t add = (threadIdx.x >= d) ? buf[threadIdx.x - d] : 0;
            __syncthreads();
            buf[threadIdx.x] += add;
            __syncthreads();
        }
        if (i < nb) counts[i] = carry + buf[threadIdx.x] - v;   // exclusive
        __syncthreads();
        if (threadIdx.x == 255) carry += buf[255];
        __syncthreads();
    }
    if (threadIdx.x == 0) *total = carry;
}

// active[pos] = t for every zero flag, in increasing t (block b writes from its offset)
__global__ __launch_bounds__(256) void write_active_kernel(const uint8_t* flags, int64_t T, const int64_t* offsets,
                                                           int64_t* active) {
    __shared__ int wsum[4];
    const int64_t t0 = (int64_t)blockIdx.x * kCompact;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    int64_t base = offsets[blockIdx.x];
    for (int i0 = 0; i0 < kCompact; i0 += 256) {
        const int64_t t = t0 + i0 + threadIdx.x;
        const bool keep = t < T && !flags[t];
        const unsigned long long m = __ballot(keep);
        if (lane == 0) wsum[wave] = __popcll(m);
        __syncthreads();
        int before = 0;
        for (int w = 0; w < wave; w++) before += wsum[w];
        const int rank = before + __popcll(m & ((1ull << lane) - 1ull));
        if (keep) active[base + rank] = t;
        base += wsum[0] + wsum[1] + wsum[2] + wsum[3];
        __syncthreads();
    }
}

// out[s, j] = in[s, active[j]], j < n_active
__global__ __launch_bounds__(256) void gather_instants_kernel(const double* __restrict__ in, double* __restrict__ out,
                                                              const int64_t* __restrict__ active, int64_t n_active,
                                                              int64_t ld_in, int64_t ld_out) {
    const int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int64_t s = blockIdx.y;
    if (j < n_active) out[s * ld_out + j] = in[s * ld_in + active[j]];
}

// toInstants: out[t, s] = in[s, t] (T x S, instant-major), 64 x 64 tiles through LDS
__global__ __launch_bounds__(256) void transpose_kernel(const double* __restrict__ in, double* __restrict__ out,
                                                        int64_t S, int64_t T, int64_t ld_in, int64_t ld_out) {
    __shared__ double tile[64][65];
    const int64_t t0 = (int64_t)blockIdx.x * 64, s0 = (int64_t)blockIdx.y * 64;
    const int lx = threadIdx.x & 63, ly = threadIdx.x >> 6;
    for (int r = ly; r < 64; r += 4) {
        const int64_t s = s0 + r, t = t0 + lx;
        if (s < S && t < T) tile[r][lx] = in[s * ld_in + t];
    }
    __syncthreads();
    for (int r = ly; r < 64; r += 4) {
        const int64_t t = t0 + r, s = s0 + lx;
        if (s < S && t < T) out[t * ld_out + s] = tile[lx][r];
    }
}

}  // namespace

hipError_t launch_series_stats(const double* in, double* out, int64_t S, int64_t T, int64_t ld, hipStream_t st) {
    if (S <= 0) return hipSuccess;
    constexpr int SPW = 64, CH = 32;   // A/B on 1M x 390: 1.00 ms vs 1.44 (32 x 64), 1.96 (16 x 64)
    hipLaunchKernelGGL((stats_kernel<SPW, CH>), dim3((unsigned)((S + SPW - 1) / SPW)), dim3(64), 0, st, in, out, S, T,
                       ld);
    return hipGetLastError();
}

hipError_t launch_nan_instants(const double* in, uint8_t* flags, int64_t S, int64_t T, int64_t ld, hipStream_t st) {
    if (S <= 0 || T <= 0) return hipSuccess;
    const int64_t gy = (S + kNanSeries - 1) / kNanSeries;
    if (gy > 65535) {   // grid.y limit: split the series range
        for (int64_t s = 0; s < S; s += 65535LL * kNanSeries) {
            const int64_t n = (S - s < 65535LL * kNanSeries) ? S - s : 65535LL * kNanSeries;
            hipError_t e = launch_nan_instants(in + s * ld, flags, n, T, ld, st);
            if (e != hipSuccess) return e;
        }
        return hipSuccess;
    }
    dim3 grid((unsigned)((T + kNanT - 1) / kNanT), (unsigned)gy);
    hipLaunchKernelGGL(nan_instants_kernel, grid, dim3(kNanT), 0, st, in, flags, S, T, ld);
    return hipGetLastError();
}

int64_t active_scratch_elems(int64_t T) { return (T + kCompact - 1) / kCompact + 1; }

hipError_t launch_active_instants(const uint8_t* flags, int64_t T, int64_t* active, int64_t* n_active,
                                  int64_t* scratch, hipStream_t st) {
    const int64_t nb = (T + kCompact - 1) / kCompact;
    if (nb == 0) return hipMemsetAsync(n_active, 0, sizeof(int64_t), st);
    hipLaunchKernelGGL(count_active_kernel, dim3((unsigned)nb), dim3(256), 0, st, flags, T, scratch);
    hipLaunchKernelGGL(scan_counts_kernel, dim3(1), dim3(256), 0, st, scratch, nb, n_active);
    hipLaunchKernelGGL(write_active_kernel, dim3((unsigned)nb), dim3(256), 0, st, flags, T, scratch, active);
    return hipGetLastError();
}

hipError_t launch_gather_instants(const double* in, double* out, const int64_t* active, int64_t n_active, int64_t S,
                                  int64_t ld_in, int64_t ld_out, hipStream_t st) {
    if (S <= 0 || n_active <= 0) return hipSuccess;
    for (int64_t s = 0; s < S; s += 65535) {
        const int64_t n = (S - s < 65535) ? S - s : 65535;
        dim3 grid((unsigned)((n_active + 255) / 256), (unsigned)n);
        hipLaunchKernelGGL(gather_instants_kernel, grid, dim3(256), 0, st, in + s * ld_in, out + s * ld_out, active,
                           n_active, ld_in, ld_out);
    }
    return hipGetLastError();
}

hipError_t launch_transpose(const double* in, double* out, int64_t S, int64_t T, int64_t ld_in, int64_t ld_out,
                            hipStream_t st) {
    if (S <= 0 || T <= 0) return hipSuccess;
    for (int64_t s = 0; s < S; s += 64LL * 65535) {
        const int64_t n = (S - s < 64LL * 65535) ? S - s : 64LL * 65535;
        dim3 grid((unsigned)((T + 63) / 64), (unsigned)((n + 63) / 64));
        hipLaunchKernelGGL(transpose_kernel, grid, dim3(256), 0, st, in + s * ld_in, out + s, n, T, ld_in, ld_out);
    }
    return hipGetLastError();
}

}  // namespace sts
