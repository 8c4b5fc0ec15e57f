// sts_acf_wide.hip -- autocorr for any numLags (UnivariateTimeSeries.autocorr,
// S/UnivariateTimeSeries.scala:68-93; callers with user-chosen lags: lbtest
// stats/TimeSeriesStatisticalTests.scala:290, acfPlot EasyPlot.scala:63).
//
// The fused tile / segment kernels carry lags 1..63 (one 64-wide lag block beside the
// imputation).  numLags > 63 runs here, on the filled panel F (the fill runs first through
// the same kernels with no ACF), in LAG BLOCKS of 61 lags:
//
//   * T > 2K: y = F - c (c = the robust shift of sts_acf.hpp, computed on F), lag products
//     P_i = sum_j y_j y_{j+i} on FP64 MFMA with the shifted-window decomposition of the tile
//     kernel (sts_tile.hip header): 4 v_mfma_f64_16x16x4_f64 per 64 steps serve
//     61 lags; lag block b adds the offset L0 = 1 + 61 b to the B operand, so its MFMAs
//     accumulate lags L0 .. L0 + 60.  One workgroup owns (series, a 64 K-step time range,
//     lag block) and walks its range in 2048-step sub-tiles staged in LDS (an A window at
//     the range's positions and a B window L0 steps later, y = 0 outside [0, T)).  Block-0
//     workgroups also sum y and y^2 over the middle [K, T - K).  acf_wide_finalize_kernel
//     combines the time ranges in a fixed order and applies acf_combine_e with edge E = K
//     (head / tail terms added per lag, never "total minus head").
//   * T <= 2K: the reference's two-pass loop per lag (one thread per lag), which also
//     reproduces its NaN pattern for lags whose slices miss an interior NaN, and NaN for
//     lags >= T (empty slices).
#include "sts_internal.hpp"
#include "sts_acf.hpp"

#include <hip/hip_runtime.h>

namespace sts {
namespace {

typedef double d4 __attribute__((ext_vector_type(4)));

constexpr int kWideLags = 61;            // lags per block (shifted-window NT = 4)
constexpr int kWideStride = 66;          // partial: [0, 64) lags of the block, [64] sum y, [65] sum y^2
constexpr int kWideSub = 2048;           // steps per LDS sub-tile
constexpr int64_t kWideRange = 65536;    // steps per workgroup time range
constexpr int kWideA = kWideSub + 128;   // A window: positions [st - 64, st + W + 64)
constexpr int kWideB = kWideSub + 192;   // B window: A positions + L0, reaching 124 past a chunk
constexpr int kQS = 4, kNT = 4;

__device__ __forceinline__ int px(int q) { return q + ((q >> 5) << 2); }   // 4 doubles of pad per 32

__global__ __launch_bounds__(256) void acf_wide_kernel(const double* __restrict__ F, int64_t S, int64_t T,
                                                       int64_t ld, const double* __restrict__ shift, int K,
                                                       int64_t nrange, int nblock, double* __restrict__ part) {
    __shared__ __attribute__((aligned(16))) double Aw[kWideA + kWideA / 8];
    __shared__ __attribute__((aligned(16))) double Bw[kWideB + kWideB / 8];
    __shared__ double red[4 * 66];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int64_t g = blockIdx.x;
    const int b = (int)(g % nblock);
    const int64_t r = (g / nblock) % nrange;
    const int64_t s = g / ((int64_t)nblock * nrange);
    const double* x = F + s * ld;
    const double c = shift[s];
    const int L0 = 1 + kWideLags * b;
    const int64_t t0 = r * kWideRange;
    const int64_t t1 = (t0 + kWideRange < T) ? t0 + kWideRange : T;
    const int64_t E = K;
    auto Y = [&](int64_t p) -> double { return (p >= 0 && p < T) ? x[p] - c : 0.0; };

    // per-lane operand offsets (unpadded) relative to a chunk start, as in tile_kernel
    int oa[kNT], ob[kNT];
#pragma unroll
    for (int t = 0; t < kNT; t++) {
        const int j = lane & 15;
        oa[t] = kQS * t + lane;
        ob[t] = kQS * t + 16 * (lane >> 4) + 16 * (j / kQS) + (16 - kQS) + (j % kQS);
    }
    d4 U0 = {0, 0, 0, 0}, U1 = {0, 0, 0, 0};
    double acc_s = 0.0, acc_q = 0.0;
    for (int64_t st = t0; st < t1; st += kWideSub) {
        const int64_t se = (st + kWideSub < t1) ? st + kWideSub : t1;
        // stage y: Aw[q] = y(st - 64 + q), Bw[q] = y(st - 64 + q + L0)
        for (int q = tid; q < kWideA; q += 256) Aw[px(q)] = Y(st - 64 + q);
        for (int q = tid; q < kWideB; q += 256) Bw[px(q)] = Y(st - 64 + q + L0);
        if (b == 0) {   // middle sums over this sub-tile's own positions
            for (int64_t p = st + tid; p < se; p += 256) {
                if (p >= E && p < T - E) {
                    const double y = x[p] - c;
                    acc_s += y;
                    acc_q = __builtin_fma(y, y, acc_q);
                }
            }
        }
        __syncthreads();
        // chunks at base = st + 64 cc (cc >= 0) of this sub-tile, plus base = -64 (the
        // shifted windows' look-back) once per series; wave w takes chunks w, w + 4, ...
        const int nch = (int)((se - st + 63) / 64);
        const int first = (st == 0) ? -1 : 0;
        for (int cc = first + wave; cc < nch; cc += 4) {
            const int rel = 64 * (cc + 1);      // window index of base (multiple of 64)
            const int cb = px(rel);
            double av[kNT], bv[kNT];
#pragma unroll
            for (int t = 0; t < kNT; t++) {
                av[t] = Aw[cb + px(oa[t])];
                bv[t] = Bw[cb + px(ob[t])];
            }
            U0 = __builtin_amdgcn_mfma_f64_16x16x4f64(av[0], bv[0], U0, 0, 0, 0);
            U1 = __builtin_amdgcn_mfma_f64_16x16x4f64(av[1], bv[1], U1, 0, 0, 0);
            U0 = __builtin_amdgcn_mfma_f64_16x16x4f64(av[2], bv[2], U0, 0, 0, 0);
            U1 = __builtin_amdgcn_mfma_f64_16x16x4f64(av[3], bv[3], U1, 0, 0, 0);
        }
        __syncthreads();
    }

    // ---- diagonal extraction: lane d accumulates lag L0 + d (d < 61) in a fixed order ----
    double* scr = Aw + wave * 256;
    const d4 D = U0 + U1;
#pragma unroll
    for (int rr = 0; rr < 4; rr++) scr[((lane >> 4) + 4 * rr) * 16 + (lane & 15)] = D[rr];
    __syncthreads();
    double lagacc = 0.0;
#pragma unroll
    for (int j = 0; j < 16; j++) {
        const int i = 16 * (j / kQS) + (16 - kQS) + (j % kQS) - lane;   // entry (i, j): lag h(j) - i
        if (i >= 0 && i < 16) lagacc += scr[i * 16 + j];
    }
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        acc_s += __shfl_xor(acc_s, d);
        acc_q += __shfl_xor(acc_q, d);
    }
    red[wave * 66 + lane] = lagacc;
    if (lane == 0) {
        red[wave * 66 + 64] = acc_s;
        red[wave * 66 + 65] = acc_q;
    }
    __syncthreads();
    if (wave == 0) {
        double* out = part + ((s * nrange + r) * nblock + b) * kWideStride;
        out[lane] = ((red[lane] + red[66 + lane]) + red[132 + lane]) + red[198 + lane];
        if (lane < 2) out[64 + lane] = ((red[64 + lane] + red[66 + 64 + lane]) + red[132 + 64 + lane]) +
                                       red[198 + 64 + lane];
    }
}

// One thread per (series, lag i = 1..K).
__global__ __launch_bounds__(256) void acf_wide_finalize_kernel(const double* __restrict__ F, int64_t S, int64_t T,
                                                                int64_t ld, const double* __restrict__ shift, int K,
                                                                int64_t nrange, int nblock,
                                                                const double* __restrict__ part,
                                                                double* __restrict__ acf,
                                                                int32_t* __restrict__ exact) {
    const int64_t s = blockIdx.y;
    const int i = blockIdx.x * 256 + threadIdx.x + 1;
    if (s >= S || i > K) return;
    const double* x = F + s * ld;
    double out;
    if (i >= T) {
        out = __builtin_nan("");
    } else if (T <= 2 * (int64_t)K) {
        // the reference's loop (S/UnivariateTimeSeries.scala:71-89), means first
        out = acf_exact_lag(x, T, i);
    } else {
        const int b = (i - 1) / kWideLags, d = (i - 1) % kWideLags;
        const double c = shift[s];
        double Pi = 0.0, Sm = 0.0, Qm = 0.0;
        for (int64_t r = 0; r < nrange; r++) {
            const double* pr = part + (s * nrange + r) * nblock * kWideStride;
            Pi += pr[b * kWideStride + d];
            Sm += pr[64];
            Qm += pr[65];
        }
        bool sus;
        out = acf_combine_e(Pi, Sm, Qm, i, T, K, [&](int j) { return x[j] - c; },
                            [&](int j) { return x[T - 1 - j] - c; }, c, &sus);
        // sts_acf.hpp rule 3: a suspect lag flags the series; launch_acf_exact recomputes all its
        // lags by the reference's loop
        if (__ballot(sus) && (threadIdx.x & 63) == 0) exact[s] = 1;
    }
    acf[s * K + (i - 1)] = out;
}

}  // namespace

size_t acf_wide_partials(int64_t S, int64_t T, int K) {
    if (T <= 2 * (int64_t)K) return 0;
    const int64_t nrange = (T + kWideRange - 1) / kWideRange;
    const int nblock = (K + kWideLags - 1) / kWideLags;
    return (size_t)(S * nrange * nblock) * kWideStride;
}

hipError_t launch_acf_wide(const double* F, int64_t S, int64_t T, int64_t ld, const double* shift, int K,
                           double* part, double* acf, int32_t* exact, hipStream_t st) {
    if (S <= 0 || K <= 0) return hipSuccess;
    const int64_t nrange = (T + kWideRange - 1) / kWideRange;
    const int nblock = (K + kWideLags - 1) / kWideLags;
    if (T > 2 * (int64_t)K) {
        const int64_t n = S * nrange * nblock;
        if (n > 0x7fffffffLL) return hipErrorInvalidValue;
        hipLaunchKernelGGL(acf_wide_kernel, dim3((unsigned)n), dim3(256), 0, st, F, S, T, ld, shift, K, nrange, nblock,
                           part);
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    if (S > 65535) {   // grid.y limit: finalize in slices of series
        for (int64_t s0 = 0; s0 < S; s0 += 65535) {
            const int64_t n = (S - s0 < 65535) ? S - s0 : 65535;
            hipLaunchKernelGGL(acf_wide_finalize_kernel, dim3((unsigned)((K + 255) / 256), (unsigned)n), dim3(256), 0,
                               st, F + s0 * ld, n, T, ld, shift ? shift + s0 : nullptr, K, nrange, nblock,
                               part ? part + s0 * nrange * nblock * kWideStride : nullptr, acf + s0 * K, exact + s0);
            const hipError_t e = hipGetLastError();
            if (e != hipSuccess) return e;
        }
    } else {
        hipLaunchKernelGGL(acf_wide_finalize_kernel, dim3((unsigned)((K + 255) / 256), (unsigned)S), dim3(256), 0, st, F,
                           S, T, ld, shift, K, nrange, nblock, part, acf, exact);
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return launch_acf_exact(F, S, T, ld, K, exact, acf, st);
}

}  // namespace sts
