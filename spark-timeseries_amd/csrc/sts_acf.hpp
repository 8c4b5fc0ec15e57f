// sts_acf.hpp -- the numerically robust pieces of autocorr shared by the tile kernel
// (sts_tile.hip), the segment kernel (sts_seg.hip) and acf_finalize_kernel.
//
// Reference: autocorr, S/UnivariateTimeSeries.scala:68-93.  For lag i it takes the means
// m1 of x[i..n) and m2 of x[0..n-i) FIRST and then sums centred products
//   v1 = sum (x[j+i] - m1)^2,  v2 = sum (x[j] - m2)^2,  c = sum (x[j+i] - m1)(x[j] - m2),
// which stays accurate whatever the level of the series.  The kernels cannot afford two
// passes over HBM, so they accumulate moments of y = x - c in one pass and centre at the
// end (v1 = sum1_sq - sum1^2 / N, ...).  That is exact algebra for ANY constant c, and it is
// accurate when c lies inside the bulk of the series: the rounding error of sum y^2 is
// about eps * N * (sigma^2 + (mean - c)^2), so (mean - c)^2 / sigma^2 is the number of
// bits lost.  Two rules keep that ratio O(1):
//
//  1. c is the MEDIAN of the valid values among 64 samples of the series (an outlier at
//     x[0] or a level far from x[0] cannot move it; |median - mean| <= sigma for the sampled
//     population): spread evenly over the whole series in the tile kernel (robust_shift),
//     and over its first 512-step tile in the segment kernel (T <= 16384 there, so a first
//     tile at another level is >= 1/32 of the series and bounds (mean - c)^2 / sigma^2 by
//     ~32).  Every workgroup / segment of a series computes it from the same raw samples the
//     same way, so all of them agree bit for bit and the partials combine.
//  2. sum y and sum y^2 are accumulated only over the MIDDLE [kAcfEdge, T - kAcfEdge) of
//     the series; the head and tail (the only positions that differ between the lag
//     slices, since K <= kAcfEdge) are added explicitly per lag (acf_combine).  The lag
//     slice sums are thus sums of their own terms, never "total minus head": an outlier in
//     the first or last kAcfEdge steps cannot cancel digits out of them.
//
// The lag products P_i = sum_j y_j y_{j+i} (j + i < T) need no correction at all.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "sts_internal.hpp"   // kAcfEdge

namespace sts {

__device__ __forceinline__ double acf_readlane(double v, int l) {
    const unsigned long long u = __builtin_bit_cast(unsigned long long, v);
    const unsigned lo = __builtin_amdgcn_readlane((unsigned)u, l);
    const unsigned hi = __builtin_amdgcn_readlane((unsigned)(u >> 32), l);
    return __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lo);
}

// The lower median of the valid per-lane samples v (ok: valid) of one wave, in the total
// order (value, lane): a ballot quickselect -- each round takes the middle remaining
// candidate as the pivot, counts the candidates below it with one ballot and keeps the side
// that holds the wanted rank (a few scalar rounds; a sorted sample needs one).  0.0 when no
// sample is valid.  Wave-uniform, deterministic (a pure function of the samples).
__device__ __forceinline__ double median_of_lanes(double v, bool ok, int lane) {
    unsigned long long cand = __ballot(ok);
    int n = __popcll(cand);
    if (n == 0) return 0.0;
    int k = (n - 1) >> 1;                          // rank wanted among the candidates
    for (;;) {
        // pivot lane: the first candidate at or after the middle of the candidates' lane range
        // (scalar; for a monotone sample that is its median)
        const int lo = __ffsll((long long)cand) - 1, hi = 63 - __clzll(cand);
        const int mid = (lo + hi) >> 1;
        const int pl = mid + __ffsll((long long)(cand >> mid)) - 1;
        const double pv = acf_readlane(v, pl);
        const bool in = (cand >> lane) & 1ull;
        const unsigned long long lt = __ballot(in && (v < pv || (v == pv && lane < pl)));
        const int cnt = __popcll(lt);
        if (cnt == k) return pv;
        if (cnt > k) {
            cand = lt;
        } else {
            cand &= ~lt & ~(1ull << pl);
            k -= cnt + 1;
        }
        n = __popcll(cand);
    }
}

// Robust shift of series `src` (length T >= 1), computed by one whole wave: lane l samples
// x[t_l] (or x[t_l + 1] when x[t_l] is NaN), t_l = l * T / 64, spread over the whole series;
// the result is the lower median of the valid samples.
__device__ __forceinline__ double robust_shift(const double* src, int64_t T, int lane) {
    const int64_t t = (int64_t)lane * T / 64;
    double v = src[t];
    if (__builtin_isnan(v) && t + 1 < T) v = src[t + 1];
    return median_of_lanes(v, !__builtin_isnan(v), lane);
}

// True when series position t contributes to the middle sums (rule 2).
__device__ __forceinline__ bool acf_mid(int64_t t, int64_t T) { return t >= kAcfEdge && t < T - kAcfEdge; }

// The reference's correlation for lag i (1 <= i <= kAcfEdge, T >= 2 * kAcfEdge) from
//   Pi = sum_{j < T-i} y_j y_{j+i},  Sm / Qm = sum / sum of squares of y over the middle,
//   hy(j) = y_j and tz(j) = y_{T-1-j} for j < kAcfEdge.
// Slice 1 = x[i..T): head positions j >= i plus the whole tail; slice 2 = x[0..T-i): the
// whole head plus tail positions T-1-j with j >= i.  Callers must run this with the same
// operands in the same order to get the same bits (the fused and separate finalizes do).
// The edge length E is kAcfEdge on the fused K <= 63 paths and K itself on the wide path
// (sts_acf_wide.hip); T >= 2E, i <= E.
template <class HY, class TZ>
__device__ __forceinline__ double acf_combine_e(double Pi, double Sm, double Qm, int i, int64_t T, int E, HY hy,
                                                TZ tz) {
    double sum1 = Sm, sq1 = Qm, sum2 = Sm, sq2 = Qm;
    for (int j = 0; j < E; j++) {
        const double y = hy(j), z = tz(j);
        const double yy = y * y, zz = z * z;
        sum2 += y;
        sq2 += yy;
        sum1 += z;
        sq1 += zz;
        if (j >= i) {
            sum1 += y;
            sq1 += yy;
            sum2 += z;
            sq2 += zz;
        }
    }
    const double N = (double)(T - i);
    const double v1 = sq1 - sum1 * sum1 / N;
    const double v2 = sq2 - sum2 * sum2 / N;
    const double cv = Pi - sum1 * sum2 / N;
    return cv / (__builtin_sqrt(v1) * __builtin_sqrt(v2));   // S/UnivariateTimeSeries.scala:89
}

template <class HY, class TZ>
__device__ __forceinline__ double acf_combine(double Pi, double Sm, double Qm, int i, int64_t T, HY hy, TZ tz) {
    return acf_combine_e(Pi, Sm, Qm, i, T, kAcfEdge, hy, tz);
}

}  // namespace sts
