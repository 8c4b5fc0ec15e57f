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
//  1. c is the MEDIAN of 64 samples that stand for the FILLED series, one per 1/64 of it
//     (robust_shift below: the first valid step of each range, a NaN-only range taking the
//     next range's; an outlier at x[0], a level far from x[0], a long leading NaN run or a
//     98 %-NaN series cannot move it; |median - mean| <= sigma for the sampled population).
//     The tile kernel loads it per series from acf_shift_kernel, the segment kernel computes
//     it at its start; both use this one function, so every workgroup / segment of a series
//     agrees bit for bit and the partials combine.
//  2. sum y and sum y^2 are accumulated only over the MIDDLE [kAcfEdge, T - kAcfEdge) of
//     the series; the head and tail (the only positions that differ between the lag
//     slices, since K <= kAcfEdge) are added explicitly per lag (acf_combine).  The lag
//     slice sums are thus sums of their own terms, never "total minus head": an outlier in
//     the first or last kAcfEdge steps cannot cancel digits out of them.
//
// The lag products P_i = sum_j y_j y_{j+i} (j + i < T) need no correction at all.
//
//  3. (round 4) Where the one-pass value can still differ from the reference's, the
//     reference's own loop runs instead.  acf_suspect bounds, per lag, the one-pass rounding
//     error (cancellation R = sum y^2 / variance) and the deviation the reference's rounded
//     means put into ITS result (a constant 100.1 series: the mean rounds to 100.1 - d, every
//     diff is d, and the reference returns 1.0 where the exact answer is 0/0); a series with
//     any suspect lag is recomputed by acf_exact_lag -- the reference's two passes, means first,
//     in its order -- so its NaN pattern and bits are the reference's.  On well-conditioned
//     series (every bench panel) nothing is flagged and the one-pass path stands.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "sts_dma.hpp"        // wave_lds_sync
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

__device__ __forceinline__ int64_t acf_readlane64(int64_t v, int l) {
    const unsigned long long u = (unsigned long long)v;
    const unsigned lo = __builtin_amdgcn_readlane((unsigned)u, l);
    const unsigned hi = __builtin_amdgcn_readlane((unsigned)(u >> 32), l);
    return (int64_t)(((unsigned long long)hi << 32) | lo);
}

// Robust shift of series `src` (length T >= 1), computed by one whole wave from what the
// FILLED series looks like, whatever the NaN pattern of the raw one (round 3: the round-2
// shift sampled raw steps and fell to 0.0 -- or to an outlier x[0] -- when they were NaN,
// e.g. fillNext over a long leading NaN run or a 98 %-NaN panel).
//   * Lane l owns the positions [t0, t1) = [l T / 64, (l + 1) T / 64) and finds the first
//     valid step in them: lane-parallel probes of 4 steps (kProbeRounds rounds; at 5 % NaN
//     the first round finds one in every lane but ~1 in 10^5), then, for the lanes still
//     without one, a wave-cooperative scan of the rest of their range, 512 steps per trip.
//     Every valid step is a value of the filled series too (no fill rewrites a valid step).
//   * A lane whose range holds no valid step takes the sample of the next lane that has one
//     -- the first valid step after t0, i.e. exactly F(t0) of fillNext, and the right end of
//     a linear / nearest gap -- else that of the last lane before it with one (a trailing
//     run).  Under fillPrevious (prev_fill) the order is reversed: a run is filled with the
//     value before it, so the lane takes the last sampled lane before it, else the next one
//     (round 3: with the fillNext order, a long interior run under fillPrevious followed by a
//     level change put the shift on the far side of the change).  So every lane stands for its 1/64 of the filled series, and a long run filled
//     by copies of one value weighs in the sample as it weighs in the series.
//   * c = the lower median of the 64 samples.  0.0 only when the series has no valid step at
//     all (its ACF is NaN for every fill then).
// A pure function of the series' values: every workgroup / segment that computes it gets the
// same bits.
constexpr int kProbeRounds = 4;
// the lane whose sample a lane without a valid step takes (see robust_shift)
__device__ __forceinline__ int shift_fallback_lane(unsigned long long above, unsigned long long below, bool prev_fill) {
    const int next = above ? __ffsll((long long)above) - 1 : -1;
    const int prev = below ? 63 - __clzll(below) : -1;
    return prev_fill ? (prev >= 0 ? prev : next) : (next >= 0 ? next : prev);
}
__device__ __forceinline__ double robust_shift(const double* src, int64_t T, int lane, bool prev_fill = false) {
    const int64_t t0 = (int64_t)lane * T / 64, t1 = (int64_t)(lane + 1) * T / 64;
    int64_t cur = t0;
    double v = 0.0;
    bool found = false;
    for (int r = 0; r < kProbeRounds; r++) {
        const bool pend = !found && cur < t1;
        if (__ballot(pend) == 0ull) break;
        if (pend) {
            double p[4];
#pragma unroll
            for (int k = 0; k < 4; k++) p[k] = (cur + k < t1) ? src[cur + k] : __builtin_nan("");
#pragma unroll
            for (int k = 3; k >= 0; k--) {   // the first valid of the four
                if (!__builtin_isnan(p[k])) {
                    v = p[k];
                    found = true;
                }
            }
            cur += 4;
        }
    }
    unsigned long long pendm = __ballot(!found && cur < t1);
    while (pendm) {   // wave-uniform: one pending lane's range at a time, coalesced
        const int l = __ffsll((long long)pendm) - 1;
        int64_t c = acf_readlane64(cur, l);
        const int64_t e = acf_readlane64(t1, l);
        bool ff = false;
        double fv = 0.0;
        while (c < e && !ff) {
            double q[8];
#pragma unroll
            for (int k = 0; k < 8; k++) {
                const int64_t t = c + 64 * k + lane;
                q[k] = (t < e) ? src[t] : __builtin_nan("");
            }
#pragma unroll
            for (int k = 0; k < 8; k++) {
                const unsigned long long m = __ballot(!__builtin_isnan(q[k]));
                if (!ff && m) {
                    fv = acf_readlane(q[k], __ffsll((long long)m) - 1);
                    ff = true;
                }
            }
            c += 512;
        }
        if (ff && lane == l) {
            v = fv;
            found = true;
        }
        pendm &= pendm - 1ull;
    }
    const unsigned long long vm = __ballot(found);
    if (vm == 0ull) return 0.0;
    const unsigned long long above = vm & ~((2ull << lane) - 1ull);   // lanes > lane (lane 63: none)
    const unsigned long long below = vm & ((1ull << lane) - 1ull);
    const int from = found ? lane : shift_fallback_lane(above, below, prev_fill);
    v = __shfl(v, from);
    return median_of_lanes(v, true, lane);
}

// True when series position t contributes to the middle sums (rule 2).
__device__ __forceinline__ bool acf_mid(int64_t t, int64_t T) { return t >= kAcfEdge && t < T - kAcfEdge; }

// Rule 3: may the one-pass result r of one lag differ from the reference's by more than the
// ACF tolerance?  sum / sq: the slice sums of y = x - c and of y^2, v = sq - sum^2 / N.
//   * NaN / inf data (a non-finite sum): both paths give NaN -- not suspect.
//   * v <= 0 or a non-finite r: a (near-)constant slice; the reference's rounded mean makes
//     its variance N d^2 > 0 (1.0 for a constant 100.1, tiny values for a constant-but-one-end
//     series) -- suspect.
//   * one-pass error: |dr| ~ eps G (sqrt(R1 R2) + |r| (R1 + R2) / 2) with R = sq / v (digits
//     cancelled; 1 when c is the mean) and G = max(sqrt(N) / 8, 16); the numpy emulation
//     (tests/test_acf_robust.py) measures G <= 4 on the spike-train rows.
//   * the reference's own deviation from its rounded means: recursive summation of N values
//     errs by at most u N rms(x) in the mean (u = 2^-53; a constant series reaches ~0.1 of
//     that: the bound's quarter is used), which moves the covariance by N d1 d2 and the
//     variances by N d^2.
// Suspect when their sum exceeds 1e-11 |r| (a tenth of the 1e-10 bar) and the reference's own
// rounding-noise level eps sqrt(N) (below which its value is noise: white-noise correlations).
__device__ __forceinline__ bool acf_suspect(double r, double sum1, double sq1, double sum2, double sq2, double v1,
                                            double v2, double N, double c) {
    if (!(__builtin_isfinite(sum1) && __builtin_isfinite(sq1) && __builtin_isfinite(sum2) && __builtin_isfinite(sq2)))
        return false;
    if (!(v1 > 0.0) || !(v2 > 0.0) || !__builtin_isfinite(r)) return true;
    constexpr double eps = 0x1p-52;
    const double R1 = sq1 / v1, R2 = sq2 / v2, ar = __builtin_fabs(r), rn = __builtin_sqrt(N);
    const double G = __builtin_fmax(rn * 0.125, 16.0);
    const double e_ours = eps * G * (__builtin_sqrt(R1 * R2) + ar * 0.5 * (R1 + R2));
    const double d1 = 0x1p-55 * N * (__builtin_fabs(c) + __builtin_sqrt(sq1 / N));
    const double d2 = 0x1p-55 * N * (__builtin_fabs(c) + __builtin_sqrt(sq2 / N));
    const double e_ref = N * d1 * d2 / __builtin_sqrt(v1 * v2) + ar * 0.5 * (N * d1 * d1 / v1 + N * d2 * d2 / v2);
    return e_ours + e_ref > __builtin_fmax(1e-11 * ar, eps * rn);
}

// The same test at a fraction of its VALU (round 6, the issue-bound short kernel): hardware
// reciprocal / reciprocal-square-root approximations instead of IEEE divisions and square
// roots (~40 instead of ~200 instructions).  Their error (far below 1e-6 relative) is covered
// by the 1.001 factor on the estimate, so this flags every series acf_suspect flags (a
// superset within 0.1 % of the threshold, which then takes the reference's own loop).
__device__ __forceinline__ bool acf_suspect_fast(double r, double sum1, double sq1, double sum2, double sq2,
                                                 double v1, double v2, double N, double c) {
    if (!(__builtin_isfinite(sum1) && __builtin_isfinite(sq1) && __builtin_isfinite(sum2) && __builtin_isfinite(sq2)))
        return false;
    if (!(v1 > 0.0) || !(v2 > 0.0) || !__builtin_isfinite(r)) return true;
    constexpr double eps = 0x1p-52;
    const double iv1 = __builtin_amdgcn_rcp(v1), iv2 = __builtin_amdgcn_rcp(v2), iN = __builtin_amdgcn_rcp(N);
    const double R1 = sq1 * iv1, R2 = sq2 * iv2, ar = __builtin_fabs(r);
    const double rn = N * __builtin_amdgcn_rsq(N);                      // sqrt(N)
    const double G = __builtin_fmax(rn * 0.125, 16.0);
    const double R12 = R1 * R2;
    const double e_ours = eps * G * (R12 * __builtin_amdgcn_rsq(R12) + ar * 0.5 * (R1 + R2));
    const double m1 = sq1 * iN, m2 = sq2 * iN;
    const double d1 = 0x1p-55 * N * (__builtin_fabs(c) + m1 * __builtin_amdgcn_rsq(m1));
    const double d2 = 0x1p-55 * N * (__builtin_fabs(c) + m2 * __builtin_amdgcn_rsq(m2));
    const double e_ref = N * d1 * d2 * __builtin_amdgcn_rsq(v1 * v2) + ar * 0.5 * (N * d1 * d1 * iv1 + N * d2 * d2 * iv2);
    return (e_ours + e_ref) * 1.001 > __builtin_fmax(1e-11 * ar, eps * rn);
}

// The reference's autocorr of lag i (1 <= i < T) over F (S/UnivariateTimeSeries.scala:71-89,
// Breeze mean = left-to-right sum / count): means first, then the centred sums, every sum
// sequential in the reference's order (-ffp-contract=off): the reference's bits.  One lane per
// lag; adjacent lags read adjacent addresses (coalesced), F[j] is wave-uniform.  Cost ~3 T
// dependent steps per lane: the fallback of rule 3 and the T <= 2K path only.
__device__ __forceinline__ double acf_exact_lag(const double* F, int64_t T, int i) {
    const int64_t len = T - i;
    const double* a = F + i;
    double s1 = 0.0, s2 = 0.0;
    int64_t j = 0;
    for (; j + 8 <= len; j += 8) {
        double p[8], q[8];
#pragma unroll
        for (int k = 0; k < 8; k++) {
            p[k] = a[j + k];
            q[k] = F[j + k];
        }
#pragma unroll
        for (int k = 0; k < 8; k++) {
            s1 += p[k];
            s2 += q[k];
        }
    }
    for (; j < len; j++) {
        s1 += a[j];
        s2 += F[j];
    }
    const double m1 = s1 / (double)len, m2 = s2 / (double)len;
    double v1 = 0.0, v2 = 0.0, cv = 0.0;
    j = 0;
    for (; j + 8 <= len; j += 8) {
        double p[8], q[8];
#pragma unroll
        for (int k = 0; k < 8; k++) {
            p[k] = a[j + k];
            q[k] = F[j + k];
        }
#pragma unroll
        for (int k = 0; k < 8; k++) {
            const double d1 = p[k] - m1, d2 = q[k] - m2;
            v1 += d1 * d1;
            v2 += d2 * d2;
            cv += d1 * d2;
        }
    }
    for (; j < len; j++) {
        const double d1 = a[j] - m1, d2 = F[j] - m2;
        v1 += d1 * d1;
        v2 += d2 * d2;
        cv += d1 * d2;
    }
    return cv / (__builtin_sqrt(v1) * __builtin_sqrt(v2));
}

// Rule 3's fallback on long series, streamed through LDS (round 6): acf_exact_lag's two passes
// -- the same operations in the same order, so the same bits -- but F arrives in chunks of C
// steps through the wave's own LDS buffers.  The whole wave loads the NEXT chunk with coalesced
// 8-B loads (512 B per instruction) into registers before it sums the current one, so each
// lane's dependent add chains wait on the FP64 pipe, not on HBM round trips (acf_exact_lag
// issues its loads 8 steps ahead of each chain: ~2 x T / 8 HBM latencies, 107.7 ms for
// 1 000 x 982 800 at K = 60).
// Lane l computes lag i, L0 < i <= L0 + 64 (L0 = 64 b for lag block b), increasing with the lane
// among the active lanes; !active lanes read inside the halo and add nothing.  bufa[C + 64]
// holds the window F[L0 + j0 .. L0 + j0 + C + 64) (the lagged operand F[j + i]); for L0 > 0
// (WIDE) bufb[C] holds F[j0 .. j0 + C) (the unlagged one), for L0 = 0 that is bufa itself.  Every
// lane of the wave must call it (wave-uniform loop).  Sums start at +0.0 and so are never -0.0:
// a masked step adds +0.0, the identity on them.
template <int C, bool WIDE = false>
__device__ double acf_exact_stream(const double* F, int64_t T, int i, bool active, double* bufa, int lane,
                                   int L0 = 0, double* bufb = nullptr) {
    static_assert(C % 64 == 0 && C >= 64, "chunk: whole wave rows");
    constexpr int PL = C / 64;
    const unsigned long long am = __ballot(active);
    if (am == 0ull) return 0.0;
    const int lf = __ffsll((long long)am) - 1, ll = 63 - __clzll(am);
    const int64_t maxlen = T - __builtin_amdgcn_readlane(i, lf);   // the smallest active lag
    const int64_t minlen = T - __builtin_amdgcn_readlane(i, ll);   // the largest
    if (!WIDE) L0 = 0;
    const double* FA = F + L0;
    const int64_t TA = T - L0;                 // FA's length
    const int ia = active ? i - L0 : 64;       // 1 .. 64
    const int64_t len = active ? T - i : 0;
    const double* pb = WIDE ? bufb : bufa;     // F[j0 + k] at pb[k]
    double s1 = 0.0, s2 = 0.0, m1 = 0.0, m2 = 0.0, v1 = 0.0, v2 = 0.0, cv = 0.0;
    for (int pass = 0; pass < 2; pass++) {
        wave_lds_sync();   // the caller's (or the previous pass's) reads of the buffers are done
        // bufa[0 .. C + 64) = FA[0 .. C + 64), bufb[0 .. C) = F[0 .. C) (0.0 past the end: never
        // summed, j + i < T for j < len)
#pragma unroll
        for (int k = 0; k <= PL; k++) {
            const int64_t t = (int64_t)k * 64 + lane;
            bufa[t] = t < TA ? FA[t] : 0.0;
            if (WIDE && k < PL) bufb[t] = t < T ? F[t] : 0.0;
        }
        for (int64_t j0 = 0; j0 < maxlen; j0 += C) {
            double pf[PL], pg[WIDE ? PL : 1];
#pragma unroll
            for (int k = 0; k < PL; k++) {   // the next chunk's new steps, in flight meanwhile
                const int64_t t = j0 + C + 64 + (int64_t)k * 64 + lane;
                pf[k] = t < TA ? FA[t] : 0.0;
                if (WIDE) {
                    const int64_t u = j0 + C + (int64_t)k * 64 + lane;
                    pg[k] = u < T ? F[u] : 0.0;
                }
            }
            wave_lds_sync();
            const double* pa = bufa + ia;   // F[j0 + i + k] at pa[k]
            const bool full = j0 + C <= minlen;
            // groups of 8 steps: 16 LDS reads, then the chains (a register double buffer of the
            // next group's reads measured slower: its 16 moves per group cost VALU issue)
            for (int k0 = 0; k0 < C; k0 += 8) {
                double a[8], b[8];
#pragma unroll
                for (int q = 0; q < 8; q++) {
                    a[q] = pa[k0 + q];
                    b[q] = pb[k0 + q];
                }
                if (full) {
                    if (pass == 0) {
#pragma unroll
                        for (int q = 0; q < 8; q++) {
                            s1 += a[q];
                            s2 += b[q];
                        }
                    } else {
#pragma unroll
                        for (int q = 0; q < 8; q++) {
                            const double d1 = a[q] - m1, d2 = b[q] - m2;
                            v1 += d1 * d1;
                            v2 += d2 * d2;
                            cv += d1 * d2;
                        }
                    }
                } else {
#pragma unroll
                    for (int q = 0; q < 8; q++) {
                        const bool in = j0 + k0 + q < len;
                        if (pass == 0) {
                            s1 += in ? a[q] : 0.0;
                            s2 += in ? b[q] : 0.0;
                        } else {
                            const double d1 = a[q] - m1, d2 = b[q] - m2;
                            v1 += in ? d1 * d1 : 0.0;
                            v2 += in ? d2 * d2 : 0.0;
                            cv += in ? d1 * d2 : 0.0;
                        }
                    }
                }
            }
            wave_lds_sync();   // every lane's reads of this chunk are done
            const double h = bufa[C + lane];   // the halo moves to the front ...
            bufa[lane] = h;
#pragma unroll
            for (int k = 0; k < PL; k++) {     // ... the next steps behind it
                bufa[64 + k * 64 + lane] = pf[k];
                if (WIDE) bufb[k * 64 + lane] = pg[k];
            }
        }
        if (pass == 0) {
            m1 = s1 / (double)len;
            m2 = s2 / (double)len;
        }
    }
    return cv / (__builtin_sqrt(v1) * __builtin_sqrt(v2));
}

// The reference's correlation for lag i (1 <= i <= kAcfEdge, T >= 2 * kAcfEdge) from
//   Pi = sum_{j < T-i} y_j y_{j+i},  Sm / Qm = sum / sum of squares of y over the middle,
//   hy(j) = y_j and tz(j) = y_{T-1-j} for j < kAcfEdge.
// Slice 1 = x[i..T): head positions j >= i plus the whole tail; slice 2 = x[0..T-i): the
// whole head plus tail positions T-1-j with j >= i.  Callers must run this with the same
// operands in the same order to get the same bits (the fused and separate finalizes do).
// The edge length E is kAcfEdge on the fused K <= 63 paths and K itself on the wide path
// (sts_acf_wide.hip); T >= 2E, i <= E.
// c: the shift of y = x - c; *suspect: rule 3's verdict on the result.
template <class HY, class TZ>
__device__ __forceinline__ double acf_combine_e(double Pi, double Sm, double Qm, int i, int64_t T, int E, HY hy,
                                                TZ tz, double c, bool* suspect) {
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
    const double r = cv / (__builtin_sqrt(v1) * __builtin_sqrt(v2));   // S/UnivariateTimeSeries.scala:89
    *suspect = acf_suspect(r, sum1, sq1, sum2, sq2, v1, v2, N, c);
    return r;
}

template <class HY, class TZ>
__device__ __forceinline__ double acf_combine(double Pi, double Sm, double Qm, int i, int64_t T, HY hy, TZ tz,
                                              double c, bool* suspect) {
    return acf_combine_e(Pi, Sm, Qm, i, T, kAcfEdge, hy, tz, c, suspect);
}

}  // namespace sts
