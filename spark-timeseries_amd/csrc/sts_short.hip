// sts_short.hip -- fillts (linear / previous / next / nearest) + autocorr(numLags <= 24) for short
// series held whole in one wave's registers (round 3: C1, the 10-year daily panels, T <= 2 560).
//
// Reference path: TimeSeriesRDD.fill("linear") then mapSeries(autocorr(_, K))
// (S/TimeSeriesRDD.scala:180-182, S/UnivariateTimeSeries.scala:247-266 fillLinear,
// :68-93 autocorr).  The segment kernel (sts_seg.hip) walks a short series in 512-step tiles
// with its lag products on FP64 MFMA; at T = 2 520 that is five tiles of ~1 500 instructions
// per wave, and the SIMDs' issue ports bound it.  Here one wave owns one series
// the way the AR fit does (§5.6): the series arrives by LDS-DMA into a per-wave LDS block,
// lane l takes the contiguous steps [l B, l B + B) into registers, and
//   * the linear fill runs in registers: every lane learns the last valid step before its
//     block and the first one after it (one ballot and two lane reads), then fills its NaN
//     runs by the reference's SEQUENTIAL accumulation r[j] = r[j-1] + increment, a run that
//     enters the block from the left being replayed from its start (bit-exact; a long run
//     costs its length in adds per lane it crosses).  Filled steps are written back into the
//     LDS block, which thus holds the filled series (unfillable NaNs keep their raw bits);
//   * the lag products P_1..P_KM of y = F - c (c: the robust shift, sts_acf.hpp) are
//     lane-local FP64 FMAs over a rolling window whose first KM values come from the previous
//     lane (DPP shifts); the middle sums, the wave sums and the per-lag finalize
//     (acf_combine: the head and tail read from the LDS block) follow sts_acf.hpp exactly;
//   * the filled series leaves from the LDS block as coalesced 1-KB stores.
// Tolerance as every ACF path: 1e-10 relative to the oracle; the fill is bit-exact.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdint>

#include "sts.h"
#include "sts_acf.hpp"
#include "sts_dma.hpp"
#include "sts_internal.hpp"
#include "sts_lanes.hpp"

namespace sts {
namespace {

#ifndef STS_SHORT_WAVES
#define STS_SHORT_WAVES 1   // waves (= series) per workgroup: the waves never synchronise, and
                            // one-wave workgroups free each 20-KB block as soon as its wave
                            // ends (C1: 0.1003-0.1012 ms vs 0.1036-0.1051 for 2, 0.108 for 4)
#endif
constexpr int kShortWaves = STS_SHORT_WAVES;

#ifndef STS_SHORT_TRIM
#define STS_SHORT_TRIM 5   // fewer VALU per series (round 6): 1 = bounds as masks, a c0-filled tail;
                           // 2 = + the middle sums under scalar lane masks, scalar-based DMA,
                           // validity bits by add-with-carry; 3 = + the wave sums through LDS rows;
                           // 4 = + rule 3's test on hardware reciprocals (acf_suspect_fast);
                           // 5 = + the store pass's LDS reads batched
#endif

#ifndef STS_SHORT_COMPACT
#define STS_SHORT_COMPACT 0   // the fill's in-block runs as one wave-wide list (A/B)
#endif

#ifndef STS_SHORT_DIAG
#define STS_SHORT_DIAG 0   // timing-only cost models (tools/variant.sh): 1 no ACF, 2 no fill,
                           // 3 no per-lag finalize, 4 no robust shift, 5 no lag products;
                           // wrong results
#endif

// v in the lanes of the wave-uniform mask m, +0.0 elsewhere (v_cndmask on the SGPR pair: no
// per-lane compare)
__device__ __forceinline__ double lanes_keep(double v, unsigned long long m) {
    const unsigned long long u = __builtin_bit_cast(unsigned long long, v);
    unsigned lo, hi;
    asm("v_cndmask_b32_e64 %0, 0, %1, %2" : "=v"(lo) : "v"((unsigned)u), "s"(m));
    asm("v_cndmask_b32_e64 %0, 0, %1, %2" : "=v"(hi) : "v"((unsigned)(u >> 32)), "s"(m));
    return __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lo);
}

// robust_shift (sts_acf.hpp) from the lanes' validity masks: lane l's sample is the first
// valid RAW step of [l T / 64, (l + 1) T / 64) -- a range of < B steps, so inside the blocks
// of at most two lanes -- read from the LDS block (the fill never rewrites a valid step).
// The same samples, fallbacks and median as robust_shift: the same bits.
template <int B>
__device__ __forceinline__ double shift_from_masks(const double* buf, unsigned long long vm, int T, int lane,
                                                   bool prev_fill) {
    const int a = (int)((int64_t)lane * T / 64), b = (int)((int64_t)(lane + 1) * T / 64);
    const int ba = a / B;
    const unsigned long long m0 = __shfl(vm, ba), m1 = __shfl(vm, ba + 1 < 64 ? ba + 1 : 63);
    const int o = a - ba * B;                                  // offset of a in block ba
    const int e0 = (b - ba * B < B) ? b - ba * B : B;          // end of the range in block ba
    const unsigned long long w0 = (m0 >> o) & ((e0 - o >= 64) ? ~0ull : ((1ull << (e0 - o)) - 1ull));
    const int e1 = b - (ba + 1) * B;                           // range steps in block ba + 1
    const unsigned long long w1 = (e1 > 0) ? (m1 & ((1ull << e1) - 1ull)) : 0ull;
    const bool found = a < b && (w0 || w1);
    const int idx = w0 ? a + __builtin_ctzll(w0) : (ba + 1) * B + (w1 ? __builtin_ctzll(w1) : 0);
    double v = found ? buf[idx] : 0.0;
    const unsigned long long vmk = __ballot(found);
    if (vmk == 0ull) return 0.0;
    const unsigned long long above = vmk & ~((2ull << lane) - 1ull);
    const unsigned long long below = vmk & ((1ull << lane) - 1ull);
    const int from = found ? lane : shift_fallback_lane(above, below, prev_fill);
    v = __shfl(v, from);
    return median_of_lanes(v, true, lane);
}

// ---- the pieces both kernels share ----

// the series into the LDS block by LDS-DMA (T even, 16-B aligned rows: whole 16-B pieces);
// returns the lane's validity mask (bit j: step t0 + j is inside the series and valid)
template <int B>
__device__ __forceinline__ unsigned long long short_load(double* buf, const double* src, int T, int lane, int t0) {
    const unsigned lb = lds_addr(buf);
#pragma unroll
    for (int i = 0; i < B / 2; i++) {
        const int u = 2 * (i * 64 + lane);
        if (STS_SHORT_TRIM >= 2 && (i + 1) * 128 <= T)   // a whole piece: scalar base + the lane's 16 B, no VALU
            glds16_s(src + i * 128, 16u * (unsigned)lane, lb + i * 1024);
        else   // past the series end: a copy of its last pair (T even), never read as data
            glds16(src + (STS_SHORT_TRIM ? (u < T - 2 ? u : T - 2) : (u < T ? u : 0)), lb + i * 1024);
    }
    dma_wait();
    wave_lds_sync();
    unsigned long long vm = 0ull;
    if (STS_SHORT_TRIM >= 2) {
        // bits shifted in from the top step down: acc = 2 acc + (v ordered), one compare and one
        // add-with-carry per step (the low word holds steps 0..31, the high word 32..B-1)
        unsigned wlo = 0u, whi = 0u;
#pragma unroll
        for (int j = B / 2 - 1; j >= 0; j--) {
            const double2 v = *reinterpret_cast<const double2*>(buf + t0 + 2 * j);
            if (2 * j >= 32) {
                asm volatile("v_cmp_o_f64 vcc, %1, %1\n\tv_addc_co_u32 %0, vcc, %0, %0, vcc" : "+v"(whi) : "v"(v.y) : "vcc");
                asm volatile("v_cmp_o_f64 vcc, %1, %1\n\tv_addc_co_u32 %0, vcc, %0, %0, vcc" : "+v"(whi) : "v"(v.x) : "vcc");
            } else {
                asm volatile("v_cmp_o_f64 vcc, %1, %1\n\tv_addc_co_u32 %0, vcc, %0, %0, vcc" : "+v"(wlo) : "v"(v.y) : "vcc");
                asm volatile("v_cmp_o_f64 vcc, %1, %1\n\tv_addc_co_u32 %0, vcc, %0, %0, vcc" : "+v"(wlo) : "v"(v.x) : "vcc");
            }
        }
        vm = ((unsigned long long)whi << 32) | wlo;
        const int n = T - t0;   // steps of this block inside the series
        vm &= n >= 64 ? ~0ull : n <= 0 ? 0ull : (1ull << n) - 1ull;
    } else if (STS_SHORT_TRIM) {   // the bound as one mask instead of a test per step
#pragma unroll
        for (int j = 0; j < B / 2; j++) {
            const double2 v = *reinterpret_cast<const double2*>(buf + t0 + 2 * j);
            if (!__builtin_isnan(v.x)) vm |= 1ull << (2 * j);
            if (!__builtin_isnan(v.y)) vm |= 1ull << (2 * j + 1);
        }
        const int n = T - t0;   // steps of this block inside the series
        vm &= n >= 64 ? ~0ull : n <= 0 ? 0ull : (1ull << n) - 1ull;
    } else {
#pragma unroll
        for (int j = 0; j < B / 2; j++) {
            const double2 v = *reinterpret_cast<const double2*>(buf + t0 + 2 * j);
            if (t0 + 2 * j < T && !__builtin_isnan(v.x)) vm |= 1ull << (2 * j);
            if (t0 + 2 * j + 1 < T && !__builtin_isnan(v.y)) vm |= 1ull << (2 * j + 1);
        }
    }
    return vm;
}

// The fill, run by run into the LDS block (a lane walks only its own runs).  A run is a
// maximal NaN stretch with valid ends L (or none, -1) and R (or none, T):
//   linear   (S/UnivariateTimeSeries.scala:247-266): both ends needed, r[t] = r[t-1] +
//            (x_R - x_L) / (R - L), sequentially from L;
//   previous (:194-204) x_L;  next (:214-224) x_R;
//   nearest  (:156-184) x_L while t - L < R - t, else x_R (ties to R), one end enough;
//            index 0 is never rewritten and never an end; no end at all throws.
// Returns fillNearest's "Input is all NaNs!" (no valid step after index 0).
template <int B, int M>
__device__ __forceinline__ bool short_fill(double* buf, unsigned long long vm, int T, int lane, int t0) {
    static_assert(M == STS_FILL_LINEAR || M == STS_FILL_PREVIOUS || M == STS_FILL_NEXT || M == STS_FILL_NEAREST,
                  "fill method");
    // fillNearest's index 0 is not a valid end: out of its mask (the shift keeps using vm)
    const unsigned long long vf = (M == STS_FILL_NEAREST && lane == 0) ? vm & ~1ull : vm;
    const int fv = vf ? t0 + __builtin_ctzll(vf) : T;          // first valid step of the block
    const int lv = vf ? t0 + 63 - __builtin_clzll(vf) : -1;    // last valid step of the block
    const unsigned long long hv = __ballot(vf != 0ull);
    const unsigned long long below = hv & ((1ull << lane) - 1ull);
    const unsigned long long above = hv & ~((2ull << lane) - 1ull);   // lane 63: none
    const int Lsrc = below ? 63 - __builtin_clzll(below) : lane;
    const int Rsrc = above ? __builtin_ctzll(above) : lane;
    const int lvs = __shfl(lv, Lsrc), fvs = __shfl(fv, Rsrc);
    const int Lc = below ? lvs : -1;   // last valid step before the block (-1: none)
    const int Rc = above ? fvs : T;    // first valid step after the block (T: none)
    const int tend = (t0 + B < T) ? t0 + B : T;   // end of this block inside the series
    const bool all_nan = (M == STS_FILL_NEAREST) && hv == 0ull && T >= 2;
    // steps [q0, q1) of a run with ends L, R
    auto fill_run = [&](int q0, int q1, int L, int R) {
        if (M == STS_FILL_PREVIOUS || M == STS_FILL_NEXT) {
            if (M == STS_FILL_PREVIOUS ? L >= 0 : R < T) {
                const double v = buf[M == STS_FILL_PREVIOUS ? L : R];
                for (int q = q0; q < q1; q++) buf[q] = v;
            }
        } else if (M == STS_FILL_NEAREST) {
            if (L >= 0 || R < T) {
                const double xL = (L >= 0) ? buf[L] : 0.0, xR = (R < T) ? buf[R] : 0.0;
                for (int q = q0; q < q1; q++) buf[q] = (R >= T || (L >= 0 && q - L < R - q)) ? xL : xR;
            }
        } else if (L >= 0 && R < T) {   // linear
            const double xL = buf[L];
            const double inc = (buf[R] - xL) / (double)(R - L);
            double cur = xL;
            for (int q = L + 1; q < q0; q++) cur = cur + inc;   // the run's steps in earlier blocks
            for (int q = q0; q < q1; q++) {
                cur = cur + inc;
                buf[q] = cur;
            }
        }
    };
    if (STS_SHORT_DIAG != 2 && !all_nan) {
        // the block opens inside a run (or at a NaN at t = 0): its left end is Lc, its right
        // end the block's first valid step or Rc
        if (!(vf & 1ull) && t0 < T) {
            const int R = vf ? fv : Rc;
            const int q0 = (M == STS_FILL_NEAREST && t0 == 0) ? 1 : t0;
            fill_run(q0, R < tend ? R : tend, Lc, R);
        }
        // runs that start inside the block: step t NaN, t - 1 valid
        const unsigned long long inT = (tend - t0 >= 64) ? ~0ull : ((1ull << (tend > t0 ? tend - t0 : 0)) - 1ull);
        unsigned long long rs = ~vf & (vf << 1) & inT;
        if (STS_SHORT_COMPACT) {
            // the wave's runs as one list, 64 at a time (a lane-by-lane loop runs as many rounds as
            // the lane with the most runs): run g is the k-th run of the largest lane l with
            // excl(l) <= g, excl = the runs of the lanes below (bit-sliced: nr <= B < 64)
            const int nr = __popcll(rs);
            int excl = 0, total = 0;
#pragma unroll
            for (int b = 0; b < 6; b++) {
                const unsigned long long m = __ballot((nr >> b) & 1);
                excl += (int)__builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u)) << b;
                total += __popcll(m) << b;
            }
            for (int base = 0; base < total; base += 64) {
                const int g = base + lane;
                int lo = 0;   // every lane searches (bpermute sources must be active)
#pragma unroll
                for (int st = 32; st >= 1; st >>= 1)
                    if (__shfl(excl, lo + st) <= g) lo += st;
                const int k = g - __shfl(excl, lo);
                const unsigned long long rso = __shfl(rs, lo), vfo = __shfl(vf, lo);
                const int Rco = __shfl(Rc, lo);
                if (g < total) {
                    unsigned long long m = rso;
                    for (int i = 0; i < k; i++) m &= m - 1ull;
                    const int j = __builtin_ctzll(m);
                    const int to = lo * B;
                    const int t = to + j;
                    const int tendo = (to + B < T) ? to + B : T;
                    const unsigned long long hi = (j + 1 < 64) ? vfo >> (j + 1) : 0ull;
                    const int R = hi ? t + 1 + __builtin_ctzll(hi) : Rco;
                    fill_run(t, R < tendo ? R : tendo, t - 1, R);
                }
            }
        } else {
            while (rs) {
                const int j = __builtin_ctzll(rs);
                rs &= rs - 1ull;
                const int t = t0 + j;
                const unsigned long long hi = (j + 1 < 64) ? vf >> (j + 1) : 0ull;
                const int R = hi ? t + 1 + __builtin_ctzll(hi) : Rc;
                fill_run(t, R < tend ? R : tend, t - 1, R);
            }
        }
    }
    return all_nan;
}

// the filled series out of the block: coalesced 1-KB stores
template <int B>
__device__ __forceinline__ void short_store(double* dst, const double* buf, int T, int lane) {
    if (STS_SHORT_TRIM >= 5) {
        // every piece read first (the block holds 64 B doubles: no bound on the reads), then the
        // stores: one LDS wait instead of one per store behind its exec-masked branch
        typedef double d2_t __attribute__((ext_vector_type(2)));
        d2_t v[B / 2];
#pragma unroll
        for (int i = 0; i < B / 2; i++) v[i] = *reinterpret_cast<const d2_t*>(buf + 2 * (i * 64 + lane));
#pragma unroll
        for (int i = 0; i < B / 2; i++) {
            const int u = 2 * (i * 64 + lane);
            if ((i + 1) * 128 <= T || u < T) __builtin_nontemporal_store(v[i], reinterpret_cast<d2_t*>(dst + u));
        }
        return;
    }
#pragma unroll
    for (int i = 0; i < B / 2; i++) {
        const int u = 2 * (i * 64 + lane);
        if (u < T) store_pair16<true>(dst + u, buf + u);   // nt stores: C1 0.0926 vs 0.1030 ms (nt loads too: 0.098)
    }
}

// Finalize per lag i = lane + 1 (sts_acf.hpp acf_combine's sums, regrouped): slice 1 = y[i..64)
// of the head + the whole tail + the middle, slice 2 = the whole head + z[i..64) of the tail +
// the middle; every partial is a sum of its own terms (suffix scans over the lanes, no "total
// minus head").  Pi: lag i's lag product, Sm / Qm: the middle sums, yh = y(lane), zt =
// y(T - 1 - lane).  `suspect`: sts_acf.hpp rule 3 for this lane's lag.
__device__ __forceinline__ double short_finalize(double Pi, double Sm, double Qm, double yh, double zt, double c0,
                                                 int T, int lane, bool& suspect) {
    // suffix sums from lane .. 63 by DPP (round 5: the ds_bpermute scan it replaces was ~1/3 of the
    // finalize's latency)
    const double ys = suffix_sum_dpp(yh, lane), yq = suffix_sum_dpp(yh * yh, lane);
    const double zs = suffix_sum_dpp(zt, lane), zq = suffix_sum_dpp(zt * zt, lane);
    const double Yall = lane_bcast(ys, 0), YQall = lane_bcast(yq, 0), Zall = lane_bcast(zs, 0),
                 ZQall = lane_bcast(zq, 0);
    // lag i = lane + 1 wants the suffixes from position i: lane i's (none for i = 64)
    const double ysi = lane_next(ys), yqi = lane_next(yq), zsi = lane_next(zs), zqi = lane_next(zq);
    const double sum1 = (Sm + Zall) + ysi, sq1 = (Qm + ZQall) + yqi;
    const double sum2 = (Sm + Yall) + zsi, sq2 = (Qm + YQall) + zqi;
    const double N = (double)(T - (lane + 1));
    const double v1 = sq1 - sum1 * sum1 / N;
    const double v2 = sq2 - sum2 * sum2 / N;
    const double cv = Pi - sum1 * sum2 / N;
    const double r = cv / (__builtin_sqrt(v1) * __builtin_sqrt(v2));   // :89
    suspect = STS_SHORT_TRIM >= 4 ? acf_suspect_fast(r, sum1, sq1, sum2, sq2, v1, v2, N, c0)
                                  : acf_suspect(r, sum1, sq1, sum2, sq2, v1, v2, N, c0);
    return r;
}

template <int B, int KM, int M>
__global__ __launch_bounds__(64 * kShortWaves, 2) void short_fill_acf_kernel(TileArgs a) {
    constexpr int BUFD = 64 * B;   // doubles per wave block: the whole series
    __shared__ __attribute__((aligned(16))) double buf_mem[kShortWaves * BUFD];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int64_t s = (int64_t)blockIdx.x * kShortWaves + wave;   // (an XCD-contiguous remap: 0.1025-0.1029 vs 0.1028-0.1030 ms, round 4)
    if (s >= a.S) return;
    double* buf = buf_mem + wave * BUFD;
    const int T = (int)a.T;
    const int t0 = lane * B;

    const unsigned long long vm = short_load<B>(buf, a.in + s * a.ld_in, T, lane, t0);
    const bool all_nan = short_fill<B, M>(buf, vm, T, lane, t0);
    wave_lds_sync();   // the LDS block now holds the filled series
    if (a.out) short_store<B>(a.out + s * a.ld_out, buf, T, lane);
    if (a.err && lane == 0) a.err[s] = all_nan ? STS_ERR_ALL_NAN : STS_OK;
    const int K = a.K;
    if (K <= 0 || a.acf_fused == nullptr || STS_SHORT_DIAG == 1) return;
    // the ACF shift of the RAW series (sts_acf.hpp robust_shift) while the stores drain
    const double c0 = (STS_SHORT_DIAG != 4) ? shift_from_masks<B>(buf, vm, T, lane, M == STS_FILL_PREVIOUS) : buf[0];

    // ---- ACF: y = F - c, lag products P_d = sum_t y_t y_{t-d}, middle sums ----
    double x[B];
    if (STS_SHORT_TRIM) {
        // the block past the series end holds c0, so y there is c0 - c0 = 0 without a select per
        // step (a non-finite c0 makes every y NaN anyway)
        for (int t = T + lane; t < BUFD; t += 64) buf[t] = c0;
        wave_lds_sync();
#pragma unroll
        for (int j = 0; j < B / 2; j++) {
            const double2 v = *reinterpret_cast<const double2*>(buf + t0 + 2 * j);
            x[2 * j] = v.x - c0;
            x[2 * j + 1] = v.y - c0;
        }
    } else {
#pragma unroll
        for (int j = 0; j < B / 2; j++) {
            const double2 v = *reinterpret_cast<const double2*>(buf + t0 + 2 * j);
            x[2 * j] = (t0 + 2 * j < T) ? v.x - c0 : 0.0;
            x[2 * j + 1] = (t0 + 2 * j + 1 < T) ? v.y - c0 : 0.0;
        }
    }
    // the head y(0..63) and the tail y(T-1-j), one per lane (T >= 128: disjoint)
    const double yh = buf[lane] - c0, zt = buf[T - 1 - lane] - c0;
    static_assert(KM <= B, "the window reaches one lane back only");
    double win[KM + 1];
#pragma unroll
    for (int k = 1; k <= KM; k++) win[k] = lane_prev(x[B - k]);
    double P[KM + 1];
#pragma unroll
    for (int d = 0; d <= KM; d++) P[d] = 0.0;
    double sm = 0.0, qm = 0.0, sm2 = 0.0, qm2 = 0.0;
    // the middle's last step T - kAcfEdge - 1 sits in lane mid_l at offset mid_o: steps j <= mid_o
    // of lanes <= mid_l are below the tail, steps j > mid_o only of lanes < mid_l (wave-uniform)
    const int mid_l = (T - kAcfEdge - 1) / B, mid_o = T - kAcfEdge - 1 - mid_l * B;
    const unsigned long long mid_m1 = mid_l >= 63 ? ~0ull : (2ull << mid_l) - 1ull;
    const unsigned long long mid_m0 = (1ull << mid_l) - 1ull;
#pragma unroll
    for (int j = 0; j < B; j++) {
        const double yj = x[j];
        if (STS_SHORT_TRIM >= 2) {
            // rule 2's middle [kAcfEdge, T - kAcfEdge) holds step t0 + j for the lanes l in [lo, hi):
            // a wave-uniform lane mask per j (scalar work), one masked copy of y for both sums, and
            // two chains (even / odd j) for the latency
            const int lo = j >= kAcfEdge ? 0 : (kAcfEdge - j + B - 1) / B;   // a constant after unrolling
            const unsigned long long mm = (j <= mid_o ? mid_m1 : mid_m0) & ~((1ull << lo) - 1ull);
            const double ym = lanes_keep(yj, mm);
            if (j & 1) {
                sm2 += ym;
                qm2 = __builtin_fma(ym, ym, qm2);
            } else {
                sm += ym;
                qm = __builtin_fma(ym, ym, qm);
            }
        } else if (acf_mid(t0 + j, T)) {
            sm += yj;
            qm = __builtin_fma(yj, yj, qm);
        }
#pragma unroll
        for (int d = 1; d <= KM; d++)
            if (STS_SHORT_DIAG != 5) P[d] = __builtin_fma(yj, win[d], P[d]);
#pragma unroll
        for (int k = KM; k >= 2; k--) win[k] = win[k - 1];
        win[1] = yj;
    }
    // ---- wave sums: rows by DPP, the four row sums of each quantity through the block
    //      (lane d - 1 collects lag d), added in wave_sum_dpp's order ----
    wave_lds_sync();   // every read of the filled block is done: it becomes scratch
    double* scr = buf;
    if (STS_SHORT_TRIM >= 2) {
        sm += sm2;
        qm += qm2;
    }
    double Pi, Sm, Qm;
    // the V = KM + 2 quantities (0: sm, d: P_d, KM + 1: qm) of every lane as LDS rows of RS
    // doubles (RS odd: conflict-free writes), then lane (v, q) sums quantity v over the q-th of
    // G lane groups and a second pass adds the G partials -- ~V + G adds per lane where the DPP
    // row sums cost 12 VALU per quantity (round 6)
    constexpr int V = KM + 2, RS = V | 1, G = 64 / V, LG = (64 + G - 1) / G;
    if (STS_SHORT_TRIM >= 3 && 64 * RS + G * V <= BUFD) {
#pragma unroll
        for (int v = 0; v < V; v++) scr[lane * RS + v] = v == 0 ? sm : v == KM + 1 ? qm : P[v];
        wave_lds_sync();
        double* part = scr + 64 * RS;
        if (lane < G * V) {
            const int v = lane % V, q = lane / V;
            const double* col = scr + q * LG * RS + v;
            double a0 = 0.0, a1 = 0.0;
#pragma unroll
            for (int k = 0; k < LG; k += 2) {
                if (q * LG + k < 64) a0 += col[k * RS];
                if (k + 1 < LG && q * LG + k + 1 < 64) a1 += col[(k + 1) * RS];
            }
            part[q * V + v] = a0 + a1;
        }
        wave_lds_sync();
        const int li = (lane < KM) ? lane + 1 : KM;
        Pi = part[li];
        Sm = part[0];
        Qm = part[KM + 1];
#pragma unroll
        for (int q = 1; q < G; q++) {
            Pi += part[q * V + li];
            Sm += part[q * V];
            Qm += part[q * V + KM + 1];
        }
    } else {
        const int row = lane >> 4;
        const bool row_lead = (lane & 15) == 0;
#pragma unroll
        for (int d = 1; d <= KM; d++) {
            const double v = row_sum_dpp(P[d]);
            if (row_lead) scr[4 * d + row] = v;
        }
        {
            const double v0 = row_sum_dpp(sm), v1 = row_sum_dpp(qm);
            if (row_lead) {
                scr[row] = v0;
                scr[4 * (KM + 1) + row] = v1;
            }
        }
        wave_lds_sync();
        const int li = (lane < KM) ? lane + 1 : KM;
        const double4 pr = *reinterpret_cast<const double4*>(scr + 4 * li);
        Pi = (pr.x + pr.y) + (pr.z + pr.w);
        const double4 sr = *reinterpret_cast<const double4*>(scr);
        const double4 qr = *reinterpret_cast<const double4*>(scr + 4 * (KM + 1));
        Sm = (sr.x + sr.y) + (sr.z + sr.w);
        Qm = (qr.x + qr.y) + (qr.z + qr.w);
    }
    if (STS_SHORT_DIAG == 3) {
        if (lane < K) a.acf_fused[s * K + lane] = Pi + Sm + Qm;
        return;
    }
    bool sus;
    double r = short_finalize(Pi, Sm, Qm, yh, zt, c0, T, lane, sus);
    // sts_acf.hpp rule 3: a suspect series takes the reference's loop over the filled series
    // this wave stored (the LDS block is scratch by now): order the stores before the reads
    if (__ballot(lane < K && sus)) {
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
        // F streams back through the (now free) block: the reference's loop, every sum from LDS
        // (sts_acf.hpp acf_exact_stream; in this kernel, so the normal case pays no extra launch)
        constexpr int CX = 64 * B - 64 < 512 ? 64 * B - 64 : 512;
        const double e = acf_exact_stream<CX>(a.out + s * a.ld_out, T, lane + 1, lane < K, buf, lane);
        if (lane < K) r = e;
    }
    if (lane < K) a.acf_fused[s * K + lane] = r;
}

// LDS barrier of the two waves of a pair workgroup (LDS ordering only: the block changes hands;
// global stores stay in flight)
__device__ __forceinline__ void pair_lds_barrier() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// Round 6: two waves per workgroup on ONE LDS block, ping-pong.  The one-wave
// kernel above holds its 20-KB block through the whole ACF although the block is only needed
// until y is in registers.  Here the workgroup is persistent over the series g, g + G, g + 2G, ...
// (G workgroups) and its two waves alternate: in phase p the block's owner (wave p % 2) streams
// series slot p in, fills it, stores it and takes y into registers, while the other wave runs the
// lag products and the finalize of slot p - 1 from its registers; an LDS barrier ends the phase.
// So each block is always streaming, and a CU holds 8 blocks with 16 waves -- which needs <= 128
// VGPRs: y stays resident (2B VGPRs), the lag products run in passes of <= 12 lags with the
// previous lane's steps fetched one at a time (no rolling window), and the wave sums go by DPP
// (no LDS scratch: the block belongs to the partner).  Rule 3 runs after the loop, when the block
// is free (half per wave), for the slots a wave recorded (the 64 first; later ones read global
// memory directly, sts_acf.hpp acf_exact_lag: the same bits).
#ifndef STS_PAIR_LAGS
#define STS_PAIR_LAGS 8   // lags per pass of the pair kernel's lag products
#endif
constexpr int kPairLags = STS_PAIR_LAGS;

template <int B, int KM, int M>
__global__ __launch_bounds__(128, 4) void short_pair_kernel(TileArgs a) {
    constexpr int BUFD = 64 * B;
    __shared__ __attribute__((aligned(16))) double buf[BUFD];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int64_t G = gridDim.x, g = blockIdx.x;
    const int64_t nslots = g < a.S ? (a.S - g + G - 1) / G : 0;
    const int T = (int)a.T;
    const int t0 = lane * B;
    const int K = a.K;
    const bool acf = K > 0 && a.acf_fused != nullptr;
    static_assert(KM <= B, "the lag partners reach one lane back only");
    double x[B];
    double yh = 0.0, zt = 0.0, c0 = 0.0;
    unsigned long long sus_slots = 0ull;   // bit j: this wave's slot 2j + wave needs rule 3
    for (int64_t p = 0; p <= nslots; p++) {
        // per-phase opaque copies: the per-step predicates and addresses derived from them are
        // recomputed in each phase instead of hoisted out of the loop (and spilled)
        int lane_q = lane, T_q = T;
        asm volatile("" : "+v"(lane_q));
        asm volatile("" : "+s"(T_q));
        const int lane = lane_q, T = T_q, t0 = lane * B;
        if ((int)(p & 1) == wave) {
            if (p < nslots) {   // ---- the block's owner: series in, fill, out, y -> registers ----
                const int64_t s = g + p * G;
                const unsigned long long vm = short_load<B>(buf, a.in + s * a.ld_in, T, lane, t0);
                const bool all_nan = short_fill<B, M>(buf, vm, T, lane, t0);
                wave_lds_sync();
                if (a.out) short_store<B>(a.out + s * a.ld_out, buf, T, lane);
                if (a.err && lane == 0) a.err[s] = all_nan ? STS_ERR_ALL_NAN : STS_OK;
                if (acf) c0 = shift_from_masks<B>(buf, vm, T, lane, M == STS_FILL_PREVIOUS);
            }
            // y into registers on EVERY path through this branch (past the last slot: whatever the
            // block holds, never used), so the previous slot's y is dead during the fill instead of
            // carried around the loop
#pragma unroll
            for (int j = 0; j < B / 2; j++) {
                const double2 v = *reinterpret_cast<const double2*>(buf + t0 + 2 * j);
                x[2 * j] = (t0 + 2 * j < T) ? v.x - c0 : 0.0;
                x[2 * j + 1] = (t0 + 2 * j + 1 < T) ? v.y - c0 : 0.0;
            }
            yh = buf[lane] - c0;
            zt = buf[T - 1 - lane] - c0;
        } else if (p >= 1 && acf && STS_SHORT_DIAG != 1) {   // ---- the other wave: slot p - 1's ACF from registers ----
            const int64_t s = g + (p - 1) * G;
            constexpr int NP = (KM + kPairLags - 1) / kPairLags, LP = (KM + NP - 1) / NP;
            double Pi = 0.0, sm = 0.0, qm = 0.0;
#pragma unroll
            for (int pass = 0; pass < NP; pass++) {
                const int d0 = 1 + pass * LP;   // lags d0 .. d0 + LP - 1 (past KM: zero, never read)
                double P[LP];
#pragma unroll
                for (int q = 0; q < LP; q++) P[q] = 0.0;
                // partners in the previous lane's block: y(t0 - m), one at a time (lane 0: 0)
#pragma unroll
                for (int m = 1; m < d0 + LP && m <= KM; m++) {
                    const double pv = lane_prev(x[B - m]);
#pragma unroll
                    for (int q = 0; q < LP; q++)
                        if (d0 + q >= m && d0 + q <= KM) P[q] = __builtin_fma(x[d0 + q - m], pv, P[q]);
                }
#pragma unroll
                for (int j = 0; j < B; j++) {
                    if (pass == 0 && acf_mid(t0 + j, T)) {
                        sm += x[j];
                        qm = __builtin_fma(x[j], x[j], qm);
                    }
#pragma unroll
                    for (int q = 0; q < LP; q++)
                        if (j >= d0 + q && d0 + q <= KM && STS_SHORT_DIAG != 5) P[q] = __builtin_fma(x[j], x[j - d0 - q], P[q]);
                }
                // wave sums into lane 63 (DPP only), then lag d's to lane d - 1
#pragma unroll
                for (int q = 0; q < LP && d0 + q <= KM; q++) {
                    const double tot = lane_bcast(wave_sum_to_63(P[q]), 63);
                    if (lane == d0 + q - 1) Pi = tot;
                }
            }
            const double Sm = lane_bcast(wave_sum_to_63(sm), 63), Qm = lane_bcast(wave_sum_to_63(qm), 63);
            bool sus;
            double r = short_finalize(Pi, Sm, Qm, yh, zt, c0, T, lane, sus);
            if (__ballot(lane < K && sus)) sus_slots |= 1ull << ((p - 1) >> 1);   // < 64: the launcher caps nslots
            if (lane < K) a.acf_fused[s * K + lane] = r;
        }
        pair_lds_barrier();   // the block changes hands
    }
    // ---- rule 3 (sts_acf.hpp) for the recorded slots: the reference's loop over the filled series
    //      this wave stored, streamed through its half of the (now free) block ----
    if (sus_slots) __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    while (sus_slots) {
        const int j = __builtin_ctzll(sus_slots);
        sus_slots &= sus_slots - 1ull;
        const int64_t s = g + (2 * (int64_t)j + wave) * G;
        constexpr int CX = 32 * B - 64 < 512 ? 32 * B - 64 : 512;
        const double e = acf_exact_stream<CX>(a.out + s * a.ld_out, T, lane + 1, lane < K, buf + wave * (BUFD / 2), lane);
        if (lane < K) a.acf_fused[s * K + lane] = e;
    }
}

}  // namespace

// fill('linear') + fused ACF for 128 <= T <= 2 560, T even, K <= 24, 16-B aligned rows
bool short_ok(int method, int64_t T, int K) {
    return (method == STS_FILL_LINEAR || method == STS_FILL_PREVIOUS || method == STS_FILL_NEXT ||
            method == STS_FILL_NEAREST) &&
           T >= 2 * kAcfEdge && T <= 64 * 40 && !(T & 1) && K > 0 && K <= 24 &&
           T > 2 * (int64_t)K;
}

// compute units of the current device (cached per device; 256 on MI355X)
int cu_count() {
    static std::atomic<int> cache[64];
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0) dev = 0;
    const int slot = dev < 64 ? dev : 63;
    int n = cache[slot].load(std::memory_order_relaxed);
    if (n <= 0) {
        if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
        cache[slot].store(n, std::memory_order_relaxed);
    }
    return n;
}

template <int M>
hipError_t launch_short_m(const TileArgs& a, hipStream_t st, bool pair) {
    if (a.S <= 0) return hipSuccess;
    // the pair form is persistent: two series per workgroup and 8 workgroups (LDS blocks) per CU at most
    // (>= S / 128 workgroups: a wave's rule-3 record holds 64 slots)
    const int64_t nblk = pair ? std::max<int64_t>(std::min<int64_t>((a.S + 1) / 2, 8 * (int64_t)cu_count()), (a.S + 127) / 128)
                              : (a.S + kShortWaves - 1) / kShortWaves;
    if (nblk > 0x7fffffffLL) return hipErrorInvalidValue;
    dim3 g((unsigned)nblk), b(pair ? 128 : 64 * kShortWaves);
    const int64_t need = (a.T + 63) / 64;
    // the lag window (KM >= K, a multiple of 4) reaches back KM steps: blocks of >= KM steps
    const int KM = (a.K + 3) / 4 * 4 < 8 ? 8 : (a.K + 3) / 4 * 4;
    const int64_t nb = need < KM ? KM : need;
    const int B = nb <= 8 ? 8 : nb <= 16 ? 16 : nb <= 24 ? 24 : nb <= 32 ? 32 : 40;
#define STS_SHORT_K(BB, KK)                                                                        \
    case KK:                                                                                       \
        if (pair) hipLaunchKernelGGL((short_pair_kernel<BB, (KK <= BB ? KK : BB), M>), g, b, 0, st, a); \
        else hipLaunchKernelGGL((short_fill_acf_kernel<BB, (KK <= BB ? KK : BB), M>), g, b, 0, st, a);  \
        break;
#define STS_SHORT(BB)                                                                              \
    case BB:                                                                                       \
        switch (KM) {                                                                              \
            STS_SHORT_K(BB, 8) STS_SHORT_K(BB, 12) STS_SHORT_K(BB, 16) STS_SHORT_K(BB, 20)         \
            STS_SHORT_K(BB, 24)                                                                    \
        default: return hipErrorInvalidValue;                                                      \
        }                                                                                          \
        break;
    switch (B) {
        STS_SHORT(8) STS_SHORT(16) STS_SHORT(24) STS_SHORT(32) STS_SHORT(40)
    default: return hipErrorInvalidValue;
    }
#undef STS_SHORT
#undef STS_SHORT_K
    return hipGetLastError();
}

hipError_t launch_short(int method, const TileArgs& a, hipStream_t st, bool pair) {
    switch (method) {
    case STS_FILL_LINEAR: return launch_short_m<STS_FILL_LINEAR>(a, st, pair);
    case STS_FILL_PREVIOUS: return launch_short_m<STS_FILL_PREVIOUS>(a, st, pair);
    case STS_FILL_NEXT: return launch_short_m<STS_FILL_NEXT>(a, st, pair);
    case STS_FILL_NEAREST: return launch_short_m<STS_FILL_NEAREST>(a, st, pair);
    default: return hipErrorInvalidValue;
    }
}

}  // namespace sts
