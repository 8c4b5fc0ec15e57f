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

#ifndef STS_SHORT_DIAG
#define STS_SHORT_DIAG 0   // timing-only cost models (tools/variant.sh): 1 no ACF, 2 no fill,
                           // 3 no per-lag finalize, 4 no robust shift, 5 no lag products;
                           // wrong results
#endif

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

template <int B, int KM, int M>
__global__ __launch_bounds__(64 * kShortWaves, 2) void short_fill_acf_kernel(TileArgs a) {
    static_assert(M == STS_FILL_LINEAR || M == STS_FILL_PREVIOUS || M == STS_FILL_NEXT || M == STS_FILL_NEAREST,
                  "fill method");
    constexpr int BUFD = 64 * B;   // doubles per wave block: the whole series
    __shared__ __attribute__((aligned(16))) double buf_mem[kShortWaves * BUFD];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int64_t s = (int64_t)blockIdx.x * kShortWaves + wave;   // (an XCD-contiguous remap: 0.1025-0.1029 vs 0.1028-0.1030 ms, round 4)
    if (s >= a.S) return;
    double* buf = buf_mem + wave * BUFD;
    const int T = (int)a.T;
    const int t0 = lane * B;
    const double* src = a.in + s * a.ld_in;

    // ---- the series into the LDS block (T even, 16-B aligned rows: whole 16-B pieces) ----
    {
        const unsigned lb = lds_addr(buf);
#pragma unroll
        for (int i = 0; i < B / 2; i++) {
            const int u = 2 * (i * 64 + lane);
            glds16(src + (u < T ? u : 0), lb + i * 1024);
        }
        dma_wait();
        wave_lds_sync();
    }
    unsigned long long vm = 0ull;   // bit j: step t0 + j is inside the series and valid
#pragma unroll
    for (int j = 0; j < B / 2; j++) {
        const double2 v = *reinterpret_cast<const double2*>(buf + t0 + 2 * j);
        if (t0 + 2 * j < T && !__builtin_isnan(v.x)) vm |= 1ull << (2 * j);
        if (t0 + 2 * j + 1 < T && !__builtin_isnan(v.y)) vm |= 1ull << (2 * j + 1);
    }

    // ---- the fill, run by run into the LDS block (a lane walks only its own runs).  A run is a
    //      maximal NaN stretch with valid ends L (or none, -1) and R (or none, T):
    //      linear   (S/UnivariateTimeSeries.scala:247-266): both ends needed, r[t] = r[t-1] +
    //               (x_R - x_L) / (R - L), sequentially from L;
    //      previous (:194-204) x_L;  next (:214-224) x_R;
    //      nearest  (:156-184) x_L while t - L < R - t, else x_R (ties to R), one end enough;
    //               index 0 is never rewritten and never an end; no end at all throws. ----
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
    // fillNearest over a series with no valid step after index 0: "Input is all NaNs!"
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
        while (rs) {
            const int j = __builtin_ctzll(rs);
            rs &= rs - 1ull;
            const int t = t0 + j;
            const unsigned long long hi = (j + 1 < 64) ? vf >> (j + 1) : 0ull;
            const int R = hi ? t + 1 + __builtin_ctzll(hi) : Rc;
            fill_run(t, R < tend ? R : tend, t - 1, R);
        }
    }
    wave_lds_sync();   // the LDS block now holds the filled series

    // ---- filled series out: coalesced 1-KB stores from the block ----
    if (a.out) {
        double* dst = a.out + s * a.ld_out;
#pragma unroll
        for (int i = 0; i < B / 2; i++) {
            const int u = 2 * (i * 64 + lane);
            if (u < T) store_pair16<true>(dst + u, buf + u);   // nt stores: C1 0.0926 vs 0.1030 ms (nt loads too: 0.098)
        }
    }
    if (a.err && lane == 0) a.err[s] = all_nan ? STS_ERR_ALL_NAN : STS_OK;
    const int K = a.K;
    if (K <= 0 || a.acf_fused == nullptr || STS_SHORT_DIAG == 1) return;
    // the ACF shift of the RAW series (sts_acf.hpp robust_shift) while the stores drain
    const double c0 = (STS_SHORT_DIAG != 4) ? shift_from_masks<B>(buf, vm, T, lane, M == STS_FILL_PREVIOUS) : buf[0];

    // ---- ACF: y = F - c, lag products P_d = sum_t y_t y_{t-d}, middle sums ----
    double x[B];
#pragma unroll
    for (int j = 0; j < B / 2; j++) {
        const double2 v = *reinterpret_cast<const double2*>(buf + t0 + 2 * j);
        x[2 * j] = (t0 + 2 * j < T) ? v.x - c0 : 0.0;
        x[2 * j + 1] = (t0 + 2 * j + 1 < T) ? v.y - c0 : 0.0;
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
    double sm = 0.0, qm = 0.0;
#pragma unroll
    for (int j = 0; j < B; j++) {
        const double yj = x[j];
        if (acf_mid(t0 + j, T)) {
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
    const double Pi = (pr.x + pr.y) + (pr.z + pr.w);
    const double4 sr = *reinterpret_cast<const double4*>(scr);
    const double4 qr = *reinterpret_cast<const double4*>(scr + 4 * (KM + 1));
    const double Sm = (sr.x + sr.y) + (sr.z + sr.w), Qm = (qr.x + qr.y) + (qr.z + qr.w);
    if (STS_SHORT_DIAG == 3) {
        if (lane < K) a.acf_fused[s * K + lane] = Pi + Sm + Qm;
        return;
    }
    // ---- finalize per lag i = lane + 1 (sts_acf.hpp acf_combine's sums, regrouped): slice 1
    //      = y[i..64) of the head + the whole tail + the middle, slice 2 = the whole head +
    //      z[i..64) of the tail + the middle; every partial is a sum of its own terms (suffix
    //      scans over the lanes, no "total minus head") ----
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
    double r = cv / (__builtin_sqrt(v1) * __builtin_sqrt(v2));   // :89
    // sts_acf.hpp rule 3: a suspect series takes the reference's loop over the filled series
    // this wave stored (the LDS block is scratch by now): order the stores before the reads
    if (__ballot(lane < K && acf_suspect(r, sum1, sq1, sum2, sq2, v1, v2, N, c0))) {
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
        // F streams back through the (now free) block: the reference's loop, every sum from LDS
        // (sts_acf.hpp acf_exact_stream; in this kernel, so the normal case pays no extra launch)
        constexpr int CX = 64 * B - 64 < 512 ? 64 * B - 64 : 512;
        const double e = acf_exact_stream<CX>(a.out + s * a.ld_out, T, lane + 1, lane < K, buf, lane);
        if (lane < K) r = e;
    }
    if (lane < K) a.acf_fused[s * K + lane] = r;
}

}  // namespace

// fill('linear') + fused ACF for 128 <= T <= 2 560, T even, K <= 24, 16-B aligned rows
bool short_ok(int method, int64_t T, int K) {
    return (method == STS_FILL_LINEAR || method == STS_FILL_PREVIOUS || method == STS_FILL_NEXT ||
            method == STS_FILL_NEAREST) &&
           T >= 2 * kAcfEdge && T <= 64 * 40 && !(T & 1) && K > 0 && K <= 24 &&
           T > 2 * (int64_t)K;
}

template <int M>
hipError_t launch_short_m(const TileArgs& a, hipStream_t st) {
    if (a.S <= 0) return hipSuccess;
    const int64_t nblk = (a.S + kShortWaves - 1) / kShortWaves;
    if (nblk > 0x7fffffffLL) return hipErrorInvalidValue;
    dim3 g((unsigned)nblk), b(64 * kShortWaves);
    const int64_t need = (a.T + 63) / 64;
    // the lag window (KM >= K, a multiple of 4) reaches back KM steps: blocks of >= KM steps
    const int KM = (a.K + 3) / 4 * 4 < 8 ? 8 : (a.K + 3) / 4 * 4;
    const int64_t nb = need < KM ? KM : need;
    const int B = nb <= 8 ? 8 : nb <= 16 ? 16 : nb <= 24 ? 24 : nb <= 32 ? 32 : 40;
#define STS_SHORT_K(BB, KK) \
    case KK: hipLaunchKernelGGL((short_fill_acf_kernel<BB, (KK <= BB ? KK : BB), M>), g, b, 0, st, a); break;
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

hipError_t launch_short(int method, const TileArgs& a, hipStream_t st) {
    switch (method) {
    case STS_FILL_LINEAR: return launch_short_m<STS_FILL_LINEAR>(a, st);
    case STS_FILL_PREVIOUS: return launch_short_m<STS_FILL_PREVIOUS>(a, st);
    case STS_FILL_NEXT: return launch_short_m<STS_FILL_NEXT>(a, st);
    case STS_FILL_NEAREST: return launch_short_m<STS_FILL_NEAREST>(a, st);
    default: return hipErrorInvalidValue;
    }
}

}  // namespace sts
