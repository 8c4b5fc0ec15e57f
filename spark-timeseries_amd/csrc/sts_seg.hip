// sts_seg.hip -- the wave-private SEGMENT kernel: NaN imputation (fillts) of long series
// with optional fused multi-lag autocorrelation partial sums on FP64 MFMA.  It serves
// sts_fill / sts_fill_autocorr / sts_autocorr whenever the panel is 16-B aligned and
// K <= 60 (sts_tile.hip keeps the lag-matrix output and K = 61..63).
//
// Reference operators (S/ = src/main/scala/com/cloudera/sparkts/):
//   fillPrevious   S/UnivariateTimeSeries.scala:194-204
//   fillNext       S/UnivariateTimeSeries.scala:214-224
//   fillNearest    S/UnivariateTimeSeries.scala:156-184
//   fillLinear     S/UnivariateTimeSeries.scala:247-266
//   autocorr       S/UnivariateTimeSeries.scala:68-93
//
// Work decomposition.  One WAVE owns one segment of kSegTiles tiles of kW = 512 steps of
// one series and walks it sequentially; the four waves of a workgroup are independent
// (no __syncthreads anywhere), each with a private LDS ring, so loads, imputation,
// stores and MFMA phases of different waves interleave freely on a CU.  Per tile:
//   * the tile arrived in registers one iteration earlier (4 x 16 B per lane, 1 KB
//     contiguous per load instruction) and was copied raw into the ring;
//   * validity ballots (one 64-bit mask per 64 steps) of this tile and of the NEXT tile
//     (which is in registers) give every NaN its last valid index L <= t (carried across
//     tiles) and first valid index N >= t (looking into the next tile) in O(1);
//   * the NaN positions are compacted and imputed with every lane busy; linear replays
//     the reference's sequential accumulation r = r + inc (t - L adds) -- bit-exact, the
//     library is built with -ffp-contract=off;
//   * the filled tile goes out with 16-B stores and y = F - c replaces it in the ring (c =
//     the robust shift of sts_acf.hpp; sum y and sum y^2 over the series' middle are
//     accumulated here);
//   * the PREVIOUS tile's lag products run on MFMA (its ring slot plus this tile's head).
//
// Lag products with 4 MFMAs per 64 steps for K <= 60 (2 for K <= 24).  With
// A[i][k] = y(m0 + c + i + 16k) and B[k][j] = y(m0 + c + 16k + h(j)), the 16x16x4 FP64
// MFMA accumulates D[i][j] += sum_k y_m y_{m + h(j) - i} (m = m0 + c + i + 16k): entry
// (i, j) holds lag h(j) - i.  MFMA number t of a 64-step chunk uses the window shift
// c = q t (q = 16 / NT) and h(j) = 16 (j / q) + 16 - q + (j % q).  A position m with
// m mod 16 = rho sits in row (rho - q t) mod 16 of MFMA t, so across t its lag sets are
// 16 (j / q) + 16 - q + (j % q) - ((rho - q t) mod 16): the q-wide residue windows of the
// NT MFMAs tile the 16 residues and every lag 0 .. 16 NT - q is hit exactly once per
// position (waste: lags -q+1..-1 and > 16 NT - q).  For K = 60 that is 64 MACs per step
// for 61 needed (the plain Toeplitz blocking needs 5 MFMAs = 80).  The lag map is the
// same for every t, so the NT accumulators are summed before the diagonal extraction.
#include "sts_internal.hpp"
#include "sts_acf.hpp"
#include "sts_scan.hpp"
#include "sts_lanes.hpp"

#include <hip/hip_runtime.h>

#include <type_traits>

namespace sts {
namespace {

typedef double d4 __attribute__((ext_vector_type(4)));
// native vector (HIP's double2 is a struct: arrays of it are not promoted to registers)
typedef double v2d __attribute__((ext_vector_type(2)));

#ifndef STS_SEG_VTAB
#define STS_SEG_VTAB 1                // word tables lane-parallel (DPP scans) instead of a scalar loop
#endif

constexpr int kW = 512;               // steps per tile
constexpr int kWords = kW / 64;       // validity words per tile
constexpr int kRing = 2 * kW + 128;   // two slots + a mirror of slot 0's head
constexpr int kWaves = 4;             // waves per workgroup (independent)
constexpr int kBig = 0x7fffffff;

struct WaveLds {
    double ring[kRing];
    unsigned long long m2[2][kWords]; // validity masks of the tiles in ring slots 0 / 1
    unsigned long long need[kWords];  // NaN positions to impute
    int lastUp[kWords];               // last valid global index in words <= w (carry: < tile)
    int firstFrom[kWords];            // first valid global index in words >= w (look-ahead)
    int wbase[kWords + 1];            // exclusive prefix count of need bits
    // linear fill, long runs (as in sts_tile.hip): the chain value at the last step of the
    // previous tile (by tile parity)
    int carry_L[2], carry_t[2];
    double carry_r[2];
    int cN_pos, cN;                   // cache of the global look-ahead scan: first valid >= cN_pos is cN
};

__device__ __forceinline__ bool isnan_d(double v) { return __builtin_isnan(v); }

// Order LDS traffic between lanes of ONE wave: LDS instructions of a wave execute in
// order, so only the compiler has to be kept from reordering across the hand-off.
// (LDS-only fences: a fence on all address spaces would also emit s_waitcnt vmcnt(0) and
// drain the register prefetch and the stores at every hand-off.)
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
}

__device__ __forceinline__ unsigned long long bitrep(unsigned x) {
    unsigned long long r;
    asm("s_bitreplicate_b64_b32 %0, %1" : "=s"(r) : "s"(x));
    return r;
}
// bit i of ev -> bit 2i, bit i of od -> bit 2i + 1
__device__ __forceinline__ unsigned long long interleave2(unsigned ev, unsigned od) {
    return (bitrep(ev) & 0x5555555555555555ull) | (bitrep(od) & 0xAAAAAAAAAAAAAAAAull);
}

__device__ __forceinline__ double readlane_d(double v, int l) {
    const unsigned long long u = __builtin_bit_cast(unsigned long long, v);
    const unsigned lo = __builtin_amdgcn_readlane((unsigned)u, l);
    const unsigned hi = __builtin_amdgcn_readlane((unsigned)(u >> 32), l);
    return __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lo);
}

// One tile into registers: lane l, register u holds steps kb + 128u + 2l (+1).
__device__ __forceinline__ void load_tile(v2d (&R)[4], const double* src, int kb, int T, int lane) {
    const v2d* s2 = reinterpret_cast<const v2d*>(src + kb) + lane;
    if (kb + kW <= T) {
#pragma unroll
        for (int u = 0; u < 4; u++) R[u] = s2[64 * u];
    } else {
        const double nan = __builtin_nan("");
#pragma unroll
        for (int u = 0; u < 4; u++) {   // clamped loads + selects: no branches around R
            const int t = kb + 128 * u + 2 * lane;
            const double a = src[t < T ? t : T - 1];
            const double b = src[t + 1 < T ? t + 1 : T - 1];
            v2d v;
            v.x = (t < T) ? a : nan;
            v.y = (t + 1 < T) ? b : nan;
            R[u] = v;
        }
    }
}

__device__ __forceinline__ double pick_reg(const v2d (&R)[4], int p) {
    const int u = p >> 7, ln = (p & 127) >> 1, e = p & 1;
    double v = 0.0;
#pragma unroll
    for (int uu = 0; uu < 4; uu++)
        if (uu == u) v = e ? R[uu].y : R[uu].x;
    return readlane_d(v, ln);
}

template <int NT>
struct Mfma {
    static constexpr int Q = (NT > 0) ? 16 / NT : 16;
    static constexpr int NA = (NT > 2) ? 2 : (NT > 0 ? NT : 1);   // accumulators (the lag map is t-independent)
    __device__ static __forceinline__ int offB(int lane) {
        const int j = lane & 15;
        return 16 * (lane >> 4) + 16 * (j / Q) + (16 - Q) + (j % Q);
    }
    // lag products of the chunks [c_lo, 8) of the tile in ring slot SLOT
    template <int SLOT>
    __device__ static __forceinline__ void tile(const double* ring, int c_lo, d4 (&U)[Mfma<NT>::NA], int lane,
                                                int offb) {
        const double* pa = ring + SLOT * kW + lane;
        const double* pb = ring + SLOT * kW + offb;
        // software pipeline, one chunk deep: chunk c + 1's operands load while chunk c's
        // MFMAs run; the sched barrier stops the scheduler hoisting every chunk's loads
        // (that alone would take 128 VGPRs)
        double a[NT], b[NT];
#pragma unroll
        for (int t = 0; t < NT; t++) {
            a[t] = pa[64 * c_lo + Q * t];
            b[t] = pb[64 * c_lo + Q * t];
        }
#pragma unroll
        for (int c = 0; c < kWords; c++) {
            if (c < c_lo) continue;
            double an[NT], bn[NT];
            if (c + 1 < kWords) {
#pragma unroll
                for (int t = 0; t < NT; t++) {
                    an[t] = pa[64 * (c + 1) + Q * t];
                    bn[t] = pb[64 * (c + 1) + Q * t];
                }
            }
#pragma unroll
            for (int t = 0; t < NT; t++) U[t % NA] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[t], b[t], U[t % NA], 0, 0, 0);
            __builtin_amdgcn_sched_barrier(0);
            if (c + 1 < kWords) {
#pragma unroll
                for (int t = 0; t < NT; t++) {
                    a[t] = an[t];
                    b[t] = bn[t];
                }
            }
        }
    }
};

struct SegState {
    int Lc;          // last valid index before the tile being imputed (-1: none)
    double Lv;       // its value
    double c0;       // ACF shift (sts_acf.hpp robust_shift)
    double sm, qm;   // this lane's sum y / sum y^2 over the series' middle (sts_acf.hpp)
    bool err;        // nearest: "Input is all NaNs!"
};

__device__ __forceinline__ unsigned long long uni64(unsigned long long v) {
    const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)v);
    const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(v >> 32));
    return ((unsigned long long)hi << 32) | lo;
}

// Validity masks of a tile held in registers -> LDS (word 2u: lanes 0..31 of register u,
// word 2u + 1: lanes 32..63); returns the tile position of its first valid step (-1: none).
__device__ __forceinline__ int masks_to_lds(const v2d (&R)[4], unsigned long long* dstm, int lane) {
    int f = -1;
#pragma unroll
    for (int u = 3; u >= 0; u--) {
        const unsigned long long bx = __ballot(!isnan_d(R[u].x));
        const unsigned long long by = __ballot(!isnan_d(R[u].y));
        const unsigned long long m0 = interleave2((unsigned)bx, (unsigned)by);
        const unsigned long long m1 = interleave2((unsigned)(bx >> 32), (unsigned)(by >> 32));
        if (m1) f = 128 * u + 64 + __ffsll(m1) - 1;
        if (m0) f = 128 * u + __ffsll(m0) - 1;
        if (lane == 0) {
            dstm[2 * u] = m0;
            dstm[2 * u + 1] = m1;
        }
    }
    return f;
}

// Impute tile k (ring slot SLOT, raw; masks in w.m2[SLOT]) and turn it into y; optionally
// store it.  look: first valid index >= kb + kW when known (kBig: unknown, then scan
// global memory from scan_from); lookv its value.
template <int NT, int SLOT>
__device__ __forceinline__ void impute_tile(WaveLds& w, const double* src, double* dst, int kb, int T, int method,
                                            int look, double lookv, int scan_from, bool store, bool own,
                                            SegState& st, int lane, v2d& head) {
    double* ring = w.ring + SLOT * kW;
    const bool needL = (method == STS_FILL_LINEAR || method == STS_FILL_PREVIOUS || method == STS_FILL_NEAREST);
    const bool needN = (method == STS_FILL_LINEAR || method == STS_FILL_NEXT || method == STS_FILL_NEAREST);
    const int tend = (kb + kW < T) ? kb + kW : T;     // end of the real steps of this tile
    if (method != STS_FILL_NONE) {
#if STS_SEG_VTAB
        // ---- word tables, lane-parallel: lane i < kWords owns word i (DPP scans within row 0,
        //      v_readlane for the few values every lane needs) ----
        const int wl = lane & (kWords - 1);
        const unsigned long long m = w.m2[SLOT][wl];
        const bool own_w = lane < kWords;
        const int gbase = kb + 64 * wl;
        const int hiw = tend - gbase;                       // real steps of word wl: bits [0, hiw)
        unsigned long long r = 0ull;
        if (own_w && hiw > 0) {
            r = ~m;
            if (hiw < 64) r &= (1ull << hiw) - 1ull;
        }
        const int cnt = __popcll(r);
        int incl = cnt;                                     // inclusive prefix count over words
        incl += __builtin_amdgcn_update_dpp(0, incl, 0x111, 0xf, 0xf, false);
        incl += __builtin_amdgcn_update_dpp(0, incl, 0x112, 0xf, 0xf, false);
        incl += __builtin_amdgcn_update_dpp(0, incl, 0x114, 0xf, 0xf, false);
        const int excl = incl - cnt;
        int lvw = (own_w && m) ? gbase + 63 - __clzll(m) : -1;   // last valid index in words <= wl
        lvw = max(lvw, __builtin_amdgcn_update_dpp(-1, lvw, 0x111, 0xf, 0xf, false));
        lvw = max(lvw, __builtin_amdgcn_update_dpp(-1, lvw, 0x112, 0xf, 0xf, false));
        lvw = max(lvw, __builtin_amdgcn_update_dpp(-1, lvw, 0x114, 0xf, 0xf, false));
        const int runw = max(lvw, st.Lc);
        int lnw = r ? gbase + 63 - __clzll(r) : -1;         // last NaN to impute in words <= wl
        lnw = max(lnw, __builtin_amdgcn_update_dpp(-1, lnw, 0x111, 0xf, 0xf, false));
        lnw = max(lnw, __builtin_amdgcn_update_dpp(-1, lnw, 0x112, 0xf, 0xf, false));
        lnw = max(lnw, __builtin_amdgcn_update_dpp(-1, lnw, 0x114, 0xf, 0xf, false));
        bool lg = false;   // linear: can a step lie more than kLongRun past its last valid index?
        if (method == STS_FILL_LINEAR) {   // (conservative, as in sts_tile.hip)
            const int tz = m ? __ffsll(m) - 1 : 64;
            lg = __ballot(own_w && (__popcll(~m) > kLongRun / 2 ||
                                    (lane == 0 && tz > 0 && kb + tz - 1 - st.Lc > kLongRun))) != 0ull;
        }
        if (own_w) {
            w.need[lane] = r;
            w.lastUp[lane] = runw;
            w.wbase[lane] = excl;
        }
        int wb[kWords + 1];
#pragma unroll
        for (int i = 0; i < kWords; i++) wb[i] = __builtin_amdgcn_readlane(excl, i);
        wb[kWords] = __builtin_amdgcn_readlane(incl, kWords - 1);
        const int run = __builtin_amdgcn_readlane(runw, kWords - 1);
        const int lastneed = __builtin_amdgcn_readlane(lnw, kWords - 1);
#else
        // ---- word tables (wave-uniform scalars, short-lived) ----
        int wb[kWords + 1];
        int run = st.Lc, lastneed = -1;
        bool lg = false;   // linear: can a step lie more than kLongRun past its last valid index?
        wb[0] = 0;
#pragma unroll
        for (int i = 0; i < kWords; i++) {
            const unsigned long long m = uni64(w.m2[SLOT][i]);
            if (method == STS_FILL_LINEAR) {   // (conservative, as in sts_tile.hip: a long run
                // puts > kLongRun / 2 NaNs into one word, or reaches into the tile's first word
                // from more than kLongRun before it)
                const int tz = m ? __ffsll(m) - 1 : 64;
                lg = lg || __popcll(~m) > kLongRun / 2 || (i == 0 && tz > 0 && kb + tz - 1 - run > kLongRun);
            }
            if (m) run = kb + 64 * i + 63 - __clzll(m);
            const int hi = tend - (kb + 64 * i);               // real steps of word i: bits [0, hi)
            unsigned long long r = 0ull;
            if (hi > 0) {
                r = ~m;
                if (hi < 64) r &= (1ull << hi) - 1ull;
            }
            if (r) lastneed = kb + 64 * i + 63 - __clzll(r);
            wb[i + 1] = wb[i] + __popcll(r);
            if (lane == 0) {
                w.need[i] = r;
                w.lastUp[i] = run;
                w.wbase[i] = wb[i];
            }
        }
#endif
        const int lastv = (run >= kb) ? run : -1;     // last valid index in this tile
        const int nnan = wb[kWords];
        if (nnan > 0) {
            // look-ahead: only when a NaN lies after the tile's last valid index
            int f = T;
            double fv = 0.0;
            if (needN) {
                f = look;
                fv = lookv;
                if (look == kBig) {
                    if (lastneed > lastv) {   // a long gap is scanned once, not once per tile
                        const int cp = w.cN_pos, cn = w.cN;
                        f = (cp >= 0 && cp <= scan_from && cn >= scan_from) ? cn : (int)scan_fwd(src, scan_from, T, lane);
                        if (lane == 0) {
                            w.cN_pos = scan_from;
                            w.cN = f;
                        }
                        fv = (f < T) ? src[f] : 0.0;
                    } else {
                        f = T;
                    }
                }
#if STS_SEG_VTAB
                int fw = (own_w && m) ? gbase + __ffsll(m) - 1 : kBig;   // first valid in words >= wl
                fw = min(fw, __builtin_amdgcn_update_dpp(kBig, fw, 0x101, 0xf, 0xf, false));
                fw = min(fw, __builtin_amdgcn_update_dpp(kBig, fw, 0x102, 0xf, 0xf, false));
                fw = min(fw, __builtin_amdgcn_update_dpp(kBig, fw, 0x104, 0xf, 0xf, false));
                if (own_w) w.firstFrom[lane] = min(fw, f);
#else
                int ff = f;
#pragma unroll
                for (int i = kWords - 1; i >= 0; i--) {
                    const unsigned long long m = uni64(w.m2[SLOT][i]);
                    if (m) ff = kb + 64 * i + __ffsll(m) - 1;
                    if (lane == 0) w.firstFrom[i] = ff;
                }
#endif
            }
            wave_sync();
            // ---- impute the compacted NaN positions; F goes into the ring in place
            //      (every (L, N) source is a valid position, never rewritten) ----
            const int Lc = st.Lc;
            const double Lcv = st.Lv;
            // two versions of the loop: only a flagged tile carries the long-run chain code
            auto impute = [&](auto long_tag) {
            constexpr bool LONG = decltype(long_tag)::value;
            for (int idx = lane; idx < nnan; idx += 64) {
                int wd = 0;
#pragma unroll
                for (int i = 1; i < kWords; i++) wd += (idx >= wb[i]) ? 1 : 0;
                unsigned long long nm = w.need[wd];
                int kk = idx - w.wbase[wd], bit = 0;
#pragma unroll
                for (int width = 32; width >= 1; width >>= 1) {
                    const int c = __popcll(nm & ((1ull << width) - 1ull));
                    if (kk >= c) { kk -= c; nm >>= width; bit += width; }
                }
                const int q = wd * 64 + bit;
                const int t = kb + q;
                const unsigned long long m = w.m2[SLOT][wd];
                int Lt = -1, Nt = T;
                double Lv = 0.0, Nv = 0.0;
                if (needL) {
                    const unsigned long long lo = m & ((1ull << bit) - 1ull);
                    Lt = lo ? kb + wd * 64 + 63 - __clzll(lo) : (wd > 0 ? w.lastUp[wd - 1] : Lc);
                    Lv = (Lt >= kb) ? ring[Lt - kb] : Lcv;
                }
                if (needN) {
                    const unsigned long long hi = (bit == 63) ? 0ull : (m & (~0ull << (bit + 1)));
                    Nt = hi ? kb + wd * 64 + __ffsll(hi) - 1 : (wd + 1 < kWords ? w.firstFrom[wd + 1] : f);
                    Nv = (Nt < kb + kW) ? ring[Nt - kb] : fv;
                }
                double r = __builtin_nan("");
                switch (method) {
                case STS_FILL_PREVIOUS:
                    if (Lt >= 0) r = Lv;
                    break;
                case STS_FILL_NEXT:
                    if (Nt < T) r = Nv;
                    break;
                case STS_FILL_NEAREST: {
                    if (t == 0) break;                        // index 0 is never modified
                    const int P = (Lt >= 1) ? Lt : -1;        // index 0 is never a previous source
                    if (P < 0 && Nt >= T) { st.err = true; break; }
                    r = (Nt >= T || (P >= 0 && t - P < Nt - t)) ? Lv : Nv;   // ties go to next
                    break;
                }
                case STS_FILL_LINEAR: {
                    if (Lt < 0 || Nt >= T) break;             // runs touching index 0 or n-1 stay NaN
                    if (LONG && t - Lt > kLongRun) {
                        // a step more than kLongRun past L: the lane holding the run's first
                        // such step in this tile walks the chain through all of them (O(run)),
                        // from the previous tile's carried value when the run continues from
                        // it, else replaying from L; the other lanes skip theirs
                        if (t - Lt == kLongRun + 1 || q == 0) {
                            const double inc = (Nv - Lv) / (double)(Nt - Lt);
                            const int rd = ((kb / kW) + 1) & 1, wr = (kb / kW) & 1;
                            double v;
                            if (w.carry_L[rd] == Lt && w.carry_t[rd] == t - 1) {
                                v = w.carry_r[rd];
                            } else {
                                v = Lv;
                                int j = t - 1 - Lt;   // replay from L, 8 dependent adds per trip
                                for (; j >= 8; j -= 8) {
                                    v = v + inc; v = v + inc; v = v + inc; v = v + inc;
                                    v = v + inc; v = v + inc; v = v + inc; v = v + inc;
                                }
                                for (; j > 0; j--) v = v + inc;
                            }
                            for (int qq = q; kb + qq < tend && kb + qq < Nt; qq++) {
                                v = v + inc;
                                ring[qq] = v;
                                if (qq == kW - 1) {
                                    w.carry_L[wr] = Lt;
                                    w.carry_t[wr] = kb + kW - 1;
                                    w.carry_r[wr] = v;
                                }
                            }
                        }
                        continue;
                    }
                    const double inc = (Nv - Lv) / (double)(Nt - Lt);
                    double acc = Lv;
                    for (int j = t - Lt; j > 0; j--) acc = acc + inc;   // sequential, as :259-261
                    r = acc;
                    break;
                }
                default:
                    break;
                }
                ring[q] = r;
            }
            };
            if (lg) impute(std::true_type{});
            else impute(std::false_type{});
        }
        wave_sync();
        if (lastv >= 0) {
            st.Lc = lastv;
            st.Lv = ring[lastv - kb];
        }
    } else {
        wave_sync();
    }

    // ---- filled output (16-B stores), then y = F - c0 (0 past the series end); a tile of
    //      this segment (own) adds its middle positions to the lane's sums ----
    v2d* r2 = reinterpret_cast<v2d*>(ring) + lane;
    const bool full = (kb + kW <= T);
#pragma unroll
    for (int u = 0; u < 4; u++) {
        const v2d f = r2[64 * u];
        const int t = kb + 128 * u + 2 * lane;
        if (store) {
            if (full) {
                __builtin_nontemporal_store(f, reinterpret_cast<v2d*>(dst + t));   // nt: C1 step 0.148 -> 0.140 ms
            } else {
                if (t < T) dst[t] = f.x;
                if (t + 1 < T) dst[t + 1] = f.y;
            }
        }
        if constexpr (NT > 0) {
            v2d y;
            y.x = (full || t < T) ? f.x - st.c0 : 0.0;
            y.y = (full || t + 1 < T) ? f.y - st.c0 : 0.0;
            r2[64 * u] = y;
            if (own) {   // sum y / sum y^2 over the series' middle (sts_acf.hpp rule 2)
                const bool mid_tile = kb >= kAcfEdge && kb + kW + kAcfEdge <= T;   // wave-uniform
                const double zx = (mid_tile || acf_mid(t, T)) ? y.x : 0.0;
                const double zy = (mid_tile || acf_mid(t + 1, T)) ? y.y : 0.0;
                st.sm += zx;
                st.sm += zy;
                st.qm = __builtin_fma(zx, zx, st.qm);
                st.qm = __builtin_fma(zy, zy, st.qm);
            }
            if (SLOT == 0 && u == 0) reinterpret_cast<v2d*>(w.ring + 2 * kW)[lane] = y;
            if (u == 0 && kb == 0) head = y;          // y(2 lane), y(2 lane + 1): fused ACF finalize
        }
    }
    wave_sync();
}

template <int SLOT>
__device__ __forceinline__ void zero_slot(WaveLds& w, int lane) {
    v2d* r2 = reinterpret_cast<v2d*>(w.ring + SLOT * kW) + lane;
    const v2d z = {0.0, 0.0};
#pragma unroll
    for (int u = 0; u < 4; u++) r2[64 * u] = z;
    if (SLOT == 0) reinterpret_cast<v2d*>(w.ring + 2 * kW)[lane] = z;
    wave_sync();
}

__device__ __forceinline__ void raw_to_slot(double* slot, const v2d (&R)[4], int lane) {
    v2d* r2 = reinterpret_cast<v2d*>(slot) + lane;
#pragma unroll
    for (int u = 0; u < 4; u++) r2[64 * u] = R[u];
}

struct SegCtx {
    const double* src;
    double* dst;
    int T, ntiles, k0, k1, kLast, kEnd, method;
};

// MFMA work of one step on the previous tile: none, the pre-chunk of a series (chunk 7
// of the all-zero "tile -1"), or the whole tile.
enum { kMmNone = 0, kMmPre = 1, kMmFull = 2 };

// Iteration k (ring slot SLOT holds tile k raw, its masks in w.m2[SLOT]):
// Rn = tile k + 1 (in flight), Rnn = free (receives tile k + 2).
template <int NT, int SLOT, int MM>
__device__ __forceinline__ void seg_step(WaveLds& w, const SegCtx& cx, int k, v2d (&Rnn)[4], v2d (&Rn)[4],
                                         SegState& st, d4 (&U)[Mfma<NT>::NA], int lane, int offb, v2d& head) {
    if (k + 2 <= cx.kLast) load_tile(Rnn, cx.src, (k + 2) * kW, cx.T, lane);
    const bool have_next = (k + 1 <= cx.kLast);
    int look = kBig, scan_from = (k + 1) * kW;
    double lookv = 0.0;
    if (have_next) {
        const int f = masks_to_lds(Rn, w.m2[SLOT ^ 1], lane);
        if (f >= 0) {
            look = (k + 1) * kW + f;
            lookv = pick_reg(Rn, f);
        } else {
            scan_from = (k + 2) * kW;
        }
    } else if ((k + 1) * kW >= cx.T) {
        look = cx.T;                                  // nothing after this tile
    }
    if (k < cx.ntiles) {
        impute_tile<NT, SLOT>(w, cx.src, cx.dst, k * kW, cx.T, cx.method, look, lookv, scan_from,
                              cx.dst != nullptr && k < cx.k1, k < cx.k1, st, lane, head);
    } else if constexpr (NT > 0) {
        zero_slot<SLOT>(w, lane);
    }
    if constexpr (NT > 0 && MM != kMmNone)
        Mfma<NT>::template tile<SLOT ^ 1>(w.ring, MM == kMmPre ? kWords - 1 : 0, U, lane, offb);
    if (have_next) {
        wave_sync();
        raw_to_slot(w.ring + (SLOT ^ 1) * kW, Rn, lane);
        wave_sync();
    }
}

template <int NT>
__global__ __launch_bounds__(256, 4) void seg_kernel(TileArgs a, int method) {
    __shared__ WaveLds lds[kWaves];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // wave-uniform: scalar state
    const int64_t unit = (int64_t)blockIdx.x * kWaves + wave;
    if (unit >= a.S * a.chunks_per_series) return;
    WaveLds& w = lds[wave];
    const int64_t s = unit / a.chunks_per_series;
    const int g = (int)(unit - s * a.chunks_per_series);
    SegCtx cx;
    cx.src = a.in + s * a.ld_in;
    cx.dst = a.out ? a.out + s * a.ld_out : nullptr;
    cx.T = (int)a.T;
    cx.ntiles = (int)a.tiles_per_series;
    cx.k0 = g * (int)a.tiles_per_chunk;
    cx.k1 = (cx.k0 + (int)a.tiles_per_chunk < cx.ntiles) ? cx.k0 + (int)a.tiles_per_chunk : cx.ntiles;
    cx.kLast = (cx.k1 < cx.ntiles - 1) ? cx.k1 : cx.ntiles - 1;
    cx.kEnd = (NT > 0) ? cx.k1 : cx.k1 - 1;
    cx.method = method;
    const bool needL = (method == STS_FILL_LINEAR || method == STS_FILL_PREVIOUS || method == STS_FILL_NEAREST);

    SegState st;
    st.err = false;
    st.c0 = 0.0;
    st.sm = 0.0;
    st.qm = 0.0;
    if (lane == 0) w.cN_pos = -1;
    if (lane < 2) {
        w.carry_L[lane] = -1;
        w.carry_t[lane] = -kBig;   // matches no tile start
    }
    st.Lc = -1;
    st.Lv = 0.0;
    if (needL && cx.k0 > 0) {
        st.Lc = (int)scan_back(cx.src, cx.k0 * kW, lane);
        st.Lv = (st.Lc >= 0) ? cx.src[st.Lc] : 0.0;
    }

    const int offb = Mfma<NT>::offB(lane);
    d4 U[Mfma<NT>::NA];
#pragma unroll
    for (int t = 0; t < Mfma<NT>::NA; t++) U[t] = d4{0.0, 0.0, 0.0, 0.0};

    v2d RA[4], RB[4];
    load_tile(RA, cx.src, cx.k0 * kW, cx.T, lane);
    if (cx.k0 + 1 <= cx.kLast) load_tile(RB, cx.src, (cx.k0 + 1) * kW, cx.T, lane);
    // ACF shift (sts_acf.hpp robust_shift): 64 samples spread over the whole series that
    // stand for the filled values; its probe loads are in flight with the first two tiles'
    if (NT > 0) st.c0 = robust_shift(cx.src, cx.T, lane, method == STS_FILL_PREVIOUS);
    masks_to_lds(RA, w.m2[0], lane);
    raw_to_slot(w.ring, RA, lane);
    if (NT > 0 && g == 0) zero_slot<1>(w, lane);     // "tile -1": y = 0 before the series
    wave_sync();

    // first step peeled: its MFMA work is the pre-chunk (segment 0) or nothing
    v2d head = {0.0, 0.0};
    if (NT > 0 && g == 0) seg_step<NT, 0, kMmPre>(w, cx, cx.k0, RA, RB, st, U, lane, offb, head);
    else seg_step<NT, 0, kMmNone>(w, cx, cx.k0, RA, RB, st, U, lane, offb, head);
    for (int k = cx.k0 + 1; k <= cx.kEnd; k += 2) {
        seg_step<NT, 1, kMmFull>(w, cx, k, RB, RA, st, U, lane, offb, head);
        if (k + 1 > cx.kEnd) break;
        seg_step<NT, 0, kMmFull>(w, cx, k + 1, RA, RB, st, U, lane, offb, head);
    }
    const int klast_slot = (cx.ntiles - 1 - cx.k0) & 1;   // ring slot of the series' last tile
    // st.err is per lane (the lane that imputed the failing NaN): one wave-wide answer
    const bool any_err = __ballot(st.err) != 0ull;
    if (a.err && lane == 0 && (any_err || a.err_all)) a.err[s] = any_err ? STS_ERR_ALL_NAN : STS_OK;

    if constexpr (NT > 0) {
        // fused finalize: the last tile's y survives in its ring slot; the extraction below
        // uses the first 256 doubles of the ring as scratch, so slot 0 is first copied up
        // into slot 1's place when it holds the last tile (slot 1 = the zeroed look-ahead)
        const int kb_last = (cx.ntiles - 1) * kW;
        const double* tail_base = w.ring + klast_slot * kW;
        if (a.acf_fused != nullptr && klast_slot == 0) {
            wave_sync();
            v2d* r2 = reinterpret_cast<v2d*>(w.ring) + lane;
#pragma unroll
            for (int u = 0; u < 4; u++) r2[256 + 64 * u] = r2[64 * u];
            tail_base = w.ring + kW;
        }
        // ---- diagonal extraction: lane d sums the entries (i, j) with h(j) - i = d ----
        constexpr int Q = Mfma<NT>::Q;
        d4 D = U[0];
#pragma unroll
        for (int t = 1; t < Mfma<NT>::NA; t++) D += U[t];
        wave_sync();
        double* scr = w.ring;
#pragma unroll
        for (int r = 0; r < 4; r++) scr[((lane >> 4) + 4 * r) * 16 + (lane & 15)] = D[r];
        wave_sync();
        double lagacc = 0.0;
#pragma unroll
        for (int j = 0; j < 16; j++) {
            const int i = 16 * (j / Q) + (16 - Q) + (j % Q) - lane;
            if (i >= 0 && i < 16) lagacc += scr[i * 16 + j];
        }
        const double sm = wave_sum_dpp(st.sm), qm = wave_sum_dpp(st.qm);
        if (a.acf_fused == nullptr) {
            double* part = a.partials + unit * kPartStride;
            part[lane] = lagacc;
            if (lane == 0) {
                part[kPartSum] = sm;
                part[kPartSq] = qm;
                part[kPartShift] = st.c0;
            }
        } else {
            // ---- one segment per series: acf_finalize_kernel's general path (T >= 2 kAcfEdge,
            //      T > 2K) right here, with the head y(0..63) from tile 0 (registers) and the
            //      tail y(T-64..T) from the last tile's ring slot (host guarantees it holds
            //      >= 64 steps).  Same operations in the same order -> the same bits. ----
            const int K = a.K, T = cx.T;
            const int i = lane + 1;
            const double Pi = 0.0 + __shfl(lagacc, (lane + 1) & 63), Sm = 0.0 + sm, Qm = 0.0 + qm;
            const double* tail = tail_base;   // y of the last tile, indexed by series position - kb_last
            bool sus;
            double r = acf_combine(
                Pi, Sm, Qm, i, T,
                [&](int j) {   // j is wave-uniform: a scalar lane select, not an LDS-crossbar shuffle
                    return readlane_d((j & 1) ? head.y : head.x, j >> 1);
                },
                [&](int j) { return tail[T - 1 - j - kb_last]; }, st.c0, &sus);
            // sts_acf.hpp rule 3: a suspect series takes the reference's loop over F, which this
            // wave wrote itself (one segment per series): order its stores before the reads
            if (__ballot(sus && lane < K)) {
                __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
                const double* F = cx.dst ? cx.dst : cx.src;
                // the ring is free now: F streams through it (sts_acf.hpp acf_exact_stream)
                static_assert(kRing >= 512 + 64, "the exact fallback's chunk buffer");
                const double e = acf_exact_stream<512>(F, T, i, lane < K && i < T, w.ring, lane);
                if (lane < K) r = e;
            }
            if (lane < K) a.acf_fused[s * K + lane] = r;
        }
    }
}

}  // namespace

int seg_nt(int K) { return K <= 0 ? 0 : (K <= 24 ? 2 : (K <= 60 ? 4 : -1)); }

hipError_t launch_segment(int method, const TileArgs& a, hipStream_t st) {
    const int64_t units = a.S * a.chunks_per_series;
    if (units <= 0) return hipSuccess;
    const int64_t nblk = (units + kWaves - 1) / kWaves;
    if (nblk > 0x7fffffffLL || a.T > 0x7fffffffLL - 2 * kW) return hipErrorInvalidValue;
    dim3 grid((unsigned)nblk), block(64 * kWaves);
    switch (seg_nt(a.K)) {
    case 0: hipLaunchKernelGGL((seg_kernel<0>), grid, block, 0, st, a, method); break;
    case 2: hipLaunchKernelGGL((seg_kernel<2>), grid, block, 0, st, a, method); break;
    case 4: hipLaunchKernelGGL((seg_kernel<4>), grid, block, 0, st, a, method); break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace sts
