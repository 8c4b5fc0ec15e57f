// sts_tile.hip -- the series-tile kernel: NaN imputation (fillts), optional fused
// multi-lag autocorrelation partial sums on FP64 MFMA, optional lag-matrix output.
//
// Reference operators (S/ = src/main/scala/com/cloudera/sparkts/):
//   fillPrevious   S/UnivariateTimeSeries.scala:194-204
//   fillNext       S/UnivariateTimeSeries.scala:214-224
//   fillNearest    S/UnivariateTimeSeries.scala:156-184
//   fillLinear     S/UnivariateTimeSeries.scala:247-266
//   autocorr       S/UnivariateTimeSeries.scala:68-93
//   lagMatTrimBoth S/Lag.scala:62-77
//
// One workgroup (4 waves) owns one TILE: TW consecutive steps [t0, t1) of one series,
// staged in LDS together with kHB steps before and kHA steps after it (extended range
// E).  Imputation is index driven: a 64-bit validity ballot per 64 steps plus a
// word-level max/min scan give, in O(1) per step, the last valid index L(t) <= t and
// the first valid index N(t) >= t.  From (L, N) every method is a copy except linear,
// whose reference loop accumulates r[j] = r[j-1] + inc SEQUENTIALLY from the run
// start: each NaN step replays that chain from L (t - L adds), which reproduces the
// reference bit for bit (no FMA: the library is built with -ffp-contract=off).  Steps more
// than kLongRun past L are instead produced by one lane walking the run's chain once,
// carrying its value across the workgroup's tiles), so a gap of G steps costs O(G), not
// O(G^2).  Runs longer than the halos find L / N with a 512-step-wide scan of global
// memory whose answer is cached for the workgroup's next tiles.
//
// Autocorrelation: with y = F - c (c = the robust shift of sts_acf.hpp: the median of 64
// samples of the series; exact algebra for a correlation), the kernel accumulates per
// chunk P_i = sum_j y_j * y_{j+i} (i = 0..63) with y = 0 past the series end, and sum y /
// sum y^2 over the series' middle [64, T - 64) in the store pass.  The lag products are
// FP64 MFMA rank-4 updates: viewing the series as rows of 16, U_t = sum_a A_a^T A_{a+t}
// (A_a = 16 consecutive steps) holds every pair at lag 16t + c - b; lane l of a wave
// feeds element j0 + l as the A operand and j0 + 16t + l as the B operand of
// v_mfma_f64_16x16x4_f64, so both operands are contiguous LDS reads.  A finalize
// kernel (sts_acf_finalize) combines the tiles in a fixed order (deterministic).
#include "sts_internal.hpp"
#include "sts_lanes.hpp"
#include "sts_acf.hpp"
#include "sts_scan.hpp"

#include <hip/hip_runtime.h>

#include <type_traits>

// Measured-negative variants of this kernel (rounds 1-3: double-buffered tiles with the lag
// products interleaved into the next tile, LDS-DMA tile prefetch, early / split prefetch issue,
// middle sums in the y pass, the no-MFMA / no-operand diagnostics and the I8 Ozaki cost models)
// are not in this source: their records are in DESIGN.md §5.2 / profiles/INDEX.md and their code
// at commit bd59bf8 (tools/var_rev.sh builds a library from any revision for same-box A/B).

#ifndef STS_FILL_PRIO
#define STS_FILL_PRIO 2   // wave priority outside the MFMA phase (s_setprio; same-box A/B on C3, profiles/r04_v8_ab_c3_prio.jsonl:
                          // 41.36-41.55 ms against 41.98-42.12 without priorities, 41.60-41.63 when raised from the second tile on)
#endif
#ifndef STS_TILE_WGS
#define STS_TILE_WGS 4    // workgroups per CU the register budget is sized for (128 VGPRs; LDS 40.5 KB x 4 fits)
#endif


namespace sts {
namespace {

// Workgroup barrier ordering LDS only.  The tile kernel never reads global data another
// thread of the kernel wrote, so global loads (the register prefetch) and stores need no
// ordering here -- and a fence on all address spaces would pin them in program order.
__device__ __forceinline__ void lds_barrier() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

typedef double d4 __attribute__((ext_vector_type(4)));
typedef double d2v __attribute__((ext_vector_type(2)));   // 16-B lag-matrix stores

constexpr int kThreads = 256;
constexpr int kBig = 1 << 30;

__device__ __forceinline__ bool isnan_d(double v) { return __builtin_isnan(v); }

// Diagnostic build only (-DSTS_STAMPS, `make stamps`): per-phase s_memtime accumulation,
// summed over waves into a device array read back by sts_debug_stamps().  The shipped
// library has no stamps.
#ifdef STS_STAMPS
__device__ unsigned long long g_stamps[16];
#define STAMP(i)                                                                            \
    do {                                                                                    \
        const unsigned long long now_ = __builtin_amdgcn_s_memtime();                      \
        st_acc[i] += now_ - st_prev;                                                        \
        st_prev = now_;                                                                     \
    } while (0)
#else
#define STAMP(i) \
    do {         \
    } while (0)
#endif

// Interleave two 32-step validity ballots into one 64-step word: bit i of ev -> bit 2i,
// bit i of od -> bit 2i + 1.  s_bitreplicate_b64_b32 doubles every bit (i -> 2i, 2i + 1)
// in one scalar op; the masks keep the even / odd copy.
__device__ __forceinline__ unsigned long long bitrep(unsigned x) {
    unsigned long long r;
    asm("s_bitreplicate_b64_b32 %0, %1" : "=s"(r) : "s"(x));
    return r;
}
__device__ __forceinline__ unsigned long long interleave2(unsigned ev, unsigned od) {
    return (bitrep(ev) & 0x5555555555555555ull) | (bitrep(od) & 0xAAAAAAAAAAAAAAAAull);
}

// An opaque copy of a per-lane value: computed where it is used, per tile, instead of being
// hoisted out of the tile loop by LICM and kept live in a VGPR for the whole kernel (round 3:
// ~50 VGPRs of hoisted per-lane LDS addresses that are one base plus immediate offsets)
__device__ __forceinline__ int opq(int x) {
    asm volatile("" : "+v"(x));
    return x;
}

// v_writelane with a constant lane: lane L of v takes the wave-uniform x (no exec change)
template <int L>
__device__ __forceinline__ void wlane(int& v, unsigned x) {
    asm("v_writelane_b32 %0, %1, %2" : "+v"(v) : "s"(x), "n"(L));
}

// Wave-wide scans of one int per lane for wave 0's word scan: DPP within rows of 16 lanes
// (row_shr / row_shl 1, 2, 4, 8; lanes without a source keep the identity) and readlane
// carries across the four rows -- VALU-latency steps instead of one ds_bpermute round trip
// per step.  dpp controls: row_shl:n = 0x100 + n, row_shr:n = 0x110 + n, wave_shl:1 = 0x130,
// wave_shr:1 = 0x138.
template <int CTRL>
__device__ __forceinline__ int dpp(int old, int v) {
    return __builtin_amdgcn_update_dpp(old, v, CTRL, 0xf, 0xf, false);
}
__device__ __forceinline__ int rl(int v, int l) { return __builtin_amdgcn_readlane(v, l); }
__device__ __forceinline__ int imax(int a, int b) { return a > b ? a : b; }
__device__ __forceinline__ int imin(int a, int b) { return a < b ? a : b; }
// inclusive prefix max over lanes 0..lane
__device__ __forceinline__ int wave_prefix_max(int v, int lane) {
    constexpr int I = -0x7fffffff - 1;
    v = imax(v, dpp<0x111>(I, v));
    v = imax(v, dpp<0x112>(I, v));
    v = imax(v, dpp<0x114>(I, v));
    v = imax(v, dpp<0x118>(I, v));
    const int p1 = rl(v, 15), p2 = imax(p1, rl(v, 31)), p3 = imax(p2, rl(v, 47));
    const int r = opq(lane) >> 4;   // opaque: the row masks are recomputed per use, not hoisted into spilled SGPRs
    return imax(v, r == 0 ? I : r == 1 ? p1 : r == 2 ? p2 : p3);
}
// inclusive prefix sum over lanes 0..lane
__device__ __forceinline__ int wave_prefix_sum(int v, int lane) {
    v += dpp<0x111>(0, v);
    v += dpp<0x112>(0, v);
    v += dpp<0x114>(0, v);
    v += dpp<0x118>(0, v);
    const int p1 = rl(v, 15), p2 = p1 + rl(v, 31), p3 = p2 + rl(v, 47);
    const int r = opq(lane) >> 4;   // opaque: the row masks are recomputed per use, not hoisted into spilled SGPRs
    return v + (r == 0 ? 0 : r == 1 ? p1 : r == 2 ? p2 : p3);
}
// inclusive suffix min over lanes lane..63
__device__ __forceinline__ int wave_suffix_min(int v, int lane) {
    constexpr int I = 0x7fffffff;
    v = imin(v, dpp<0x101>(I, v));
    v = imin(v, dpp<0x102>(I, v));
    v = imin(v, dpp<0x104>(I, v));
    v = imin(v, dpp<0x108>(I, v));
    const int s3 = rl(v, 48), s2 = imin(s3, rl(v, 32)), s1 = imin(s2, rl(v, 16));
    const int r = opq(lane) >> 4;   // opaque: the row masks are recomputed per use, not hoisted into spilled SGPRs
    return imin(v, r == 0 ? s1 : r == 1 ? s2 : r == 2 ? s3 : I);
}

// Padded LDS index of extended-tile position q: 4 doubles of padding per 32.  Keeps the
// lag-product B-operand gathers (16-step-spaced groups, see below) conflict-free across the
// 64 LDS banks; 16-B pairs (even q) never straddle a pad.
template <bool PAD>
__device__ __forceinline__ int px_(int q) { return PAD ? q + ((q >> 5) << 2) : q; }
template <bool PAD>
__device__ __forceinline__ int px2_(int q2) { return PAD ? q2 + ((q2 >> 4) << 1) : q2; }   // double2 index

// Lag-product decompositions (see the header): SHIFTED (K <= 60) uses NT = 2 or 4 MFMAs
// per 64 steps with window shifts q*t (q = 16 / NT) and B columns h(j) = 16(j/q) + 16 - q
// + j%q -- every lag 0 .. 16 NT - q exactly once per step, and the same lag map h(j) - i in
// every accumulator; TOEPLITZ (K = 61..63) uses NT = floor((K + 15) / 16) + 1 MFMAs with
// U_t holding lag 16t + j - i.
// M: the fill method (STS_FILL_*), a template parameter (round 4: as a kernel argument its tests
// were hoisted out of the tile loop as masks and spilled; compile-time, every method-dependent
// branch folds away)
template <int TW, int NT, bool SHIFTED, int NTH, int M>
__global__ __launch_bounds__(NTH, STS_TILE_WGS) void tile_kernel(TileArgs a) {
    constexpr int method = M;
    if constexpr (NT > 0) __builtin_amdgcn_s_setprio(STS_FILL_PRIO);   // see the MFMA phase below
    constexpr int kThreads = NTH;          // 256 (4 waves) or 128 (2 waves, TW = 2048)
    constexpr int kWaves = NTH / 64;
    static_assert(TW / 64 % kWaves == 0, "whole 64-step chunks per wave");
    constexpr int EW = kHB + TW + kHA;
    constexpr int NA = SHIFTED ? 2 : (NT > 0 ? NT : 1);      // MFMA accumulators
    constexpr int QS = (SHIFTED && NT > 0) ? 16 / NT : 16;   // window shift step (shifted scheme)
    // y is needed this far past the written range (A windows reach 4t <= 12 past the
    // tile, and the used lags <= 60 past that; the Toeplitz scheme reaches 16 NT)
    constexpr int REACH = (NT == 0) ? 0 : (SHIFTED ? 80 : 16 * NT);
    constexpr bool PAD = SHIFTED && NT > 0;                  // padded LDS layout (B gathers)
    constexpr int EWP = PAD ? EW + EW / 8 : EW;
    auto px = [](int q) { return px_<PAD>(q); };
    auto px2 = [](int q2) { return px2_<PAD>(q2); };
    // px2(q2 + kThreads) - px2(q2) (kThreads is a multiple of 16) and px(q + 64) - px(q)
    constexpr int PX2S = PAD ? kThreads + 2 * (kThreads / 16) : kThreads;
    constexpr int PXW = PAD ? 72 : 64;
    static_assert(kThreads % 16 == 0, "linear padded strides");
    constexpr int NW = EW / 64;
    constexpr int NP2 = EW / 2;                              // double2 per extended tile
    constexpr int RPT = (NP2 + kThreads - 1) / kThreads;     // prefetch registers per thread
    static_assert(EW % 64 == 0, "extended tile must be whole words");
    static_assert(NW <= 128, "word scan handles at most 128 words");
    // padded (px) for the shifted scheme
    __shared__ __attribute__((aligned(16))) double vals[EWP];
    __shared__ unsigned long long mask[NW];
    __shared__ int lastUpTo[NW];           // last valid E-position in words <= w (-1: none)
    __shared__ int firstFrom[NW];          // first valid E-position in words >= w (kBig: none)
    __shared__ int wbase[NW + 1];          // NaN-list offset of each word (exclusive prefix count)
    __shared__ unsigned long long wneed[NW];   // NaN positions to impute, per word
    __shared__ int sh_i[4];                // lext, next (series positions), NaN count, long-run flag
    __shared__ double sh_d[3];             // (unused), value at lext, value at next
    // linear fill, long runs: the chain value at the last step of the previous tile
    // (double-buffered by tile parity: read [(k + 1) & 1], write [k & 1])
    __shared__ int carry_L[2], carry_t[2];
    __shared__ double carry_r[2];
    // wave 0's caches of the global scans (series positions; LDS, not registers: nothing is
    // live across tiles for them): the last valid index before sh_c[0] is sh_c[1]; the first
    // valid index at or after sh_c[2] is sh_c[3]
    __shared__ int sh_c[4];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave-uniform: scalar loop control
    // one workgroup = one CHUNK of tiles_per_chunk consecutive tiles of one series
    const int64_t nchunk = a.S * a.chunks_per_series;
    const int64_t ch = xcd_remap(blockIdx.x, nchunk);
    const int64_t s = ch / a.chunks_per_series;
    const int64_t cidx = ch - s * a.chunks_per_series;
    const int64_t k_begin = cidx * a.tiles_per_chunk;
    const int64_t k_end = (k_begin + a.tiles_per_chunk < a.tiles_per_series) ? k_begin + a.tiles_per_chunk
                                                                              : a.tiles_per_series;
    const int64_t T = a.T;
    const double* src = a.in + s * a.ld_in;
    const bool src_al = (reinterpret_cast<uintptr_t>(src) & 15) == 0;
    constexpr bool needL = (method == STS_FILL_LINEAR || method == STS_FILL_PREVIOUS || method == STS_FILL_NEAREST);
    constexpr bool needN = (method == STS_FILL_LINEAR || method == STS_FILL_NEXT || method == STS_FILL_NEAREST);
    double* dst = a.out ? a.out + s * a.ld_out : nullptr;
    const int64_t lrows = T - a.max_lag;
    const int ncols = a.max_lag + (a.include_original ? 1 : 0);
    const int init = a.include_original ? 0 : 1;

    if (tid < 2) {
        carry_L[tid] = -1;
        carry_t[tid] = -kBig;   // matches no tile start
    }
    if (tid == 0) {
        sh_c[0] = -kBig;
        sh_c[2] = -1;
    }
    double acc_s = 0.0, acc_q = 0.0;   // sum y, sum y^2 over this thread's middle positions

    // register prefetch of one INTERIOR extended tile [e0, e0 + EW); the first and last tile
    // of a series (which touch its ends) are loaded synchronously with bounds checks
    static_assert(RPT <= 9, "prefetch registers are spelled out for RPT <= 9");
    double2 R0, R1, R2, R3, R4, R5, R6, R7, R8;   // named: an array here ends up in scratch
    auto interior = [&](int64_t kk) {
        const int64_t e0 = kk * TW - kHB;
        return e0 >= 0 && e0 + EW <= T && src_al;
    };
    // (a macro, not a lambda: a captured register array would be forced to scratch)
// non-temporal loads on the fused-ACF instantiations (same-box A/B on the C3 shard, five rounds:
// 40.83-41.26 against 41.10-41.55 ms, profiles/r05_s19_ab_c3_c5_ntload.jsonl); the fill-only ones
// (C5) keep plain loads (1.850-1.856 against 1.820-1.826 ms)
#define STS_LD1(j)                                                                          \
    if constexpr (j < RPT) {                                                                \
        const int q2_ = tid + j * kThreads;                                                 \
        const double2* p_ = &s2_[q2_ < NP2 ? q2_ : NP2 - 1];                                \
        if constexpr (NT > 0) {                                                             \
            const d2v v_ = __builtin_nontemporal_load(reinterpret_cast<const d2v*>(p_));    \
            R##j = make_double2(v_.x, v_.y);                                                \
        } else {                                                                            \
            R##j = *p_;                                                                     \
        }                                                                                   \
    }
#define STS_ISSUE(kk)                                                                       \
    do {                                                                                    \
        const double2* s2_ = reinterpret_cast<const double2*>(src + ((kk) * TW - kHB));     \
        STS_LD1(0) STS_LD1(1) STS_LD1(2) STS_LD1(3) STS_LD1(4)                              \
        STS_LD1(5) STS_LD1(6) STS_LD1(7) STS_LD1(8)                                         \
    } while (0)
// define R on the no-prefetch path too, so the registers are dead between their store to
// LDS and the next issue (otherwise the loop-carried values stay live across the body).  An
// empty asm that "writes" them defines them with no instruction (round 3: the zeroing moves
// it replaced were hoisted above the prefetch branch, 18 VALU per wave and tile); the values
// are never read (every read of R sits behind `have`).
#define STS_CLEAR()                                                                         \
    do {                                                                                    \
        asm volatile("" : "=v"(R0), "=v"(R1), "=v"(R2), "=v"(R3), "=v"(R4));               \
        asm volatile("" : "=v"(R5), "=v"(R6), "=v"(R7), "=v"(R8));                         \
    } while (0)
// (the bound test only where it can fail: a runtime test on every register kept a spilled
// exec mask per register alive across the tile loop)
#define STS_ST1(j)                                                                          \
    if constexpr (j < RPT) {                                                                \
        const int q2_ = tid + j * kThreads;                                                 \
        if ((j + 1) * kThreads <= NP2 || q2_ < NP2) v2_[pst_ + j * PX2S] = R##j;            \
    }

    d4 U[NA];
#pragma unroll
    for (int t = 0; t < NA; t++) U[t] = d4{0.0, 0.0, 0.0, 0.0};
    bool series_err = false;
#ifdef STS_STAMPS
    unsigned long long st_acc[12] = {0};
    unsigned long long st_prev = __builtin_amdgcn_s_memtime();
#endif
    bool have = interior(k_begin);
    if (have) STS_ISSUE(k_begin);
    else STS_CLEAR();
    // ACF shift (sts_acf.hpp: median of 64 raw samples of the series), computed once per
    // series by acf_shift_kernel before this launch: a scalar load
    // (made wave-uniform in SGPRs here: a VGPR load result used inside the tile loop gets a
    // vmcnt(0) at its use in every tile, which would also wait for the next tile's prefetch)
    const double c0 = [&] {
        if constexpr (NT == 0) return 0.0;
        const double v = a.shift[s];
        const unsigned long long u = __builtin_bit_cast(unsigned long long, v);
        const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)u);
        const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(u >> 32));
        return __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lo);
    }();

    // ---- lag products on MFMA (§ header) for chunks [FROM, TO) of this wave's CPW chunks of a
    //      tile whose y sits in buffer vb; chunk order (and so the accumulation order) is the
    //      same however the range is split into groups ----
    constexpr int qA0 = kHB;                // E-position of the tile's first step
    constexpr int NTA = NT > 0 ? NT : 1;    // array extent (NT = 0 instantiates no MFMA code)
    constexpr int CPW = TW / 64 / kWaves;   // 64-step chunks per wave
    auto mid_sums = [&](int p, double y) {
        // sum y / sum y^2 over the series' middle (sts_acf.hpp rule 2): lane l of the chunk
        // at series position p holds y(p + l)
        const double z = acf_mid(p + lane, T) ? y : 0.0;
        acc_s += z;
        acc_q = __builtin_fma(z, z, acc_q);
    };
    auto mfma_group = [&](auto FROM, auto TO, const double* vb, int64_t kk, int tt0, int tt1) {
        constexpr int F = decltype(FROM)::value, TE = decltype(TO)::value;
        if constexpr (NT > 0 && F < TE) {
            // a tile wholly inside the middle takes the unrolled loop with plain sums; the
            // series' first and last tiles take the per-chunk loop with the per-lane test
            const bool tile_mid = tt0 >= kAcfEdge && tt1 + kAcfEdge <= T;
            const int tlen = tt1 - tt0;
            const int nch = (tlen + 63) / 64;
            const bool full = wave * CPW + CPW <= nch;
            int c = wave * CPW + F;
            int cend = wave * CPW + TE;
            if (cend > nch) cend = nch;
            if constexpr (SHIFTED) {
                // A = y(chunk + QS t + lane), B = y(chunk + QS t + 16 (lane >> 4) + h(lane & 15));
                // per-lane operand offsets (padded) relative to a chunk start
                int oa[NTA], ob[NTA];
#pragma unroll
                for (int t = 0; t < NT; t++) {
                    const int j = lane & 15;
                    const int ra = QS * t + lane;
                    const int rb = QS * t + 16 * (lane >> 4) + 16 * (j / QS) + (16 - QS) + (j % QS);
                    oa[t] = opq(px(ra));
                    ob[t] = opq(px(rb));
                }
                auto chunk_mfma = [&](const double* yb) {
                    double av[NTA], bv[NTA];
#pragma unroll
                    for (int t = 0; t < NT; t++) {
                        av[t] = yb[oa[t]];
                        bv[t] = yb[ob[t]];
                    }
#pragma unroll
                    for (int t = 0; t < NT; t++)
                        U[t % NA] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[t], bv[t], U[t % NA], 0, 0, 0);
                    return av[0];   // y at chunk position lane
                };
                // wave 0 of the first tile also runs chunk -1 (the look-back, y = 0), whose
                // shifted windows hold the series' first QS t steps
                if (F == 0 && kk == 0 && wave == 0) chunk_mfma(vb);   // y = 0 there: no middle-sum term
                if (full && tile_mid) {
                    // full chunk range, unrolled: per-lane LDS indices made opaque once per
                    // group (else LICM hoists all of them out of the tile loop and spills),
                    // chunk offsets (72 doubles per padded chunk) fold into the ds_read
                    // immediates
                    int ia[NTA], ib[NTA];
                    const int cb = px(qA0 + 64 * (wave * CPW));
#pragma unroll
                    for (int t = 0; t < NT; t++) {
                        ia[t] = cb + oa[t];
                        ib[t] = cb + ob[t];
                        asm volatile("" : "+v"(ia[t]), "+v"(ib[t]));
                    }
#pragma unroll
                    for (int cc = F; cc < TE; cc++) {
                        double av[NTA], bv[NTA];
#pragma unroll
                        for (int t = 0; t < NT; t++) {
                            av[t] = vb[ia[t] + 72 * cc];
                            bv[t] = vb[ib[t] + 72 * cc];
                        }
#pragma unroll
                        for (int t = 0; t < NT; t++)
                            U[t % NA] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[t], bv[t], U[t % NA], 0, 0, 0);
                        acc_s += av[0];   // middle sums: VALU under the MFMA pipe
                        acc_q = __builtin_fma(av[0], av[0], acc_q);
                        __builtin_amdgcn_sched_barrier(0);   // one chunk's operands live at a time
                    }
                    c = cend;
                }
                for (; c < cend; c++) mid_sums(tt0 + 64 * c, chunk_mfma(vb + px(qA0 + 64 * c)));   // chunk start: a multiple of 32
            } else {
                // U_t += y(j0 + l) x y(j0 + 16t + l)
                for (; c < cend; c++) {
                    const int jrel = 64 * c + lane;
                    double bv[NTA];
#pragma unroll
                    for (int t = 0; t < NT; t++) bv[t] = vb[px(qA0 + jrel + 16 * t)];
                    const double av = (jrel < tlen) ? bv[0] : 0.0;   // A only inside the tile
#pragma unroll
                    for (int t = 0; t < NT; t++) U[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv[t], U[t], 0, 0, 0);
                    mid_sums(tt0 + 64 * c, av);
                }
            }
        }
    };
    for (int64_t k = k_begin; k < k_end; k++) {
        const int t0 = (int)(k * TW);
        const int t1 = (t0 + TW < T) ? t0 + TW : (int)T;
        const int e0 = t0 - kHB;

        // ---- 1. prefetched registers (or a bounds-checked edge load) -> LDS; for prefetched
        //      tiles the validity ballots come straight from the registers: register j of
        //      wave v holds steps 128v + 512j + 2*lane (+1), i.e. words 2v + 8j and 2v + 8j + 1
        //      as an even/odd bit interleave ----
        if (have) {
            double2* v2_ = reinterpret_cast<double2*>(vals);
            const int pst_ = opq(px2(tid));   // px2(tid + j kThreads) = px2(tid) + j PX2S
            STS_ST1(0) STS_ST1(1) STS_ST1(2) STS_ST1(3) STS_ST1(4) STS_ST1(5) STS_ST1(6) STS_ST1(7) STS_ST1(8)
// The two words of register j go into lanes 4j .. 4j + 3 of one VGPR (v_writelane, no
// branch), and one LDS store per wave writes them all (round 3: a lane-0 store per word
// behind per-word bound tests cost ~20 SALU and 4 spilled-mask reloads per register).
#define STS_BAL1(j)                                                                         \
    if constexpr (j < RPT) {                                                                \
        const unsigned long long bx_ = __ballot(!isnan_d(R##j.x));                          \
        const unsigned long long by_ = __ballot(!isnan_d(R##j.y));                          \
        const unsigned long long lo_ = interleave2((unsigned)bx_, (unsigned)by_);           \
        const unsigned long long hi_ = interleave2((unsigned)(bx_ >> 32), (unsigned)(by_ >> 32)); \
        wlane<4 * j + 0>(mv_, (unsigned)lo_);                                               \
        wlane<4 * j + 1>(mv_, (unsigned)(lo_ >> 32));                                       \
        wlane<4 * j + 2>(mv_, (unsigned)hi_);                                               \
        wlane<4 * j + 3>(mv_, (unsigned)(hi_ >> 32));                                       \
    }
            {
                int mv_ = 0;
                STS_BAL1(0) STS_BAL1(1) STS_BAL1(2) STS_BAL1(3) STS_BAL1(4) STS_BAL1(5) STS_BAL1(6)
                STS_BAL1(7) STS_BAL1(8)
                // lane i: dword (i & 1) of word 2 wave + 2 kWaves (i / 4) + ((i >> 1) & 1)
                const int w_ = 2 * wave + 2 * kWaves * (lane >> 2) + ((lane >> 1) & 1);
                if (lane < 4 * RPT && w_ < NW) reinterpret_cast<int*>(mask)[2 * w_ + (lane & 1)] = mv_;
            }
#undef STS_BAL1
        } else {
            for (int q = tid; q < EW; q += kThreads) {
                const int t = e0 + q;
                vals[px(q)] = (t >= 0 && t < T) ? src[t] : __builtin_nan("");
            }
        }
        const bool have_next = (k + 1 < k_end) && interior(k + 1);
        STAMP(0);
        lds_barrier();
        STAMP(1);

        // positions to produce: [qA, qB) (E-relative); the ACF needs REACH steps past the tile
        const int qA = kHB;
        const int qW = kHB + (t1 - t0);                  // end of the written range
        int qB = qW + REACH;
        if (e0 + qB > T) qB = (int)T - e0;

        // ---- 2. validity ballots from LDS for the edge tiles (wave v owns words v, v+4, ...) ----
        if (!have) {
            const int pb = opq(px(lane) + PXW * wave);   // px(64 w + lane) = px(lane) + PXW w
            // (not unrolled: unrolled, its per-trip tests w < NW were hoisted out of the tile loop
            // as 16 wave-uniform 64-bit masks, spilled, and cost the common path 42 SGPRs of spill
            // slots: 78 -> 36 spilled SGPRs, round 4)
#pragma unroll 1
            for (int i = 0; i < (NW + kWaves - 1) / kWaves; i++) {
                const int w = wave + i * kWaves;
                if (w < NW) {
                    const unsigned long long m = __ballot(!isnan_d(vals[pb + PXW * kWaves * i]));
                    if (lane == 0) mask[w] = m;
                }
            }
            STAMP(2);
            lds_barrier();
        }
        STAMP(3);

        // ---- 3. word scans (wave 0; lane l: words 2l, 2l+1): last valid position up to each
        //      word, first valid from each word, and the NaN-list offset of each word.  The
        //      workgroup's other waves wait at the barrier, so with the MFMA phase wave 0 runs at
        //      the top priority (same-box A/B on C3, profiles/r04_v8_ab_c3_prio.jsonl: 5 of 5
        //      rounds faster, 0.03-0.5 ms) ----
        if (wave == 0) {
            if constexpr (NT > 0) __builtin_amdgcn_s_setprio(3);
            // opaque: recomputed per tile (two VALU ops) instead of hoisted out of the tile loop,
            // where the derived LDS addresses were spilled to scratch and reloaded behind a
            // vmcnt(0) on wave 0's critical path
            int w0 = 2 * lane;
            asm volatile("" : "+v"(w0));
            const int w1 = w0 + 1;
            const unsigned long long m0 = (w0 < NW) ? mask[w0] : ~0ull;
            const unsigned long long m1 = (w1 < NW) ? mask[w1] : ~0ull;
            const int l0 = (w0 < NW && m0) ? w0 * 64 + 63 - __clzll(m0) : -1;
            const int l1 = (w1 < NW && m1) ? w1 * 64 + 63 - __clzll(m1) : -1;
            const int f0 = (w0 < NW && m0) ? w0 * 64 + __ffsll(m0) - 1 : kBig;
            const int f1 = (w1 < NW && m1) ? w1 * 64 + __ffsll(m1) - 1 : kBig;
            // NaN positions to impute: invalid AND inside [qA, qB)
            auto need = [&](int w, unsigned long long m) -> unsigned long long {
                const int lo = qA - w * 64, hi = qB - w * 64;      // bit range [lo, hi)
                if (method == STS_FILL_NONE || hi <= 0 || lo >= 64) return 0ull;
                unsigned long long r = ~m;
                if (lo > 0) r &= ~0ull << lo;
                if (hi < 64) r &= (1ull << hi) - 1ull;
                return r;
            };
            const unsigned long long n0 = (w0 < NW) ? need(w0, m0) : 0ull;
            const unsigned long long n1 = (w1 < NW) ? need(w1, m1) : 0ull;
            const int pm = wave_prefix_max(l1 > l0 ? l1 : l0, lane);           // inclusive prefix max
            const int sm = wave_suffix_min(f0 < f1 ? f0 : f1, lane);           // inclusive suffix min
            const int pc = wave_prefix_sum(__popcll(n0) + __popcll(n1), lane); // inclusive prefix count
            const int ex = dpp<0x138>(-1, pm);       // exclusive: lane - 1's value (wave_shr:1)
            const int exc = dpp<0x138>(0, pc);
            const int exs = dpp<0x130>(kBig, sm);    // lane + 1's value (wave_shl:1)
            const int nnan = rl(pc, 63);
            const int firstValidE = rl(sm, 0);
            const int lastValidE = rl(pm, 63);
            // linear fill: can a step of this tile lie more than kLongRun past its last valid
            // index?  Such a step ends a run of > kLongRun NaNs, which puts more than half of
            // that many NaNs into one word of the extended tile (a run reaching in from before
            // the tile fills the whole look-back word).  Conservative: a false alarm only
            // selects the loop that carries the long-run code, and the per-step replay is exact
            // for any run length.
            const bool lg = method == STS_FILL_LINEAR &&
                            __ballot((w0 < NW && __popcll(~m0) > kLongRun / 2) ||
                                     (w1 < NW && __popcll(~m1) > kLongRun / 2)) != 0ull;
            if (w0 < NW) {
                lastUpTo[w0] = ex > l0 ? ex : l0;
                const int a0 = f1 < exs ? f1 : exs;
                firstFrom[w0] = f0 < a0 ? f0 : a0;
                wbase[w0] = exc;
                wneed[w0] = n0;
            }
            if (w1 < NW) {
                const int a1 = ex > l0 ? ex : l0;
                lastUpTo[w1] = a1 > l1 ? a1 : l1;
                firstFrom[w1] = f1 < exs ? f1 : exs;
                wbase[w1] = exc + __popcll(n0);
                wneed[w1] = n1;
            }
            // slow paths: a NaN run longer than the halos (rare); the answers are cached for
            // the next tiles of this workgroup, so a long gap is scanned once per workgroup
            int lext = -1, next = (int)T;
            if (needL && e0 > 0 && firstValidE > qA && nnan > 0)
                lext = (sh_c[0] == e0) ? sh_c[1] : (int)scan_back(src, e0, lane);
            if (needN && e0 + EW < T && qB > qA && lastValidE < qB - 1 && nnan > 0) {
                const int from = e0 + EW;
                const int cN_pos = sh_c[2], cN = sh_c[3];
                next = (cN_pos >= 0 && cN_pos <= from && cN >= from) ? cN : (int)scan_fwd(src, from, T, lane);
                if (lane == 0) {
                    sh_c[2] = from;
                    sh_c[3] = next;
                }
            }
            // the last valid index before the next tile's e0 = e0 + TW: in this tile's words
            // [0, TW / 64) (lane TW / 128 - 1's inclusive prefix max), else lext
            if (needL) {
                const int lq = rl(pm, TW / 128 - 1);
                if (lane == 0) {
                    sh_c[0] = e0 + TW;
                    sh_c[1] = (lq >= 0) ? e0 + lq : lext;
                }
            }
            if (lane == 0) {
                wbase[NW] = nnan;
                sh_i[0] = lext;
                sh_i[1] = next;
                sh_i[2] = nnan;
                sh_i[3] = lg ? 1 : 0;
            }
            // the global loads stay inside their (rare, wave-uniform) branches together with
            // their use, so the vmcnt wait they need is not executed on the common path (it
            // would also wait for every prefetch load in flight)
            if (lext >= 0) {
                const double v = src[lext];
                if (lane == 0) sh_d[1] = v;
            }
            if (next < T) {
                const double v = src[next];
                if (lane == 0) sh_d[2] = v;
            }
        }
        if constexpr (NT > 0) __builtin_amdgcn_s_setprio(STS_FILL_PRIO);
        STAMP(4);
        lds_barrier();
        STAMP(5);

        // ---- 4. impute the compacted NaN positions, all lanes busy; F goes back into
        //      vals IN PLACE (every (L, N) source is a valid position, never rewritten) ----
        {
            const int nnan = sh_i[2];
            const int lext = sh_i[0], next = sh_i[1];
            const double lextv = sh_d[1], nextv = sh_d[2];
            // two versions of the loop: only a tile flagged by the word scan carries the
            // long-run chain code
            auto impute = [&](auto long_tag) {
            constexpr bool LONG = decltype(long_tag)::value;
            for (int idx = tid; idx < nnan; idx += kThreads) {
                // the word holding NaN #idx: last w with wbase[w] <= idx (binary search) ...
                int lo = 0, hi = NW;
                while (hi - lo > 1) {
                    const int mid = (lo + hi) >> 1;
                    if (wbase[mid] <= idx) lo = mid;
                    else hi = mid;
                }
                // ... and the position of its (idx - wbase[w])-th set need-bit (popcount bisection)
                unsigned long long nm = wneed[lo];
                int kk = idx - wbase[lo], bit = 0;
#pragma unroll
                for (int width = 32; width >= 1; width >>= 1) {
                    const int c = __popcll(nm & ((1ull << width) - 1ull));
                    if (kk >= c) { kk -= c; nm >>= width; bit += width; }
                }
                const int q = lo * 64 + bit;
                const int t = e0 + q;
                const int w = q >> 6, b = q & 63;
                const unsigned long long m = mask[w];
                int Lt = -1, Nt = (int)T;
                double Lv = 0.0, Nv = 0.0;
                if (needL) {
                    const unsigned long long lo = m & ((1ull << b) - 1ull);
                    const int Lq = lo ? w * 64 + 63 - __clzll(lo) : (w > 0 ? lastUpTo[w - 1] : -1);
                    if (Lq >= 0) { Lt = e0 + Lq; Lv = vals[px(Lq)]; }
                    else { Lt = lext; Lv = lextv; }
                }
                if (needN) {
                    const unsigned long long hi = (b == 63) ? 0ull : (m & (~0ull << (b + 1)));
                    const int Nq = hi ? w * 64 + __ffsll(hi) - 1 : (w + 1 < NW ? firstFrom[w + 1] : kBig);
                    if (Nq < kBig) { Nt = e0 + Nq; Nv = vals[px(Nq)]; }
                    else { Nt = next; Nv = nextv; }
                }
                double f = __builtin_nan("");
                switch (method) {
                case STS_FILL_PREVIOUS:
                    if (Lt >= 0) f = Lv;
                    break;
                case STS_FILL_NEXT:
                    if (Nt < T) f = Nv;
                    break;
                case STS_FILL_NEAREST: {
                    if (t == 0) break;                        // index 0 is never modified
                    const int P = (Lt >= 1) ? Lt : -1;        // index 0 is never a previous source
                    if (P < 0 && Nt >= T) { series_err = true; break; }
                    f = (Nt >= T || (P >= 0 && t - P < Nt - t)) ? Lv : Nv;   // ties go to next
                    break;
                }
                case STS_FILL_LINEAR: {
                    if (Lt < 0 || Nt >= T) break;             // runs touching index 0 or n-1 stay NaN
                    if (LONG && t - Lt > kLongRun) {
                        // a step more than kLongRun past L: the lane holding the run's first
                        // such step in this tile walks the chain r = r + inc through all of
                        // them (O(run), not O(run^2)), starting from the previous tile's
                        // carried value when the run continues from it, else replaying from L;
                        // the other lanes skip theirs
                        if (t - Lt == kLongRun + 1 || q == qA) {
                            const double inc = (Nv - Lv) / (double)(Nt - Lt);
                            const int rd = (int)((k + 1) & 1), wr = (int)(k & 1);
                            double v;
                            if (carry_L[rd] == Lt && carry_t[rd] == t - 1) {
                                v = carry_r[rd];
                            } else {
                                v = Lv;
                                int j = t - 1 - Lt;   // replay from L, 8 dependent adds per trip
                                for (; j >= 8; j -= 8) {
                                    v = v + inc; v = v + inc; v = v + inc; v = v + inc;
                                    v = v + inc; v = v + inc; v = v + inc; v = v + inc;
                                }
                                for (; j > 0; j--) v = v + inc;
                            }
                            const int qend = (Nt - e0 < qB) ? Nt - e0 : qB;
                            for (int qq = q; qq < qend; qq++) {
                                v = v + inc;
                                vals[px(qq)] = v;
                                if (e0 + qq == t1 - 1) {
                                    carry_L[wr] = Lt;
                                    carry_t[wr] = t1 - 1;
                                    carry_r[wr] = v;
                                }
                            }
                        }
                        continue;
                    }
                    const double inc = (Nv - Lv) / (double)(Nt - Lt);
                    double r = Lv;
                    for (int j = t - Lt; j > 0; j--) r = r + inc;   // sequential, as :259-261
                    f = r;
                    break;
                }
                default:
                    break;
                }
                vals[px(q)] = f;
            }
        };
            if (sh_i[3]) impute(std::true_type{});
            else impute(std::false_type{});
        }
        STAMP(6);
        lds_barrier();
        STAMP(7);

        // ---- 5. filled output + lag matrix (16-B stores), then y = F - F(0) in place
        //      (0 past the series end) for the MFMA phase; start the next tile's loads ----
        {
            const bool al = dst && ((reinterpret_cast<uintptr_t>(dst) & 15) == 0);
            double2* v2 = reinterpret_cast<double2*>(vals);
            const int qBfull = (NT > 0) ? ((SHIFTED || qW + 64 + 16 * NT >= EW) ? EW : qW + 64 + 16 * NT) : 0;
            // fast path: a full tile not at the series end -- the written range is exactly
            // [kHB, kHB + TW) and every y the MFMA phase reads is F - c0 (no zero tail), so
            // every index and guard below is a compile-time constant
            const bool fast = (dst == nullptr || al) && (t1 - t0 == TW) && (NT == 0 || e0 + qW + REACH <= T);
            if (fast) {
                constexpr int FS = TW / 2 / kThreads;                          // stored double2
                constexpr int FY = NT > 0 ? (NP2 - kHB / 2 + kThreads - 1) / kThreads : FS;
                constexpr int FH = (FY + 1) / 2;     // two halves: fewer live registers
                const int vq = (kHB >> 1) + tid;
                const int pvq = opq(px2(vq));   // px2(vq + jj kThreads) = pvq + jj PX2S
                const bool wr = dst != nullptr;   // wave-uniform (a null test of dp is per lane)
                // uniform tile base (SGPRs) + a 32-bit lane offset: the saddr store form, no
                // 64-bit per-lane pointer kept live across the tile loop
                char* const dpb = reinterpret_cast<char*>(dst + t0);
                unsigned dpo = (unsigned)tid * 16u;
                asm volatile("" : "+v"(dpo));   // per tile: else LICM keeps dst + dpo as a 64-bit VGPR pair
#pragma unroll
                for (int h = 0; h < 2; h++) {
                    double2 fv[FH];
#pragma unroll
                    for (int j = 0; j < FH; j++) {
                        const int jj = h * FH + j;
                        if (jj < FY && (jj * kThreads + kThreads <= NP2 - kHB / 2 ||
                                        tid + jj * kThreads < NP2 - kHB / 2))
                            fv[j] = v2[pvq + jj * PX2S];
                    }
#pragma unroll
                    for (int j = 0; j < FH; j++) {
                        const int jj = h * FH + j;
                        if (jj >= FY) continue;
                        const bool in = jj * kThreads + kThreads <= NP2 - kHB / 2 ||
                                        tid + jj * kThreads < NP2 - kHB / 2;
                        if (jj < FS && wr) {   // non-temporal: A/B on C3 +1 %
                            double2* dq = reinterpret_cast<double2*>(dpb + jj * kThreads * 16 + dpo);
                            __builtin_nontemporal_store(fv[j].x, &dq->x);
                            __builtin_nontemporal_store(fv[j].y, &dq->y);
                        }
                        if (NT > 0 && in) {
                            double2 y;
                            y.x = fv[j].x - c0;
                            y.y = fv[j].y - c0;
                            v2[pvq + jj * PX2S] = y;
                        }
                    }
                }
            } else
            for (int q2 = (qA >> 1) + tid; 2 * q2 < qW || 2 * q2 < qBfull; q2 += kThreads) {
                const int q = 2 * q2;
                double2 f = v2[px2(q2)];
                if (q < qW) {
                    const int t = e0 + q;
                    if (dst) {
                        if (al && q + 1 < qW) {
                            *reinterpret_cast<double2*>(dst + t) = f;
                        } else {
                            dst[t] = f.x;
                            if (q + 1 < qW) dst[t + 1] = f.y;
                        }
                    }
                }
                if (NT > 0 && q < qBfull) {
                    f.x = (q < qB) ? f.x - c0 : 0.0;
                    f.y = (q + 1 < qB) ? f.y - c0 : 0.0;
                    v2[px2(q2)] = f;
                }
            }
            // shifted scheme, first tile: the pre-chunk (positions [0, 4t) of the series) reads
            // the look-back range as y = 0
            if (SHIFTED && NT > 0 && e0 < 0 && tid < kHB / 2) v2[px2(tid)] = make_double2(0.0, 0.0);
        }
        if (have_next) STS_ISSUE(k + 1);   // in flight during the MFMA phase of tile k
        else STS_CLEAR();
        // lag matrix (fill only; S/Lag.scala:62-77): column c - init holds x[r + max_lag - c] at
        // row r.  Each column's rows of this tile go out as 16-B pairs aligned on the column's
        // own address (one wave instruction = 1 KB of one column; round 3 stored the two halves
        // of every pair with separate 8-B stores); the pair straddling the tile's first / last
        // row is stored per element.  Plain stores: non-temporal ones ran C5 at 1.80 ms against
        // 1.64-1.66 (profiles/r04_v4_c5_forms.jsonl).
        if constexpr (NT == 0) {
            if (a.lagmat) {
                double* lm = a.lagmat + s * lrows * ncols;
                for (int c = init; c <= a.max_lag; c++) {
                    double* col = lm + (int64_t)(c - init) * lrows;
                    const int sh = a.max_lag - c;
                    const int rlo = t0 - sh > 0 ? t0 - sh : 0;
                    const int rhi = (int64_t)(t1 - sh) < lrows ? t1 - sh : (int)lrows;
                    if (rlo >= rhi) continue;
                    const int par = (int)((reinterpret_cast<uintptr_t>(col) >> 3) & 1);   // col + r 16-B aligned iff r + par even
                    const int rp = rlo - ((rlo + par) & 1);
                    for (int r = rp + 2 * tid; r < rhi; r += 2 * kThreads) {
                        const int q = r + sh - e0;
                        if (r >= rlo && r + 1 < rhi) {
                            *reinterpret_cast<d2v*>(col + r) = d2v{vals[px(q)], vals[px(q + 1)]};
                        } else {
                            if (r >= rlo) col[r] = vals[px(q)];
                            if (r + 1 < rhi) col[r + 1] = vals[px(q + 1)];
                        }
                    }
                }
            }
        }
        STAMP(8);

        if constexpr (NT > 0) {
            lds_barrier();
            STAMP(9);
            // ---- 6. lag products on MFMA, at wave priority 0; the rest of the tile loop runs at
            //      STS_FILL_PRIO, so a SIMD's arbiter favours the waves of workgroups in their fill
            //      and store phases (memory issue) over the MFMA stream of the others ----
            __builtin_amdgcn_s_setprio(0);
            mfma_group(std::integral_constant<int, 0>{}, std::integral_constant<int, CPW>{}, vals, k, t0, t1);
            __builtin_amdgcn_s_setprio(STS_FILL_PRIO);
        }
        have = have_next;
        STAMP(10);
        lds_barrier();   // vals / mask / lists are reused by the next tile
        STAMP(11);
    }
#undef STS_ISSUE
#undef STS_LD1
#undef STS_ST1
#undef STS_CLEAR
    if (series_err && a.err) a.err[s] = STS_ERR_ALL_NAN;
#ifdef STS_STAMPS
    if (lane == 0) {
#pragma unroll
        for (int i = 0; i < 12; i++) atomicAdd(&g_stamps[i], st_acc[i]);
        atomicAdd(&g_stamps[12], 1ull);
    }
#endif

    if constexpr (NT > 0) {
        // ---- 7. diagonal extraction: lane d accumulates lag d in a fixed order ----
        double* scr = vals + wave * 256;
        double lagacc = 0.0;
        if constexpr (SHIFTED) {
            d4 D = U[0];
#pragma unroll
            for (int t = 1; t < NA; t++) D += U[t];
#pragma unroll
            for (int r = 0; r < 4; r++) scr[((lane >> 4) + 4 * r) * 16 + (lane & 15)] = D[r];
            lds_barrier();
#pragma unroll
            for (int j = 0; j < 16; j++) {
                const int i = 16 * (j / QS) + (16 - QS) + (j % QS) - lane;   // entry (i, j) holds lag h(j) - i
                if (i >= 0 && i < 16) lagacc += scr[i * 16 + j];
            }
            lds_barrier();
        } else {
#pragma unroll
            for (int t = 0; t < NT; t++) {
#pragma unroll
                for (int r = 0; r < 4; r++) scr[((lane >> 4) + 4 * r) * 16 + (lane & 15)] = U[t][r];
                lds_barrier();
#pragma unroll
                for (int b = 0; b < 16; b++)
                    if (((b + lane) >> 4) == t) lagacc += scr[b * 16 + ((b + lane) & 15)];
                lds_barrier();
            }
        }
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) {
            acc_s += __shfl_xor(acc_s, d);
            acc_q += __shfl_xor(acc_q, d);
        }
        double* wsum = vals + kWaves * 256;
        wsum[wave * kPartStride + lane] = lagacc;
        if (lane == 0) {
            wsum[wave * kPartStride + kPartSum] = acc_s;
            wsum[wave * kPartStride + kPartSq] = acc_q;
        }
        lds_barrier();
        if (wave == 0) {
            double* part = a.partials + ch * kPartStride;
            double tot = 0.0;
#pragma unroll
            for (int w = 0; w < kWaves; w++) tot += wsum[w * kPartStride + lane];
            part[lane] = tot;
            if (lane == 0) {
                double ts = 0.0, tq = 0.0;
#pragma unroll
                for (int w = 0; w < kWaves; w++) {
                    ts += wsum[w * kPartStride + kPartSum];
                    tq += wsum[w * kPartStride + kPartSq];
                }
                part[kPartSum] = ts;
                part[kPartSq] = tq;
                part[kPartShift] = c0;
            }
        }
    }
}

// One wave per series: combine the chunk partials in chunk order (deterministic) and form
// the reference's correlation cov / (sqrt(var1) * sqrt(var2)) (S/UnivariateTimeSeries.scala:
// 80-89) with the robust head / tail handling of sts_acf.hpp.  Lane l computes lag i = l + 1.
// Series with T <= 2K (or shorter than the two edges) run the reference's two-pass loop
// directly (reproduces its NaN pattern exactly when a NaN sits in the middle of a short
// series), and so does every series with a lag sts_acf.hpp's rule 3 finds suspect.
__global__ __launch_bounds__(256) void acf_finalize_kernel(FinalizeArgs a) {
    const int lane = threadIdx.x & 63;
    const int64_t s = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (s >= a.S) return;
    const int K = a.K;
    const int i = lane + 1;
    const int64_t T = a.T;
    const double* F = a.F + s * a.ldF;
    if (lane >= K) return;
    double out;
    if (i >= T) {
        out = __builtin_nan("");
    } else if (T <= 2 * (int64_t)K || T < 2 * kAcfEdge) {
        out = acf_exact_lag(F, T, i);
    } else {
        double Pi = 0.0, Sm = 0.0, Qm = 0.0;
        const double* pp = a.partials + s * a.parts_per_series * kPartStride;
        const double c = pp[kPartShift];
        for (int64_t k = 0; k < a.parts_per_series; k++, pp += kPartStride) {
            Pi += pp[i];
            Sm += pp[kPartSum];
            Qm += pp[kPartSq];
        }
        bool sus;
        out = acf_combine(Pi, Sm, Qm, i, T, [&](int j) { return F[j] - c; },
                          [&](int j) { return F[T - 1 - j] - c; }, c, &sus);
        // sts_acf.hpp rule 3: a series with any suspect lag takes the reference's loop (all lags):
        // flagged here, recomputed by acf_exact_kernel (F streamed through LDS)
        if (__ballot(sus) && lane == 0) a.exact[s] = 1;
    }
    a.acf[s * K + lane] = out;
}

// Rule 3's fallback (sts_acf.hpp): one wave per (flagged series, block of 64 lags), every lag by
// the reference's two-pass loop over F streamed through the wave's LDS chunk buffer.  Waves of
// unflagged series exit at once (one flag load).
// One wave per (series, 64-lag block), four per workgroup (so the four land on the CU's four
// SIMDs: a flagged series' wave is one latency-bound chain per SIMD); waves of unflagged
// series read their flag and end.  WIDE: the blocks past the first (numLags > 64) keep a second
// chunk buffer for the unlagged operand.
constexpr int kExactChunk = 512;
template <bool WIDE>
__global__ __launch_bounds__(256) void acf_exact_kernel(const double* __restrict__ F, int64_t S, int64_t T,
                                                        int64_t ld, int K, int nblk, const int32_t* __restrict__ flags,
                                                        double* __restrict__ acf) {
    __shared__ double lds[4][kExactChunk + 64];
    __shared__ double ldsb[4][WIDE ? kExactChunk : 1];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int nb = WIDE ? nblk - 1 : 1;
    const int64_t u = (int64_t)blockIdx.x * 4 + wave;
    const int64_t s = u / nb;
    if (s >= S || !flags[s]) return;
    const int b = WIDE ? 1 + (int)(u % nb) : 0;
    const int i = b * 64 + lane + 1;
    const bool active = i <= K && (int64_t)i < T;
    const double r = WIDE ? acf_exact_stream<kExactChunk, true>(F + s * ld, T, i, active, lds[wave], lane, b * 64,
                                                                ldsb[wave])
                          : acf_exact_stream<kExactChunk>(F + s * ld, T, i, active, lds[wave], lane);
    if (active) acf[s * K + (i - 1)] = r;
}

// One wave per series: the robust ACF shift (sts_acf.hpp) of every series, once per call,
// for the tile kernel's workgroups to load (instead of each of a series' ~15 workgroups
// sampling and ranking it again).
__global__ __launch_bounds__(256) void acf_shift_kernel(const double* in, int64_t S, int64_t T, int64_t ld, int prev,
                                                        double* shift) {
    const int lane = threadIdx.x & 63;
    const int64_t s = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (s >= S) return;
    const double c = robust_shift(in + s * ld, T, lane, prev != 0);
    if (lane == 0) shift[s] = c;
}

}  // namespace

hipError_t launch_acf_shift(const double* in, int64_t S, int64_t T, int64_t ld, int method, double* shift,
                            hipStream_t st) {
    if (S <= 0 || T <= 0) return hipSuccess;
    dim3 grid((unsigned)((S + 3) / 4)), block(256);
    hipLaunchKernelGGL(acf_shift_kernel, grid, block, 0, st, in, S, T, ld, method == STS_FILL_PREVIOUS ? 1 : 0,
                       shift);
    return hipGetLastError();
}

// one launch of tile_kernel<TW, NT, SHIFTED, NTH, method>
template <int TW, int NT, bool SHIFTED, int NTH>
hipError_t launch_m(int method, dim3 grid, const TileArgs& a, hipStream_t st) {
    const dim3 block(NTH);
    switch (method) {
    case STS_FILL_NONE: hipLaunchKernelGGL((tile_kernel<TW, NT, SHIFTED, NTH, STS_FILL_NONE>), grid, block, 0, st, a); break;
    case STS_FILL_LINEAR: hipLaunchKernelGGL((tile_kernel<TW, NT, SHIFTED, NTH, STS_FILL_LINEAR>), grid, block, 0, st, a); break;
    case STS_FILL_NEAREST: hipLaunchKernelGGL((tile_kernel<TW, NT, SHIFTED, NTH, STS_FILL_NEAREST>), grid, block, 0, st, a); break;
    case STS_FILL_NEXT: hipLaunchKernelGGL((tile_kernel<TW, NT, SHIFTED, NTH, STS_FILL_NEXT>), grid, block, 0, st, a); break;
    case STS_FILL_PREVIOUS: hipLaunchKernelGGL((tile_kernel<TW, NT, SHIFTED, NTH, STS_FILL_PREVIOUS>), grid, block, 0, st, a); break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t launch_tile(int method, int tw, const TileArgs& a, hipStream_t st) {
    const int64_t nchunk = a.S * a.chunks_per_series;
    if (nchunk <= 0) return hipSuccess;
    if (nchunk > 0x7fffffffLL) return hipErrorInvalidValue;
    dim3 grid((unsigned)nchunk);
    if (tw == 512 && a.K == 0) return launch_m<512, 0, false, kThreads>(method, grid, a, st);
#ifdef STS_AB
    if (tw == 2048 && a.K > 0 && a.K <= 60) {   // 2-wave workgroups (A/B build: STS_TILE_W=2048)
        if (a.K <= 24) return launch_m<2048, 2, true, kThreads / 2>(method, grid, a, st);
        return launch_m<2048, 4, true, kThreads / 2>(method, grid, a, st);
    }
#endif
    if (tw != 4096) return hipErrorInvalidValue;
    if (a.K == 0) return launch_m<4096, 0, false, kThreads>(method, grid, a, st);
    if (a.K <= 24) return launch_m<4096, 2, true, kThreads>(method, grid, a, st);
    if (a.K <= 60) return launch_m<4096, 4, true, kThreads>(method, grid, a, st);
    if (a.K <= 63) return launch_m<4096, 5, false, kThreads>(method, grid, a, st);
    return hipErrorInvalidValue;
}

#ifdef STS_STAMPS
extern "C" int sts_debug_stamps(unsigned long long* out16) {
    if (hipMemcpyFromSymbol(out16, HIP_SYMBOL(g_stamps), sizeof(unsigned long long) * 16) != hipSuccess) return 4;
    unsigned long long z[16] = {0};
    return hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), z, sizeof(z)) == hipSuccess ? 0 : 4;
}
#endif

hipError_t launch_acf_finalize(const FinalizeArgs& a, hipStream_t st) {
    if (a.S <= 0 || a.K <= 0) return hipSuccess;
    dim3 grid((unsigned)((a.S + 3) / 4)), block(256);
    hipLaunchKernelGGL(acf_finalize_kernel, grid, block, 0, st, a);
    return hipGetLastError();
}

hipError_t launch_acf_exact(const double* F, int64_t S, int64_t T, int64_t ldF, int K, const int32_t* exact,
                            double* acf, hipStream_t st) {
    if (S <= 0 || K <= 0 || T <= 0) return hipSuccess;
    const int nblk = (K + 63) / 64;
    if ((S * nblk + 3) / 4 > 0x7fffffffLL) return hipErrorInvalidValue;
    hipLaunchKernelGGL(acf_exact_kernel<false>, dim3((unsigned)((S + 3) / 4)), dim3(256), 0, st, F, S, T, ldF, K, nblk,
                       exact, acf);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess || nblk == 1) return e;
    hipLaunchKernelGGL(acf_exact_kernel<true>, dim3((unsigned)((S * (nblk - 1) + 3) / 4)), dim3(256), 0, st, F, S, T,
                       ldF, K, nblk, exact, acf);
    return hipGetLastError();
}

}  // namespace sts
