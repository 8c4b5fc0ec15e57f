// sts_recur.hip -- first-order and p-th order recurrences along time, bit-exact by
// construction (the reference's own sequential order):
//   EWMAModel.addTimeDependentEffects     S/models/EWMA.scala:135-142
//   EWMAModel.removeTimeDependentEffects  S/models/EWMA.scala:125-133 (dest eq ts)
//   ARModel.addTimeDependentEffects       S/models/Autoregression.scala:75-88 (IIR)
//   ARModel.removeTimeDependentEffects    S/models/Autoregression.scala:60-73 (dest eq ts)
//   differencesAtLag                      S/UnivariateTimeSeries.scala:356-376 (dest eq ts)
//   C2 pipeline fillPrevious -> differencesAtLag(lag) -> EWMA add, fused (one HBM pass)
//
// Two kernels:
//  * recur_row_kernel (C2 and EWMA add on 16-B aligned rows of <= 1 024 steps): whole rows, 32
//    lanes per series, the sequential pieces made lane-parallel (carry by ballot, lag by DPP,
//    EWMA by an affine-map scan whose guess is verified bit for bit lane by lane);
//  * recur_kernel (everything else): one LANE per series; a wave owns SPW series and moves
//    SPW x CH blocks through LDS (the next chunk's loads in flight while the current one runs),
//    transposed so each lane runs its series' recurrence over the chunk in registers.
#include "sts_internal.hpp"
#include "sts_dma.hpp"
#include "sts_lanes.hpp"

#include <hip/hip_runtime.h>

#ifndef STS_FDE_SPW
#define STS_FDE_SPW 16   // series per wave (A/B on C2, 1M x 390: 16 x 128 1.40 ms, 24 x 128 1.41-1.43,
#define STS_FDE_CH 128   // 8 x 128 1.42, 32 x 128 1.50-1.52, 32 x 64 1.59-1.67, 16 x 192 2.35, 16 x 256 2.24)
#endif

#ifndef STS_RECUR_V2
#define STS_RECUR_V2 1   // 16-B global accesses in the C2 recurrence kernel (A/B: 1.673 vs 1.687 ms on C2)
#endif

namespace sts {
namespace {

constexpr int kSpw = STS_FDE_SPW, kCh = STS_FDE_CH;
// recur_row_kernel's launch shape (C2 A/B, profiles/r04_v9_ab_c2_lps.jsonl, r04_v10_ab_c2_shape.jsonl):
// 16 / 32 / 64 lanes per series 1.176-1.185 / 1.162-1.170 / 1.173-1.177 ms; 1 / 2 / 4 waves per
// workgroup 1.248-1.252 / 1.202-1.204 / 1.170-1.174 ms; XCD-contiguous spans 1.068-1.070 against
// 1.160-1.170 ms without
constexpr int kRowLps = 32;
constexpr int kRowWpg = 4;

// One lane's recurrence state and step, shared by the chunk and row kernels (the
// reference's statement order; -ffp-contract=off keeps every product / sum separate).
template <int OP, int H>
struct RecurLane {
    double sm = 0.0, oms = 0.0, cc = 0.0;
    double cf[H];
    double h[H];                   // value at t-1-j (outputs, or filled values for kFillDiffEwma)
    double e = 0.0;                // EWMA state
    double carry;                  // fillPrevious carry
    int hp;
    int64_t start;
    // load: the state and the raw per-series parameters (plain loads from clamped indices, no
    // arithmetic on them, so nothing waits for them until finish()); finish: derived values
    __device__ __forceinline__ void load(const RecurArgs& a, int64_t sl, bool live) {
        carry = __builtin_nan("");
        hp = (OP == kArAdd || OP == kArRemoveInplace) ? a.p : a.lag;   // history length used
        start = (OP == kFillDiffEwma) ? a.lag : a.start;
        e = 0.0;
        const int64_t si = live ? sl : 0;
#pragma unroll
        for (int j = 0; j < H; j++) {
            cf[j] = 0.0;
            h[j] = 0.0;
        }
        if (OP == kEwmaAdd || OP == kEwmaRemoveInplace || OP == kFillDiffEwma) sm = a.sm[si];
        if (OP == kArAdd || OP == kArRemoveInplace) {
            cc = a.c[si];
#pragma unroll
            for (int j = 0; j < H; j++) cf[j] = a.coef[si * a.p + (j < a.p ? j : 0)];
        }
    }
    __device__ __forceinline__ void finish(const RecurArgs& a) {
        if (OP == kEwmaAdd || OP == kEwmaRemoveInplace || OP == kFillDiffEwma) oms = 1.0 - sm;
        if (OP == kArAdd || OP == kArRemoveInplace) {
#pragma unroll
            for (int j = 0; j < H; j++) cf[j] = (j < a.p) ? cf[j] : 0.0;
        }
    }
    __device__ __forceinline__ void init(const RecurArgs& a, int64_t sl, bool live) {
        load(a, sl, live);
        finish(a);
    }
    // STEADY: t >= steady_from() (every t-guard below is then a constant; same operations)
    __device__ __forceinline__ int64_t steady_from() const {
        int64_t f = start > H ? start : H;
        return f > 1 ? f : 1;
    }
    template <bool STEADY = false>
    __device__ __forceinline__ double step(double x, int64_t t) {
        const bool first = !STEADY && t == 0;
        const bool before = !STEADY && t < start;
        double y;
        if (OP == kEwmaAdd) {
            // dest(i) = smoothing * ts(i) + (1 - smoothing) * dest(i - 1)
            e = first ? x : sm * x + oms * e;
            y = e;
        } else if (OP == kEwmaRemoveInplace) {
            // ts(i - 1) already overwritten by dest(i - 1)
            y = first ? x : (x - oms * h[0]) / sm;
        } else if (OP == kArAdd) {
            y = cc + x;
#pragma unroll
            for (int j = 0; j < H; j++)
                if (j < hp && (STEADY || t - j - 1 >= 0)) y += h[j] * cf[j];
        } else if (OP == kArRemoveInplace) {
            y = x - cc;
#pragma unroll
            for (int j = 0; j < H; j++)
                if (j < hp && (STEADY || t - j - 1 >= 0)) y -= h[j] * cf[j];
        } else if (OP == kDiffInplace) {
            // ts(i - lag) already overwritten when i - lag >= start; for i - lag < start it
            // equals the original, so h (the outputs) is right in both cases
            double hl = 0.0;
#pragma unroll
            for (int j = 0; j < H; j++) hl = (j == hp - 1) ? h[j] : hl;   // static indexing
            y = before ? x : x - hl;
        } else {  // kFillDiffEwma: fillPrevious -> differencesAtLag(lag, start=lag) -> EWMA add
            carry = (x != x) ? carry : x;
            const double f = carry;
            double hl = 0.0;
#pragma unroll
            for (int j = 0; j < H; j++) hl = (j == hp - 1) ? h[j] : hl;   // static indexing
            const double d = before ? f : f - hl;
            e = first ? d : sm * d + oms * e;
            // history of FILLED values
#pragma unroll
            for (int j = H - 1; j > 0; j--) h[j] = h[j - 1];
            h[0] = f;
            return e;
        }
#pragma unroll
        for (int j = H - 1; j > 0; j--) h[j] = h[j - 1];
        h[0] = y;
        return y;
    }
};

// SPW series per wave, CH steps per chunk: the chunk's SPW x CH block moves through LDS
// with every load / store instruction covering 64 consecutive steps of ONE series (512
// contiguous bytes); lanes < SPW then run their series' recurrence over the chunk.
// Longer row segments (fewer series, longer chunks) keep HBM pages open: C2's 1M series
// x 390 steps are only 3 KB each.
template <int OP, int H, int SPW = 64, int CH = 32, bool V2 = false>
__global__ __launch_bounds__(64) void recur_kernel(RecurArgs a) {
    // V2: 16-B loads / stores (two consecutive steps per lane, half the memory instructions);
    // rows padded to an even stride so the 16-B LDS accesses stay aligned
    // (round 4: 130-step chunks -- three for C2's 390 steps instead of 3 x 128 + 6 -- ran 2.14
    // against 1.43 ms: a 130-step row does not fill whole 128-double load instructions, so every
    // instruction then spans two rows; profiles/r04_v4_ab_c2.jsonl)
    constexpr int kRow = V2 ? CH + 2 : CH + 1;
    constexpr int EPL = V2 ? 2 : 1;               // elements per lane per instruction
    constexpr int NLD = SPW * CH / (64 * EPL);    // load instructions per chunk per lane
    static_assert(SPW * CH % (64 * EPL) == 0 && (V2 ? CH % 2 == 0 : (CH % 64 == 0 || 64 % CH == 0)), "chunk shape");
    __shared__ __attribute__((aligned(16))) double tile[SPW * kRow];
    const int lane = threadIdx.x;
    const int64_t s0 = (int64_t)blockIdx.x * SPW;
    const int64_t sl = s0 + lane;                 // this lane's series (lanes < SPW)
    const bool live = lane < SPW && sl < a.S;
    const int ns = (a.S - s0 < SPW) ? (int)(a.S - s0) : SPW;
    const int64_t T = a.T;

    RecurLane<OP, H> rl;
    rl.init(a, sl, live);

    // load instruction i of a chunk: element e = (i * 64 + lane) * EPL, row e / CH, column e % CH
    double2 pre[NLD];
    auto fetch = [&](int64_t tc) {
        const int len = (T - tc < CH) ? (int)(T - tc) : CH;
#pragma unroll
        for (int i = 0; i < NLD; i++) {
            const int e = (i * 64 + lane) * EPL;
            const int row = e / CH, col = e % CH;
            const double* src = a.in + (s0 + row) * a.ld_in + tc + col;
            if (V2) {
                if (row < ns && col + 1 < len) {
                    pre[i] = *reinterpret_cast<const double2*>(src);
                } else {
                    pre[i].x = (row < ns && col < len) ? src[0] : 0.0;
                    pre[i].y = 0.0;
                }
            } else {
                pre[i].x = (row < ns && col < len) ? src[0] : 0.0;
            }
        }
    };
    fetch(0);
    for (int64_t tc = 0; tc < T; tc += CH) {
        const int len = (T - tc < CH) ? (int)(T - tc) : CH;
#pragma unroll
        for (int i = 0; i < NLD; i++) {
            const int e = (i * 64 + lane) * EPL;
            const int row = e / CH, col = e % CH;
            if (V2) {
                if (row < ns && col < len) *reinterpret_cast<double2*>(&tile[row * kRow + col]) = pre[i];
            } else {
                if (row < ns && col < len) tile[row * kRow + col] = pre[i].x;
            }
        }
        if (tc + CH < T) fetch(tc + CH);   // next chunk in flight during this one
        __syncthreads();
        if (live) {
            double* myrow = tile + lane * kRow;
            for (int c = 0; c < len; c++) myrow[c] = rl.step(myrow[c], tc + c);
        }
        __syncthreads();
#pragma unroll
        for (int i = 0; i < NLD; i++) {
            const int e = (i * 64 + lane) * EPL;
            const int row = e / CH, col = e % CH;
            double* d = a.out + (s0 + row) * a.ld_out + tc + col;
            if (V2) {
                if (row < ns && col + 1 < len) *reinterpret_cast<double2*>(d) = *reinterpret_cast<const double2*>(&tile[row * kRow + col]);
                else if (row < ns && col < len) d[0] = tile[row * kRow + col];
            } else {
                if (row < ns && col < len) d[0] = tile[row * kRow + col];
            }
        }
        __syncthreads();
    }
}

// ---------------------------------------------------------------------------------------
// Whole rows, LPS lanes per series (64 / LPS series per wave; T <= LPS B; C2 with LPS = 32:
// B = 14, two series per wave): lane r of a series holds the steps [rB, rB + B) in registers,
// and the sequential recurrences run lane-parallel yet bit-exact:
//  * fillPrevious: the carry into a lane is the last valid value of the nearest lower lane of
//    its series that has one (ballot + one bpermute); inside the block the reference's carry loop;
//  * differencesAtLag(lag <= H): the previous lane's last H filled values by DPP wave shift;
//  * EWMA add: e_t = s d_t + (1 - s) e_{t-1} is affine in e_{t-1}.  Each lane composes its
//    block's map (A, B); a scan of the maps (DPP row_shr 1, 2, 4, 8 inside rows of 16, readlanes
//    across rows) gives every lane a GUESS of its incoming state; one pass of the reference's own
//    step from the guess gives each lane's outgoing state, which becomes the next lane's incoming
//    state; a second pass computes and stores the outputs and is verified: a lane's incoming
//    state must equal, bit for bit, the previous lane's outgoing state as computed from that
//    lane's incoming state.  Mismatching lanes take their predecessor's value and run (and
//    store) again.  A series' first lane starts exactly (e_0 = d_0), so after round r lanes
//    0..r+1 are exact and the loop ends after at most LPS - 1 rounds; with a block's contraction
//    (1 - s)^B (0.8^14 = 0.04 for C2) it ends after the first almost always.  The outputs are the
//    sequential loop's bits.
// Only the fused C2 pipeline and EWMA add take this kernel (the maps of in-place EWMA remove
// expand by (1 - s) / s, and AR add's state is a p-vector).

template <int CTRL>
__device__ __forceinline__ double dpp_shift(double v) {   // row_shr:k (0x110 + k) or wave_shr:1 (0x138); lanes without a source get 0
    const unsigned long long u = __builtin_bit_cast(unsigned long long, v);
    // bound_ctrl: a lane without a source reads 0, so no old value to zero first (round 6)
    const int lo = __builtin_amdgcn_mov_dpp((int)(unsigned)u, CTRL, 0xf, 0xf, true);
    const int hi = __builtin_amdgcn_mov_dpp((int)(unsigned)(u >> 32), CTRL, 0xf, 0xf, true);
    return __builtin_bit_cast(double, ((unsigned long long)(unsigned)hi << 32) | (unsigned)lo);
}
__device__ __forceinline__ unsigned long long dbits(double v) { return __builtin_bit_cast(unsigned long long, v); }
[[maybe_unused]] __device__ __forceinline__ double lane_get(double v, int l) {   // v_readlane: lane l's value, uniform
    const unsigned long long u = __builtin_bit_cast(unsigned long long, v);
    const unsigned lo = __builtin_amdgcn_readlane((unsigned)u, l);
    const unsigned hi = __builtin_amdgcn_readlane((unsigned)(u >> 32), l);
    return __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lo);
}

// IO: the wave's rows move as one contiguous span (ld == T, T even) through a per-wave LDS
// block: in by LDS-DMA (1 KB of consecutive doubles per instruction), out by 16-B LDS reads and
// coalesced 16-B stores; each lane reads / writes its block in LDS.  Without IO every load / store
// instruction touches 16 B per lane at an 8B-byte lane stride (up to 64 cache lines per
// instruction).  LPS: lanes per series (16: one DPP row; 32 / 64: two / four rows, joined by
// readlanes).
template <int OP, int H, int B, bool IO, int LPS>
__global__ __launch_bounds__(64 * kRowWpg) void recur_row_kernel(RecurArgs a) {
    static_assert(B % 2 == 0 && H <= B, "lane blocks of whole 16-B pairs, history inside one block");
    static_assert(LPS == 16 || LPS == 32 || LPS == 64, "one, two or four DPP rows per series");
    constexpr int SPW = 64 / LPS;  // series per wave
    constexpr int WD = 64 * B;     // doubles per wave block: SPW rows of up to LPS B steps
    constexpr unsigned long long kGroup = LPS == 64 ? ~0ull : (1ull << (LPS % 64)) - 1ull;   // a series' lanes
    __shared__ __attribute__((aligned(16))) double blk_mem[IO ? kRowWpg * WD : 2];
    const int lane = threadIdx.x & 63;
    const int rl = lane & (LPS - 1);
    const int wave = threadIdx.x >> 6;
    const int64_t bid = xcd_remap(blockIdx.x, gridDim.x);   // XCD x streams one contiguous range of spans
    const int64_t s0 = (bid * kRowWpg + wave) * SPW;   // the wave's first series
    if (s0 >= a.S) return;                                       // wave-uniform
    const int64_t s = s0 + lane / LPS;
    const bool live = s < a.S;
    const int64_t sc = live ? s : a.S - 1;   // a dead row computes on a copy and stores nothing
    const int T = (int)a.T;
    const int t0 = rl * B;
    const double* src = a.in + sc * a.ld_in;
    double* dst = a.out + sc * a.ld_out;
    const double sm = a.sm[sc];
    const double oms = 1.0 - sm;
    const bool even = (T & 1) == 0;   // uniform
    double* blk = blk_mem + (IO ? wave * WD : 0);
    const int nrow = (a.S - s0 < SPW) ? (int)(a.S - s0) : SPW;
    const int span = nrow * T;                       // doubles of the wave's rows (even)
    const int lo = (lane / LPS) * T + t0;            // this lane's block in the LDS span

    // clamped addresses, no branches: steps past the row read some other valid step; they only
    // feed lanes past the row and the row's last lane's own steps past T, never a store
    double v[B];
    if constexpr (IO) {
        const double* g = a.in + s0 * a.ld_in;      // ld == T: the rows are one span
        const unsigned lb = lds_addr(blk);
#pragma unroll
        for (int i = 0; i < WD / 128; i++) {
            const int u = 128 * i + 2 * lane;
            if (128 * i < span) glds16<true>(g + (u < span ? u : span - 2), lb + i * 1024);   // nt: C2 0.979-0.982 vs 1.003-1.007 ms
        }
        dma_wait();
        wave_lds_sync();
#pragma unroll
        for (int j = 0; j < B; j += 2) {
            const double2 p = *reinterpret_cast<const double2*>(blk + lo + j);
            v[j] = p.x;
            v[j + 1] = p.y;
        }
        wave_lds_sync();   // every lane has its block: the span's LDS takes the outputs
    } else if (even) {
#pragma unroll
        for (int j = 0; j < B; j += 2) {
            const int t = (t0 + j < T - 2) ? t0 + j : T - 2;
            const double2 p = *reinterpret_cast<const double2*>(src + t);
            v[j] = p.x;
            v[j + 1] = p.y;
        }
    } else {
#pragma unroll
        for (int j = 0; j < B; j++) v[j] = src[(t0 + j < T - 1) ? t0 + j : T - 1];
    }

    double d0;   // d at the block's first step (the EWMA's e_0 when t0 == 0)
    if constexpr (OP == kFillDiffEwma) {
        // ---- fillPrevious (S/UnivariateTimeSeries.scala:186-204) ----
        double lastv = __builtin_nan("");
#pragma unroll
        for (int j = 0; j < B; j++) lastv = (v[j] != v[j]) ? lastv : v[j];
        const unsigned long long below =
            __ballot(!(lastv != lastv)) & ((1ull << lane) - 1ull) & (kGroup << (lane & (64 - LPS)));
        const double cin = __shfl(lastv, below ? 63 - __builtin_clzll(below) : lane);
        double carry = below ? cin : __builtin_nan("");
#pragma unroll
        for (int j = 0; j < B; j++) {
            carry = (v[j] != v[j]) ? carry : v[j];
            v[j] = carry;
        }
        // ---- differencesAtLag(lag, start = lag) of the FILLED values (:356-376), in place from
        //      the block's end ----
        double pv[H + 1];   // pv[k]: the filled value at t0 - k (row lane 0: never read, t < lag)
        pv[0] = 0.0;
#pragma unroll
        for (int k = 1; k <= H; k++) pv[k] = dpp_shift<0x138>(v[B - k]);
        if constexpr (H == 1) {
#pragma unroll
            for (int j = B - 1; j >= 1; j--) v[j] = v[j] - v[j - 1];
            v[0] = (t0 == 0) ? v[0] : v[0] - pv[1];
        } else {
            const int L = a.lag;   // 1 <= L <= H
#pragma unroll
            for (int j = B - 1; j >= 0; j--) {
                double hl = 0.0;
#pragma unroll
                for (int k = 1; k <= H; k++) hl = (k == L) ? (j >= k ? v[j - k] : pv[k - j]) : hl;
                v[j] = (j < H && t0 + j < L) ? v[j] : v[j] - hl;
            }
        }
    }
    d0 = v[0];
    // sm * d once per step: the reference's step is then one product and one sum,
    // e = (s d) + ((1 - s) e), rounded in the same order
#pragma unroll
    for (int j = 0; j < B; j++) v[j] = sm * v[j];
    const bool first = (t0 == 0);
    auto enter = [&](double ein) -> double { return first ? d0 : v[0] + oms * ein; };

    // ---- EWMA add (S/models/EWMA.scala:135-142): the guess ----
    double Bm = first ? d0 : v[0];   // e_out = A e_in + Bm over the block (FMAs: a guess only)
#pragma unroll
    for (int j = 1; j < B; j++) Bm = __builtin_fma(oms, Bm, v[j]);
    double A = 1.0, pw = oms;   // oms^B by squaring
#pragma unroll
    for (int b = B; b > 0; b >>= 1) {
        if (b & 1) A *= pw;
        pw *= pw;
    }
    A = first ? 0.0 : A;
#define STS_ROWSCAN_STEP(K)                                                                  \
    {                                                                                        \
        const double Ap = dpp_shift<0x110 + K>(A), Bp = dpp_shift<0x110 + K>(Bm);                \
        if ((lane & 15) >= K) {                                                              \
            Bm = __builtin_fma(A, Bp, Bm);                                                   \
            A = A * Ap;                                                                      \
        }                                                                                    \
    }
    STS_ROWSCAN_STEP(1) STS_ROWSCAN_STEP(2) STS_ROWSCAN_STEP(4) STS_ROWSCAN_STEP(8)
#undef STS_ROWSCAN_STEP
    if constexpr (LPS == 32) {   // the second row of a series continues from its first row's total
        const double a0 = lane_get(A, 15), b0 = lane_get(Bm, 15), a1 = lane_get(A, 47), b1 = lane_get(Bm, 47);
        const double Ap = lane < 32 ? a0 : a1, Bp = lane < 32 ? b0 : b1;
        if (rl >= 16) {
            Bm = __builtin_fma(A, Bp, Bm);
            A = A * Ap;
        }
    } else if constexpr (LPS == 64) {   // rows 1..3 continue from the state at the end of the row before
        const double E0 = lane_get(Bm, 15);   // row 0 holds t = 0: its prefix is a constant
        const double E1 = __builtin_fma(lane_get(A, 31), E0, lane_get(Bm, 31));
        const double E2 = __builtin_fma(lane_get(A, 47), E1, lane_get(Bm, 47));
        const int row = lane >> 4;
        const double Ein = row == 1 ? E0 : (row == 2 ? E1 : E2);
        Bm = row == 0 ? Bm : __builtin_fma(A, Ein, Bm);
    }
    double ein = dpp_shift<0x138>(Bm);   // the inclusive prefix of the lane before: the state entering this one
    // one pass of the reference's step from the guess; its outgoing state is the next guess
    {
        double e = enter(ein);
#pragma unroll
        for (int j = 1; j < B; j++) e = v[j] + oms * e;
        const double nx = dpp_shift<0x138>(e);
        ein = (rl > 0) ? nx : ein;
    }

    // ---- outputs from the reference's step, stored, verified lane by lane ----
    const bool act = live && t0 < T;
    bool dirty = true;
    for (int round = 0; round < LPS; round++) {   // round r: lanes 0..r+1 of the series exact
        double e = enter(ein);
        double ep = e;
#pragma unroll
        for (int j = 1; j < B; j++) {
            e = v[j] + oms * e;
            if (j & 1) {
                const int t = t0 + j - 1;
                if (act && dirty) {
                    if (IO) {
                        if (t < T) *reinterpret_cast<double2*>(blk + lo + j - 1) = make_double2(ep, e);
                    } else if (even) {
                        if (t < T) *reinterpret_cast<double2*>(dst + t) = make_double2(ep, e);
                    } else {
                        if (t + 1 < T) *reinterpret_cast<double2*>(dst + t) = make_double2(ep, e);
                        else if (t < T) dst[t] = ep;
                    }
                }
            }
            ep = e;
        }
        const double eprev = dpp_shift<0x138>(e);
        // dead rows (past S) never redo: their garbage NaN patterns must not force rounds
        const bool redo = act && rl > 0 && dbits(eprev) != dbits(ein);
        if (!__ballot(redo)) break;
        ein = redo ? eprev : ein;
        dirty = redo;
    }
    if constexpr (IO) {   // the span out in 1-KB coalesced pieces
        wave_lds_sync();
        double* g = a.out + s0 * a.ld_out;
#pragma unroll
        for (int i = 0; i < WD / 128; i++) {
            const int u = 128 * i + 2 * lane;
            if (u < span) *reinterpret_cast<double2*>(g + u) = *reinterpret_cast<const double2*>(blk + u);
        }
    }
}

// Fallbacks for histories longer than 32 steps (correct, not tuned):
// in-place differencing decomposes into `lag` independent chains t = r, r+lag, ...
__global__ __launch_bounds__(256) void diff_chain_kernel(double* x, int64_t S, int64_t T, int64_t ld, int lag,
                                                         int start) {
    const int64_t g = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (g >= S * lag) return;
    const int64_t s = g / lag;
    const int r = (int)(g - s * lag);
    double* v = x + s * ld;
    for (int64_t t = r; t < T; t += lag)
        if (t >= start) v[t] = v[t] - v[t - lag];
}

// AR add / in-place AR remove of order p > 32: one thread per series on global memory
template <int OP>
__global__ __launch_bounds__(256) void ar_naive_kernel(RecurArgs a) {
    const int64_t s = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (s >= a.S) return;
    const double* x = a.in + s * a.ld_in;
    double* d = a.out + s * a.ld_out;
    const double* cf = a.coef + s * a.p;
    const double c = a.c[s];
    for (int64_t i = 0; i < a.T; i++) {
        if (OP == kArAdd) {
            double v = c + x[i];
            for (int j = 0; j < a.p && i - j - 1 >= 0; j++) v += d[i - j - 1] * cf[j];
            d[i] = v;
        } else {
            double v = x[i] - c;
            for (int j = 0; j < a.p && i - j - 1 >= 0; j++) v -= d[i - j - 1] * cf[j];
            d[i] = v;
        }
    }
}

// 16-B accesses need 16-B aligned rows (base and ld even)
inline bool rows16(const RecurArgs& a) {
    return STS_RECUR_V2 && ((reinterpret_cast<uintptr_t>(a.in) | reinterpret_cast<uintptr_t>(a.out)) & 15) == 0 &&
           a.ld_in % 2 == 0 && a.ld_out % 2 == 0;
}

template <int OP>
hipError_t launch_h(const RecurArgs& a, int need, hipStream_t st) {
    if constexpr (OP == kFillDiffEwma || OP == kEwmaAdd) {
        if (need <= 8 && rows16(a) && a.T <= kRowLps * 32) {   // whole rows, kRowLps lanes per series
            dim3 g((unsigned)((a.S + kRowWpg * (64 / kRowLps) - 1) / (kRowWpg * (64 / kRowLps)))), b(64 * kRowWpg);
            const int B = (int)(((a.T + kRowLps - 1) / kRowLps + 1) & ~1);   // even, >= 2
            const bool h1 = OP == kEwmaAdd || need <= 1;
            if (!h1 && need > B) goto chunks;                   // the lag reaches past the previous lane
            // one contiguous span per wave through LDS (in place too: a wave reads and rewrites
            // only its own span)
            const bool io = a.ld_in == a.T && a.ld_out == a.T && (a.T & 1) == 0;
#define STS_ROW_B(BB)                                                                          \
            case BB:                                                                           \
                if (io) {                                                                      \
                    if (h1) hipLaunchKernelGGL((recur_row_kernel<OP, 1, BB, true, kRowLps>), g, b, 0, st, a); \
                    else hipLaunchKernelGGL((recur_row_kernel<OP, (OP == kEwmaAdd ? 1 : (BB < 8 ? BB : 8)), BB, true, kRowLps>), g, b, 0, st, a); \
                } else {                                                                       \
                    if (h1) hipLaunchKernelGGL((recur_row_kernel<OP, 1, BB, false, kRowLps>), g, b, 0, st, a); \
                    else hipLaunchKernelGGL((recur_row_kernel<OP, (OP == kEwmaAdd ? 1 : (BB < 8 ? BB : 8)), BB, false, kRowLps>), g, b, 0, st, a); \
                }                                                                              \
                break;
            switch (B) {
                STS_ROW_B(2) STS_ROW_B(4) STS_ROW_B(6) STS_ROW_B(8) STS_ROW_B(10) STS_ROW_B(12) STS_ROW_B(14)
                STS_ROW_B(16) STS_ROW_B(18) STS_ROW_B(20) STS_ROW_B(22) STS_ROW_B(24) STS_ROW_B(26) STS_ROW_B(28)
                STS_ROW_B(30) STS_ROW_B(32)
            default: return hipErrorInvalidValue;
            }
#undef STS_ROW_B
            return hipGetLastError();
        }
    }
chunks:
    if (need <= 8 && rows16(a)) {   // the C2 shape: 16 series x 128-step chunks, 16-B accesses
        dim3 g((unsigned)((a.S + kSpw - 1) / kSpw)), b(64);
        if (need <= 1) hipLaunchKernelGGL((recur_kernel<OP, 1, kSpw, kCh, true>), g, b, 0, st, a);
        else if (need <= 2) hipLaunchKernelGGL((recur_kernel<OP, 2, kSpw, kCh, true>), g, b, 0, st, a);
        else if (need <= 4) hipLaunchKernelGGL((recur_kernel<OP, 4, kSpw, kCh, true>), g, b, 0, st, a);
        else hipLaunchKernelGGL((recur_kernel<OP, 8, kSpw, kCh, true>), g, b, 0, st, a);
        return hipGetLastError();
    }
    dim3 grid((unsigned)((a.S + 63) / 64)), block(64);
    if (need <= 1) hipLaunchKernelGGL((recur_kernel<OP, 1>), grid, block, 0, st, a);
    else if (need <= 2) hipLaunchKernelGGL((recur_kernel<OP, 2>), grid, block, 0, st, a);
    else if (need <= 4) hipLaunchKernelGGL((recur_kernel<OP, 4>), grid, block, 0, st, a);
    else if (need <= 8) hipLaunchKernelGGL((recur_kernel<OP, 8>), grid, block, 0, st, a);
    else if (need <= 16) hipLaunchKernelGGL((recur_kernel<OP, 16>), grid, block, 0, st, a);
    else if (need <= 32) hipLaunchKernelGGL((recur_kernel<OP, 32>), grid, block, 0, st, a);
    else if (OP == kArAdd || OP == kArRemoveInplace)
        hipLaunchKernelGGL((ar_naive_kernel<OP>), dim3((unsigned)((a.S + 255) / 256)), dim3(256), 0, st, a);
    else if (OP == kDiffInplace)
        hipLaunchKernelGGL(diff_chain_kernel, dim3((unsigned)((a.S * a.lag + 255) / 256)), dim3(256), 0, st,
                           a.out, a.S, a.T, a.ld_out, a.lag, a.start);
    else return hipErrorInvalidValue;
    return hipGetLastError();
}

}  // namespace

hipError_t launch_recur(RecurOp op, const RecurArgs& a, hipStream_t st) {
    if (a.S <= 0 || a.T <= 0) return hipSuccess;
    switch (op) {
    case kEwmaAdd: return launch_h<kEwmaAdd>(a, 1, st);
    case kEwmaRemoveInplace: return launch_h<kEwmaRemoveInplace>(a, 1, st);
    case kArAdd: return launch_h<kArAdd>(a, a.p, st);
    case kArRemoveInplace: return launch_h<kArRemoveInplace>(a, a.p, st);
    case kDiffInplace: return launch_h<kDiffInplace>(a, a.lag, st);
    case kFillDiffEwma:
        return launch_h<kFillDiffEwma>(a, a.lag, st);
    }
    return hipErrorInvalidValue;
}

hipError_t launch_diff_inplace(double* x, int64_t S, int64_t T, int64_t ld, int lag, int start,
                               hipStream_t st) {
    RecurArgs a{};
    a.in = x;
    a.out = x;
    a.S = S;
    a.T = T;
    a.ld_in = ld;
    a.ld_out = ld;
    a.lag = lag;
    a.start = start;
    return launch_recur(kDiffInplace, a, st);
}

}  // namespace sts
