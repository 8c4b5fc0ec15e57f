// sts_recur.hip -- first-order and p-th order recurrences along time, one LANE per
// series, bit-exact by construction (the reference's own sequential order):
//   EWMAModel.addTimeDependentEffects     S/models/EWMA.scala:135-142
//   EWMAModel.removeTimeDependentEffects  S/models/EWMA.scala:125-133 (dest eq ts)
//   ARModel.addTimeDependentEffects       S/models/Autoregression.scala:75-88 (IIR)
//   ARModel.removeTimeDependentEffects    S/models/Autoregression.scala:60-73 (dest eq ts)
//   differencesAtLag                      S/UnivariateTimeSeries.scala:356-376 (dest eq ts)
//   C2 pipeline fillPrevious -> differencesAtLag(lag) -> EWMA add, fused (one HBM pass)
//
// A wave owns SPW series (64 by default; 32 for the fused C2 pipeline).  Time is processed
// in chunks of CH steps: the wave loads an SPW x CH block through LDS (each load
// instruction covers 64 consecutive steps of one series, 512 contiguous bytes; the next
// chunk's loads are in flight while the current chunk runs), transposes it (row stride
// CH+1 doubles: the per-lane row reads hit distinct banks), runs each lane's recurrence
// over the chunk in registers, and stores the block back the same way.  Measured on the C2
// shape (1M series x 390 steps): 64-step row segments beat 32 (1.68 vs 1.98 ms) and 128
// (2.86 ms); the series count per wave (16 / 32 / 64) hardly matters.
#include "sts_internal.hpp"
#include "sts_dma.hpp"

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
    // EWMA ops with the smoothing value already at hand (rows_kernel: from LDS, so that no
    // vector-memory load -- and no vmcnt wait behind the in-flight DMA -- sits in its loop)
    __device__ __forceinline__ void init_sm(const RecurArgs& a, double smv) {
        carry = __builtin_nan("");
        hp = a.lag;
        start = (OP == kFillDiffEwma) ? a.lag : a.start;
        e = 0.0;
#pragma unroll
        for (int j = 0; j < H; j++) {
            cf[j] = 0.0;
            h[j] = 0.0;
        }
        sm = smv;
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
    // rows padded to an even stride so the 16-B LDS accesses stay aligned, and = 2 mod 4
    // doubles so the 16 lanes' per-row 8-B reads hit distinct bank pairs.  (Round 4: 130-step
    // chunks -- three for C2's 390 steps instead of 3 x 128 + 6 -- ran 2.14 against 1.43 ms:
    // a 130-step row does not fill whole 128-double load instructions, so every instruction
    // then spans two rows; profiles/r04_v4_ab_c2.jsonl.)
    constexpr int kRow = V2 ? (CH % 4 == 2 ? CH : CH + 2) : CH + 1;
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

// Whole-row batches for panels stored row after row (ld == T): a batch of NS series is one
// contiguous span of the panel, so it moves in address order -- LDS-DMA in, 16-B stores out,
// every row read and written whole (the DRAM-page pattern of a straight copy; the chunk kernel
// above reads each row in ~1-KB pieces at different times).  One persistent 4-wave workgroup
// per CU double-buffers the batches in LDS: batch i+1 streams in while lanes 0..NS-1 of waves
// 0 and 1 run their series' recurrence over batch i in place and all four waves then store it.
// Every wave issues the same number of DMA pieces (kRowPcsW) and stores (kRowStW) per batch --
// tail lanes re-store the batch's last pair with its own bytes and tail pieces re-read
// in-bounds data into unused LDS -- so the wait for batch i is a constant vmcnt: the younger
// stores of batch i-1 and the pieces of batch i+1 stay in flight.  The last piece carries the
// batch's smoothing values (4-B DMA), so the loop holds no vector-memory load hipcc would wait
// for with a vmcnt(0) (that would also wait for the DMA in flight).
constexpr int kRowPcsW = 19;                       // DMA pieces (1 KB) per wave per batch
constexpr int kRowBufD = 4 * kRowPcsW * 128;       // doubles per buffer (76 KB): two fit one CU's LDS
constexpr int kRowSpan = kRowBufD - 128;           // panel part of a buffer; the last piece holds sm
constexpr int kRowStW = kRowSpan / 2 / 256 + 1;    // 16-B store rounds per thread per batch (19)
static_assert(kRowStW * 512 >= kRowSpan, "store rounds cover the span");
static_assert(kRowPcsW + kRowStW <= 63, "vmcnt field");

template <int N>
__device__ __forceinline__ void vm_wait() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }

template <int OP, int H>
__global__ __launch_bounds__(256, 1) void rows_kernel(RecurArgs a, int NS, int64_t nb) {
    __shared__ __attribute__((aligned(16))) double buf[2 * kRowBufD];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int64_t T = a.T;
    const int64_t last2 = a.S * T - 2;             // last in-bounds 16-B pair of the panel
    const int64_t G = gridDim.x;
    auto dma = [&](int64_t b, int slot) {          // batch b -> buffer slot (kRowPcsW pieces per wave)
        const double* src = a.in + b * NS * T;
        const int64_t room = last2 - b * NS * T;   // clamp: tail pieces re-read in-bounds bytes
        const unsigned base = lds_addr(buf + slot * kRowBufD);
#pragma unroll 1
        for (int j = 0; j < kRowPcsW; j++) {
            const int m = wave * kRowPcsW + j;
            if (m == 4 * kRowPcsW - 1) {
                // the last piece: smoothing of the batch's series (dwords 0 .. 2 NS - 1)
                const int64_t d = b * NS * 2 + (lane < 2 * NS ? lane : 0);
                const int64_t dl = 2 * a.S - 1;
                glds4(reinterpret_cast<const unsigned*>(a.sm) + (d < dl ? d : dl), base + (unsigned)(kRowSpan * 8));
            } else {
                int64_t q = (int64_t)m * 128 + 2 * lane;
                q = q < room ? q : room;
                glds16(src + q, base + (unsigned)(m << 10));
            }
        }
    };
    int64_t b = blockIdx.x;
    if (b >= nb) return;
    dma(b, 0);
    bool next_issued = b + G < nb;
    if (next_issued) dma(b + G, 1);
    for (int it = 0; b < nb; it++, b += G) {
        const int slot = it & 1;
        // batch b has landed: younger are this wave's stores of the previous batch (it > 0) and
        // the pieces of batch b + G (if issued)
        if (it > 0) {
            if (next_issued) vm_wait<kRowStW + kRowPcsW>();
            else vm_wait<kRowStW>();
        } else {
            if (next_issued) vm_wait<kRowPcsW>();
            else vm_wait<0>();
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
        const int nsb = (int)((a.S - b * NS < NS) ? a.S - b * NS : NS);   // series in this batch
        double* bb = buf + slot * kRowBufD;
        // recurrence: series j of the batch on lane j / 3 of wave j % 3 (waves 0..2: each step is a
        // dependent FP64 chain, so three waves on three SIMDs instead of one); the row moves
        // through registers 16 steps at a time, the next 16 read before the current ones run
        // (an LDS round trip per step cost ~100 cycles: 2.98 against 1.42 ms on C2)
        if (wave < 3) {
            const int j = lane * 3 + wave;
            if (j < nsb) {
                RecurLane<OP, H> rl;
                rl.init_sm(a, bb[kRowSpan + j]);
                double2* row = reinterpret_cast<double2*>(bb + (int64_t)j * T);
                const int np = (int)(T >> 1);          // pairs (T even)
                const int nblk = np >> 3;
                double2 cur[8];
                if (nblk > 0) {
#pragma unroll
                    for (int i = 0; i < 8; i++) cur[i] = row[i];
                }
                for (int bk = 0; bk < nblk; bk++) {
                    double2 nxt[8];
                    const bool more = bk + 1 < nblk;
                    if (more) {
#pragma unroll
                        for (int i = 0; i < 8; i++) nxt[i] = row[(bk + 1) * 8 + i];
                    }
                    const int64_t t0 = (int64_t)bk * 16;
                    if (bk == 0) {   // steady_from() <= 8 (H, lag <= 8)
#pragma unroll
                        for (int i = 0; i < 8; i++) {
                            cur[i].x = rl.step(cur[i].x, t0 + 2 * i);
                            cur[i].y = rl.step(cur[i].y, t0 + 2 * i + 1);
                        }
                    } else {
#pragma unroll
                        for (int i = 0; i < 8; i++) {
                            cur[i].x = rl.template step<true>(cur[i].x, t0 + 2 * i);
                            cur[i].y = rl.template step<true>(cur[i].y, t0 + 2 * i + 1);
                        }
                    }
#pragma unroll
                    for (int i = 0; i < 8; i++) row[bk * 8 + i] = cur[i];
                    if (more) {
#pragma unroll
                        for (int i = 0; i < 8; i++) cur[i] = nxt[i];
                    }
                }
                for (int p2 = nblk * 8; p2 < np; p2++) {
                    double2 v = row[p2];
                    v.x = rl.step(v.x, 2 * (int64_t)p2);
                    v.y = rl.step(v.y, 2 * (int64_t)p2 + 1);
                    row[p2] = v;
                }
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
        // store the batch: kRowStW 16-B rounds per thread, tail lanes repeat the last pair
        {
            const int64_t np = (int64_t)nsb * T / 2;
            double2* dst = reinterpret_cast<double2*>(a.out + b * NS * T);
            const double2* src2 = reinterpret_cast<const double2*>(bb);
#pragma unroll
            for (int r = 0; r < kRowStW; r++) {
                int64_t p = (int64_t)r * 256 + tid;
                p = p < np ? p : np - 1;
                dst[p] = src2[p];
            }
        }
        // every LDS read of this slot is done before any wave refills it
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
        next_issued = b + 2 * G < nb;
        if (next_issued) dma(b + 2 * G, slot);
    }
}

// rows_kernel applies: a row-contiguous 16-B aligned panel (ld == T, T even) of rows short
// enough for 8+ series per batch
inline int rows_ns(const RecurArgs& a) {
    if (a.ld_in != a.T || a.ld_out != a.T || (a.T & 1) || a.T < 2) return 0;
    if (((reinterpret_cast<uintptr_t>(a.in) | reinterpret_cast<uintptr_t>(a.out)) & 15) != 0) return 0;
    int64_t ns = kRowSpan / a.T;
    if (ns > 32) ns = 32;                    // the smoothing piece holds 64 dwords (and 3 x 11 lanes compute)
    return ns >= 8 ? (int)ns : 0;
}

inline int cu_count() {
    static int n[64] = {0};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
    if (n[dev] <= 0) {
        int v = 0;
        if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0) v = 256;
        n[dev] = v;
    }
    return n[dev];
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
#ifdef STS_ROWS
    // the fused C2 pipeline on row-contiguous panels: whole-row batches (rows_kernel)
    if constexpr (OP == kFillDiffEwma) if (need <= 8) {
        const int ns = rows_ns(a);
        if (ns > 0) {
            const int64_t nb = (a.S + ns - 1) / ns;
            const int64_t g = nb < cu_count() ? nb : cu_count();
            dim3 grid((unsigned)g), block(256);
            if (need <= 1) hipLaunchKernelGGL((rows_kernel<OP, 1>), grid, block, 0, st, a, ns, nb);
            else if (need <= 2) hipLaunchKernelGGL((rows_kernel<OP, 2>), grid, block, 0, st, a, ns, nb);
            else if (need <= 4) hipLaunchKernelGGL((rows_kernel<OP, 4>), grid, block, 0, st, a, ns, nb);
            else hipLaunchKernelGGL((rows_kernel<OP, 8>), grid, block, 0, st, a, ns, nb);
            return hipGetLastError();
        }
    }
#endif
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
