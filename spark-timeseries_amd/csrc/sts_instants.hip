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
#include "sts_lanes.hpp"

#include <hip/hip_runtime.h>

#ifndef STS_TR16
#define STS_TR16 1                    // 16-B transpose when shapes allow
#endif
#ifndef STS_TR_NT
#define STS_TR_NT 1                   // non-temporal transpose stores (+2.5 %, r02_v10)
#endif
#ifndef STS_GATHER_BATCH
#define STS_GATHER_BATCH 1            // instant gather: batched loads before the stores
#endif
#ifndef STS_TR_XCD
#define STS_TR_XCD 1                  // transpose tiles XCD-contiguous (see transpose16_kernel)
#endif
#ifndef STS_NAN16
#define STS_NAN16 1                   // 16-B NaN-instant scan when shapes allow
#endif
#ifndef STS_STATS_FAST
#define STS_STATS_FAST 1              // seriesStats division off the step chain (see stats_fast_kernel)
#endif
#ifndef STS_STATS_CH
#define STS_STATS_CH 16               // seriesStats chunk (steps staged per series)
#endif
#ifndef STS_STATS_LA
#define STS_STATS_LA 1                // seriesStats chunks on 128-B line boundaries (stats_fast_kernel)
#endif

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

// Branch-free forms of jmax / jmin (same results, selects instead of early returns).
__device__ __forceinline__ double jmax_sel(double a, double b) {
    double r = (a >= b) ? a : b;
    r = (a == 0.0 && b == 0.0 && __builtin_signbit(a)) ? b : r;
    return (a != a) ? a : r;
}
__device__ __forceinline__ double jmin_sel(double a, double b) {
    double r = (a <= b) ? a : b;
    r = (a == 0.0 && b == 0.0 && __builtin_signbit(b)) ? b : r;
    return (a != a) ? a : r;
}

// The same StatCounter with the Welford division delta / n taken off the per-step chain.
// The compiler's IEEE f64 division is a Markstein sequence: y = 1/b refined by two Newton
// steps from v_rcp_f64 (a function of b alone), q0 = a y, r = fma(-b, q0, a), q = fma(r, y,
// q0), with v_div_scale / v_div_fmas / v_div_fixup scaling or patching only when the operands'
// exponents are extreme or a is 0 / inf / NaN.  b = n here is the step count, the same in
// every lane, so y(n) and -n for a chunk's steps are computed once into LDS (lane c: step
// c) and broadcast; a lane whose delta lies outside [2^-900, 2^700] (or is inf / NaN)
// takes the library division instead, so every quotient has the division's bits
// (tests/test_parity_gpu.py::test_series_stats* include the extreme and special values).
__device__ __forceinline__ double newton_rcp(double b) {
    double y = __builtin_amdgcn_rcp(b);
    double e = __builtin_fma(-b, y, 1.0);
    y = __builtin_fma(y, e, y);
    e = __builtin_fma(-b, y, 1.0);
    return __builtin_fma(y, e, y);
}

// LA (line-aligned chunks): the chunks of row r start at the 128-B line boundaries of ITS
// addresses, t = tc + col - off(r) with off(r) = (address of step 0 / 8) mod 16, so every
// staged row segment is whole L2 lines.  With chunks aligned on the series' steps
// instead, a row whose stride is not a multiple of 128 B (390 steps: 3 120 B) straddles two
// lines per chunk and the other half is evicted before the next chunk asks for it: 1.74x the
// panel's bytes fetched on 1M x 390 (profiles/r05_final_stats_traffic.json).  The per-step
// arithmetic and its order are unchanged (same bits); only which chunk a step is staged in moves.
template <int SPW, int CH, bool LA>
__global__ __launch_bounds__(64) void stats_fast_kernel(const double* __restrict__ in, double* __restrict__ out,
                                                        int64_t S, int64_t T, int64_t ld) {
    constexpr int kRow = CH + 1;
    constexpr int NLD = SPW * CH / 64;
    constexpr int kOff = LA ? CH - 1 : 0;   // largest lead-in of a row (doubles before its step 0)
    static_assert(CH + kOff <= 64, "one lane per step of the reciprocal table");
    static_assert(!LA || (CH % 16 == 0), "LA: a chunk row is whole 128-B lines");
    __shared__ double tile[SPW * kRow];
    __shared__ double ytab[CH + kOff], nbtab[CH + kOff];
    const int lane = threadIdx.x;
    const int64_t s0 = (int64_t)blockIdx.x * SPW;
    const bool live = lane < SPW && s0 + lane < S;
    const int ns = (S - s0 < SPW) ? (int)(S - s0) : SPW;
    const double* base = in + s0 * ld;
    // off(row) = (address of row's step 0 / 8) mod CH (only the low bits of row * ld matter)
    const unsigned o0 = (unsigned)(reinterpret_cast<uintptr_t>(base) >> 3), lm = (unsigned)ld;
    auto roff = [&](int row) -> int { return LA ? (int)((o0 + (unsigned)row * lm) & 15u) : 0; };
    int tend = (int)T;   // chunks run while some row of the wave still has steps: tc < T + max off
    if (LA) {
        int mo = live ? roff(lane) : 0;
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) {
            const int o = __shfl_xor(mo, d);
            mo = o > mo ? o : mo;
        }
        tend += mo;
    }
    if (T <= 0) tend = 0;   // empty series: no loads at all (the panel pointer may be null)
    double mu = 0.0, m2 = 0.0, mx = -__builtin_inf(), mn = __builtin_inf();
    // LA: 16-B loads of whole lines (8 lanes per row line): the doubles before step 0 / after
    // step T - 1 share a line with a step of the row (mapped memory: lines never cross pages)
    // and are never used; else element loads clamped into the row
    constexpr int NLQ = LA ? NLD / 2 : NLD;
    double2 pq[LA ? NLQ : 1];
    double pre[LA ? 1 : NLD];
    auto fetch = [&](int64_t tc) {   // no branches around the prefetch registers
#pragma unroll
        for (int i = 0; i < NLQ; i++) {
            if constexpr (LA) {
                const int row = (i * 64 + lane) / (CH / 2), cp = (i * 64 + lane) % (CH / 2);
                const int rr = row < ns ? row : ns - 1;
                const int o = roff(rr);
                // a pair past the row's last line (its steps ended, or the chunk's next line)
                // re-reads that line's last pair: never a line past the row (the panel's end
                // may be unmapped)
                const int64_t pl = ((T - 1 + o) | 15) - 1, pos = tc + 2 * cp;
                pq[i] = *reinterpret_cast<const double2*>(base + rr * ld - o + (pos < pl ? pos : pl));
            } else {
                const int row = (i * 64 + lane) / CH, col = (i * 64 + lane) % CH;
                const int rr = row < ns ? row : ns - 1;
                const int64_t cc = (tc + col < T) ? tc + col : T - 1;
                pre[i] = base[rr * ld + cc];
            }
        }
    };
    const int myoff = live ? roff(lane) : 0;
    auto step = [&](double v, double y, double nb) {
        const double delta = v - mu;            // StatCounter.merge(value)
        const double ad = __builtin_fabs(delta);
        const double q0 = delta * y;
        const double r = __builtin_fma(nb, q0, delta);
        double q = __builtin_fma(r, y, q0);
        q = (ad == 0.0) ? delta : q;            // 0 / n = 0 with the sign of delta
        if (!(ad == 0.0 || (ad >= 0x1p-900 && ad <= 0x1p700))) q = delta / (-nb);
        mu += q;
        m2 += delta * (v - mu);
        mx = jmax_sel(mx, v);
        mn = jmin_sel(mn, v);
    };
    if (tend > 0) fetch(0);
    for (int64_t tc = 0; tc < tend; tc += CH) {
#pragma unroll
        for (int i = 0; i < NLQ; i++) {
            if constexpr (LA) {
                const int row = (i * 64 + lane) / (CH / 2), cp = (i * 64 + lane) % (CH / 2);
                tile[row * kRow + 2 * cp] = pq[i].x;
                tile[row * kRow + 2 * cp + 1] = pq[i].y;
            } else {
                const int row = (i * 64 + lane) / CH, col = (i * 64 + lane) % CH;
                tile[row * kRow + col] = pre[i];
            }
        }
        if (lane < CH + kOff) {   // entry j: step count n = tc + j - kOff + 1 (unused where n < 1)
            const double n = (double)(tc + lane - kOff + 1);   // exact (T < 2^52)
            ytab[lane] = newton_rcp(n);
            nbtab[lane] = -n;
        }
        if (tc + CH < tend) fetch(tc + CH);
        __syncthreads();
        if (live) {
            const double* row = tile + lane * kRow;
            const double* yt = ytab + kOff - myoff;   // column c: step tc + c - off, entry c - off + kOff
            const double* nt = nbtab + kOff - myoff;
            // steps of this row in the chunk: columns [cs, ce) (all CH of them inside the series)
            const int cs = (myoff - tc > 0) ? (int)(myoff - tc) : 0;
            const int ce = (T - tc + myoff < CH) ? (int)(T - tc + myoff) : CH;
            for (int c = cs; c < ce; c++) step(row[c], yt[c], nt[c]);
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

// The same scan with 16-B loads (T and ld even, 16-B aligned panel): a lane tests two
// consecutive instants of each series, every load instruction covering 1 KB of a row.
__global__ __launch_bounds__(kNanT) void nan_instants16_kernel(const double* __restrict__ in, uint8_t* flags,
                                                               int64_t S, int64_t T, int64_t ld) {
    typedef double v2n __attribute__((ext_vector_type(2)));
    const int64_t t = 2 * ((int64_t)blockIdx.x * kNanT + threadIdx.x);
    const int64_t sa = (int64_t)blockIdx.y * kNanSeries;
    const int64_t sb = (sa + kNanSeries < S) ? sa + kNanSeries : S;
    if (t >= T) return;
    bool a0 = false, a1 = false;
    const double* p = in + sa * ld + t;
#pragma unroll 8
    for (int64_t s = sa; s < sb; s++, p += ld) {
        const v2n v = *reinterpret_cast<const v2n*>(p);
        a0 |= __builtin_isnan(v.x);
        a1 |= __builtin_isnan(v.y);
    }
    if (a0) flags[t] = 1;
    if (a1) flags[t + 1] = 1;
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

// out[s, j] = in[s, active[j]], j < n_active: one wave per series row (4 rows per block), so a
// short row (a few hundred kept instants) does not leave most of a 256-wide block idle
constexpr int kGatherRows = 4;
__global__ __launch_bounds__(64 * kGatherRows) void gather_instants_kernel(const double* __restrict__ in,
                                                                           double* __restrict__ out,
                                                                           const int64_t* __restrict__ active,
                                                                           int64_t n_active, int64_t S, int64_t ld_in,
                                                                           int64_t ld_out) {
    const int64_t s = (int64_t)blockIdx.x * kGatherRows + (threadIdx.x >> 6);
    if (s >= S) return;
    const double* src = in + s * ld_in;
    double* dst = out + s * ld_out;
    const int lane = threadIdx.x & 63;
    if (STS_GATHER_BATCH) {
        // 8 loads in flight per lane before the stores (512 kept instants per pass)
        for (int64_t j0 = 0; j0 < n_active; j0 += 512) {
            double v[8];
#pragma unroll
            for (int k = 0; k < 8; k++) {
                const int64_t j = j0 + lane + 64 * k;
                v[k] = src[active[j < n_active ? j : n_active - 1]];
            }
#pragma unroll
            for (int k = 0; k < 8; k++) {
                const int64_t j = j0 + lane + 64 * k;
                if (j < n_active) dst[j] = v[k];
            }
        }
    } else {
        for (int64_t j = lane; j < n_active; j += 64) dst[j] = src[active[j]];
    }
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

// The same with 16-B accesses (T, S, both leading dimensions even, 16-B aligned panels): a
// lane moves two consecutive instants of a series in and two consecutive series of an instant
// out, every load and store instruction covering 2 x 512 B.  The tile is kept t-major with
// an odd pitch, so the column reads of the store phase spread over the banks.
typedef double v2t __attribute__((ext_vector_type(2)));
constexpr int kTrPitch = 64 + 1;
// Tiles are XCD-contiguous (STS_TR_XCD): the instant tiles of one series block share the lines
// that straddle their boundaries (a 64-instant row segment of a 390-step row covers 5 lines for
// 4), so they run on one XCD and its L2 serves the shared line once; dispatched round-robin over
// the 8 XCDs (linear id x-fastest), the neighbours sat on different L2s and the panel was read
// 1.25 x (profiles/r05_final_to_instants_traffic.json).
__device__ __forceinline__ void tr_tile(int64_t& t0, int64_t& s0) {
    int64_t bx = blockIdx.x, by = blockIdx.y;
    if (STS_TR_XCD) {
        const int64_t nx = gridDim.x, b = xcd_remap(bx + by * nx, nx * (int64_t)gridDim.y);
        bx = b % nx;
        by = b / nx;
    }
    t0 = bx * 64;
    s0 = by * 64;
}
__global__ __launch_bounds__(256) void transpose16_kernel(const double* __restrict__ in, double* __restrict__ out,
                                                          int64_t S, int64_t T, int64_t ld_in, int64_t ld_out) {
    __shared__ double tile[64 * kTrPitch];   // tile[t * pitch + s]
    int64_t t0, s0;
    tr_tile(t0, s0);
    const int p = threadIdx.x & 31, r0 = threadIdx.x >> 5;   // pair p, row r0 + 8 i
    v2t v[8];
#pragma unroll
    for (int i = 0; i < 8; i++) {
        const int64_t s = s0 + r0 + 8 * i, t = t0 + 2 * p;
        v[i] = (s < S && t < T) ? *reinterpret_cast<const v2t*>(in + s * ld_in + t) : v2t{0.0, 0.0};
    }
#pragma unroll
    for (int i = 0; i < 8; i++) {
        const int sr = r0 + 8 * i;
        tile[(2 * p) * kTrPitch + sr] = v[i].x;
        tile[(2 * p + 1) * kTrPitch + sr] = v[i].y;
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 8; i++) {
        const int tr = r0 + 8 * i;
        const int64_t t = t0 + tr, s = s0 + 2 * p;
        if (s < S && t < T) {
            const v2t o = {tile[tr * kTrPitch + 2 * p], tile[tr * kTrPitch + 2 * p + 1]};
            if (STS_TR_NT) __builtin_nontemporal_store(o, reinterpret_cast<v2t*>(out + t * ld_out + s));
            else *reinterpret_cast<v2t*>(out + t * ld_out + s) = o;
        }
    }
}

}  // namespace

hipError_t launch_series_stats(const double* in, double* out, int64_t S, int64_t T, int64_t ld, hipStream_t st) {
    if (S <= 0) return hipSuccess;
    constexpr int SPW = 64, CH = STS_STATS_CH;   // A/B on 1M x 390: 1.00 ms vs 1.44 (32 x 64), 1.96 (16 x 64)
    if (STS_STATS_FAST && T < (1LL << 52))
        hipLaunchKernelGGL((stats_fast_kernel<SPW, CH, STS_STATS_LA != 0 && CH % 16 == 0>), dim3((unsigned)((S + SPW - 1) / SPW)), dim3(64), 0, st, in, out,
                           S, T, ld);
    else
        hipLaunchKernelGGL((stats_kernel<SPW, CH>), dim3((unsigned)((S + SPW - 1) / SPW)), dim3(64), 0, st, in, out, S,
                           T, ld);
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
    if (STS_NAN16 && T % 2 == 0 && ld % 2 == 0 && reinterpret_cast<uintptr_t>(in) % 16 == 0) {
        dim3 grid((unsigned)((T / 2 + kNanT - 1) / kNanT), (unsigned)gy);
        hipLaunchKernelGGL(nan_instants16_kernel, grid, dim3(kNanT), 0, st, in, flags, S, T, ld);
        return hipGetLastError();
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
    const int64_t nblk = (S + kGatherRows - 1) / kGatherRows;
    if (nblk > 0x7fffffffLL) return hipErrorInvalidValue;
    hipLaunchKernelGGL(gather_instants_kernel, dim3((unsigned)nblk), dim3(64 * kGatherRows), 0, st, in, out, active,
                       n_active, S, ld_in, ld_out);
    return hipGetLastError();
}

hipError_t launch_transpose(const double* in, double* out, int64_t S, int64_t T, int64_t ld_in, int64_t ld_out,
                            hipStream_t st) {
    if (S <= 0 || T <= 0) return hipSuccess;
    const bool v16 = STS_TR16 && (T % 2 == 0) && (S % 2 == 0) && (ld_in % 2 == 0) && (ld_out % 2 == 0) &&
                     (reinterpret_cast<uintptr_t>(in) % 16 == 0) && (reinterpret_cast<uintptr_t>(out) % 16 == 0);
    for (int64_t s = 0; s < S; s += 64LL * 65535) {
        const int64_t n = (S - s < 64LL * 65535) ? S - s : 64LL * 65535;
        dim3 grid((unsigned)((T + 63) / 64), (unsigned)((n + 63) / 64));
        if (v16)
            hipLaunchKernelGGL(transpose16_kernel, grid, dim3(256), 0, st, in + s * ld_in, out + s, n, T, ld_in, ld_out);
        else
            hipLaunchKernelGGL(transpose_kernel, grid, dim3(256), 0, st, in + s * ld_in, out + s, n, T, ld_in, ld_out);
    }
    return hipGetLastError();
}

}  // namespace sts
