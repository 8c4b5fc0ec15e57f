// sts_tile2.hip -- ROLE-SPLIT variant of the C3 tile kernel (fill linear/... + ACF, K <= 60):
// the imputation work and the lag-product MFMAs of one workgroup run on different waves,
// on different tiles, at the same time.
//
// Reference operators: as sts_tile.hip (S/UnivariateTimeSeries.scala:68-93, 156-266).
//
// Why: in tile_kernel every wave does both jobs in sequence (load -> scan -> impute ->
// store + y -> MFMA), so a workgroup's MFMA phase and its memory / integer phases only
// overlap with OTHER workgroups' phases; FP64 MFMA is ~45 % of a tile's SIMD time and
// overlaps badly with the same SIMD's other work.  Here a 512-thread
// workgroup has 4 FILL waves and 4 MFMA waves and two LDS tile slots: while the fill waves
// load, impute, store and turn tile k+1 into y in one slot, the MFMA waves run the lag
// products of tile k from the other slot.  Both roles pass the same workgroup barriers
// (gfx950 has no named barriers); the MFMA waves' 16 chunks per tile are spread over the
// four fill intervals (STS_T2_C1..C3).  The fill code is tile_kernel's, statement for
// statement (bit-identical fills and partials: tested against both the oracle and
// tile_kernel).  2 workgroups per CU: 2 x 79 KB LDS, <= 128 VGPRs.
#include "sts_internal.hpp"

#include <hip/hip_runtime.h>

#ifndef STS_T2_WAVES_PER_EU
#define STS_T2_WAVES_PER_EU 2   // 2: one 512-thread workgroup per CU, 256 VGPRs; 4: two, 128 VGPRs
#endif

#ifndef STS_T2_C1
#define STS_T2_C1 6    // MFMA chunks done while the fill waves wait for / stage the tile
#endif
#ifndef STS_T2_C2
#define STS_T2_C2 7    // ... during the word scan
#endif
#ifndef STS_T2_C3
#define STS_T2_C3 11   // ... during the imputation; the rest during store + y
#endif

namespace sts {
namespace {

__device__ __forceinline__ void lds_barrier2() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

typedef double d4 __attribute__((ext_vector_type(4)));

constexpr int kFT = 256;          // fill threads (waves 0-3)
constexpr int kBig2 = 1 << 30;

__device__ __forceinline__ bool isnan2(double v) { return __builtin_isnan(v); }

__device__ __forceinline__ int64_t xcd_remap2(int64_t b, int64_t n) {
    int64_t q = n / 8, r = n % 8, x = b % 8;
    return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + b / 8;
}

__device__ __forceinline__ unsigned long long bitrep2(unsigned x) {
    unsigned long long r;
    asm("s_bitreplicate_b64_b32 %0, %1" : "=s"(r) : "s"(x));
    return r;
}
__device__ __forceinline__ unsigned long long interleave2b(unsigned ev, unsigned od) {
    return (bitrep2(ev) & 0x5555555555555555ull) | (bitrep2(od) & 0xAAAAAAAAAAAAAAAAull);
}

__device__ int64_t scan_back2(const double* src, int64_t from, int lane) {
    for (int64_t base = from - 64;; base -= 64) {
        int64_t t = base + lane;
        bool v = (t >= 0 && t < from) ? !isnan2(src[t]) : false;
        unsigned long long m = __ballot(v);
        if (m) return base + 63 - __clzll(m);
        if (base <= 0) return -1;
    }
}

__device__ int64_t scan_fwd2(const double* src, int64_t from, int64_t T, int lane) {
    for (int64_t base = from;; base += 64) {
        int64_t t = base + lane;
        bool v = (t < T) ? !isnan2(src[t]) : false;
        unsigned long long m = __ballot(v);
        if (m) return base + __ffsll(m) - 1;
        if (base + 64 >= T) return T;
    }
}

__device__ __forceinline__ int pxs(int q) { return q + ((q >> 5) << 2); }     // padded LDS index
__device__ __forceinline__ int px2s(int q2) { return q2 + ((q2 >> 4) << 1); }  // double2 index

template <int NT>
__global__ __launch_bounds__(512, STS_T2_WAVES_PER_EU) void tile2_kernel(TileArgs a, int method) {
    constexpr int TW = 4096;
    constexpr int EW = kHB + TW + kHA;
    constexpr int NA = 2;
    constexpr int QS = 16 / NT;
    constexpr int REACH = 80;
    constexpr int EWP = EW + EW / 8;
    constexpr int NW = EW / 64;
    constexpr int NP2 = EW / 2;
    constexpr int RPT = (NP2 + kFT - 1) / kFT;
    constexpr int CPW = TW / 64 / 4;             // chunks per MFMA wave per tile
    static_assert(NW <= 128 && RPT <= 9, "tile geometry");
    __shared__ __attribute__((aligned(16))) double vals[2][EWP];
    __shared__ unsigned long long mask[NW];
    __shared__ int lastUpTo[NW];
    __shared__ int firstFrom[NW];
    __shared__ int wbase[NW + 1];
    __shared__ unsigned long long wneed[NW];
    __shared__ int sh_i[3];
    __shared__ double sh_d[3];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const bool filler = wave < 4;
    const int mwave = wave - 4;
    const int64_t nchunk = a.S * a.chunks_per_series;
    const int64_t ch = xcd_remap2(blockIdx.x, nchunk);
    const int64_t s = ch / a.chunks_per_series;
    const int64_t cidx = ch - s * a.chunks_per_series;
    const int64_t k_begin = cidx * a.tiles_per_chunk;
    const int64_t k_end = (k_begin + a.tiles_per_chunk < a.tiles_per_series) ? k_begin + a.tiles_per_chunk
                                                                              : a.tiles_per_series;
    const int64_t T = a.T;
    const double* src = a.in + s * a.ld_in;
    const bool src_al = (reinterpret_cast<uintptr_t>(src) & 15) == 0;
    const bool needL = (method == STS_FILL_LINEAR || method == STS_FILL_PREVIOUS || method == STS_FILL_NEAREST);
    const bool needN = (method == STS_FILL_LINEAR || method == STS_FILL_NEXT || method == STS_FILL_NEAREST);
    double* dst = a.out ? a.out + s * a.ld_out : nullptr;

    // ACF shift c0 = F(0)
    if (wave == 0) {
        double x0 = src[0];
        if (method == STS_FILL_NEXT && isnan2(x0)) {
            const int64_t f = scan_fwd2(src, 0, T, lane);
            x0 = (f < T) ? src[f] : __builtin_nan("");
        }
        if (lane == 0) sh_d[0] = x0;
    }
    lds_barrier2();
    const double c0 = sh_d[0];
    lds_barrier2();

    double2 R0, R1, R2, R3, R4, R5, R6, R7, R8;
    auto interior = [&](int64_t kk) {
        const int64_t e0 = kk * TW - kHB;
        return e0 >= 0 && e0 + EW <= T && src_al;
    };
#define T2_LD1(j)                                                                           \
    if constexpr (j < RPT) {                                                                \
        const int q2_ = tid + j * kFT;                                                      \
        R##j = s2_[q2_ < NP2 ? q2_ : NP2 - 1];                                              \
    }
#define T2_ISSUE(kk)                                                                        \
    do {                                                                                    \
        const double2* s2_ = reinterpret_cast<const double2*>(src + ((kk) * TW - kHB));     \
        T2_LD1(0) T2_LD1(1) T2_LD1(2) T2_LD1(3) T2_LD1(4)                                   \
        T2_LD1(5) T2_LD1(6) T2_LD1(7) T2_LD1(8)                                             \
    } while (0)
#define T2_CLEAR()                                                                          \
    do {                                                                                    \
        R0 = R1 = R2 = R3 = R4 = R5 = R6 = R7 = R8 = make_double2(0.0, 0.0);                \
    } while (0)
#define T2_ST1(j)                                                                           \
    if constexpr (j < RPT) {                                                                \
        const int q2_ = tid + j * kFT;                                                      \
        if (q2_ < NP2) v2_[px2s(q2_)] = R##j;                                               \
    }

    // MFMA-wave state
    d4 U[NA];
#pragma unroll
    for (int t = 0; t < NA; t++) U[t] = d4{0.0, 0.0, 0.0, 0.0};
    double sy = 0.0;
    int oa[NT], ob[NT];
#pragma unroll
    for (int t = 0; t < NT; t++) {
        const int j = lane & 15;
        oa[t] = pxs(QS * t + lane);
        ob[t] = pxs(QS * t + 16 * (lane >> 4) + 16 * (j / QS) + (16 - QS) + (j % QS));
    }
    auto chunk_mfma = [&](const double* yb) {
        double av[NT], bv[NT];
#pragma unroll
        for (int t = 0; t < NT; t++) {
            av[t] = yb[oa[t]];
            bv[t] = yb[ob[t]];
        }
#pragma unroll
        for (int t = 0; t < NT; t++)
            U[t % NA] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[t], bv[t], U[t % NA], 0, 0, 0);
        sy += av[0];
    };
    // chunks [from, to) of this MFMA wave's share of the consumed tile kc
    auto mfma_part = [&](const double* cv, int64_t kc, int from, int to) {
        const int64_t t0c = kc * TW;
        const int64_t t1c = (t0c + TW < T) ? t0c + TW : T;
        const int nch = (int)((t1c - t0c + 63) / 64);
        int c = mwave * CPW + from;
        int cend = mwave * CPW + to;
        if (cend > nch) cend = nch;
        for (; c < cend; c++) chunk_mfma(cv + pxs(kHB + 64 * c));
    };

    bool series_err = false;
    bool have = false;
    if (filler) {
        have = interior(k_begin);
        if (have) T2_ISSUE(k_begin);
        else T2_CLEAR();
    }
    const int64_t ntile = k_end - k_begin;
    for (int64_t i = 0; i <= ntile; i++) {
        const int64_t k = k_begin + i;        // tile produced (filled) this step
        const int64_t kc = k - 1;             // tile consumed (MFMA) this step
        const bool produce = i < ntile;
        const bool consume = i > 0;
        double* vals_p = vals[i & 1];
        const double* vals_c = vals[(i + 1) & 1];
        const bool have_p = produce && interior(k);   // workgroup-uniform (== `have` on fill waves)
        const int t0 = (int)(k * TW);
        const int t1 = (t0 + TW < T) ? t0 + TW : (int)T;
        const int e0 = t0 - kHB;
        const int qA = kHB;
        const int qW = kHB + (t1 - t0);
        int qB = qW + REACH;
        if (e0 + qB > T) qB = (int)T - e0;
        const bool have_next = (k + 1 < k_end) && interior(k + 1);

        // ===== interval 1: tile k -> LDS (fill) | MFMA chunks [0, C1) of tile k-1 =====
        if (filler && produce) {
            if (have) {
                double2* v2_ = reinterpret_cast<double2*>(vals_p);
                T2_ST1(0) T2_ST1(1) T2_ST1(2) T2_ST1(3) T2_ST1(4) T2_ST1(5) T2_ST1(6) T2_ST1(7) T2_ST1(8)
#define T2_BAL1(j)                                                                          \
    if constexpr (j < RPT) {                                                                \
        const unsigned long long bx_ = __ballot(!isnan2(R##j.x));                           \
        const unsigned long long by_ = __ballot(!isnan2(R##j.y));                           \
        const int w_ = 2 * wave + 8 * j;                                                    \
        if (lane == 0) {                                                                    \
            if (w_ < NW) mask[w_] = interleave2b((unsigned)bx_, (unsigned)by_);             \
            if (w_ + 1 < NW) mask[w_ + 1] = interleave2b((unsigned)(bx_ >> 32), (unsigned)(by_ >> 32)); \
        }                                                                                   \
    }
                T2_BAL1(0) T2_BAL1(1) T2_BAL1(2) T2_BAL1(3) T2_BAL1(4) T2_BAL1(5) T2_BAL1(6) T2_BAL1(7)
                T2_BAL1(8)
#undef T2_BAL1
            } else {
                for (int q = tid; q < EW; q += kFT) {
                    const int t = e0 + q;
                    vals_p[pxs(q)] = (t >= 0 && t < T) ? src[t] : __builtin_nan("");
                }
            }
        }
        if (!filler && consume) {
            if (kc == 0 && mwave == 0) chunk_mfma(vals_c);   // pre-chunk: the series' first QS t steps
            mfma_part(vals_c, kc, 0, STS_T2_C1);
        }
        lds_barrier2();
        if (produce && !have_p) {   // edge tiles: ballots from LDS (workgroup-uniform branch)
            if (filler) {
#pragma unroll 2
                for (int ii = 0; ii < (NW + 3) / 4; ii++) {
                    const int w = wave + ii * 4;
                    if (w < NW) {
                        const unsigned long long m = __ballot(!isnan2(vals_p[pxs(w * 64 + lane)]));
                        if (lane == 0) mask[w] = m;
                    }
                }
            }
            lds_barrier2();
        }

        // ===== interval 2: word scans (fill wave 0) | MFMA chunks [C1, C2) =====
        if (filler && produce && wave == 0) {
            const int w0 = 2 * lane, w1 = 2 * lane + 1;
            const unsigned long long m0 = (w0 < NW) ? mask[w0] : ~0ull;
            const unsigned long long m1 = (w1 < NW) ? mask[w1] : ~0ull;
            const int l0 = (w0 < NW && m0) ? w0 * 64 + 63 - __clzll(m0) : -1;
            const int l1 = (w1 < NW && m1) ? w1 * 64 + 63 - __clzll(m1) : -1;
            const int f0 = (w0 < NW && m0) ? w0 * 64 + __ffsll(m0) - 1 : kBig2;
            const int f1 = (w1 < NW && m1) ? w1 * 64 + __ffsll(m1) - 1 : kBig2;
            auto need = [&](int w, unsigned long long m) -> unsigned long long {
                const int lo = qA - w * 64, hi = qB - w * 64;
                if (method == STS_FILL_NONE || hi <= 0 || lo >= 64) return 0ull;
                unsigned long long r = ~m;
                if (lo > 0) r &= ~0ull << lo;
                if (hi < 64) r &= (1ull << hi) - 1ull;
                return r;
            };
            const unsigned long long n0 = (w0 < NW) ? need(w0, m0) : 0ull;
            const unsigned long long n1 = (w1 < NW) ? need(w1, m1) : 0ull;
            int pm = l1 > l0 ? l1 : l0;
            int sm = f0 < f1 ? f0 : f1;
            int pc = __popcll(n0) + __popcll(n1);
#pragma unroll
            for (int d = 1; d < 64; d <<= 1) {
                const int o = __shfl_up(pm, d);
                const int c = __shfl_up(pc, d);
                const int u = __shfl_down(sm, d);
                if (lane >= d) { pm = o > pm ? o : pm; pc += c; }
                if (lane + d < 64) sm = u < sm ? u : sm;
            }
            int ex = __shfl_up(pm, 1);
            int exc = __shfl_up(pc, 1);
            int exs = __shfl_down(sm, 1);
            if (lane == 0) { ex = -1; exc = 0; }
            if (lane == 63) exs = kBig2;
            const int nnan = __shfl(pc, 63);
            const int firstValidE = __shfl(sm, 0);
            const int lastValidE = __shfl(pm, 63);
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
            int lext = -1, next = (int)T;
            if (needL && e0 > 0 && firstValidE > qA && nnan > 0) lext = (int)scan_back2(src, e0, lane);
            if (needN && e0 + EW < T && qB > qA && lastValidE < qB - 1 && nnan > 0)
                next = (int)scan_fwd2(src, e0 + EW, T, lane);
            if (lane == 0) {
                wbase[NW] = nnan;
                sh_i[0] = lext;
                sh_i[1] = next;
                sh_i[2] = nnan;
                sh_d[1] = (lext >= 0) ? src[lext] : 0.0;
                sh_d[2] = (next < T) ? src[next] : 0.0;
            }
        }
        if (!filler && consume) mfma_part(vals_c, kc, STS_T2_C1, STS_T2_C2);
        lds_barrier2();

        // ===== interval 3: impute the compacted NaN positions | MFMA chunks [C2, C3) =====
        if (filler && produce) {
            const int nnan = sh_i[2];
            const int lext = sh_i[0], next = sh_i[1];
            const double lextv = sh_d[1], nextv = sh_d[2];
            for (int idx = tid; idx < nnan; idx += kFT) {
                int lo = 0, hi = NW;
                while (hi - lo > 1) {
                    const int mid = (lo + hi) >> 1;
                    if (wbase[mid] <= idx) lo = mid;
                    else hi = mid;
                }
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
                    const unsigned long long lom = m & ((1ull << b) - 1ull);
                    const int Lq = lom ? w * 64 + 63 - __clzll(lom) : (w > 0 ? lastUpTo[w - 1] : -1);
                    if (Lq >= 0) { Lt = e0 + Lq; Lv = vals_p[pxs(Lq)]; }
                    else { Lt = lext; Lv = lextv; }
                }
                if (needN) {
                    const unsigned long long him = (b == 63) ? 0ull : (m & (~0ull << (b + 1)));
                    const int Nq = him ? w * 64 + __ffsll(him) - 1 : (w + 1 < NW ? firstFrom[w + 1] : kBig2);
                    if (Nq < kBig2) { Nt = e0 + Nq; Nv = vals_p[pxs(Nq)]; }
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
                    if (t == 0) break;
                    const int P = (Lt >= 1) ? Lt : -1;
                    if (P < 0 && Nt >= T) { series_err = true; break; }
                    f = (Nt >= T || (P >= 0 && t - P < Nt - t)) ? Lv : Nv;
                    break;
                }
                case STS_FILL_LINEAR: {
                    if (Lt < 0 || Nt >= T) break;
                    const double inc = (Nv - Lv) / (double)(Nt - Lt);
                    double r = Lv;
                    for (int j = t - Lt; j > 0; j--) r = r + inc;   // sequential, as :259-261
                    f = r;
                    break;
                }
                default:
                    break;
                }
                vals_p[pxs(q)] = f;
            }
        }
        if (!filler && consume) mfma_part(vals_c, kc, STS_T2_C2, STS_T2_C3);
        lds_barrier2();

        // ===== interval 4: filled output + y = F - c0 in place; next prefetch |
        //       MFMA chunks [C3, CPW) =====
        if (filler && produce) {
            const bool al = dst && ((reinterpret_cast<uintptr_t>(dst) & 15) == 0);
            double2* v2 = reinterpret_cast<double2*>(vals_p);
            const bool fast = (dst == nullptr || al) && (t1 - t0 == TW) && (e0 + qW + REACH <= T);
            if (fast) {
                constexpr int FS = TW / 2 / kFT;
                constexpr int FY = (NP2 - kHB / 2 + kFT - 1) / kFT;
                constexpr int FH = (FY + 1) / 2;
                const int vq = (kHB >> 1) + tid;
                const bool wr = dst != nullptr;
                double2* dp = reinterpret_cast<double2*>(dst + t0) + tid;
#pragma unroll
                for (int h = 0; h < 2; h++) {
                    double2 fv[FH];
#pragma unroll
                    for (int j = 0; j < FH; j++) {
                        const int jj = h * FH + j;
                        if (jj < FY && (jj * kFT + kFT <= NP2 - kHB / 2 || tid + jj * kFT < NP2 - kHB / 2))
                            fv[j] = v2[px2s(vq + jj * kFT)];
                    }
#pragma unroll
                    for (int j = 0; j < FH; j++) {
                        const int jj = h * FH + j;
                        if (jj >= FY) continue;
                        const bool in = jj * kFT + kFT <= NP2 - kHB / 2 || tid + jj * kFT < NP2 - kHB / 2;
                        if (jj < FS && wr) {
                            __builtin_nontemporal_store(fv[j].x, &dp[jj * kFT].x);
                            __builtin_nontemporal_store(fv[j].y, &dp[jj * kFT].y);
                        }
                        if (in) {
                            double2 y;
                            y.x = fv[j].x - c0;
                            y.y = fv[j].y - c0;
                            v2[px2s(vq + jj * kFT)] = y;
                        }
                    }
                }
            } else {
                for (int q2 = (qA >> 1) + tid; 2 * q2 < EW; q2 += kFT) {
                    const int q = 2 * q2;
                    double2 f = v2[px2s(q2)];
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
                    f.x = (q < qB) ? f.x - c0 : 0.0;
                    f.y = (q + 1 < qB) ? f.y - c0 : 0.0;
                    v2[px2s(q2)] = f;
                }
            }
            if (e0 < 0 && tid < kHB / 2) v2[px2s(tid)] = make_double2(0.0, 0.0);   // y = 0 before the series
            if (have_next) T2_ISSUE(k + 1);
            else T2_CLEAR();
            have = have_next;
        }
        if (!filler && consume) mfma_part(vals_c, kc, STS_T2_C3, CPW);
        lds_barrier2();
    }
#undef T2_ISSUE
#undef T2_LD1
#undef T2_ST1
#undef T2_CLEAR
    if (series_err && a.err) a.err[s] = STS_ERR_ALL_NAN;

    // ---- diagonal extraction by the MFMA waves: lane d accumulates lag d in a fixed order ----
    double* scr = &vals[0][0] + (filler ? 0 : mwave) * 256;
    double lagacc = 0.0;
    {
        d4 D = U[0];
#pragma unroll
        for (int t = 1; t < NA; t++) D += U[t];
        if (!filler) {
#pragma unroll
            for (int r = 0; r < 4; r++) scr[((lane >> 4) + 4 * r) * 16 + (lane & 15)] = D[r];
        }
        lds_barrier2();
        if (!filler) {
#pragma unroll
            for (int j = 0; j < 16; j++) {
                const int ii = 16 * (j / QS) + (16 - QS) + (j % QS) - lane;
                if (ii >= 0 && ii < 16) lagacc += scr[ii * 16 + j];
            }
        }
        lds_barrier2();
    }
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) sy += __shfl_xor(sy, d);
    double* wsum = &vals[0][0] + 4 * 256;
    if (!filler) {
        wsum[mwave * kPartStride + lane] = lagacc;
        if (lane == 0) wsum[mwave * kPartStride + 64] = sy;
    }
    lds_barrier2();
    if (wave == 4) {
        double* part = a.partials + ch * kPartStride;
        double tot = 0.0;
#pragma unroll
        for (int w = 0; w < 4; w++) tot += wsum[w * kPartStride + lane];
        part[lane] = tot;
        if (lane == 0) {
            double ts = 0.0;
#pragma unroll
            for (int w = 0; w < 4; w++) ts += wsum[w * kPartStride + 64];
            part[64] = ts;
        }
    }
}

}  // namespace

bool tile2_supported(int K, const TileArgs& a) {
    return K > 0 && K <= 60 && a.lagmat == nullptr && a.T < 0x7fff0000LL;
}

hipError_t launch_tile2(int method, const TileArgs& a, hipStream_t st) {
    const int64_t nchunk = a.S * a.chunks_per_series;
    if (nchunk <= 0) return hipSuccess;
    if (nchunk > 0x7fffffffLL) return hipErrorInvalidValue;
    dim3 grid((unsigned)nchunk), block(512);
    if (a.K <= 24) hipLaunchKernelGGL((tile2_kernel<2>), grid, block, 0, st, a, method);
    else hipLaunchKernelGGL((tile2_kernel<4>), grid, block, 0, st, a, method);
    return hipGetLastError();
}

}  // namespace sts
