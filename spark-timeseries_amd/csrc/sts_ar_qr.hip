// sts_ar_qr.hip -- the reference's own least-squares arithmetic for the AR fits that the fast
// fit kernels (sts_ar.hip) flag ("AR rule").
//
// Autoregression.fitModel (S/models/Autoregression.scala:38-53) solves the lag-design OLS with
// commons-math3 3.4.1 OLSMultipleLinearRegression: Householder QR of X^T (threshold 0), the
// reflections applied to y, back-substitution of R (restated statement by statement in
// oracle/sts_oracle.c, orc_ols_householder).  On a well-conditioned series the fast kernels'
// centred normal equations + refinement land within ~1e-12 of the exact solution and so within
// 1e-10 of the reference.  On an ill-conditioned one (a price level far above the series'
// spread, nearly collinear lags, an intercept that is a small difference of large means) the
// reference itself sits up to ~1e-5 from exact: matching it means repeating its roundings.
// The fit kernels therefore flag such series (ar_rule_flags in sts_ar.hip) into a list, and
// the kernels below recompute exactly those series with the reference's operation order:
// every sum sequential in row order, no contraction (-ffp-contract=off), correctly rounded
// sqrt and division -- the same bits as the oracle's restatement.
//
// ar_qr_lane_kernel<P, INT> (p <= 8): one flagged series per LANE, no scratch.  A column of
// the partly reduced design is never stored: its value at row r after reflection k is
//   c_j^(k)[r] = c_j^(k-1)[r] - alpha_j^(k) * c_k^(k-1)[r]       (r > k; y: + delta^(k) * ...)
// so each pass over the rows REPLAYS reflections 0..k-1 on the row's raw lag window, with
// the alpha / delta scalars of the earlier reflections in registers.  Per reflection k two
// sequential passes: the squared norm of pivot column k (its reflection vector), then the
// alpha / delta dot products of every later column and y.  R's rows and Q^T y are replayed
// again for the back-substitution (rows 0..NC-1 only).  Cost: ~250 flops per row and series
// for AR(5), no memory beyond the series.
//
// ar_qr_wave_kernel (any p <= 31): one flagged series per WAVE, lane j = column j (lane NC =
// y), the reduced design row-major in a global scratch slot, two passes per reflection (dot
// products, update + next pivot's norm), lane 0 back-substitutes.
#include "sts_internal.hpp"

#include <hip/hip_runtime.h>

#include <type_traits>

namespace sts {
namespace {

template <int I>
using IC = std::integral_constant<int, I>;

template <int B, int E, class F>
__device__ __forceinline__ void static_for(F&& f) {
    if constexpr (B < E) {
        f(IC<B>{});
        static_for<B + 1, E>(f);
    }
}

// descending: f(E-1), ..., f(B)
template <int B, int E, class F>
__device__ __forceinline__ void static_rfor(F&& f) {
    if constexpr (B < E) {
        f(IC<E - 1>{});
        static_rfor<B, E - 1>(f);
    }
}

template <int P, bool INT>
struct QrShape {
    static constexpr int NC = P + (INT ? 1 : 0);   // design columns (intercept first)
};

// the raw design row r from its lag window w[q] = x[r + q] (q = 0..P): the reference's
// row [1?, x(r+P-1), .., x(r)] (Lag.lagMatTrimBoth, S/Lag.scala:62-77), y = x(r + P)
template <int P, bool INT>
__device__ __forceinline__ void qr_row(const double (&w)[P + 1], double (&c)[QrShape<P, INT>::NC + 1]) {
    constexpr int NC = QrShape<P, INT>::NC;
    if constexpr (INT) {
        c[0] = 1.0;
#pragma unroll
        for (int j = 1; j <= P; j++) c[j] = w[P - j];
    } else {
#pragma unroll
        for (int j = 0; j < P; j++) c[j] = w[P - 1 - j];
    }
    c[NC] = w[P];
}

// raw values in flight per lane in a row sweep.  Measured on the all-flagged C4 shape
// (bench.py --workload c4_levels): 8 values at one wave per SIMD (256 VGPRs) 49.4 ms, 4 values at
// two waves per SIMD (251 VGPRs, __launch_bounds__(64, 2)) 57.8 ms -- the per-lane loads (64
// series, 64 cache lines per load instruction) bound it, not latency: more waves only thrash L1
constexpr int kQrPf = 8;

template <int P, bool INT>
__global__ __launch_bounds__(64) void ar_qr_lane_kernel(ArArgs a, const int64_t* __restrict__ list,
                                                        const uint32_t* __restrict__ count, int64_t n_direct) {
    constexpr int NC = QrShape<P, INT>::NC;
    const int64_t n = list ? (int64_t)*count : n_direct;
    const int64_t T = a.T;
    const int64_t m = T - P;
    for (int64_t base = (int64_t)blockIdx.x * 64; base < n; base += (int64_t)gridDim.x * 64) {
        const int64_t i = base + threadIdx.x;
        const bool act = i < n;
        // inactive lanes repeat the wave's first series and store nothing: the row loops stay
        // wave-uniform (every series of a call has the same T)
        const int64_t li = act ? i : base;
        const int64_t s = list ? list[li] : li;
        const double* xs = a.in + s * a.ld_in;
        auto ld = [&](int64_t t) -> double { return xs[t < T ? t : T - 1]; };

        // sweep(r0, body): body(r, w) for r = r0 .. m-1 with w[q] = x[r + q], the next kQrPf
        // raw values in flight while kQrPf rows are processed
        auto sweep = [&](int64_t r0, auto&& body) {
            double w[P + 1];
#pragma unroll
            for (int q = 0; q <= P; q++) w[q] = ld(r0 + q);
            double nx[kQrPf];
#pragma unroll
            for (int u = 0; u < kQrPf; u++) nx[u] = ld(r0 + P + 1 + u);
            for (int64_t r = r0; r < m; r += kQrPf) {
                double cur[kQrPf];
#pragma unroll
                for (int u = 0; u < kQrPf; u++) {
                    cur[u] = nx[u];
                    nx[u] = ld(r + kQrPf + P + 1 + u);
                }
#pragma unroll
                for (int u = 0; u < kQrPf; u++) {
                    if (r + u < m) {
                        body(r + u, w);
#pragma unroll
                        for (int q = 0; q < P; q++) w[q] = w[q + 1];
                        w[P] = cur[u];
                    }
                }
            }
        };

        double al[NC][NC];   // al[k][j]: alpha_j of reflection k (j > k)
        double dl[NC];       // delta of reflection k (applied to y)
        double ra[NC];       // rDiag = a_k
        double pv[NC];       // the modified pivot entry qrt[k][k] - a_k
        bool singular = false;

        // reflections 0 .. K-1 on a raw row (r > every k' < K), columns J0.. only where asked
        auto replay = [&](auto KK, double (&c)[NC + 1], auto JMAX) {
            constexpr int K = decltype(KK)::value;
            constexpr int JM = decltype(JMAX)::value;   // last column replayed (NC = with y)
            static_for<0, K>([&](auto kq) {
                constexpr int k = decltype(kq)::value;
                static_for<k + 1, (JM < NC ? JM + 1 : NC)>([&](auto jq) {
                    constexpr int j = decltype(jq)::value;
                    c[j] = c[j] - al[k][j] * c[k];
                });
                if constexpr (JM == NC) c[NC] = c[NC] + dl[k] * c[k];
            });
        };

        static_for<0, NC>([&](auto kq) {
            constexpr int k = decltype(kq)::value;
            // ---- squared norm of pivot column k over rows k..m-1 (sequential, row order) ----
            double ns = 0.0, ck = 0.0;
            if constexpr (INT && k == 0) {
                // the intercept column: 1.0 * 1.0 summed m times is exactly m
                ns = (double)m;
                ck = 1.0;
            } else {
                sweep(k, [&](int64_t r, const double (&w)[P + 1]) {
                    double c[NC + 1];
                    qr_row<P, INT>(w, c);
                    replay(IC<k>{}, c, IC<k>{});
                    if (r == k) ck = c[k];
                    ns = ns + c[k] * c[k];
                });
            }
            const double av = (ck > 0) ? -__builtin_sqrt(ns) : __builtin_sqrt(ns);
            ra[k] = av;
            singular = singular || (av == 0.0);
            pv[k] = ck - av;
            // ---- alpha_j (j > k) and delta: sequential dot products with the reflection vector ----
            {
                double acc[NC + 1];
#pragma unroll
                for (int j = 0; j <= NC; j++) acc[j] = 0.0;
                sweep(k, [&](int64_t r, const double (&w)[P + 1]) {
                    double c[NC + 1];
                    qr_row<P, INT>(w, c);
                    replay(IC<k>{}, c, IC<NC>{});
                    const double v = (r == k) ? pv[k] : c[k];
                    static_for<k + 1, NC>([&](auto jq) {
                        constexpr int j = decltype(jq)::value;
                        acc[j] = acc[j] - c[j] * v;
                    });
                    acc[NC] = acc[NC] + c[NC] * v;
                });
                const double den = av * pv[k];
                static_for<k + 1, NC>([&](auto jq) {
                    constexpr int j = decltype(jq)::value;
                    al[k][j] = acc[j] / den;
                });
                dl[k] = acc[NC] / den;
            }
        });

        // ---- back-substitution (Solver.solve): row i of R and of Q^T y replayed, rows NC-1 .. 0 ----
        double b[NC];
        static_rfor<0, NC>([&](auto iq) {
            constexpr int i = decltype(iq)::value;
            double w[P + 1];
#pragma unroll
            for (int q = 0; q <= P; q++) w[q] = ld(i + q);
            double c[NC + 1];
            qr_row<P, INT>(w, c);
            replay(IC<i>{}, c, IC<NC>{});
            // reflection i at its own pivot row uses the modified entry
            static_for<i + 1, NC>([&](auto jq) {
                constexpr int j = decltype(jq)::value;
                c[j] = c[j] - al[i][j] * pv[i];
            });
            c[NC] = c[NC] + dl[i] * pv[i];
            double yi = c[NC];
            static_rfor<i + 1, NC>([&](auto rq) {
                constexpr int row = decltype(rq)::value;
                yi = yi - b[row] * c[row];
            });
            b[i] = yi / ra[i];
        });

        if (act) {
            const double nan = __builtin_nan("");
            double cc = INT ? (singular ? nan : b[0]) : (singular ? nan : 0.0);
            a.c[s] = cc;
#pragma unroll
            for (int j = 0; j < P; j++) a.coef[s * P + j] = singular ? nan : b[(INT ? 1 : 0) + j];
            if (a.err) a.err[s] = singular ? STS_ERR_SINGULAR : STS_OK;
        }
        if (a.out) {
            // fused removeTimeDependentEffects with the reference's model, in its order
            // (S/models/Autoregression.scala:60-73)
            const double nan = __builtin_nan("");
            const double cc = singular ? nan : (INT ? b[0] : 0.0);
            double ph[P];
#pragma unroll
            for (int j = 0; j < P; j++) ph[j] = singular ? nan : b[(INT ? 1 : 0) + j];
            double* dst = a.out + s * a.ld_out;
            double xw[P + 1];   // xw[k] = x_{t-k}
#pragma unroll
            for (int k = 1; k <= P; k++) xw[k] = 0.0;
            constexpr int U = 16;   // raw values of the next 16 steps in flight
            double nx[U];
#pragma unroll
            for (int u = 0; u < U; u++) nx[u] = ld(u);
            for (int64_t t0 = 0; t0 < T; t0 += U) {
                double cur[U];
#pragma unroll
                for (int u = 0; u < U; u++) {
                    cur[u] = nx[u];
                    nx[u] = ld(t0 + U + u);
                }
#pragma unroll
                for (int u = 0; u < U; u++) {
                    const int64_t t = t0 + u;
                    if (t < T) {
                        const double xt = cur[u];
                        double d = xt - cc;
#pragma unroll
                        for (int j = 0; j < P; j++)
                            if (t - j - 1 >= 0) d = d - xw[j + 1] * ph[j];
#pragma unroll
                        for (int k = P; k >= 2; k--) xw[k] = xw[k - 1];
                        xw[1] = xt;
                        if (act) dst[t] = d;
                    }
                }
            }
        }
    }
}

// ---------------------------------------------------------------------------------------
// General p (<= 31): one wave per flagged series, lane j <-> design column j, lane NC <-> y.
// scr: the wave's slot of m x ldc doubles, row-major (a row = one design row: lanes read
// consecutive doubles).
__global__ __launch_bounds__(64) void ar_qr_wave_kernel(ArArgs a, const int64_t* __restrict__ list,
                                                        const uint32_t* __restrict__ count, int64_t n_direct,
                                                        double* __restrict__ scratch, int64_t slot_elems, int ldc) {
    const int64_t n = list ? (int64_t)*count : n_direct;
    const int lane = threadIdx.x;
    const int p = a.p;
    const bool INT = !a.no_intercept;
    const int NC = p + (INT ? 1 : 0);
    const int64_t T = a.T;
    const int64_t m = T - p;
    double* S = scratch + (int64_t)blockIdx.x * slot_elems;
    __shared__ double sh_a[64], sh_piv[64], sh_b[64], sh_ns;
    for (int64_t it = blockIdx.x; it < n; it += gridDim.x) {
        const int64_t s = list ? list[it] : it;
        const double* xs = a.in + s * a.ld_in;
        // ---- the raw design, row-major ----
        if (lane <= NC) {
            for (int64_t r = 0; r < m; r++) {
                double v;
                if (lane == NC) v = xs[r + p];
                else if (INT && lane == 0) v = 1.0;
                else v = xs[r + p - (lane + (INT ? 0 : 1))];
                S[r * ldc + lane] = v;
            }
        }
        __syncthreads();
        // norm of column 0
        if (lane == 0) {
            double ns = 0.0;
            for (int64_t r = 0; r < m; r++) {
                const double c = S[r * ldc];
                ns = ns + c * c;
            }
            sh_ns = ns;
        }
        __syncthreads();
        for (int k = 0; k < NC; k++) {
            const double ns = sh_ns;
            const double ck = S[(int64_t)k * ldc + k];
            const double av = (ck > 0) ? -__builtin_sqrt(ns) : __builtin_sqrt(ns);
            const double piv = ck - av;
            if (lane == 0) {
                sh_a[k] = av;
                sh_piv[k] = piv;
            }
            __syncthreads();
            if (lane == k) S[(int64_t)k * ldc + k] = piv;
            __syncthreads();
            if (av != 0.0) {
                // dot products: lane j > k (columns, then y)
                double acc = 0.0;
                const bool mine = lane > k && lane <= NC;
                if (mine) {
                    if (lane < NC) {
                        for (int64_t r = k; r < m; r++) acc = acc - S[r * ldc + lane] * S[r * ldc + k];
                    } else {
                        for (int64_t r = k; r < m; r++) acc = acc + S[r * ldc + lane] * S[r * ldc + k];
                    }
                    acc = acc / (av * piv);
                }
                __syncthreads();
                // update; lane k + 1 also sums its new squares from row k + 1 (next pivot's norm)
                double nn = 0.0;
                if (mine) {
                    for (int64_t r = k; r < m; r++) {
                        const double vr = S[r * ldc + k];
                        double e = S[r * ldc + lane];
                        e = (lane < NC) ? e - acc * vr : e + acc * vr;
                        S[r * ldc + lane] = e;
                        if (r > k) nn = nn + e * e;
                    }
                }
                if (lane == k + 1) sh_ns = nn;
                __syncthreads();
            } else {
                // no reflection (the reference skips it): the next norm from unchanged values
                if (lane == k + 1 && lane < NC) {
                    double nn = 0.0;
                    for (int64_t r = k + 1; r < m; r++) {
                        const double e = S[r * ldc + lane];
                        nn = nn + e * e;
                    }
                    sh_ns = nn;
                }
                __syncthreads();
            }
        }
        // ---- singular check + back-substitution (lane 0, the reference's order) ----
        if (lane == 0) {
            bool singular = false;
            for (int k = 0; k < NC; k++) singular = singular || (sh_a[k] == 0.0);   // |rDiag| <= 0
            double bb[32];
            double yy[32];
            for (int k = 0; k < NC; k++) yy[k] = S[(int64_t)k * ldc + NC];
            for (int row = NC - 1; row >= 0; --row) {
                yy[row] = yy[row] / sh_a[row];
                const double yr = yy[row];
                bb[row] = yr;
                for (int i2 = 0; i2 < row; i2++) yy[i2] = yy[i2] - yr * S[(int64_t)i2 * ldc + row];
            }
            const double nan = __builtin_nan("");
            a.c[s] = singular ? nan : (INT ? bb[0] : 0.0);
            for (int j = 0; j < p; j++) {
                sh_b[j] = singular ? nan : bb[(INT ? 1 : 0) + j];
                a.coef[s * p + j] = sh_b[j];
            }
            if (a.err) a.err[s] = singular ? STS_ERR_SINGULAR : STS_OK;
            sh_ns = singular ? nan : (INT ? bb[0] : 0.0);
        }
        __syncthreads();
        if (a.out) {
            // fused remove, in the reference's order, one step per lane
            const double cc = sh_ns;
            double* dst = a.out + s * a.ld_out;
            for (int64_t t = lane; t < T; t += 64) {
                double d = xs[t] - cc;
                for (int j = 0; j < p && t - j - 1 >= 0; j++) d = d - xs[t - j - 1] * sh_b[j];
                dst[t] = d;
            }
        }
        __syncthreads();
    }
}

}  // namespace

bool ar_qr_lane_ok(int p) { return p >= 1 && p <= 8; }

size_t ar_qr_wave_slot_elems(int64_t T, int p, int no_intercept) {
    const int NC = p + (no_intercept ? 0 : 1);
    const int ldc = (NC + 2) & ~1;
    return (size_t)(T - p) * (size_t)ldc;
}

hipError_t launch_ar_qr(const ArArgs& a, const int64_t* list, const uint32_t* count, int64_t n_direct,
                        double* scratch, int slots, bool force_wave, hipStream_t st) {
    if (a.S <= 0) return hipSuccess;
    if (ar_qr_lane_ok(a.p) && !force_wave) {
        // one lane per flagged series; the grid covers up to 64 * 1024 series per sweep
        const int64_t want = (a.S + 63) / 64;
        dim3 g((unsigned)(want < 1024 ? want : 1024)), b(64);
#define STS_QR_LANE(PP)                                                                              \
        case PP:                                                                                     \
            if (a.no_intercept) hipLaunchKernelGGL((ar_qr_lane_kernel<PP, false>), g, b, 0, st, a, list, count, n_direct); \
            else hipLaunchKernelGGL((ar_qr_lane_kernel<PP, true>), g, b, 0, st, a, list, count, n_direct);     \
            break;
        switch (a.p) {
            STS_QR_LANE(1) STS_QR_LANE(2) STS_QR_LANE(3) STS_QR_LANE(4)
            STS_QR_LANE(5) STS_QR_LANE(6) STS_QR_LANE(7) STS_QR_LANE(8)
        default: return hipErrorInvalidValue;
        }
#undef STS_QR_LANE
        return hipGetLastError();
    }
    if (!scratch || slots < 1) return hipErrorInvalidValue;
    const int NC = a.p + (a.no_intercept ? 0 : 1);
    const int ldc = (NC + 2) & ~1;
    hipLaunchKernelGGL(ar_qr_wave_kernel, dim3((unsigned)slots), dim3(64), 0, st, a, list, count, n_direct, scratch,
                       (int64_t)ar_qr_wave_slot_elems(a.T, a.p, a.no_intercept), ldc);
    return hipGetLastError();
}

}  // namespace sts
