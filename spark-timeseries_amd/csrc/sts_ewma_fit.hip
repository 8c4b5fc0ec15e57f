// sts_ewma_fit.hip -- EWMA.fitModel batched over a panel.
//
// Reference (S/ = src/main/scala/com/cloudera/sparkts/):
//   EWMA.fitModel            S/models/EWMA.scala:44-68
//   EWMAModel.sse            S/models/EWMA.scala:80-95
//   EWMAModel.gradient       S/models/EWMA.scala:102-123
//   addTimeDependentEffects  S/models/EWMA.scala:135-142 (the smoothed series both use)
// The optimizer is commons-math3 3.4.1 (pom.xml:396-400, not vendored):
//   NonLinearConjugateGradientOptimizer(FLETCHER_REEVES, SimpleValueChecker(1e-6, 1e-6)),
//   whose LineSearch is BracketFinder(growLimit 100, 500 evaluations) from [0, 1e-8]
//   followed by BrentOptimizer(1e-15, Double.MIN_VALUE, SimpleUnivariateValueChecker(1e-8,
//   1e-8)); InitialGuess 0.94, MaxIter / MaxEval 10000.  With one parameter the search
//   direction is reset to the steepest descent every iteration (iterations % n == 0).
//
// Device design: one LANE per series runs the optimizer as a resumable state machine
// (EwmaOpt below: every objective / gradient request is a yield point).  A wave owns SPW
// series; each round the wave streams its series block through LDS once (CH-step chunks,
// every load instruction = 64 consecutive steps of one series) and every lane with a
// pending request evaluates sse AND gradient of its own series at its own smoothing value
// in one sequential pass -- the reference's own operation order, so every evaluation is
// bit-exact and the optimizer takes the reference's path.  Rows of finished series are not
// loaded.  A small per-lane cache of evaluated points serves the optimizer's repeated
// requests (the objective at the point whose gradient was just computed, the line search's
// f(0)) without a pass; the evaluation COUNTERS still count them, as commons-math3 does.
// A series containing NaN (T >= 2) makes every sse NaN, so the reference's optimizer can
// only end in TooManyEvaluationsException: that is decided after the first pass.
#include "sts_internal.hpp"

#include <hip/hip_runtime.h>

namespace sts {
namespace {

struct Pv {
    double x, v;   // (Univariate)PointValuePair
};

constexpr int kCache = 4;

struct EwmaOpt {
    double res_f, res_g;   // result of the request being resumed (sse, gradient)
    double req;            // requested smoothing value
    int pc;                // resume point (0 = start)
    int status;            // -1 running, else the final sts_status
    // NonLinearConjugateGradientOptimizer
    double point, dir, cur_v, alpha;
    int have_cur, iter, evals;
    // BracketFinder
    int bev;
    double xA, xB, xC, fA, fB, fC, w, fW, wLim, tmp1, tmp2;
    // BrentOptimizer
    double a, b, x, v, ww, d, e, fx, fv, fw, u, fu, m, tol1, tol2;
    Pv prev, cur, best;
    int have_prev;
    // evaluated points (bit patterns of s) -> (sse, gradient)
    unsigned long long cs[kCache];
    double cf[kCache], cg[kCache];
    int cn;
};

__device__ __forceinline__ unsigned long long dbits(double v) {
    return (unsigned long long)__double_as_longlong(v);
}

__device__ __forceinline__ bool cache_lookup(EwmaOpt& o) {
    const unsigned long long k = dbits(o.req);
#pragma unroll
    for (int i = 0; i < kCache; i++)
        if (i < o.cn && o.cs[i] == k) {
            o.res_f = o.cf[i];
            o.res_g = o.cg[i];
            return true;
        }
    return false;
}

__device__ __forceinline__ void cache_insert(EwmaOpt& o) {
    const int slot = o.cn < kCache ? o.cn : (int)(dbits(o.req) % kCache);
#pragma unroll
    for (int i = 0; i < kCache; i++)
        if (i == slot) {
            o.cs[i] = dbits(o.req);
            o.cf[i] = o.res_f;
            o.cg[i] = o.res_g;
        }
    if (o.cn < kCache) o.cn++;
}

// commons-math3 Precision.equals(x, y): within 1 ulp, NaN never equal
__device__ bool cm_equals(double x, double y) {
    const long long xi = __double_as_longlong(x), yi = __double_as_longlong(y);
    const unsigned long long sgn = 0x8000000000000000ull;
    bool eq;
    if ((((unsigned long long)(xi ^ yi)) & sgn) == 0) {
        const long long dd = xi - yi;
        eq = (dd < 0 ? -dd : dd) <= 1;
    } else {
        long long dp, dm;
        if (xi < yi) {
            dp = yi;
            dm = (long long)((unsigned long long)xi - sgn);
        } else {
            dp = xi;
            dm = (long long)((unsigned long long)yi - sgn);
        }
        eq = (dp > 1) ? false : (dm <= 1 - dp);
    }
    return eq && !__builtin_isnan(x) && !__builtin_isnan(y);
}

// SimpleValueChecker / SimpleUnivariateValueChecker (no iteration limit)
__device__ __forceinline__ bool cm_converged(double p, double c, double rel, double abs_) {
    const double diff = __builtin_fabs(p - c);
    const double size = __builtin_fmax(__builtin_fabs(p), __builtin_fabs(c));
    return diff <= size * rel || diff <= abs_;
}

constexpr double kGold = 1.618034;       // BracketFinder.GOLD
constexpr double kEpsMin = 1e-21;        // BracketFinder.EPS_MIN
constexpr double kBrentRel = 1e-15;      // LineSearch.REL_TOL_UNUSED
constexpr double kBrentAbs = 4.9406564584124654e-324;   // LineSearch.ABS_TOL_UNUSED = Double.MIN_VALUE

// Yield points.  Each request stores the smoothing value and the resume label; a cache
// hit falls straight through to the label.  Counted requests (computeObjectiveValue) bump
// the MaxEval counter first; bracket requests also bump BracketFinder's own counter.
#define STS_YIELD(sv)                                                                       \
    o.req = (sv);                                                                           \
    o.pc = __LINE__;                                                                        \
    if (!cache_lookup(o)) return;                                                           \
    [[fallthrough]];                                                                        \
    case __LINE__:
#define STS_FAIL(st)                                                                        \
    do {                                                                                    \
        o.status = (st);                                                                    \
        return;                                                                             \
    } while (0)
#define STS_COUNT()                                                                         \
    if (++o.evals > 10000) STS_FAIL(STS_ERR_TOO_MANY_EVALUATIONS);
#define STS_BCOUNT()                                                                        \
    if (++o.bev > 500) STS_FAIL(STS_ERR_TOO_MANY_EVALUATIONS);                              \
    STS_COUNT()

// Runs lane o's optimizer until its next uncached request (o.status stays -1) or the end.
__device__ void ewma_advance(EwmaOpt& o) {
    switch (o.pc) {
    case 0:
        o.point = 0.94;                                   // InitialGuess(Array(.94))
        STS_YIELD(o.point)                                // computeObjectiveGradient (not counted)
        o.dir = -o.res_g;                                 // MINIMIZE: r = -g; identity preconditioner
        for (;;) {
            if (++o.iter > 10000) STS_FAIL(STS_ERR_TOO_MANY_ITERATIONS);
            STS_COUNT()
            STS_YIELD(o.point)                            // objective at the current point
            if (o.have_cur && cm_converged(o.cur_v, o.res_f, 1e-6, 1e-6)) {
                o.status = STS_OK;
                return;
            }
            o.have_cur = 1;
            o.cur_v = o.res_f;

            // ---- LineSearch: BracketFinder.search(f, MINIMIZE, 0, 1e-8) ----
            o.bev = 0;
            o.xA = 0.0;
            o.xB = 1e-8;
            STS_BCOUNT()
            STS_YIELD(o.point + o.xA * o.dir)
            o.fA = o.res_f;
            STS_BCOUNT()
            STS_YIELD(o.point + o.xB * o.dir)
            o.fB = o.res_f;
            if (o.fA < o.fB) {
                o.tmp1 = o.xA; o.xA = o.xB; o.xB = o.tmp1;
                o.tmp1 = o.fA; o.fA = o.fB; o.fB = o.tmp1;
            }
            o.xC = o.xB + kGold * (o.xB - o.xA);
            STS_BCOUNT()
            STS_YIELD(o.point + o.xC * o.dir)
            o.fC = o.res_f;
            while (o.fC < o.fB) {
                o.tmp1 = (o.xB - o.xA) * (o.fB - o.fC);
                o.tmp2 = (o.xB - o.xC) * (o.fB - o.fA);
                o.w = o.tmp2 - o.tmp1;                                          // val
                o.w = __builtin_fabs(o.w) < kEpsMin ? 2 * kEpsMin : o.w;        // denom
                o.w = o.xB - ((o.xB - o.xC) * o.tmp2 - (o.xB - o.xA) * o.tmp1) / (2 * o.w);
                o.wLim = o.xB + 100 * (o.xC - o.xB);
                if ((o.w - o.xC) * (o.xB - o.w) > 0) {
                    STS_BCOUNT()
                    STS_YIELD(o.point + o.w * o.dir)
                    o.fW = o.res_f;
                    if (o.fW < o.fC) {
                        o.xA = o.xB; o.xB = o.w; o.fA = o.fB; o.fB = o.fW;
                        break;
                    } else if (o.fW > o.fB) {
                        o.xC = o.w; o.fC = o.fW;
                        break;
                    }
                    o.w = o.xC + kGold * (o.xC - o.xB);
                    STS_BCOUNT()
                    STS_YIELD(o.point + o.w * o.dir)
                    o.fW = o.res_f;
                } else if ((o.w - o.wLim) * (o.wLim - o.xC) >= 0) {
                    o.w = o.wLim;
                    STS_BCOUNT()
                    STS_YIELD(o.point + o.w * o.dir)
                    o.fW = o.res_f;
                } else if ((o.w - o.wLim) * (o.xC - o.w) > 0) {
                    STS_BCOUNT()
                    STS_YIELD(o.point + o.w * o.dir)
                    o.fW = o.res_f;
                    if (o.fW < o.fC) {
                        o.xB = o.xC; o.xC = o.w; o.w = o.xC + kGold * (o.xC - o.xB);
                        o.fB = o.fC; o.fC = o.fW;
                        STS_BCOUNT()
                        STS_YIELD(o.point + o.w * o.dir)
                        o.fW = o.res_f;
                    }
                } else {
                    o.w = o.xC + kGold * (o.xC - o.xB);
                    STS_BCOUNT()
                    STS_YIELD(o.point + o.w * o.dir)
                    o.fW = o.res_f;
                }
                o.xA = o.xB; o.fA = o.fB;
                o.xB = o.xC; o.fB = o.fC;
                o.xC = o.w; o.fC = o.fW;
            }
            // lo = xA, mid = xB, hi = xC (swapped when lo > hi); SearchInterval validation
            if (o.xA > o.xC) {
                o.tmp1 = o.xA; o.xA = o.xC; o.xC = o.tmp1;
            }
            if (!(o.xA < o.xC) || !(o.xB >= o.xA && o.xB <= o.xC)) STS_FAIL(STS_ERR_BAD_ARG);

            // ---- BrentOptimizer.doOptimize over [lo, hi] from mid, MINIMIZE ----
            o.a = o.xA;
            o.b = o.xC;
            o.x = o.xB;
            o.v = o.x;
            o.ww = o.x;
            o.d = 0.0;
            o.e = 0.0;
            STS_COUNT()
            STS_YIELD(o.point + o.x * o.dir)
            o.fx = o.res_f;
            o.fv = o.fx;
            o.fw = o.fx;
            o.cur.x = o.x;
            o.cur.v = o.fx;
            o.best = o.cur;
            o.have_prev = 0;
            for (;;) {
                o.m = 0.5 * (o.a + o.b);
                o.tol1 = kBrentRel * __builtin_fabs(o.x) + kBrentAbs;
                o.tol2 = 2 * o.tol1;
                if (__builtin_fabs(o.x - o.m) <= o.tol2 - 0.5 * (o.b - o.a)) {
                    // best(best, best(previous, current))
                    o.prev = o.have_prev ? ((o.prev.v <= o.cur.v) ? o.prev : o.cur) : o.cur;
                    o.alpha = (o.best.v <= o.prev.v) ? o.best.x : o.prev.x;
                    break;
                }
                if (__builtin_fabs(o.e) > o.tol1) {   // fit parabola (p -> tmp1, q -> tmp2, r -> u)
                    o.u = (o.x - o.ww) * (o.fv - o.fx);
                    o.tmp2 = (o.x - o.v) * (o.fw - o.fx);
                    o.tmp1 = (o.x - o.v) * o.tmp2 - (o.x - o.ww) * o.u;
                    o.tmp2 = 2 * (o.tmp2 - o.u);
                    if (o.tmp2 > 0) o.tmp1 = -o.tmp1;
                    else o.tmp2 = -o.tmp2;
                    o.u = o.e;
                    o.e = o.d;
                    if (o.tmp1 > o.tmp2 * (o.a - o.x) && o.tmp1 < o.tmp2 * (o.b - o.x) &&
                        __builtin_fabs(o.tmp1) < __builtin_fabs(0.5 * o.tmp2 * o.u)) {
                        o.d = o.tmp1 / o.tmp2;
                        o.u = o.x + o.d;
                        if (o.u - o.a < o.tol2 || o.b - o.u < o.tol2) o.d = (o.x <= o.m) ? o.tol1 : -o.tol1;
                    } else {
                        o.e = (o.x < o.m) ? o.b - o.x : o.a - o.x;
                        o.d = (0.5 * (3 - __builtin_sqrt(5.0))) * o.e;
                    }
                } else {
                    o.e = (o.x < o.m) ? o.b - o.x : o.a - o.x;
                    o.d = (0.5 * (3 - __builtin_sqrt(5.0))) * o.e;
                }
                if (__builtin_fabs(o.d) < o.tol1) o.u = (o.d >= 0) ? o.x + o.tol1 : o.x - o.tol1;
                else o.u = o.x + o.d;
                STS_COUNT()
                STS_YIELD(o.point + o.u * o.dir)
                o.fu = o.res_f;
                o.prev = o.cur;
                o.have_prev = 1;
                o.cur.x = o.u;
                o.cur.v = o.fu;
                if (!(o.best.v <= ((o.prev.v <= o.cur.v) ? o.prev.v : o.cur.v)))
                    o.best = (o.prev.v <= o.cur.v) ? o.prev : o.cur;
                if (cm_converged(o.prev.v, o.cur.v, 1e-8, 1e-8)) {
                    o.alpha = o.best.x;
                    break;
                }
                if (o.fu <= o.fx) {
                    if (o.u < o.x) o.b = o.x;
                    else o.a = o.x;
                    o.v = o.ww; o.fv = o.fw;
                    o.ww = o.x; o.fw = o.fx;
                    o.x = o.u; o.fx = o.fu;
                } else {
                    if (o.u < o.x) o.a = o.u;
                    else o.b = o.u;
                    if (o.fu <= o.fw || cm_equals(o.ww, o.x)) {
                        o.v = o.ww; o.fv = o.fw;
                        o.ww = o.u; o.fw = o.fu;
                    } else if (o.fu <= o.fv || cm_equals(o.v, o.x) || cm_equals(o.v, o.ww)) {
                        o.v = o.u; o.fv = o.fu;
                    }
                }
            }
            o.point = o.point + o.alpha * o.dir;          // point[i] += step * searchDirection[i]
            STS_YIELD(o.point)                            // computeObjectiveGradient(point)
            o.dir = -o.res_g;                             // iterations % 1 == 0: steepest descent
        }
    default:
        STS_FAIL(STS_ERR_HIP);   // unreachable
    }
}
#undef STS_YIELD
#undef STS_FAIL
#undef STS_COUNT
#undef STS_BCOUNT

// One sequential pass of EWMAModel.sse (:80-95) and .gradient (:102-123) over chunk
// [c0, len) of a series row; state carried across chunks.  Statement order and operands
// are the reference's (no FMA: the library is built with -ffp-contract=off).
struct SseGrad {
    double sm, prevS, prevD, xprev, sq, dJ;
    bool bad;
    __device__ __forceinline__ void start(double x0) {
        sm = x0;       // smoothed(0) = ts(0)
        prevS = x0;    // prevSmoothed = ts(0)
        prevD = 0.0;
        xprev = x0;
        sq = 0.0;
        dJ = 0.0;
        bad = x0 != x0;
    }
    __device__ __forceinline__ void run(const double* row, int c0, int len, double s, double oms) {
        for (int c = c0; c < len; c++) {
            const double x = row[c];
            bad |= x != x;
            const double err = x - sm;               // ts(i + 1) - smoothed(i)
            sq += err * err;                         // sqrErrors += error * error
            const double dS = xprev - prevS + oms * prevD;   // ts(i) - prevSmoothed + (1 - s) * prevDSda
            dJ += err * dS;
            prevD = dS;
            prevS = sm;
            sm = s * x + oms * sm;                   // smoothed(i + 1)
            xprev = x;
        }
    }
};

// One wave = SPW series (lanes < SPW), CH-step chunks through LDS.  Each round every lane
// with a pending request evaluates sse and gradient at its own smoothing value; FIT = false
// is the plain sse / gradient operator (one round at smoothing[s]).
template <int SPW, int CH, bool FIT>
__global__ __launch_bounds__(64) void ewma_fit_kernel(EwmaFitArgs a) {
    constexpr int kRow = CH + 1;
    constexpr int NLD = SPW * CH / 64;
    static_assert(SPW * CH % 64 == 0 && CH % 64 == 0, "chunk shape");
    __shared__ double tile[SPW * kRow];
    const int lane = threadIdx.x;
    const int64_t s0 = (int64_t)blockIdx.x * SPW;
    const int64_t sl = s0 + lane;
    const bool live = lane < SPW && sl < a.S;
    const int ns = (a.S - s0 < SPW) ? (int)(a.S - s0) : SPW;
    const int64_t T = a.T;
    const double* base = a.in + s0 * a.ld;

    EwmaOpt o;
    o.pc = 0;
    o.status = -1;
    o.iter = 0;
    o.evals = 0;
    o.have_cur = 0;
    o.cn = 0;
    o.res_f = o.res_g = 0.0;
    if (FIT) {
        if (live) ewma_advance(o);
    } else {
        o.req = live ? a.smoothing[sl] : 0.0;
    }
    bool first = true;
    for (;;) {
        const bool pending = live && o.status < 0;
        const unsigned long long want = __ballot(pending);   // rows to stream this round
        if (want == 0) break;
        const double s = o.req, oms = 1.0 - s;
        SseGrad g;
        g.start(0.0);
        double pre[NLD];
        auto fetch = [&](int64_t tc) {
#pragma unroll
            for (int i = 0; i < NLD; i++) {
                const int row = (i * 64 + lane) / CH, col = (i * 64 + lane) % CH;
                const bool want_row = row < ns && ((want >> row) & 1ull);
                pre[i] = (want_row && tc + col < T) ? base[row * a.ld + tc + col] : 0.0;
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
            if (tc + CH < T) fetch(tc + CH);   // next chunk in flight during this one
            __syncthreads();
            if (pending) {
                const double* myrow = tile + lane * kRow;
                if (tc == 0) g.start(myrow[0]);
                g.run(myrow, tc == 0 ? 1 : 0, len, s, oms);
            }
            __syncthreads();
        }
        if (pending) {
            o.res_f = g.sq;
            o.res_g = 2 * g.dJ;
            if (!FIT) {
                o.status = STS_OK;
            } else if (first && g.bad && T >= 2) {
                o.status = STS_ERR_TOO_MANY_EVALUATIONS;   // every sse is NaN (see header)
            } else {
                cache_insert(o);
                ewma_advance(o);
            }
        }
        first = false;
    }
    if (!live) return;
    if (FIT) {
        a.smoothing[sl] = (o.status == STS_OK) ? o.point : __builtin_nan("");
        if (a.err) a.err[sl] = o.status;
        if (a.evals) a.evals[sl] = o.evals;
    } else {
        if (a.sse) a.sse[sl] = o.res_f;
        if (a.grad) a.grad[sl] = o.res_g;
    }
}

constexpr int kFitSpw = 32;
constexpr int kFitCh = 64;

}  // namespace

hipError_t launch_ewma_fit(const EwmaFitArgs& a, bool fit, hipStream_t st) {
    if (a.S <= 0) return hipSuccess;
    dim3 grid((unsigned)((a.S + kFitSpw - 1) / kFitSpw)), block(64);
    if (fit) hipLaunchKernelGGL((ewma_fit_kernel<kFitSpw, kFitCh, true>), grid, block, 0, st, a);
    else hipLaunchKernelGGL((ewma_fit_kernel<kFitSpw, kFitCh, false>), grid, block, 0, st, a);
    return hipGetLastError();
}

}  // namespace sts
