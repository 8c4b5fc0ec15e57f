// sts_ewma_opt.hpp -- commons-math3 3.4.1's optimizer for EWMA.fitModel
// (S/models/EWMA.scala:44-68) as a resumable per-series state machine.
//
//   NonLinearConjugateGradientOptimizer(FLETCHER_REEVES, SimpleValueChecker(1e-6, 1e-6))
//   LineSearch = BracketFinder(growLimit 100, 500 evaluations) from [0, 1e-8], then
//                BrentOptimizer(1e-15, Double.MIN_VALUE, SimpleUnivariateValueChecker(1e-8, 1e-8))
//   InitialGuess 0.94, MaxIter 10000, MaxEval 10000
//
// ewma_advance(o) runs until the next sse / gradient request whose point is not in the
// small evaluation cache (o.req, o.status < 0) or until the optimizer ends (o.status >= 0).
// The caller evaluates EWMAModel.sse and .gradient at o.req, stores them in o.res_f /
// o.res_g, calls cache_insert(o) and ewma_advance(o) again.  Host + device: the device
// kernel (sts_ewma_fit.hip) is the product; the host build exists for the CPU test that
// checks the machine against the oracle's straight-line restatement.
#pragma once
#include "sts.h"

#if defined(__HIPCC__)
#define STS_HD __host__ __device__
#else
#define STS_HD
#endif

namespace sts {

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

STS_HD inline unsigned long long dbits(double v) { return __builtin_bit_cast(unsigned long long, v); }

STS_HD inline bool cache_lookup(EwmaOpt& o) {
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

STS_HD inline void cache_insert(EwmaOpt& o) {
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
STS_HD inline bool cm_equals(double x, double y) {
    const long long xi = (long long)dbits(x), yi = (long long)dbits(y);
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
STS_HD inline bool cm_converged(double p, double c, double rel, double abs_) {
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
__attribute__((noinline)) STS_HD void ewma_advance(EwmaOpt& o) {
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

}  // namespace sts
