// sts_garch_opt.hpp -- commons-math3 3.4.1's optimizer for GARCH.fitModel
// (S/models/GARCH.scala:33-53) as a resumable per-series state machine over a 3-D point
// (omega, alpha, beta).
//
//   NonLinearConjugateGradientOptimizer(FLETCHER_REEVES, SimpleValueChecker(1e-6, 1e-6))
//   optimize(ObjectiveFunction(logLikelihood), ObjectiveFunctionGradient(gradient),
//            InitialGuess(.2, .2, .2), MaxIter(10000), MaxEval(10000))      -- no GoalType
//
// No GoalType is passed, so getGoalType() is null and every `goal == MINIMIZE` branch of
// the optimizer, LineSearch, BracketFinder and BrentOptimizer is false: the gradient is used
// as is (ascent), BracketFinder compares with `>` and BrentOptimizer negates f internally
// and keeps the larger value in best().  These branches are restated literally, not as
// "minimise -f": BracketFinder's EPS_MIN guard is not sign-symmetric, so the two differ.
// The search direction restarts when iterations % 3 == 0 or the Fletcher-Reeves beta < 0.
//
// Same protocol as sts_ewma_opt.hpp: garch_advance(o) runs until the next evaluation whose
// point is not in the per-lane cache (o.status < 0, o.req holds the point) or the end
// (o.status >= 0).  The caller evaluates logLikelihood AND gradient at o.req into o.res_f /
// o.res_g, calls garch_cache_insert(o) and garch_advance(o) again.  Host + device: the
// device kernel (sts_garch.hip) is the product; the host build exists for the CPU test that
// checks the machine against the oracle's straight-line restatement.
#pragma once
#include "sts.h"

#if defined(__HIPCC__)
#define STS_HD __host__ __device__
#else
#define STS_HD
#endif

namespace sts {

constexpr int kGarchCache = 4;

struct GPv {
    double x, v;   // UnivariatePointValuePair
};

struct GarchOpt {
    double res_f, res_g[3];   // result of the request being resumed (logLikelihood, gradient)
    double req[3];            // requested point (omega, alpha, beta)
    int pc;                   // resume point (0 = start)
    int status;               // -1 running, else the final sts_status
    // NonLinearConjugateGradientOptimizer
    double point[3], dir[3], delta, cur_v, alpha;
    int have_cur, iter, evals;
    // BracketFinder
    int bev;
    double xA, xB, xC, fA, fB, fC, w, fW, wLim, tmp1, tmp2;
    // BrentOptimizer (f values negated internally, as isMinim == false does)
    double a, b, x, v, ww, d, e, fx, fv, fw, u, fu, m, tol1, tol2;
    GPv prev, cur, best;
    int have_prev;
    // evaluated points -> (logLikelihood, gradient)
    unsigned long long cs[kGarchCache][3];
    double cf[kGarchCache], cg[kGarchCache][3];
    int cn;
};

STS_HD inline unsigned long long gbits(double v) { return __builtin_bit_cast(unsigned long long, v); }

STS_HD inline void garch_init(GarchOpt& o) {
    o.pc = 0;
    o.status = -1;
    o.iter = 0;
    o.evals = 0;
    o.have_cur = 0;
    o.cn = 0;
    o.res_f = 0.0;
    o.res_g[0] = o.res_g[1] = o.res_g[2] = 0.0;
}

STS_HD inline bool garch_cache_lookup(GarchOpt& o) {
    const unsigned long long k0 = gbits(o.req[0]), k1 = gbits(o.req[1]), k2 = gbits(o.req[2]);
#pragma unroll
    for (int i = 0; i < kGarchCache; i++)
        if (i < o.cn && o.cs[i][0] == k0 && o.cs[i][1] == k1 && o.cs[i][2] == k2) {
            o.res_f = o.cf[i];
            o.res_g[0] = o.cg[i][0];
            o.res_g[1] = o.cg[i][1];
            o.res_g[2] = o.cg[i][2];
            return true;
        }
    return false;
}

STS_HD inline void garch_cache_insert(GarchOpt& o) {
    const int slot = o.cn < kGarchCache ? o.cn : (int)((gbits(o.req[0]) ^ gbits(o.req[1]) ^ gbits(o.req[2])) % kGarchCache);
#pragma unroll
    for (int i = 0; i < kGarchCache; i++)
        if (i == slot) {
            o.cs[i][0] = gbits(o.req[0]);
            o.cs[i][1] = gbits(o.req[1]);
            o.cs[i][2] = gbits(o.req[2]);
            o.cf[i] = o.res_f;
            o.cg[i][0] = o.res_g[0];
            o.cg[i][1] = o.res_g[1];
            o.cg[i][2] = o.res_g[2];
        }
    if (o.cn < kGarchCache) o.cn++;
}

// commons-math3 Precision.equals(x, y): within 1 ulp, NaN never equal
STS_HD inline bool g_equals(double x, double y) {
    const long long xi = (long long)gbits(x), yi = (long long)gbits(y);
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
STS_HD inline bool g_converged(double p, double c, double rel, double abs_) {
    const double diff = __builtin_fabs(p - c);
    const double size = __builtin_fmax(__builtin_fabs(p), __builtin_fabs(c));
    return diff <= size * rel || diff <= abs_;
}

// BrentOptimizer.best(a, b, isMinim = false)
STS_HD inline GPv g_best_max(const GPv& a, const GPv& b) { return (a.v >= b.v) ? a : b; }

constexpr double kGGold = 1.618034;
constexpr double kGEpsMin = 1e-21;
constexpr double kGBrentRel = 1e-15;
constexpr double kGBrentAbs = 4.9406564584124654e-324;

// Yield points: the request is point + t * dir (or the point itself); a cache hit falls
// straight through to the resume label.
#define STS_GREQ(t)                                                                         \
    o.req[0] = o.point[0] + (t) * o.dir[0];                                                 \
    o.req[1] = o.point[1] + (t) * o.dir[1];                                                 \
    o.req[2] = o.point[2] + (t) * o.dir[2];
#define STS_GYIELD()                                                                        \
    o.pc = __LINE__;                                                                        \
    if (!garch_cache_lookup(o)) return;                                                     \
    [[fallthrough]];                                                                        \
    case __LINE__:
#define STS_GFAIL(st)                                                                       \
    do {                                                                                    \
        o.status = (st);                                                                    \
        return;                                                                             \
    } while (0)
#define STS_GCOUNT()                                                                        \
    if (++o.evals > 10000) STS_GFAIL(STS_ERR_TOO_MANY_EVALUATIONS);
#define STS_GBCOUNT()                                                                       \
    if (++o.bev > 500) STS_GFAIL(STS_ERR_TOO_MANY_EVALUATIONS);                             \
    STS_GCOUNT()
#define STS_GAT(t)                                                                          \
    STS_GREQ(t)                                                                             \
    STS_GYIELD()

__attribute__((noinline)) STS_HD void garch_advance(GarchOpt& o) {
    switch (o.pc) {
    case 0:
        o.point[0] = .2;                                  // InitialGuess(Array(.2, .2, .2))
        o.point[1] = .2;
        o.point[2] = .2;
        o.req[0] = o.point[0];
        o.req[1] = o.point[1];
        o.req[2] = o.point[2];
        STS_GYIELD()                                      // computeObjectiveGradient (not counted)
        // goal != MINIMIZE: r = gradient; identity preconditioner: steepest = r
        o.dir[0] = o.res_g[0];
        o.dir[1] = o.res_g[1];
        o.dir[2] = o.res_g[2];
        o.delta = 0;
        o.delta += o.res_g[0] * o.dir[0];
        o.delta += o.res_g[1] * o.dir[1];
        o.delta += o.res_g[2] * o.dir[2];
        for (;;) {
            if (++o.iter > 10000) STS_GFAIL(STS_ERR_TOO_MANY_ITERATIONS);
            STS_GCOUNT()
            o.req[0] = o.point[0];                        // objective at the current point
            o.req[1] = o.point[1];
            o.req[2] = o.point[2];
            STS_GYIELD()
            if (o.have_cur && g_converged(o.cur_v, o.res_f, 1e-6, 1e-6)) {
                o.status = STS_OK;
                return;
            }
            o.have_cur = 1;
            o.cur_v = o.res_f;

            // ---- LineSearch: BracketFinder.search(f, null, 0, 1e-8) ----
            o.bev = 0;
            o.xA = 0.0;
            o.xB = 1e-8;
            STS_GBCOUNT()
            STS_GAT(o.xA)
            o.fA = o.res_f;
            STS_GBCOUNT()
            STS_GAT(o.xB)
            o.fB = o.res_f;
            if (o.fA > o.fB) {
                o.tmp1 = o.xA; o.xA = o.xB; o.xB = o.tmp1;
                o.tmp1 = o.fA; o.fA = o.fB; o.fB = o.tmp1;
            }
            o.xC = o.xB + kGGold * (o.xB - o.xA);
            STS_GBCOUNT()
            STS_GAT(o.xC)
            o.fC = o.res_f;
            while (o.fC > o.fB) {
                o.tmp1 = (o.xB - o.xA) * (o.fB - o.fC);
                o.tmp2 = (o.xB - o.xC) * (o.fB - o.fA);
                o.w = o.tmp2 - o.tmp1;                                           // val
                o.w = __builtin_fabs(o.w) < kGEpsMin ? 2 * kGEpsMin : o.w;       // denom
                o.w = o.xB - ((o.xB - o.xC) * o.tmp2 - (o.xB - o.xA) * o.tmp1) / (2 * o.w);
                o.wLim = o.xB + 100 * (o.xC - o.xB);
                if ((o.w - o.xC) * (o.xB - o.w) > 0) {
                    STS_GBCOUNT()
                    STS_GAT(o.w)
                    o.fW = o.res_f;
                    if (o.fW > o.fC) {
                        o.xA = o.xB; o.xB = o.w; o.fA = o.fB; o.fB = o.fW;
                        break;
                    } else if (o.fW < o.fB) {
                        o.xC = o.w; o.fC = o.fW;
                        break;
                    }
                    o.w = o.xC + kGGold * (o.xC - o.xB);
                    STS_GBCOUNT()
                    STS_GAT(o.w)
                    o.fW = o.res_f;
                } else if ((o.w - o.wLim) * (o.wLim - o.xC) >= 0) {
                    o.w = o.wLim;
                    STS_GBCOUNT()
                    STS_GAT(o.w)
                    o.fW = o.res_f;
                } else if ((o.w - o.wLim) * (o.xC - o.w) > 0) {
                    STS_GBCOUNT()
                    STS_GAT(o.w)
                    o.fW = o.res_f;
                    if (o.fW > o.fC) {
                        o.xB = o.xC; o.xC = o.w; o.w = o.xC + kGGold * (o.xC - o.xB);
                        o.fB = o.fC; o.fC = o.fW;
                        STS_GBCOUNT()
                        STS_GAT(o.w)
                        o.fW = o.res_f;
                    }
                } else {
                    o.w = o.xC + kGGold * (o.xC - o.xB);
                    STS_GBCOUNT()
                    STS_GAT(o.w)
                    o.fW = o.res_f;
                }
                o.xA = o.xB; o.fA = o.fB;
                o.xB = o.xC; o.fB = o.fC;
                o.xC = o.w; o.fC = o.fW;
            }
            if (o.xA > o.xC) {
                o.tmp1 = o.xA; o.xA = o.xC; o.xC = o.tmp1;
            }
            if (!(o.xA < o.xC) || !(o.xB >= o.xA && o.xB <= o.xC)) STS_GFAIL(STS_ERR_BAD_ARG);

            // ---- BrentOptimizer.doOptimize over [lo, hi] from mid, isMinim = false ----
            o.a = o.xA;
            o.b = o.xC;
            o.x = o.xB;
            o.v = o.x;
            o.ww = o.x;
            o.d = 0.0;
            o.e = 0.0;
            STS_GCOUNT()
            STS_GAT(o.x)
            o.fx = -o.res_f;
            o.fv = o.fx;
            o.fw = o.fx;
            o.cur.x = o.x;
            o.cur.v = -o.fx;
            o.best = o.cur;
            o.have_prev = 0;
            for (;;) {
                o.m = 0.5 * (o.a + o.b);
                o.tol1 = kGBrentRel * __builtin_fabs(o.x) + kGBrentAbs;
                o.tol2 = 2 * o.tol1;
                if (__builtin_fabs(o.x - o.m) <= o.tol2 - 0.5 * (o.b - o.a)) {
                    o.prev = o.have_prev ? g_best_max(o.prev, o.cur) : o.cur;
                    o.alpha = g_best_max(o.best, o.prev).x;
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
                STS_GCOUNT()
                STS_GAT(o.u)
                o.fu = -o.res_f;
                o.prev = o.cur;
                o.have_prev = 1;
                o.cur.x = o.u;
                o.cur.v = -o.fu;
                o.best = g_best_max(o.best, g_best_max(o.prev, o.cur));
                if (g_converged(o.prev.v, o.cur.v, 1e-8, 1e-8)) {
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
                    if (o.fu <= o.fw || g_equals(o.ww, o.x)) {
                        o.v = o.ww; o.fv = o.fw;
                        o.ww = o.u; o.fw = o.fu;
                    } else if (o.fu <= o.fv || g_equals(o.v, o.x) || g_equals(o.v, o.ww)) {
                        o.v = o.u; o.fv = o.fu;
                    }
                }
            }
            // point[i] += step * searchDirection[i]; r = gradient(point)
            o.point[0] = o.point[0] + o.alpha * o.dir[0];
            o.point[1] = o.point[1] + o.alpha * o.dir[1];
            o.point[2] = o.point[2] + o.alpha * o.dir[2];
            o.req[0] = o.point[0];
            o.req[1] = o.point[1];
            o.req[2] = o.point[2];
            STS_GYIELD()                                  // computeObjectiveGradient(point)
            {
                const double deltaOld = o.delta;
                double dl = 0;
                dl += o.res_g[0] * o.res_g[0];
                dl += o.res_g[1] * o.res_g[1];
                dl += o.res_g[2] * o.res_g[2];
                o.delta = dl;
                const double beta = o.delta / deltaOld;   // FLETCHER_REEVES
                if (o.iter % 3 == 0 || beta < 0) {
                    o.dir[0] = o.res_g[0];
                    o.dir[1] = o.res_g[1];
                    o.dir[2] = o.res_g[2];
                } else {
                    o.dir[0] = o.res_g[0] + beta * o.dir[0];
                    o.dir[1] = o.res_g[1] + beta * o.dir[1];
                    o.dir[2] = o.res_g[2] + beta * o.dir[2];
                }
            }
        }
    default:
        STS_GFAIL(STS_ERR_HIP);   // unreachable
    }
}
#undef STS_GREQ
#undef STS_GYIELD
#undef STS_GFAIL
#undef STS_GCOUNT
#undef STS_GBCOUNT
#undef STS_GAT

}  // namespace sts
