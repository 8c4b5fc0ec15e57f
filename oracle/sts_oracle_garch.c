/*
 * sts_oracle_garch.c -- CPU restatement of GARCH(1,1) and AR(1)+GARCH(1,1)
 * (S/models/GARCH.scala) for SURVEY.md §8(f) rank 1 ("ARGARCH reuse of AR fit").
 *
 * TEST INFRASTRUCTURE ONLY (see sts_oracle.h): the parity checker and the CPU
 * baseline.  Nothing in the shipped library links or calls this file.
 *
 *   GARCH.fitModel                 S/models/GARCH.scala:33-53
 *   ARGARCH.fitModel               S/models/GARCH.scala:62-68
 *   GARCHModel.logLikelihood       S/models/GARCH.scala:80-86
 *   GARCHModel.gradient            S/models/GARCH.scala:94-114 (returns the components in
 *                                  the order alpha, beta, omega while the optimizer's
 *                                  point is (omega, alpha, beta): kept, it is the code)
 *   iterateWithHAndEta             S/models/GARCH.scala:116-128
 *   GARCHModel.remove/add          S/models/GARCH.scala:130-159
 *   ARGARCHModel.remove/add        S/models/GARCH.scala:203-234
 *
 * The optimizer is commons-math3 3.4.1 (pom.xml:396-400; not vendored, restated from its
 * published algorithm): NonLinearConjugateGradientOptimizer(FLETCHER_REEVES,
 * SimpleValueChecker(1e-6, 1e-6)) called WITHOUT a GoalType, so getGoalType() is null and
 * every `goal == MINIMIZE` test is false: the gradient is not negated, BracketFinder and
 * BrentOptimizer run their maximising branches.  Written here literally in that form (the
 * device state machine is a separate restatement; tests compare the two).
 *
 * math.log: the JVM's Math.log may differ from StrictMath.log (fdlibm e_log.c) in the last
 * ulp; this restatement uses fdlibm's algorithm (orc_fdlibm_log), as the device does, so
 * device and oracle agree bit for bit.  Parity with a HotSpot Math.log intrinsic is
 * therefore unpinned at the ulp level (no JVM here).
 */
#include "sts_oracle.h"

#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* fdlibm 5.3 e_log.c (__ieee754_log) == java.lang.StrictMath.log */
double orc_fdlibm_log(double x) {
    const double ln2_hi = 6.93147180369123816490e-01, ln2_lo = 1.90821492927058770002e-10,
                 two54 = 1.80143985094819840000e+16, Lg1 = 6.666666666666735130e-01,
                 Lg2 = 3.999999999940941908e-01, Lg3 = 2.857142874366239149e-01,
                 Lg4 = 2.222219843214978396e-01, Lg5 = 1.818357216161805012e-01,
                 Lg6 = 1.531383769920937332e-01, Lg7 = 1.479819860511658591e-01;
    const double zero = 0.0;
    uint64_t b;
    memcpy(&b, &x, 8);
    int32_t hx = (int32_t)(b >> 32);
    const uint32_t lx = (uint32_t)b;
    int32_t k = 0;
    if (hx < 0x00100000) {                                   /* x < 2**-1022 */
        if (((hx & 0x7fffffff) | (int32_t)lx) == 0) return -two54 / zero;   /* log(+-0) = -inf */
        if (hx < 0) return (x - x) / zero;                   /* log(-#) = NaN */
        k -= 54;
        x *= two54;                                          /* subnormal: scale up */
        memcpy(&b, &x, 8);
        hx = (int32_t)(b >> 32);
    }
    if (hx >= 0x7ff00000) return x + x;
    k += (hx >> 20) - 1023;
    hx &= 0x000fffff;
    int32_t i = (hx + 0x95f64) & 0x100000;
    b = ((uint64_t)(uint32_t)(hx | (i ^ 0x3ff00000)) << 32) | (b & 0xffffffffull);   /* x or x/2 */
    memcpy(&x, &b, 8);
    k += (i >> 20);
    const double f = x - 1.0;
    if ((0x000fffff & (2 + hx)) < 3) {                       /* |f| < 2**-20 */
        if (f == zero) {
            if (k == 0) return zero;
            const double dk = (double)k;
            return dk * ln2_hi + dk * ln2_lo;
        }
        const double R = f * f * (0.5 - 0.33333333333333333 * f);
        if (k == 0) return f - R;
        const double dk = (double)k;
        return dk * ln2_hi - ((R - dk * ln2_lo) - f);
    }
    const double s = f / (2.0 + f);
    const double dk = (double)k;
    const double z = s * s;
    i = hx - 0x6147a;
    const double w = z * z;
    const int32_t j = 0x6b851 - hx;
    const double t1 = w * (Lg2 + w * (Lg4 + w * Lg6));
    const double t2 = z * (Lg1 + w * (Lg3 + w * (Lg5 + w * Lg7)));
    i |= j;
    const double R = t2 + t1;
    if (i > 0) {
        const double hfsq = 0.5 * f * f;
        if (k == 0) return f - (hfsq - s * (hfsq + R));
        return dk * ln2_hi - ((hfsq - (s * (hfsq + R) + dk * ln2_lo)) - f);
    }
    if (k == 0) return f - s * (f - R);
    return dk * ln2_hi - ((s * (f - R) - dk * ln2_lo) - f);
}

/* GARCHModel.logLikelihood (:80-86) over iterateWithHAndEta (:116-128) */
double orc_garch_loglik(const double* ts, int64_t n, double omega, double alpha, double beta) {
    double sum = 0.0;
    double prevH = omega / (1 - alpha - beta);
    for (int64_t i = 1; i < n; i++) {
        const double h = omega + alpha * ts[i - 1] * ts[i - 1] + beta * prevH;
        const double eta = ts[i];
        sum += -.5 * orc_fdlibm_log(h) - .5 * eta * eta / h;
        prevH = h;
    }
    return sum + -.5 * orc_fdlibm_log(2 * 3.141592653589793 /* Math.PI */) * (double)(n - 1);
}

/* GARCHModel.gradient (:94-114): g = [alpha, beta, omega] components, each * .5 */
void orc_garch_gradient(const double* ts, int64_t n, double omega, double alpha, double beta,
                        double g[3]) {
    double omegaGradient = 0.0, alphaGradient = 0.0, betaGradient = 0.0;
    double omegaDhdtheta = 0.0, alphaDhdtheta = 0.0, betaDhdtheta = 0.0;
    double prevH = omega / (1 - alpha - beta);
    for (int64_t i = 1; i < n; i++) {
        const double h = omega + alpha * ts[i - 1] * ts[i - 1] + beta * prevH;
        const double eta = ts[i], prevEta = ts[i - 1];
        omegaDhdtheta = 1 + beta * omegaDhdtheta;
        alphaDhdtheta = prevEta * prevEta + beta * alphaDhdtheta;
        betaDhdtheta = prevH + beta * betaDhdtheta;
        const double multiplier = (eta * eta / (h * h)) - (1 / h);
        omegaGradient += multiplier * omegaDhdtheta;
        alphaGradient += multiplier * alphaDhdtheta;
        betaGradient += multiplier * betaDhdtheta;
        prevH = h;
    }
    g[0] = alphaGradient * .5;
    g[1] = betaGradient * .5;
    g[2] = omegaGradient * .5;
}

/* ---------------- commons-math3 3.4.1, goal == null (maximising branches) ---------------- */

typedef struct { double x, v; } gpv_t;
typedef struct { const double* ts; int64_t n; int64_t evals; int too_many; } garch_obj_t;

/* main optimizer's computeObjectiveValue: MaxEval(10000) */
static double garch_value(garch_obj_t* o, const double p[3]) {
    if (++o->evals > 10000) o->too_many = 1;
    return o->too_many ? NAN : orc_garch_loglik(o->ts, o->n, p[0], p[1], p[2]);
}

static int prec_equals(double x, double y) {   /* Precision.equals(x, y) (1 ulp) */
    int64_t xi, yi;
    memcpy(&xi, &x, 8);
    memcpy(&yi, &y, 8);
    int eq;
    if (((xi ^ yi) & INT64_MIN) == 0) {
        const int64_t d = xi - yi;
        eq = (d < 0 ? -d : d) <= 1;
    } else {
        int64_t dp, dm;
        if (xi < yi) { dp = yi; dm = (int64_t)((uint64_t)xi - (uint64_t)INT64_MIN); }
        else { dp = xi; dm = (int64_t)((uint64_t)yi - (uint64_t)INT64_MIN); }
        eq = (dp > 1) ? 0 : (dm <= 1 - dp);
    }
    return eq && !isnan(x) && !isnan(y);
}

/* BrentOptimizer.best(a, b, isMinim = false) */
static gpv_t best_max(gpv_t a, gpv_t b) { return (a.v >= b.v) ? a : b; }

/* LineSearch.search(point, dir): BracketFinder(100, 500).search(f, null, 0, 1e-8), then
 * BrentOptimizer(1e-15, MIN_VALUE, SimpleUnivariateValueChecker(1e-8, 1e-8)).optimize(f,
 * null, [lo, hi] from mid).  *err: 1 = TooManyEvaluations, 2 = invalid search interval. */
static double garch_line_search(garch_obj_t* o, const double pt[3], const double dir[3], int* err) {
    double q[3];
    int bev = 0;
#define AT(a) (q[0] = pt[0] + (a) * dir[0], q[1] = pt[1] + (a) * dir[1], q[2] = pt[2] + (a) * dir[2], q)
#define F(a) (++bev > 500 ? (*err = 1, NAN) : garch_value(o, AT(a)))
    const double GOLD = 1.618034, EPS_MIN = 1e-21;
    double xA = 0, xB = 1e-8;
    double fA = F(xA);
    double fB = F(xB);
    if (*err || o->too_many) return NAN;
    if (fA > fB) {                                     /* isMinim ? fA < fB : fA > fB */
        double t = xA; xA = xB; xB = t;
        t = fA; fA = fB; fB = t;
    }
    double xC = xB + GOLD * (xB - xA);
    double fC = F(xC);
    while (fC > fB) {                                  /* isMinim ? fC < fB : fC > fB */
        if (*err || o->too_many) return NAN;
        const double tmp1 = (xB - xA) * (fB - fC);
        const double tmp2 = (xB - xC) * (fB - fA);
        const double val = tmp2 - tmp1;
        const double denom = fabs(val) < EPS_MIN ? 2 * EPS_MIN : val;
        double w = xB - ((xB - xC) * tmp2 - (xB - xA) * tmp1) / (2 * denom);
        const double wLim = xB + 100 * (xC - xB);
        double fW;
        if ((w - xC) * (xB - w) > 0) {
            fW = F(w);
            if (fW > fC) {
                xA = xB; xB = w; fA = fB; fB = fW;
                break;
            } else if (fW < fB) {
                xC = w; fC = fW;
                break;
            }
            w = xC + GOLD * (xC - xB);
            fW = F(w);
        } else if ((w - wLim) * (wLim - xC) >= 0) {
            w = wLim;
            fW = F(w);
        } else if ((w - wLim) * (xC - w) > 0) {
            fW = F(w);
            if (fW > fC) {
                xB = xC; xC = w; w = xC + GOLD * (xC - xB);
                fB = fC; fC = fW;
                fW = F(w);
            }
        } else {
            w = xC + GOLD * (xC - xB);
            fW = F(w);
        }
        xA = xB; fA = fB; xB = xC; fB = fC; xC = w; fC = fW;
    }
#undef F
    if (*err || o->too_many) return NAN;
    double lo = xA, mid = xB, hi = xC;
    if (lo > hi) { const double t = lo; lo = hi; hi = t; }
    if (!(lo < hi) || !(mid >= lo && mid <= hi)) { *err = 2; return NAN; }   /* SearchInterval */

    /* BrentOptimizer.doOptimize, isMinim = false: works on -f, reports f */
    const double rel = 1e-15, absT = 4.9406564584124654e-324;
    const double GS = 0.5 * (3 - sqrt(5.0));
    double a = lo, b = hi;
    double x = mid, v = x, w = x, d = 0, e = 0;
    double fx = garch_value(o, AT(x));
    fx = -fx;
    double fv = fx, fw = fx;
    gpv_t previous = {0, 0}, current = {x, -fx}, best = current;
    int have_prev = 0;
    for (;;) {
        if (o->too_many) return NAN;
        const double m = 0.5 * (a + b);
        const double tol1 = rel * fabs(x) + absT;
        const double tol2 = 2 * tol1;
        if (fabs(x - m) <= tol2 - 0.5 * (b - a)) {
            const gpv_t bb = have_prev ? best_max(previous, current) : current;
            return best_max(best, bb).x;
        }
        double p = 0, qq = 0, r = 0, u = 0;
        if (fabs(e) > tol1) {
            r = (x - w) * (fv - fx);
            qq = (x - v) * (fw - fx);
            p = (x - v) * qq - (x - w) * r;
            qq = 2 * (qq - r);
            if (qq > 0) p = -p;
            else qq = -qq;
            r = e;
            e = d;
            if (p > qq * (a - x) && p < qq * (b - x) && fabs(p) < fabs(0.5 * qq * r)) {
                d = p / qq;
                u = x + d;
                if (u - a < tol2 || b - u < tol2) d = (x <= m) ? tol1 : -tol1;
            } else {
                e = (x < m) ? b - x : a - x;
                d = GS * e;
            }
        } else {
            e = (x < m) ? b - x : a - x;
            d = GS * e;
        }
        if (fabs(d) < tol1) u = (d >= 0) ? x + tol1 : x - tol1;
        else u = x + d;
        double fu = garch_value(o, AT(u));
        fu = -fu;
        previous = current;
        have_prev = 1;
        current.x = u;
        current.v = -fu;
        best = best_max(best, best_max(previous, current));
        {   /* SimpleUnivariateValueChecker(1e-8, 1e-8) */
            const double diff = fabs(previous.v - current.v);
            const double size = fmax(fabs(previous.v), fabs(current.v));
            if (diff <= size * 1e-8 || diff <= 1e-8) return best.x;
        }
        if (fu <= fx) {
            if (u < x) b = x;
            else a = x;
            v = w; fv = fw;
            w = x; fw = fx;
            x = u; fx = fu;
        } else {
            if (u < x) a = u;
            else b = u;
            if (fu <= fw || prec_equals(w, x)) {
                v = w; fv = fw;
                w = u; fw = fu;
            } else if (fu <= fv || prec_equals(v, x) || prec_equals(v, w)) {
                v = u; fv = fu;
            }
        }
    }
#undef AT
}

/* GARCH.fitModel (:33-53): NLCG Fletcher-Reeves from (.2, .2, .2), MaxIter / MaxEval 10000 */
int orc_garch_fit(const double* ts, int64_t n, double params[3], int64_t* evaluations) {
    garch_obj_t o = {ts, n, 0, 0};
    double point[3] = {.2, .2, .2};
    double r[3];
    /* computeObjectiveGradient (not counted); goal != MINIMIZE: r is not negated */
    orc_garch_gradient(ts, n, point[0], point[1], point[2], r);
    double steepest[3] = {r[0], r[1], r[2]};            /* IdentityPreconditioner */
    double dir[3] = {steepest[0], steepest[1], steepest[2]};
    double delta = 0;
    for (int i = 0; i < 3; i++) delta += r[i] * dir[i];
    int have = 0;
    double cur_v = 0;
    int st = ORC_OK;
    for (int64_t iter = 1;; iter++) {
        if (iter > 10000) { st = ORC_ERR_TOO_MANY_ITERATIONS; break; }
        const double objective = garch_value(&o, point);
        if (o.too_many) { st = ORC_ERR_TOO_MANY_EVALUATIONS; break; }
        if (have) {   /* SimpleValueChecker(1e-6, 1e-6) on (previous, current) */
            const double diff = fabs(cur_v - objective);
            const double size = fmax(fabs(cur_v), fabs(objective));
            if (diff <= size * 1e-6 || diff <= 1e-6) break;
        }
        have = 1;
        cur_v = objective;
        int lerr = 0;
        const double step = garch_line_search(&o, point, dir, &lerr);
        if (o.too_many || lerr == 1) { st = ORC_ERR_TOO_MANY_EVALUATIONS; break; }
        if (lerr == 2) { st = ORC_ERR_BAD_ARG; break; }
        for (int i = 0; i < 3; i++) point[i] += step * dir[i];
        orc_garch_gradient(ts, n, point[0], point[1], point[2], r);
        const double deltaOld = delta;
        delta = 0;
        for (int i = 0; i < 3; i++) delta += r[i] * r[i];
        const double beta = delta / deltaOld;           /* FLETCHER_REEVES */
        for (int i = 0; i < 3; i++) steepest[i] = r[i];
        if (iter % 3 == 0 || beta < 0) {
            for (int i = 0; i < 3; i++) dir[i] = steepest[i];
        } else {
            for (int i = 0; i < 3; i++) dir[i] = steepest[i] + beta * dir[i];
        }
    }
    if (evaluations) *evaluations = o.evals;
    for (int i = 0; i < 3; i++) params[i] = (st == ORC_OK) ? point[i] : NAN;
    return st;
}

/* ARGARCH.fitModel (:62-68): AR(1) with intercept, residuals, GARCH fit of the residuals.
 * out = (c, phi, omega, alpha, beta). */
int orc_argarch_fit(const double* ts, int64_t n, double out[5], int64_t* evaluations) {
    double c = 0, phi = 0;
    int st = orc_ar_fit(ts, n, 1, 0, &c, &phi);
    if (st != ORC_OK) {
        for (int i = 0; i < 5; i++) out[i] = NAN;
        if (evaluations) *evaluations = 0;
        return st;
    }
    double* resid = (double*)malloc((size_t)(n > 0 ? n : 1) * sizeof(double));
    orc_ar_remove(ts, resid, n, c, &phi, 1);
    double g[3];
    st = orc_garch_fit(resid, n, g, evaluations);
    free(resid);
    out[0] = c;
    out[1] = phi;
    out[2] = g[0];
    out[3] = g[1];
    out[4] = g[2];
    return st;
}

/* GARCHModel.removeTimeDependentEffects (:130-142) */
void orc_garch_remove(const double* ts, double* dest, int64_t n, double omega, double alpha,
                      double beta) {
    if (n <= 0) return;
    double prevEta = ts[0];
    double prevVariance = omega / (1.0 - alpha - beta);
    dest[0] = prevEta / sqrt(prevVariance);
    for (int64_t i = 1; i < n; i++) {
        const double variance = omega + alpha * prevEta * prevEta + beta * prevVariance;
        const double eta = ts[i];
        dest[i] = eta / sqrt(variance);
        prevEta = eta;
        prevVariance = variance;
    }
}

/* GARCHModel.addTimeDependentEffects (:144-159) */
void orc_garch_add(const double* ts, double* dest, int64_t n, double omega, double alpha,
                   double beta) {
    if (n <= 0) return;
    double prevVariance = omega / (1.0 - alpha - beta);
    double prevEta = ts[0] * sqrt(prevVariance);
    dest[0] = prevEta;
    for (int64_t i = 1; i < n; i++) {
        const double variance = omega + alpha * prevEta * prevEta + beta * prevVariance;
        const double standardizedEta = ts[i];
        const double eta = standardizedEta * sqrt(variance);
        dest[i] = eta;
        prevEta = eta;
        prevVariance = variance;
    }
}

/* ARGARCHModel.removeTimeDependentEffects (:203-217); dest may alias ts (then ts(i - 1)
 * reads the overwritten value, as on the JVM) */
void orc_argarch_remove(const double* ts, double* dest, int64_t n, double c, double phi,
                        double omega, double alpha, double beta) {
    if (n <= 0) return;
    double prevEta = ts[0] - c;
    double prevVariance = omega / (1.0 - alpha - beta);
    dest[0] = prevEta / sqrt(prevVariance);
    for (int64_t i = 1; i < n; i++) {
        const double variance = omega + alpha * prevEta * prevEta + beta * prevVariance;
        const double eta = ts[i] - c - phi * ts[i - 1];
        dest[i] = eta / sqrt(variance);
        prevEta = eta;
        prevVariance = variance;
    }
}

/* ARGARCHModel.addTimeDependentEffects (:219-234) */
void orc_argarch_add(const double* ts, double* dest, int64_t n, double c, double phi,
                     double omega, double alpha, double beta) {
    if (n <= 0) return;
    double prevVariance = omega / (1.0 - alpha - beta);
    double prevEta = ts[0] * sqrt(prevVariance);
    dest[0] = c + prevEta;
    for (int64_t i = 1; i < n; i++) {
        const double variance = omega + alpha * prevEta * prevEta + beta * prevVariance;
        const double standardizedEta = ts[i];
        const double eta = standardizedEta * sqrt(variance);
        dest[i] = c + phi * dest[i - 1] + eta;
        prevEta = eta;
        prevVariance = variance;
    }
}

int orc_panel_garch_fit(const double* in, int64_t S, int64_t T, int64_t ld, double* params,
                        int32_t* err, int threads) {
    int any = 0;
#pragma omp parallel for schedule(dynamic, 16) num_threads(threads > 0 ? threads : 1) reduction(| : any)
    for (int64_t q = 0; q < S; q++) {
        const int st = orc_garch_fit(in + q * ld, T, params + 3 * q, NULL);
        if (err) err[q] = st;
        any |= st != ORC_OK;
    }
    return any ? ORC_ERR_TOO_MANY_EVALUATIONS : ORC_OK;
}

int orc_panel_argarch_fit(const double* in, int64_t S, int64_t T, int64_t ld, double* params,
                          int32_t* err, int threads) {
    int any = 0;
#pragma omp parallel for schedule(dynamic, 16) num_threads(threads > 0 ? threads : 1) reduction(| : any)
    for (int64_t q = 0; q < S; q++) {
        const int st = orc_argarch_fit(in + q * ld, T, params + 5 * q, NULL);
        if (err) err[q] = st;
        any |= st != ORC_OK;
    }
    return any ? ORC_ERR_TOO_MANY_EVALUATIONS : ORC_OK;
}
