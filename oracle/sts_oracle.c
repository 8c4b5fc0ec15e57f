/*
 * sts_oracle.c -- CPU restatement of the spark-timeseries hot path.
 *
 * TEST INFRASTRUCTURE ONLY (see sts_oracle.h): the parity checker and the
 * CPU baseline.  Nothing in the shipped library links or calls this file.
 *
 * Reference: mjayantkumar/spark-timeseries (Scala 2.10, Breeze 0.10,
 * commons-math3 3.4.1).  S/ = src/main/scala/com/cloudera/sparkts/.
 * Build flags: -O2 -ffp-contract=off (JVM double semantics: IEEE binary64,
 * round-to-nearest, no fused multiply-add).
 */
#include "sts_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#ifdef _OPENMP
#include <omp.h>
#endif

/* S/UnivariateTimeSeries.scala:194-204 (fillPrevious) */
void orc_fill_previous(const double* x, double* r, int64_t n) {
    double filler = NAN; /* initial value, :196 */
    for (int64_t i = 0; i < n; i++) {
        filler = isnan(x[i]) ? filler : x[i];
        r[i] = filler;
    }
}

/* S/UnivariateTimeSeries.scala:214-224 (fillNext) */
void orc_fill_next(const double* x, double* r, int64_t n) {
    double filler = NAN;
    for (int64_t i = n - 1; i >= 0; i--) {
        filler = isnan(x[i]) ? filler : x[i];
        r[i] = filler;
    }
}

/* S/UnivariateTimeSeries.scala:156-184 (fillNearest), statement by statement.
 * The loop starts at i = 1: index 0 is never modified and never becomes
 * lastExisting; ties go to the next value; throws
 * IllegalArgumentException("Input is all NaNs!") at :170-171. */
int orc_fill_nearest(const double* x, double* r, int64_t n) {
    if (r != x) memcpy(r, x, (size_t)n * sizeof(double));
    int64_t lastExisting = -1;
    int64_t nextExisting = -1;
    int64_t i = 1;
    while (i < n) {
        if (isnan(r[i])) {
            if (nextExisting < i) {
                nextExisting = i + 1;
                while (nextExisting < n && isnan(r[nextExisting])) nextExisting++;
            }
            if (lastExisting < 0 && nextExisting >= n) {
                return ORC_ERR_ALL_NAN;
            } else if (nextExisting >= n || (lastExisting >= 0 && i - lastExisting < nextExisting - i)) {
                r[i] = r[lastExisting];
            } else {
                r[i] = r[nextExisting];
            }
        } else {
            lastExisting = i;
        }
        i++;
    }
    return ORC_OK;
}

/* S/UnivariateTimeSeries.scala:247-266 (fillLinear).  Interior runs are filled
 * by a SEQUENTIAL accumulation r[j] = r[j-1] + increment (:259-261), not by
 * before + k*increment; the two differ in the last bits. */
void orc_fill_linear(const double* x, double* r, int64_t n) {
    if (r != x) memcpy(r, x, (size_t)n * sizeof(double));
    int64_t i = 1;
    while (i < n - 1) {
        int64_t rangeStart = i;
        while (i < n - 1 && isnan(r[i])) i++;
        double before = r[rangeStart - 1];
        double after = r[i];
        if (i != rangeStart && !isnan(before) && !isnan(after)) {
            /* Double / Int: the Int distance is widened to double */
            double increment = (after - before) / (double)(int32_t)(i - (rangeStart - 1));
            for (int64_t j = rangeStart; j < i; j++) r[j] = r[j - 1] + increment;
        }
        i++;
    }
}

/* commons-math3 3.4.1 PolynomialFunction(double[] c) + value(x): the constructor drops
 * trailing zero coefficients (`while (n > 1 && c[n - 1] == 0) --n`), value() is Horner's
 * rule `result = c[n-1]; for j = n-2..0: result = x * result + c[j]` (no FMA on the JVM).
 * The trimming matters only for signed zeros and infinities, but it is the reference's. */
static double cm3_poly_value(const double c[4], double x) {
    int n = 4;
    while (n > 1 && c[n - 1] == 0.0) --n;
    double result = c[n - 1];
    for (int j = n - 2; j >= 0; j--) result = x * result + c[j];
    return result;
}

/* java.util.Arrays.binarySearch(double[], double) for the spline's knots (strictly
 * increasing integers, never -0.0 or NaN, so the bit comparisons of the JDK's tie branch
 * never decide anything): the index of key, else -(insertion point) - 1. */
static int64_t java_binary_search(const double* a, int64_t len, double key) {
    int64_t low = 0, high = len - 1;
    while (low <= high) {
        int64_t mid = (int64_t)(((uint64_t)low + (uint64_t)high) >> 1);
        double midVal = a[mid];
        if (midVal < key) low = mid + 1;
        else if (midVal > key) high = mid - 1;
        else return mid;
    }
    return -(low + 1);
}

/* S/UnivariateTimeSeries.scala:268-297 (fillSpline): the knots are the non-NaN steps
 * (x = index as double, y = value), `new SplineInterpolator().interpolate(knotsX, knotsY)`,
 * then result(i) = filler.value(i) for EVERY i in [knotsX(0), knotsX.last) -- valid steps
 * included (the spline's value at a knot is y up to signed zeros / non-finite data) -- and
 * the raw value elsewhere.  commons-math3 3.4.1 (not vendored in /root/reference; restated
 * from its published source):
 *   SplineInterpolator.interpolate: x.length < 3 -> NumberIsTooSmallException(NUMBER_OF_POINTS,
 *     x.length, 3, true) (ORC_ERR_TOO_FEW_POINTS); n = x.length - 1; h[i] = x[i+1] - x[i];
 *     mu[0] = z[0] = 0; for i = 1..n-1: g = 2(x[i+1] - x[i-1]) - h[i-1] mu[i-1];
 *     mu[i] = h[i] / g; z[i] = (3 (y[i+1] h[i-1] - y[i] (x[i+1] - x[i-1]) + y[i-1] h[i]) /
 *     (h[i-1] h[i]) - h[i-1] z[i-1]) / g; z[n] = c[n] = 0; for j = n-1..0: c[j] = z[j] -
 *     mu[j] c[j+1]; b[j] = (y[j+1] - y[j]) / h[j] - h[j] (c[j+1] + 2 c[j]) / 3;
 *     d[j] = (c[j+1] - c[j]) / (3 h[j]); polynomial j = {y[j], b[j], c[j], d[j]}.
 *   PolynomialSplineFunction.value(v): i = binarySearch(knots, v); i < 0 -> -i - 2;
 *     i >= n -> i - 1; polynomials[i].value(v - knots[i]).
 * Every expression keeps Java's left-to-right evaluation order. */
int orc_fill_spline(const double* x, double* r, int64_t len) {
    if (r != x) memcpy(r, x, (size_t)len * sizeof(double));
    int64_t m = 0;
    for (int64_t i = 0; i < len; i++) m += !isnan(x[i]);
    if (m < 3) return ORC_ERR_TOO_FEW_POINTS;
    double* kx = (double*)malloc((size_t)m * 8 * sizeof(double));
    if (!kx) return ORC_ERR_BAD_ARG;
    double *ky = kx + m, *h = ky + m, *mu = h + m, *z = mu + m, *b = z + m, *c = b + m, *d = c + m;
    int64_t k = 0;
    for (int64_t i = 0; i < len; i++)
        if (!isnan(x[i])) {
            kx[k] = (double)i;
            ky[k] = x[i];
            k++;
        }
    const int64_t n = m - 1;
    for (int64_t i = 0; i < n; i++) h[i] = kx[i + 1] - kx[i];
    mu[0] = 0.0;
    z[0] = 0.0;
    double g = 0;
    for (int64_t i = 1; i < n; i++) {
        g = 2.0 * (kx[i + 1] - kx[i - 1]) - h[i - 1] * mu[i - 1];
        mu[i] = h[i] / g;
        z[i] = (3.0 * (ky[i + 1] * h[i - 1] - ky[i] * (kx[i + 1] - kx[i - 1]) + ky[i - 1] * h[i]) /
                    (h[i - 1] * h[i]) -
                h[i - 1] * z[i - 1]) /
               g;
    }
    z[n] = 0.0;
    c[n] = 0.0;
    for (int64_t j = n - 1; j >= 0; j--) {
        c[j] = z[j] - mu[j] * c[j + 1];
        b[j] = (ky[j + 1] - ky[j]) / h[j] - h[j] * (c[j + 1] + 2.0 * c[j]) / 3.0;
        d[j] = (c[j + 1] - c[j]) / (3.0 * h[j]);
    }
    /* :289-294: i from knotsX(0).toInt until knotsX.last.toInt */
    const int64_t end = (int64_t)kx[n];
    for (int64_t i = (int64_t)kx[0]; i < end; i++) {
        const double v = (double)i;
        int64_t s = java_binary_search(kx, m, v);
        if (s < 0) s = -s - 2;
        if (s >= n) s--;
        const double cf[4] = {ky[s], b[s], c[s], d[s]};
        r[i] = cm3_poly_value(cf, v - kx[s]);
    }
    free(kx);
    return ORC_OK;
}

/* S/UnivariateTimeSeries.scala:141-150 (fillts dispatch) */
int orc_fillts(const double* x, double* r, int64_t n, int method) {
    switch (method) {
    case ORC_FILL_LINEAR: orc_fill_linear(x, r, n); return ORC_OK;
    case ORC_FILL_NEAREST: return orc_fill_nearest(x, r, n);
    case ORC_FILL_NEXT: orc_fill_next(x, r, n); return ORC_OK;
    case ORC_FILL_PREVIOUS: orc_fill_previous(x, r, n); return ORC_OK;
    case ORC_FILL_SPLINE: return orc_fill_spline(x, r, n);
    default: return ORC_ERR_UNSUPPORTED_METHOD;
    }
}

/* Breeze 0.10 breeze.stats.mean over a DenseVector slice: sum left to right,
 * divide by the count (Breeze source is not vendored in /root/reference; the
 * form is an ASSUMPTION -- PARITY UNPINNED).  Any summation order differs by
 * << 1e-10 on ordinary series, but a running-mean update (mu += (y - mu) / n)
 * would return a constant series' mean exactly and the reference's autocorr
 * of a non-dyadic constant would then be NaN instead of 1.0.
 * The device's one copy of this form is acf_exact_lag's first pass
 * (spark-timeseries_amd/csrc/sts_acf.hpp). */
static double breeze_mean(const double* v, int64_t len) {
    double sum = 0.0;
    for (int64_t k = 0; k < len; k++) sum += v[k];
    return sum / (double)len;
}

/* S/UnivariateTimeSeries.scala:68-93 (autocorr).  For lag i >= n the slices are
 * empty (or inverted); the result is NaN (0/0), see DESIGN.md. */
void orc_autocorr(const double* ts, int64_t n, int numLags, double* corrs) {
    for (int i = 1; i <= numLags; i++) {
        if ((int64_t)i >= n) { corrs[i - 1] = NAN; continue; }
        const double* slice1 = ts + i;       /* ts(i until n)   :72 */
        const double* slice2 = ts;           /* ts(0 until n-i) :73 */
        int64_t len = n - i;
        double mean1 = breeze_mean(slice1, len);
        double mean2 = breeze_mean(slice2, len);
        double variance1 = 0.0, variance2 = 0.0, covariance = 0.0;
        for (int64_t j = 0; j < len; j++) {
            double diff1 = slice1[j] - mean1;
            double diff2 = slice2[j] - mean2;
            variance1 += diff1 * diff1;
            variance2 += diff2 * diff2;
            covariance += diff1 * diff2;
        }
        corrs[i - 1] = covariance / (sqrt(variance1) * sqrt(variance2));
    }
}

/* S/Lag.scala:62-77 (lagMatTrimBoth, Vector variant): Breeze DenseMatrix of
 * (n - maxLag) rows x (maxLag + inc) columns, column-major:
 * M(r, c - init) = x(r + maxLag - c), c = init..maxLag. */
int orc_lag_mat_trim_both(const double* x, int64_t n, int maxLag, int includeOriginal,
                          double* out) {
    int64_t numRows = n - maxLag;
    if (maxLag < 0 || numRows < 0) return ORC_ERR_BAD_ARG;
    int initialLag = includeOriginal ? 0 : 1;
    for (int64_t r = 0; r < numRows; r++)
        for (int c = initialLag; c <= maxLag; c++)
            out[(int64_t)(c - initialLag) * numRows + r] = x[r + maxLag - c];
    return ORC_OK;
}

/* S/UnivariateTimeSeries.scala:356-376 (differencesAtLag with an explicit dest).
 * dest may alias ts: the loop then reads values it has already overwritten,
 * exactly as the JVM loop does.  lag == 0 returns dest untouched (:363-364). */
int orc_differences_at_lag(const double* ts, double* dest, int64_t n, int lag, int start) {
    if (!(start >= lag)) return ORC_ERR_REQUIREMENT; /* require(), :361 */
    if (lag == 0) return ORC_OK;
    for (int64_t i = 0; i < n; i++)
        dest[i] = (i < start) ? ts[i] : ts[i] - ts[i - lag];
    return ORC_OK;
}

/* S/UnivariateTimeSeries.scala:397-417 (inverseDifferencesAtLag) */
int orc_inverse_differences_at_lag(const double* d, double* dest, int64_t n, int lag, int start) {
    if (!(start >= lag)) return ORC_ERR_REQUIREMENT;
    if (lag == 0) return ORC_OK;
    for (int64_t i = 0; i < n; i++)
        dest[i] = (i < start) ? d[i] : d[i] + dest[i - lag];
    return ORC_OK;
}

/* S/UnivariateTimeSeries.scala:438-450 (differencesOfOrderD): ping-pong of two
 * copies so that no call sees its own output. */
void orc_differences_of_order_d(const double* ts, double* out, int64_t n, int d) {
    double* a = (double*)malloc((size_t)(n > 0 ? n : 1) * sizeof(double));
    double* b = (double*)malloc((size_t)(n > 0 ? n : 1) * sizeof(double));
    memcpy(a, ts, (size_t)n * sizeof(double)); /* diffedTs */
    memcpy(b, ts, (size_t)n * sizeof(double)); /* origTs */
    double* diffed = a;
    double* orig = b;
    for (int i = 1; i <= d; i++) {
        double* swap = orig;
        orig = diffed;
        diffed = swap;
        orc_differences_at_lag(orig, diffed, n, 1, i);
    }
    memcpy(out, diffed, (size_t)n * sizeof(double));
    free(a);
    free(b);
}

/* S/models/EWMA.scala:135-142 (EWMAModel.addTimeDependentEffects):
 * dest(0) = ts(0); dest(i) = s*ts(i) + (1 - s)*dest(i-1).  In-place is safe. */
void orc_ewma_add(const double* ts, double* dest, int64_t n, double s) {
    if (n <= 0) return;
    dest[0] = ts[0];
    for (int64_t i = 1; i < n; i++) dest[i] = s * ts[i] + (1.0 - s) * dest[i - 1];
}

/* S/models/EWMA.scala:125-133 (removeTimeDependentEffects):
 * dest(i) = (ts(i) - (1 - s)*ts(i-1)) / s.  In-place is NOT equivalent
 * (reads the overwritten ts(i-1)); the loop below reproduces that too. */
void orc_ewma_remove(const double* ts, double* dest, int64_t n, double s) {
    if (n <= 0) return;
    dest[0] = ts[0];
    for (int64_t i = 1; i < n; i++) dest[i] = (ts[i] - (1.0 - s) * ts[i - 1]) / s;
}

/* S/models/Autoregression.scala:60-73 (ARModel.removeTimeDependentEffects) */
void orc_ar_remove(const double* ts, double* dest, int64_t n, double c, const double* coef, int p) {
    for (int64_t i = 0; i < n; i++) {
        dest[i] = ts[i] - c;
        for (int j = 0; j < p && i - j - 1 >= 0; j++) dest[i] -= ts[i - j - 1] * coef[j];
    }
}

/* S/models/Autoregression.scala:75-88 (ARModel.addTimeDependentEffects, IIR) */
void orc_ar_add(const double* ts, double* dest, int64_t n, double c, const double* coef, int p) {
    for (int64_t i = 0; i < n; i++) {
        dest[i] = c + ts[i];
        for (int j = 0; j < p && i - j - 1 >= 0; j++) dest[i] += dest[i - j - 1] * coef[j];
    }
}

/* commons-math3 3.4.1 OLSMultipleLinearRegression (not vendored in
 * /root/reference; restated from its published source):
 *   newSampleData -> validateSampleData (x[0].length + 1 > x.length throws
 *   NOT_ENOUGH_DATA_FOR_NUMBER_OF_PREDICTORS), intercept column of 1.0 first
 *   unless noIntercept, QRDecomposition(X, threshold = 0) on X^T rows
 *   (Householder, performHouseholderReflection), Solver.solve(y): apply the
 *   reflections to y, back-substitute R; SingularMatrixException when any
 *   |rDiag| <= 0.  Called from S/models/Autoregression.scala:47-50. */
int orc_ols_householder(const double* y, const double* x, int64_t m, int k, int no_intercept,
                        double* beta) {
    int ncol = k + (no_intercept ? 0 : 1);
    if (m == 0) return ORC_ERR_NOT_ENOUGH_DATA;
    if ((int64_t)k + 1 > m) return ORC_ERR_NOT_ENOUGH_DATA;
    /* qrt = X^T: qrt[col][row] */
    double* qrt = (double*)malloc((size_t)ncol * (size_t)m * sizeof(double));
    double* rDiag = (double*)malloc((size_t)ncol * sizeof(double));
    double* yy = (double*)malloc((size_t)m * sizeof(double));
    for (int64_t r = 0; r < m; r++) {
        int cc = 0;
        if (!no_intercept) qrt[(int64_t)(cc++) * m + r] = 1.0;
        for (int c = 0; c < k; c++) qrt[(int64_t)(cc++) * m + r] = x[r * k + c];
        yy[r] = y[r];
    }
    int64_t minmn = (int64_t)ncol < m ? ncol : m;
    for (int64_t minor = 0; minor < minmn; minor++) {
        double* qrtMinor = qrt + minor * m;
        double xNormSqr = 0.0;
        for (int64_t row = minor; row < m; row++) {
            double c = qrtMinor[row];
            xNormSqr += c * c;
        }
        double a = (qrtMinor[minor] > 0) ? -sqrt(xNormSqr) : sqrt(xNormSqr);
        rDiag[minor] = a;
        if (a != 0.0) {
            qrtMinor[minor] -= a;
            for (int64_t col = minor + 1; col < ncol; col++) {
                double* qrtCol = qrt + col * m;
                double alpha = 0.0;
                for (int64_t row = minor; row < m; row++) alpha -= qrtCol[row] * qrtMinor[row];
                alpha /= a * qrtMinor[minor];
                for (int64_t row = minor; row < m; row++) qrtCol[row] -= alpha * qrtMinor[row];
            }
        }
    }
    int status = ORC_OK;
    for (int64_t d = 0; d < minmn; d++)
        if (fabs(rDiag[d]) <= 0.0) status = ORC_ERR_SINGULAR;
    if (status == ORC_OK) {
        for (int64_t minor = 0; minor < minmn; minor++) {
            const double* qrtMinor = qrt + minor * m;
            double dotProduct = 0.0;
            for (int64_t row = minor; row < m; row++) dotProduct += yy[row] * qrtMinor[row];
            dotProduct /= rDiag[minor] * qrtMinor[minor];
            for (int64_t row = minor; row < m; row++) yy[row] += dotProduct * qrtMinor[row];
        }
        for (int64_t row = minmn - 1; row >= 0; --row) {
            yy[row] /= rDiag[row];
            double yRow = yy[row];
            const double* qrtRow = qrt + row * m;
            beta[row] = yRow;
            for (int64_t i = 0; i < row; i++) yy[i] -= yRow * qrtRow[i];
        }
    }
    free(qrt);
    free(rDiag);
    free(yy);
    return status;
}

/* S/models/Autoregression.scala:38-53 (Autoregression.fitModel):
 * Y = ts(maxLag until n), X = Lag.lagMatTrimBoth(ts, maxLag) (row r =
 * [x(r+p-1), ..., x(r)]), OLS with intercept unless noIntercept;
 * c = params.head (0 if noIntercept), coefficients = params.tail. */
int orc_ar_fit(const double* ts, int64_t n, int p, int no_intercept, double* c, double* coef) {
    int64_t m = n - p;
    if (p < 1 || m <= 0) return ORC_ERR_NOT_ENOUGH_DATA;
    double* X = (double*)malloc((size_t)m * (size_t)p * sizeof(double));
    for (int64_t r = 0; r < m; r++)
        for (int cc = 1; cc <= p; cc++) X[r * p + (cc - 1)] = ts[r + p - cc];
    double beta[64];
    if (p + 1 > 64) { free(X); return ORC_ERR_BAD_ARG; }
    int st = orc_ols_householder(ts + p, X, m, p, no_intercept, beta);
    free(X);
    if (st != ORC_OK) return st;
    if (no_intercept) {
        *c = 0.0;
        for (int j = 0; j < p; j++) coef[j] = beta[j];
    } else {
        *c = beta[0];
        for (int j = 0; j < p; j++) coef[j] = beta[j + 1];
    }
    return ORC_OK;
}

/* ---------------- EWMA.fitModel (S/models/EWMA.scala:44-68) ----------------
 *
 * EWMAModel.sse (:80-95) and .gradient (:102-123) restated statement by statement.
 * The optimizer is commons-math3 3.4.1 (pom.xml:396-400; not vendored in /root/reference),
 * restated from its published algorithm:
 *   NonLinearConjugateGradientOptimizer(FLETCHER_REEVES, SimpleValueChecker(1e-6, 1e-6))
 *     -> LineSearch(relTol 1e-8, absTol 1e-8, initialBracketingRange 1e-8)
 *        = BracketFinder(growLimit 100, maxEvaluations 500).search(f, MIN, 0, 1e-8)
 *          + BrentOptimizer(rel 1e-15, abs Double.MIN_VALUE,
 *                           SimpleUnivariateValueChecker(1e-8, 1e-8))
 *   InitialGuess 0.94, MaxIter 10000, MaxEval 10000 (:60-62).
 * One parameter (n = 1): iterations % n == 0 always resets the search direction to the
 * steepest descent, so beta never matters.  Parity is pinned only by
 * T/models/EWMASuite.scala:54-63 (the oil series -> truncated smoothing 89).
 */
double orc_ewma_sse(const double* ts, int64_t n, double s) {
    /* smoothed = addTimeDependentEffects(ts, zeros) (:82-84), then :86-92 */
    double sm = (n > 0) ? ts[0] : 0.0, sq = 0.0;
    for (int64_t i = 0; i < n - 1; i++) {
        const double error = ts[i + 1] - sm;     /* ts(i + 1) - smoothed(i) */
        sq += error * error;
        sm = s * ts[i + 1] + (1 - s) * sm;       /* smoothed(i + 1), EWMA.scala:140 */
    }
    return sq;
}

double orc_ewma_gradient(const double* ts, int64_t n, double s) {
    double sm = (n > 0) ? ts[0] : 0.0;           /* smoothed(i) */
    double prevSmoothed = (n > 0) ? ts[0] : 0.0, prevDSda = 0.0, dSda = 0.0, dJda = 0.0;
    for (int64_t i = 0; i < n - 1; i++) {
        const double error = ts[i + 1] - sm;
        dSda = ts[i] - prevSmoothed + (1 - s) * prevDSda;
        dJda += error * dSda;
        prevDSda = dSda;
        prevSmoothed = sm;
        sm = s * ts[i + 1] + (1 - s) * sm;
    }
    return 2 * dJda;
}

typedef struct { double x, v; } pv_t;   /* (Univariate)PointValuePair */

/* commons-math3 Precision.equals(x, y) = equals(x, y, 1 ulp), NaN never equal */
static int cm_precision_equals(double x, double y) {
    int64_t xi, yi;
    memcpy(&xi, &x, 8);
    memcpy(&yi, &y, 8);
    int eq;
    if (((xi ^ yi) & INT64_MIN) == 0) {
        int64_t d = xi - yi;
        eq = (d < 0 ? -d : d) <= 1;
    } else {
        int64_t dp, dm;
        if (xi < yi) { dp = yi; dm = (int64_t)((uint64_t)xi - (uint64_t)INT64_MIN); }
        else { dp = xi; dm = (int64_t)((uint64_t)yi - (uint64_t)INT64_MIN); }
        eq = (dp > 1) ? 0 : (dm <= 1 - dp);
    }
    return eq && !isnan(x) && !isnan(y);
}

/* objective with the main optimizer's evaluation counter (MaxEval 10000) */
typedef struct { const double* ts; int64_t n; int64_t evals; int too_many; } ewma_obj_t;
static double ewma_value(ewma_obj_t* o, double s) {
    if (++o->evals > 10000) o->too_many = 1;
    return o->too_many ? NAN : orc_ewma_sse(o->ts, o->n, s);
}

#define CM_GOLD 1.618034
#define CM_EPS_MIN 1e-21

/* LineSearch.search (n = 1): f(alpha) = value(point + alpha * dir) */
static double cm_line_search(ewma_obj_t* o, double point, double dir, int* err) {
    /* BracketFinder.search(f, MINIMIZE, 0, 1e-8); its own counter: 500 evaluations */
    int bev = 0;
#define F(a) (++bev > 500 ? (*err = 1, NAN) : ewma_value(o, point + (a) * dir))
    double xA = 0, xB = 1e-8;
    double fA = F(xA), fB = F(xB);
    if (*err || o->too_many) return NAN;
    if (fA < fB) {
        double t = xA; xA = xB; xB = t;
        t = fA; fA = fB; fB = t;
    }
    double xC = xB + CM_GOLD * (xB - xA);
    double fC = F(xC);
    while (fC < fB) {
        if (*err || o->too_many) return NAN;
        double tmp1 = (xB - xA) * (fB - fC);
        double tmp2 = (xB - xC) * (fB - fA);
        double val = tmp2 - tmp1;
        double denom = fabs(val) < CM_EPS_MIN ? 2 * CM_EPS_MIN : val;
        double w = xB - ((xB - xC) * tmp2 - (xB - xA) * tmp1) / (2 * denom);
        double wLim = xB + 100 * (xC - xB);
        double fW;
        if ((w - xC) * (xB - w) > 0) {
            fW = F(w);
            if (fW < fC) {
                xA = xB; xB = w; fA = fB; fB = fW;
                break;
            } else if (fW > fB) {
                xC = w; fC = fW;
                break;
            }
            w = xC + CM_GOLD * (xC - xB);
            fW = F(w);
        } else if ((w - wLim) * (wLim - xC) >= 0) {
            w = wLim;
            fW = F(w);
        } else if ((w - wLim) * (xC - w) > 0) {
            fW = F(w);
            if (fW < fC) {
                xB = xC; xC = w; w = xC + CM_GOLD * (xC - xB);
                fB = fC; fC = fW;
                fW = F(w);
            }
        } else {
            w = xC + CM_GOLD * (xC - xB);
            fW = F(w);
        }
        xA = xB; fA = fB; xB = xC; fB = fC; xC = w; fC = fW;
    }
#undef F
    if (*err || o->too_many) return NAN;
    double lo = xA, mid = xB, hi = xC;
    if (lo > hi) { double t = lo; lo = hi; hi = t; }
    if (!(lo < hi) || !(mid >= lo && mid <= hi)) { *err = 2; return NAN; }  /* SearchInterval */

    /* BrentOptimizer.doOptimize, MINIMIZE, start = mid */
    const double rel = 1e-15, absT = 4.9e-324;
    const double GS = 0.5 * (3 - sqrt(5.0));
    double a = lo, b = hi;
    double x = mid, v = x, w = x, d = 0, e = 0;
    double fx = ewma_value(o, point + x * dir);
    double fv = fx, fw = fx;
    pv_t previous = {0, 0}, current = {x, fx}, best = current;
    int have_prev = 0;
    for (;;) {
        if (o->too_many) return NAN;
        const double m = 0.5 * (a + b);
        const double tol1 = rel * fabs(x) + absT;
        const double tol2 = 2 * tol1;
        const int stop = fabs(x - m) <= tol2 - 0.5 * (b - a);
        if (stop) {
            /* best(best, best(previous, current)) */
            pv_t bb = current;
            if (have_prev) bb = (previous.v <= current.v) ? previous : current;
            return (best.v <= bb.v) ? best.x : bb.x;
        }
        double p = 0, q = 0, r = 0, u = 0;
        if (fabs(e) > tol1) {
            r = (x - w) * (fv - fx);
            q = (x - v) * (fw - fx);
            p = (x - v) * q - (x - w) * r;
            q = 2 * (q - r);
            if (q > 0) p = -p;
            else q = -q;
            r = e;
            e = d;
            if (p > q * (a - x) && p < q * (b - x) && fabs(p) < fabs(0.5 * q * r)) {
                d = p / q;
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
        double fu = ewma_value(o, point + u * dir);
        previous = current;
        have_prev = 1;
        current.x = u;
        current.v = fu;
        {
            pv_t bb = (previous.v <= current.v) ? previous : current;
            best = (best.v <= bb.v) ? best : bb;
        }
        /* SimpleUnivariateValueChecker(1e-8, 1e-8) */
        {
            const double pvv = previous.v, cvv = current.v;
            const double diff = fabs(pvv - cvv);
            const double size = fmax(fabs(pvv), fabs(cvv));
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
            if (fu <= fw || cm_precision_equals(w, x)) {
                v = w; fv = fw;
                w = u; fw = fu;
            } else if (fu <= fv || cm_precision_equals(v, x) || cm_precision_equals(v, w)) {
                v = u; fv = fu;
            }
        }
    }
}

int orc_ewma_fit(const double* ts, int64_t n, double* smoothing, int64_t* evaluations) {
    ewma_obj_t o = {ts, n, 0, 0};
    double point = 0.94;                               /* InitialGuess(Array(.94)) */
    double r = -orc_ewma_gradient(ts, n, point);       /* MINIMIZE: r = -gradient */
    double dir = r;                                    /* IdentityPreconditioner */
    int have = 0;
    double cur_v = 0;
    int st = ORC_OK;
    for (int64_t iter = 1;; iter++) {
        if (iter > 10000) { st = ORC_ERR_TOO_MANY_ITERATIONS; break; }
        const double objective = ewma_value(&o, point);
        if (o.too_many) { st = ORC_ERR_TOO_MANY_EVALUATIONS; break; }
        if (have) {
            /* SimpleValueChecker(1e-6, 1e-6) */
            const double diff = fabs(cur_v - objective);
            const double size = fmax(fabs(cur_v), fabs(objective));
            if (diff <= size * 1e-6 || diff <= 1e-6) break;
        }
        have = 1;
        cur_v = objective;
        int lerr = 0;
        const double step = cm_line_search(&o, point, dir, &lerr);
        if (o.too_many || lerr == 1) { st = ORC_ERR_TOO_MANY_EVALUATIONS; break; }
        if (lerr == 2) { st = ORC_ERR_BAD_ARG; break; }
        point += step * dir;
        r = -orc_ewma_gradient(ts, n, point);
        dir = r;                                       /* iterations % 1 == 0: reset */
    }
    if (evaluations) *evaluations = o.evals;
    *smoothing = (st == ORC_OK) ? point : NAN;
    return st;
}

int orc_panel_ewma_fit(const double* in, int64_t S, int64_t T, int64_t ld, double* smoothing,
                       int32_t* err, int threads) {
    int any = 0;
#pragma omp parallel for schedule(dynamic, 64) num_threads(threads > 0 ? threads : 1) reduction(| : any)
    for (int64_t q = 0; q < S; q++) {
        int st = orc_ewma_fit(in + q * ld, T, smoothing + q, NULL);
        if (err) err[q] = st;
        any |= (st != ORC_OK);
    }
    return any ? ORC_ERR_TOO_MANY_EVALUATIONS : ORC_OK;
}

/* ---------------- TimeSeriesRDD.seriesStats / removeInstantsWithNaNs / toInstants ---------------- */

/* java.lang.Math.max / min (Scala math.max / min): NaN propagates; signed zeros ordered */
static double jmax(double a, double b) {
    if (a != a) return a;
    if (a == 0.0 && b == 0.0 && signbit(a)) return b;
    return (a >= b) ? a : b;
}
static double jmin(double a, double b) {
    if (a != a) return a;
    if (a == 0.0 && b == 0.0 && signbit(b)) return b;
    return (a <= b) ? a : b;
}

/* S/TimeSeriesRDD.scala:204-206: new StatCounter(series.valuesIterator).  Spark 1.3.1
 * StatCounter (spark-core, not vendored) restated: n = 0, mu = 0, m2 = 0, max = -Inf,
 * min = +Inf, then per value merge(value): delta = value - mu; n += 1; mu += delta / n;
 * m2 += delta * (value - mu); maxValue = math.max(maxValue, value); minValue = math.min(...).
 * out = (mu, m2, max, min); count = n. */
void orc_stat_counter(const double* ts, int64_t n, double out[4]) {
    int64_t cnt = 0;
    double mu = 0.0, m2 = 0.0, mx = -INFINITY, mn = INFINITY;
    for (int64_t i = 0; i < n; i++) {
        const double value = ts[i];
        const double delta = value - mu;
        cnt += 1;
        mu += delta / (double)cnt;
        m2 += delta * (value - mu);
        mx = jmax(mx, value);
        mn = jmin(mn, value);
    }
    out[0] = mu;
    out[1] = m2;
    out[2] = mx;
    out[3] = mn;
}

/* S/TimeSeriesRDD.scala:131-152: nans = aggregate(zero)(merge: arr(i) |= rec(i).isNaN,
 * comb: OR); activeIndices = indices with !nans; every series -> its values at activeIndices.
 * Returns the number of active instants; out is S x n_active (ld n_active), active[] the kept
 * positions. */
int64_t orc_remove_instants_with_nans(const double* in, int64_t S, int64_t T, int64_t ld, double* out,
                                      int64_t* active) {
    unsigned char* nans = (unsigned char*)calloc((size_t)(T > 0 ? T : 1), 1);
    for (int64_t s = 0; s < S; s++)
        for (int64_t i = 0; i < T; i++) nans[i] |= isnan(in[s * ld + i]) ? 1 : 0;
    int64_t na = 0;
    for (int64_t i = 0; i < T; i++)
        if (!nans[i]) active[na++] = i;
    for (int64_t s = 0; s < S; s++)
        for (int64_t j = 0; j < na; j++) out[s * na + j] = in[s * ld + active[j]];
    free(nans);
    return na;
}

/* S/TimeSeriesRDD.scala:215-324: one record per instant, values in series order */
void orc_to_instants(const double* in, int64_t S, int64_t T, int64_t ld, double* out) {
    for (int64_t t = 0; t < T; t++)
        for (int64_t s = 0; s < S; s++) out[t * S + s] = in[s * ld + t];
}

/* ---------------- panel drivers: one "partition" per thread (local[N]) ---------------- */

static int clamp_threads(int threads) { return threads > 0 ? threads : 1; }

static double now_ns(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec * 1e9 + (double)ts.tv_nsec;
}

/* bench.py --percall: one series' fillts / autocorr on one core, as the JVM's per-record
 * closure runs it (best of reps; the C loop is a lower bound on the JIT-compiled Scala's) */
double orc_time_fill(const double* x, double* r, int64_t n, int method, int reps) {
    double best = 1e300;
    for (int i = 0; i < reps; i++) {
        const double t0 = now_ns();
        (void)orc_fillts(x, r, n, method);
        const double dt = now_ns() - t0;
        if (dt < best) best = dt;
    }
    return best;
}

double orc_time_autocorr(const double* x, int64_t n, int K, double* out, int reps) {
    double best = 1e300;
    for (int i = 0; i < reps; i++) {
        const double t0 = now_ns();
        orc_autocorr(x, n, K, out);
        const double dt = now_ns() - t0;
        if (dt < best) best = dt;
    }
    return best;
}

int orc_panel_fill(const double* in, double* out, int64_t S, int64_t T, int64_t ld, int method,
                   int32_t* err, int threads) {
    if (method < 0 || method > 4) return ORC_ERR_UNSUPPORTED_METHOD;
    int first = ORC_OK;
#pragma omp parallel for schedule(static) num_threads(clamp_threads(threads))
    for (int64_t s = 0; s < S; s++) {
        int st = orc_fillts(in + s * ld, out + s * ld, T, method);
        if (err) err[s] = st;
        if (st != ORC_OK) {
#pragma omp atomic write
            first = st;
        }
    }
    return first;
}

int orc_panel_fill_autocorr(const double* in, double* filled, int64_t S, int64_t T, int64_t ld,
                            int method, int K, double* acf, int32_t* err, int threads) {
    if (method < -1 || method > 4) return ORC_ERR_UNSUPPORTED_METHOD;
    int any = 0;
#pragma omp parallel for schedule(static) num_threads(clamp_threads(threads)) reduction(max : any)
    for (int64_t s = 0; s < S; s++) {
        int st = ORC_OK;
        if (method >= 0) st = orc_fillts(in + s * ld, filled + s * ld, T, method);
        else memcpy(filled + s * ld, in + s * ld, (size_t)T * sizeof(double));
        if (err) err[s] = st;
        if (st != ORC_OK) {
            for (int k = 0; k < K; k++) acf[s * K + k] = NAN;
            any = st;
        } else {
            orc_autocorr(filled + s * ld, T, K, acf + s * K);
        }
    }
    return any;
}

/* C2 pipeline: fillPrevious -> differencesAtLag(1) -> EWMAModel(s).add */
int orc_panel_fill_diff_ewma(const double* in, double* out, int64_t S, int64_t T, int64_t ld,
                             double s, int threads) {
#pragma omp parallel num_threads(clamp_threads(threads))
    {
        double* tmp = (double*)malloc((size_t)(T > 0 ? T : 1) * sizeof(double));
        double* dif = (double*)malloc((size_t)(T > 0 ? T : 1) * sizeof(double));
#pragma omp for schedule(static)
        for (int64_t q = 0; q < S; q++) {
            orc_fill_previous(in + q * ld, tmp, T);
            memcpy(dif, tmp, (size_t)T * sizeof(double));
            orc_differences_at_lag(tmp, dif, T, 1, 1);
            orc_ewma_add(dif, out + q * ld, T, s);
        }
        free(tmp);
        free(dif);
    }
    return ORC_OK;
}

/* C4 pipeline: Autoregression.fitModel(ts, p) -> ARModel.removeTimeDependentEffects(ts) */
int orc_panel_ar_fit_remove(const double* in, double* out, int64_t S, int64_t T, int64_t ld,
                            int p, int no_intercept, double* c, double* coef, int threads) {
    int any = 0;
#pragma omp parallel for schedule(static) num_threads(clamp_threads(threads)) reduction(| : any)
    for (int64_t q = 0; q < S; q++) {
        int st = orc_ar_fit(in + q * ld, T, p, no_intercept, c + q, coef + q * p);
        if (st != ORC_OK) {
            any = 1;
            c[q] = NAN;
            for (int j = 0; j < p; j++) coef[q * p + j] = NAN;
        }
        orc_ar_remove(in + q * ld, out + q * ld, T, c[q], coef + q * p, p);
    }
    return any ? ORC_ERR_SINGULAR : ORC_OK;
}

/* ---------------- synthetic generator ---------------- */

void orc_philox4x32_10(const uint32_t ctr_in[4], const uint32_t key_in[2], uint32_t out[4]) {
    uint32_t c0 = ctr_in[0], c1 = ctr_in[1], c2 = ctr_in[2], c3 = ctr_in[3];
    uint32_t k0 = key_in[0], k1 = key_in[1];
    for (int r = 0; r < 10; r++) {
        uint64_t p0 = (uint64_t)0xD2511F53u * c0;
        uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
        uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
        uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
        uint32_t n0 = hi1 ^ c1 ^ k0;
        uint32_t n2 = hi0 ^ c3 ^ k1;
        c0 = n0;
        c1 = lo1;
        c2 = n2;
        c3 = lo0;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    out[0] = c0;
    out[1] = c1;
    out[2] = c2;
    out[3] = c3;
}

static inline double u53(uint32_t a, uint32_t b) {
    uint64_t m = ((uint64_t)(a >> 5) << 26) | (uint64_t)(b >> 6);
    return (double)m * 0x1p-53;
}

static inline void gen_words(uint64_t seed, int64_t s, uint64_t t, uint32_t out[4]) {
    uint32_t ctr[4] = {(uint32_t)t, (uint32_t)(t >> 32), (uint32_t)(uint64_t)s,
                       (uint32_t)((uint64_t)s >> 32)};
    uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
    orc_philox4x32_10(ctr, key, out);
}

static double gen_series_u(uint64_t seed, int64_t s) {
    uint32_t w[4];
    gen_words(seed, s, ~(uint64_t)0, w);
    return u53(w[0], w[1]);
}

/* x[s,t] = 100 + 10*u_s + t/T + (u_{s,t} - 0.5) */
double orc_gen_value(uint64_t seed, int64_t s, int64_t t, int64_t T) {
    uint32_t w[4];
    gen_words(seed, s, (uint64_t)t, w);
    double us = gen_series_u(seed, s);
    double ust = u53(w[0], w[1]);
    return ((100.0 + 10.0 * us) + (double)t / (double)T) + (ust - 0.5);
}

uint32_t orc_nan_threshold(double p) {
    if (!(p > 0.0)) return 0;
    if (p >= 1.0) return 0xFFFFFFFFu;
    return (uint32_t)floor(p * 4294967296.0);
}

int orc_gen_is_nan(uint64_t seed, int64_t s, int64_t t, uint32_t thr) {
    uint32_t w[4];
    gen_words(seed, s, (uint64_t)t, w);
    return w[2] < thr;
}

void orc_gen_panel(uint64_t seed, int64_t s0, int64_t S, int64_t T, int64_t ld, double nan_p,
                   double* out) {
    uint32_t thr = orc_nan_threshold(nan_p);
    for (int64_t q = 0; q < S; q++) {
        int64_t s = s0 + q;
        double us = gen_series_u(seed, s);
        for (int64_t t = 0; t < T; t++) {
            uint32_t w[4];
            gen_words(seed, s, (uint64_t)t, w);
            double v = ((100.0 + 10.0 * us) + (double)t / (double)T) + (u53(w[0], w[1]) - 0.5);
            out[q * ld + t] = (w[2] < thr) ? NAN : v;
        }
    }
}

/* C4: AR(p) series, phi = base * (1 + 0.1*(u_s - 0.5)), c = 1, innovations
 * u_{s,t} - 0.5, built with ARModel.addTimeDependentEffects semantics. */
static const double kArBase[8] = {0.3, -0.2, 0.1, 0.05, -0.05, 0.02, -0.02, 0.01};

void orc_gen_ar_params(uint64_t seed, int64_t s, int p, double* c, double* phi) {
    double us = gen_series_u(seed, s);
    double scale = 1.0 + 0.1 * (us - 0.5);
    *c = 1.0;
    for (int j = 0; j < p; j++) phi[j] = kArBase[j & 7] * scale;
}

void orc_gen_ar_panel(uint64_t seed, int64_t s0, int64_t S, int64_t T, int64_t ld, int p,
                      double* out) {
    double phi[64];
    for (int64_t q = 0; q < S; q++) {
        int64_t s = s0 + q;
        double c;
        orc_gen_ar_params(seed, s, p, &c, phi);
        double* d = out + q * ld;
        for (int64_t t = 0; t < T; t++) {
            uint32_t w[4];
            gen_words(seed, s, (uint64_t)t, w);
            double e = u53(w[0], w[1]) - 0.5;
            d[t] = c + e;
            for (int j = 0; j < p && t - j - 1 >= 0; j++) d[t] += d[t - j - 1] * phi[j];
        }
    }
}
