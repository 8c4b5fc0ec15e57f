/*
 * sts_oracle.h -- CPU restatement of the spark-timeseries hot-path algorithms.
 *
 * TEST INFRASTRUCTURE ONLY.  This library is the parity oracle: only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it, and
 * only as the checker / the CPU baseline, never as the product path.  The
 * product is libsts_hip.so (spark-timeseries_amd/csrc), which never links or
 * calls anything here.
 *
 * Every function restates the reference loop statement by statement (citations
 * per function in sts_oracle.c; S/ = /root/reference/src/main/scala/com/
 * cloudera/sparkts/).  Arithmetic is IEEE-754 binary64, round-to-nearest, no
 * FMA contraction (build with -ffp-contract=off), i.e. the JVM's semantics.
 *
 * Panel convention: S series x T steps, series-contiguous, element (s, t) at
 * s*ld + t (Breeze DenseMatrix(T, S) column-major, S/TimeSeries.scala:25-26).
 */
#ifndef STS_ORACLE_H
#define STS_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* status codes shared with include/sts.h */
#define ORC_OK 0
#define ORC_ERR_BAD_ARG 1
#define ORC_ERR_ALL_NAN 2
#define ORC_ERR_UNSUPPORTED_METHOD 3
#define ORC_ERR_REQUIREMENT 5
#define ORC_ERR_NOT_ENOUGH_DATA 7
#define ORC_ERR_SINGULAR 8
#define ORC_ERR_TOO_MANY_EVALUATIONS 10
#define ORC_ERR_TOO_MANY_ITERATIONS 11
#define ORC_ERR_TOO_FEW_POINTS 12     /* commons-math3 NumberIsTooSmallException (spline: < 3 knots) */

/* fill methods (same numbering as include/sts.h) */
#define ORC_FILL_LINEAR 0
#define ORC_FILL_NEAREST 1
#define ORC_FILL_NEXT 2
#define ORC_FILL_PREVIOUS 3
#define ORC_FILL_SPLINE 4

/* ---- single-series restatements ---- */
void orc_fill_previous(const double* x, double* r, int64_t n);
void orc_fill_next(const double* x, double* r, int64_t n);
int  orc_fill_nearest(const double* x, double* r, int64_t n);   /* ORC_ERR_ALL_NAN on throw */
void orc_fill_linear(const double* x, double* r, int64_t n);
int  orc_fill_spline(const double* x, double* r, int64_t n);    /* ORC_ERR_TOO_FEW_POINTS on throw */
int  orc_fillts(const double* x, double* r, int64_t n, int method);
void orc_autocorr(const double* x, int64_t n, int K, double* out);
int  orc_lag_mat_trim_both(const double* x, int64_t n, int max_lag, int include_original,
                           double* out /* (n-max_lag) x ncols column-major */);
int  orc_differences_at_lag(const double* ts, double* dest, int64_t n, int lag, int start);
int  orc_inverse_differences_at_lag(const double* d, double* dest, int64_t n, int lag, int start);
void orc_differences_of_order_d(const double* ts, double* out, int64_t n, int d);
void orc_ewma_add(const double* ts, double* dest, int64_t n, double s);
void orc_ewma_remove(const double* ts, double* dest, int64_t n, double s);
void orc_ar_remove(const double* ts, double* dest, int64_t n, double c, const double* coef, int p);
void orc_ar_add(const double* ts, double* dest, int64_t n, double c, const double* coef, int p);
int  orc_ar_fit(const double* ts, int64_t n, int p, int no_intercept, double* c, double* coef);
double orc_ewma_sse(const double* ts, int64_t n, double s);
double orc_ewma_gradient(const double* ts, int64_t n, double s);
int  orc_ewma_fit(const double* ts, int64_t n, double* smoothing, int64_t* evaluations);
void orc_stat_counter(const double* ts, int64_t n, double out[4]);
int64_t orc_remove_instants_with_nans(const double* in, int64_t S, int64_t T, int64_t ld, double* out,
                                      int64_t* active);
void orc_to_instants(const double* in, int64_t S, int64_t T, int64_t ld, double* out);
int  orc_ols_householder(const double* y, const double* x /* m x k row-major */, int64_t m,
                         int k, int no_intercept, double* beta /* k(+1) */);

/* ---- GARCH(1,1), AR(1)+GARCH(1,1): sts_oracle_garch.c (S/models/GARCH.scala) ---- */
double orc_fdlibm_log(double x);   /* StrictMath.log */
double orc_garch_loglik(const double* ts, int64_t n, double omega, double alpha, double beta);
void orc_garch_gradient(const double* ts, int64_t n, double omega, double alpha, double beta,
                        double g[3]);
int  orc_garch_fit(const double* ts, int64_t n, double params[3] /* omega, alpha, beta */,
                   int64_t* evaluations);
int  orc_argarch_fit(const double* ts, int64_t n, double out[5] /* c, phi, omega, alpha, beta */,
                     int64_t* evaluations);
void orc_garch_remove(const double* ts, double* dest, int64_t n, double omega, double alpha, double beta);
void orc_garch_add(const double* ts, double* dest, int64_t n, double omega, double alpha, double beta);
void orc_argarch_remove(const double* ts, double* dest, int64_t n, double c, double phi,
                        double omega, double alpha, double beta);
void orc_argarch_add(const double* ts, double* dest, int64_t n, double c, double phi,
                     double omega, double alpha, double beta);
int  orc_panel_garch_fit(const double* in, int64_t S, int64_t T, int64_t ld, double* params,
                         int32_t* err, int threads);
int  orc_panel_argarch_fit(const double* in, int64_t S, int64_t T, int64_t ld, double* params,
                           int32_t* err, int threads);

/* ---- panel drivers (threads = 0 -> 1 thread) ---- */
int orc_panel_fill(const double* in, double* out, int64_t S, int64_t T, int64_t ld, int method,
                   int32_t* err, int threads);
int orc_panel_fill_autocorr(const double* in, double* filled, int64_t S, int64_t T, int64_t ld,
                            int method, int K, double* acf, int32_t* err, int threads);
int orc_panel_fill_diff_ewma(const double* in, double* out, int64_t S, int64_t T, int64_t ld,
                             double s, int threads);
int orc_panel_ar_fit_remove(const double* in, double* out, int64_t S, int64_t T, int64_t ld,
                            int p, int no_intercept, double* c, double* coef, int threads);

int orc_panel_ewma_fit(const double* in, int64_t S, int64_t T, int64_t ld, double* smoothing,
                       int32_t* err, int threads);

/* ---- per-call cost of one series (bench.py --percall: the CPU side of the S = 1 crossover),
 * timed inside C so no FFI overhead is counted: ns per call, best of `reps` calls. ---- */
double orc_time_fill(const double* x, double* r, int64_t n, int method, int reps);
double orc_time_autocorr(const double* x, int64_t n, int K, double* out, int reps);

/* ---- synthetic generator; bit-identical to the device generator ---- */
void   orc_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]);
double orc_gen_value(uint64_t seed, int64_t s, int64_t t, int64_t T);
int    orc_gen_is_nan(uint64_t seed, int64_t s, int64_t t, uint32_t nan_threshold);
uint32_t orc_nan_threshold(double p);
void   orc_gen_panel(uint64_t seed, int64_t s0, int64_t S, int64_t T, int64_t ld, double nan_p,
                     double* out);
void   orc_gen_ar_panel(uint64_t seed, int64_t s0, int64_t S, int64_t T, int64_t ld, int p,
                        double* out);
void   orc_gen_ar_params(uint64_t seed, int64_t s, int p, double* c, double* phi);

#ifdef __cplusplus
}
#endif
#endif
