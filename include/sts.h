/*
 * sts.h -- C ABI of libsts_hip.so, the MI355X (gfx950) engine for the
 * spark-timeseries series-wise hot path.
 *
 * Every entry point below replaces a reference operator that Spark calls once
 * per (key, series) record inside a narrow map task
 * (TimeSeriesRDD.mapSeries, S/TimeSeriesRDD.scala:188-199).  Here one call
 * processes a whole PANEL of series (a partition's records gathered into one
 * buffer), which is the batching the JNI shim performs.
 *
 *   S/ = src/main/scala/com/cloudera/sparkts/ in the reference.
 *
 * Panel layout: S series x T time steps, fp64, series-contiguous: element
 * (s, t) of a panel with leading dimension ld (ld >= T) is at p[s*ld + t].
 * This is Breeze DenseMatrix(T, S) column-major as built by
 * TimeSeriesRDD.collectAsTimeSeries (S/TimeSeriesRDD.scala:66-71) and each
 * record's DenseVector.data.  NaN marks a missing observation.
 *
 * Memory: functions without a `_host` suffix take DEVICE pointers (HBM,
 * e.g. hipMalloc'd) and are stream-ordered on `stream` (a hipStream_t; NULL
 * means hipStreamPerThread, so concurrent executor threads never serialise
 * on the legacy null stream).  `_host` variants take host pointers, stage
 * through HBM on the calling thread's stream and return when the results
 * are back on the host (the JNI path).
 *
 * Errors: every function returns an sts_status; sts_last_error() gives a
 * thread-local message.  Per-series data errors (fillNearest on an all-NaN
 * series, singular AR designs) are written to an optional device int32
 * array err_per_series[S] (0 = ok, else an sts_status); when that pointer is
 * NULL the call synchronises its stream and returns the first failing status,
 * which is the reference's exception semantics (a task exception).
 *
 * Arithmetic: IEEE binary64, no FMA contraction on the bit-exact paths
 * (fills, differencing, lag matrices, EWMA/AR add and remove); the
 * reductions (autocorr, AR fit) match the reference within 1e-10 relative.
 */
#ifndef STS_H
#define STS_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define STS_ABI_VERSION 1

/* Status codes.  The comment names the JVM exception the reference throws. */
typedef enum sts_status {
    STS_OK = 0,
    STS_ERR_BAD_ARG = 1,            /* IllegalArgumentException (argument validation)      */
    STS_ERR_ALL_NAN = 2,            /* IllegalArgumentException("Input is all NaNs!"),
                                       S/UnivariateTimeSeries.scala:170-171                */
    STS_ERR_UNSUPPORTED_METHOD = 3, /* UnsupportedOperationException, :148                  */
    STS_ERR_HIP = 4,                /* device / runtime failure                             */
    STS_ERR_REQUIREMENT = 5,        /* IllegalArgumentException("requirement failed: ..."),
                                       :361 / :402                                          */
    STS_ERR_NULL_DEST = 6,          /* NullPointerException (EWMAModel with dest = null,
                                       S/models/EWMA.scala:125-127,135-136)                 */
    STS_ERR_NOT_ENOUGH_DATA = 7,    /* commons-math3 MathIllegalArgumentException
                                       NOT_ENOUGH_DATA_FOR_NUMBER_OF_PREDICTORS              */
    STS_ERR_SINGULAR = 8,           /* commons-math3 SingularMatrixException                 */
    STS_ERR_NO_DEVICE = 9,          /* no gfx950 device visible                              */
    STS_ERR_TOO_MANY_EVALUATIONS = 10, /* commons-math3 TooManyEvaluationsException (EWMA fit) */
    STS_ERR_TOO_MANY_ITERATIONS = 11,  /* commons-math3 TooManyIterationsException (EWMA fit)  */
    STS_ERR_TOO_FEW_POINTS = 12        /* commons-math3 NumberIsTooSmallException(NUMBER_OF_POINTS,
                                          n, 3, true): fill "spline" on a series with fewer than
                                          3 non-NaN values (SplineInterpolator.interpolate)     */
} sts_status;

/* Fill methods of UnivariateTimeSeries.fillts (S/UnivariateTimeSeries.scala:141-150). */
typedef enum sts_fill_method {
    STS_FILL_NONE = -1,     /* identity (no imputation); fused kernels only */
    STS_FILL_LINEAR = 0,    /* fillLinear   :247-266 */
    STS_FILL_NEAREST = 1,   /* fillNearest  :156-184 */
    STS_FILL_NEXT = 2,      /* fillNext     :214-224 */
    STS_FILL_PREVIOUS = 3,  /* fillPrevious :194-204 */
    STS_FILL_SPLINE = 4     /* fillSpline   :268-297 (commons-math3 3.4.1 natural cubic
                               SplineInterpolator; sts_spline.hip, not fused) */
} sts_fill_method;

/* ---- library / runtime ---- */
int         sts_abi_version(void);
/* Select the HIP device for the calling thread (idempotent). */
int         sts_init(int device);
/* Thread-local description of the last non-OK status on this thread. */
const char* sts_last_error(void);
/* Map a fillts method string ("linear", "nearest", "next", "previous", "spline")
 * to sts_fill_method; returns -2 for anything else (the reference's
 * UnsupportedOperationException, S/UnivariateTimeSeries.scala:148). */
int         sts_fill_method_from_name(const char* name);
/* Wait for all work this library queued on `stream`. */
int         sts_stream_synchronize(void* stream);
/* Measurement hooks (bench.py): while on, HIP events are recorded on the launch stream
 * around every series-tile kernel launched by the calling thread; sts_profile_end waits
 * for them and returns the summed kernel time and the number of launches. */
int         sts_profile_begin(void);
int         sts_profile_end(double* kernel_ms, int64_t* launches);

/* ---- a1-a5: TimeSeriesRDD.fill(method) -> UnivariateTimeSeries.fillts
 *      (S/TimeSeriesRDD.scala:180-182, S/UnivariateTimeSeries.scala:141-297).
 * out must not alias in (the reference always fills a fresh copy, :157/:195/:215/:248/:276).
 * Per-series errors: STS_ERR_ALL_NAN (nearest), STS_ERR_TOO_FEW_POINTS (spline).  Bit-exact. */
int sts_fill(const double* in, double* out, int64_t S, int64_t T, int64_t ld_in, int64_t ld_out,
             int method, int32_t* err_per_series, void* stream);

/* ---- a6: UnivariateTimeSeries.differencesAtLag(ts, dest, lag, startIndex)
 *      (S/UnivariateTimeSeries.scala:356-376; the (ts, lag) wrapper :384-386 is start = lag).
 * out == in (same pointer and ld) reproduces the reference's in-place (dest eq ts)
 * semantics, where later elements read already-differenced values.  lag == 0
 * leaves out untouched (:363-364).  start < lag -> STS_ERR_REQUIREMENT.  Bit-exact. */
int sts_diff_at_lag(const double* in, double* out, int64_t S, int64_t T, int64_t ld_in,
                    int64_t ld_out, int lag, int start, void* stream);

/* ---- a7: UnivariateTimeSeries.lag(ts, maxLag, includeOriginal) -> Lag.lagMatTrimBoth
 *      (S/UnivariateTimeSeries.scala:37-39, S/Lag.scala:62-77).
 * Series s's (T - maxLag) x (maxLag + inc) column-major block is written at
 * out + s * (T - maxLag) * (maxLag + inc), i.e. the panel form of TimeSeries.lags
 * (S/TimeSeries.scala:50-73).  Bit-exact. */
int sts_lag_matrix(const double* in, double* out, int64_t S, int64_t T, int64_t ld_in,
                   int max_lag, int include_original, void* stream);

/* ---- a8: UnivariateTimeSeries.autocorr(ts, numLags) (S/UnivariateTimeSeries.scala:68-93).
 * acf[s*K + (i-1)] = lag-i sample autocorrelation, i = 1..K, any K >= 0 (lags >= T are NaN,
 * as the reference's empty slices give).  K <= 63 runs fused in the imputation kernels, larger
 * K in 61-lag MFMA blocks (sts_acf_wide.hip).  1e-10 relative. */
int sts_autocorr(const double* in, int64_t S, int64_t T, int64_t ld, int K, double* acf,
                 void* stream);

/* ---- a9 / a10: EWMAModel.add/removeTimeDependentEffects (S/models/EWMA.scala:125-142).
 * smoothing[s] is series s's model parameter (device array of S doubles).
 * out == in is allowed for add (safe in the reference) and for remove (reproduces the
 * reference's read-after-overwrite).  out == NULL -> STS_ERR_NULL_DEST.  Bit-exact. */
int sts_ewma_add(const double* in, double* out, int64_t S, int64_t T, int64_t ld_in,
                 int64_t ld_out, const double* smoothing, void* stream);
int sts_ewma_remove(const double* in, double* out, int64_t S, int64_t T, int64_t ld_in,
                    int64_t ld_out, const double* smoothing, void* stream);

/* ---- f1: EWMA.fitModel(ts) (S/models/EWMA.scala:44-68), every series of a panel in one
 * call.  smoothing[s] receives the fitted parameter.  The optimizer is commons-math3 3.4.1's
 * NonLinearConjugateGradientOptimizer (Fletcher-Reeves, SimpleValueChecker(1e-6, 1e-6), line
 * search = BracketFinder + BrentOptimizer, start 0.94, MaxIter / MaxEval 10000), run per
 * series on the device; every sse / gradient evaluation is the reference's sequential loop
 * (bit-exact), so the fit follows the reference's optimizer path.  A series the optimizer
 * cannot fit (any NaN: every sse is NaN) gets NaN and STS_ERR_TOO_MANY_EVALUATIONS. */
int sts_ewma_fit(const double* in, int64_t S, int64_t T, int64_t ld, double* smoothing,
                 int32_t* err_per_series, void* stream);
/* EWMAModel(smoothing[s]).sse(ts) (:80-95) and .gradient(ts) (:102-123) per series, one
 * pass; sse or gradient may be NULL.  Bit-exact. */
int sts_ewma_sse_gradient(const double* in, int64_t S, int64_t T, int64_t ld,
                          const double* smoothing, double* sse, double* gradient, void* stream);

/* ---- f1: GARCH(1,1) and AR(1)+GARCH(1,1) (S/models/GARCH.scala) ----
 * GARCH.fitModel (:33-53) per series: commons-math3 NLCG (Fletcher-Reeves) from
 * (.2, .2, .2) without a GoalType (its maximising branches), MaxIter / MaxEval 10000;
 * params[s*3 + 0..2] = (omega, alpha, beta).  A series the reference cannot fit gets NaN
 * params and its status in err_per_series (device, optional; NULL -> the first failure is
 * returned): STS_ERR_TOO_MANY_EVALUATIONS (e.g. any NaN), STS_ERR_TOO_MANY_ITERATIONS,
 * STS_ERR_BAD_ARG (invalid line-search interval).  Bit-exact against the restatement
 * (Math.log evaluated as StrictMath.log / fdlibm). */
int sts_garch_fit(const double* in, int64_t S, int64_t T, int64_t ld, double* params,
                  int32_t* err_per_series, void* stream);
/* GARCHModel(params[s]).logLikelihood(ts) (:80-86) and .gradient(ts) (:94-114) per series,
 * one pass; gradient[s*3 + 0..2] in the reference's (alpha, beta, omega) order. */
int sts_garch_loglik_gradient(const double* in, int64_t S, int64_t T, int64_t ld,
                              const double* params, double* loglik, double* gradient,
                              void* stream);
/* GARCHModel.removeTimeDependentEffects / addTimeDependentEffects (:130-159), per-series
 * omega / alpha / beta.  out == NULL -> STS_ERR_NULL_DEST; out == in is the reference's
 * dest eq ts (identical here: both read ts(i) before writing dest(i)).  Bit-exact. */
int sts_garch_remove(const double* in, double* out, int64_t S, int64_t T, int64_t ld_in,
                     int64_t ld_out, const double* omega, const double* alpha,
                     const double* beta, void* stream);
int sts_garch_add(const double* in, double* out, int64_t S, int64_t T, int64_t ld_in,
                  int64_t ld_out, const double* omega, const double* alpha,
                  const double* beta, void* stream);
/* ARGARCHModel.removeTimeDependentEffects / addTimeDependentEffects (:203-234).  remove
 * with out == in reproduces the reference's read of the overwritten ts(i - 1).  Bit-exact. */
int sts_argarch_remove(const double* in, double* out, int64_t S, int64_t T, int64_t ld_in,
                       int64_t ld_out, const double* c, const double* phi, const double* omega,
                       const double* alpha, const double* beta, void* stream);
int sts_argarch_add(const double* in, double* out, int64_t S, int64_t T, int64_t ld_in,
                    int64_t ld_out, const double* c, const double* phi, const double* omega,
                    const double* alpha, const double* beta, void* stream);
/* ARGARCH.fitModel (:62-68): Autoregression.fitModel(ts) (AR(1) with intercept, the a11
 * kernels) -> c[s], phi[s]; its residuals (a12, into a scratch panel) -> GARCH.fitModel ->
 * params[s*3 + 0..2].  T < 3 -> STS_ERR_NOT_ENOUGH_DATA.  An AR-stage failure keeps its
 * status.  c / phi within 1e-10 of the Householder-QR restatement; the GARCH stage is
 * bit-exact given the residuals. */
int sts_argarch_fit(const double* in, int64_t S, int64_t T, int64_t ld, double* c, double* phi,
                    double* params, int32_t* err_per_series, void* stream);

/* ---- f2: TimeSeriesRDD.seriesStats() (S/TimeSeriesRDD.scala:204-206): Spark 1.3.1
 * StatCounter over each series' values, NaN included, merged in order
 * (delta = v - mu; n += 1; mu += delta / n; m2 += delta * (v - mu); max / min via
 * java.lang.Math).  stats[s*4 + 0..3] = (mean, m2, max, min); count = T for every series
 * (variance = m2 / n etc. are derived exactly as StatCounter does).  Bit-exact. */
int sts_series_stats(const double* in, int64_t S, int64_t T, int64_t ld, double* stats,
                     void* stream);
/* Memory access: the kernel reads whole 128-byte lines, so it may read up to 15
 * doubles before in[0] and up to 15 after in[(S-1)*ld + T-1] -- always inside the 128-byte lines
 * (hence the pages) that hold those two elements, never a line the panel does not touch. */

/* ---- f3: TimeSeriesRDD.removeInstantsWithNaNs() (S/TimeSeriesRDD.scala:131-152) in three
 * steps, so partitions on different GPUs can combine their NaN flags in between (an
 * all-reduce MAX of `flags`, the reference's aggregate(merge, comb) of Boolean arrays):
 *   sts_nan_instants     flags[t] = 1 where any series of the panel is NaN at t (flags are
 *                        only ever set: zero them first; repeated calls OR together);
 *   sts_active_instants  active[0 .. *n_active) = the instants with flags[t] == 0, in
 *                        increasing order; n_active is a device int64;
 *   sts_gather_instants  out[s*ld_out + j] = in[s*ld_in + active[j]], j < n_active.
 * Bit-exact (copies). */
int sts_nan_instants(const double* in, int64_t S, int64_t T, int64_t ld, uint8_t* flags,
                     void* stream);
int sts_active_instants(const uint8_t* flags, int64_t T, int64_t* active, int64_t* n_active,
                        void* stream);
int sts_gather_instants(const double* in, double* out, int64_t S, int64_t ld_in, int64_t ld_out,
                        const int64_t* active, int64_t n_active, void* stream);

/* ---- f4: TimeSeriesRDD.toInstants (S/TimeSeriesRDD.scala:215-324), the local step: the
 * panel transpose out[t*ld_out + s] = in[s*ld_in + t] -- one record per instant holding
 * every series' value in partition (series) order.  Across GPUs the instants are
 * re-partitioned by time with an all-to-all (sparkts.TimeSeriesRDD.toInstants).  Bit-exact. */
int sts_to_instants(const double* in, double* out, int64_t S, int64_t T, int64_t ld_in,
                    int64_t ld_out, void* stream);

/* ---- f5: ingest / egress formats -- the step before the hot path (staging a partition
 * into the HBM panel) and the way back.
 *
 * Python wire format (S/PythonConnector.scala:47-90 BytesToKeyAndSeries / KeyAndSeriesToBytes,
 * python/sparkts/timeseriesrdd.py:239-290): a record is int32 BE keyLen | keyLen UTF-8 bytes |
 * int32 BE n | n x float64 BE; `bytes` holds records back to back.
 *   sts_wire_scan (HOST memory, no device): walks the headers; fills key_off / key_len /
 *     val_off (byte offsets) for up to max_records records, *n_records and *T.  Every record
 *     must hold the same n (one shared index): otherwise STS_ERR_BAD_ARG, as is a truncated
 *     or overrunning record.
 *   sts_wire_decode (device): panel[s*ld + t] = the BE double at bytes[val_off[s] + 8t].
 *   sts_wire_encode (device): the inverse, value blocks only (headers are the caller's).
 * Bit-exact (byte permutations). */
int sts_wire_scan(const uint8_t* bytes, int64_t nbytes, int64_t max_records, int64_t* n_records,
                  int64_t* T, int64_t* key_off, int32_t* key_len, int64_t* val_off);
int sts_wire_decode(const uint8_t* bytes, const int64_t* val_off, int64_t S, int64_t T,
                    double* panel, int64_t ld, void* stream);
int sts_wire_encode(const double* panel, int64_t S, int64_t T, int64_t ld, const int64_t* val_off,
                    uint8_t* bytes, void* stream);
/* timeSeriesRDDFromObservations (S/TimeSeriesRDD.scala:493-542): panel (S x T, ld) = NaN, then
 * observation i writes value[i] at (series_id[i], loc[i]) -- loc = targetIndex.locAtDateTime
 * of its timestamp, negative = not in the index (dropped, :529-535).  Among observations of
 * one cell the LAST in input order wins (the reference keeps the last in its (key, time) sort
 * order).  Device arrays. */
int sts_observations_to_panel(const int32_t* series_id, const int64_t* loc, const double* value,
                              int64_t n_obs, double* panel, int64_t S, int64_t T, int64_t ld,
                              void* stream);
/* timeSeriesRDDFromCsv (S/TimeSeriesRDD.scala:547-561), the per-line parse
 * `key,v1,...,vn` (HOST memory): up to max_records lines of `text`; values go row-major into
 * `values` (capacity values_cap doubles, ld = T), keys as (key_off, key_len) into text.
 * Numbers parse as java.lang.Double.parseDouble does for decimal / NaN / Infinity tokens.
 * Every line must hold the same number of values. */
int sts_csv_parse(const char* text, int64_t len, int64_t max_records, int64_t* n_records,
                  int64_t* T, int64_t* key_off, int32_t* key_len, double* values,
                  int64_t values_cap);

/* ---- a11: Autoregression.fitModel(ts, p, noIntercept) (S/models/Autoregression.scala:38-53).
 * c[s] and coef[s*p + j] receive the model; 1 <= p <= 31.  T - p < p + 1 ->
 * STS_ERR_NOT_ENOUGH_DATA.  1e-10 relative to commons-math3's Householder-QR OLS: a series
 * the fast fit flags as ill-conditioned ("AR rule": level / spread, collinear lags, fragile
 * coefficients), and every noIntercept series, is fitted with the reference's own QR
 * operation order -- bit-identical to it. */
int sts_ar_fit(const double* in, int64_t S, int64_t T, int64_t ld, int p, int no_intercept,
               double* c, double* coef, int32_t* err_per_series, void* stream);
/* Diagnostic: how many of the S series the AR rule sends to the reference-order QR for
 * sts_ar_fit(in, S, T, ld, p, no_intercept, ...) (synchronous; noIntercept: all S). */
int sts_ar_rule_count(const double* in, int64_t S, int64_t T, int64_t ld, int p, int no_intercept,
                      int64_t* count, void* stream);

/* ---- f1b: ARIMA.fitModel(p, d, 0, ts, includeIntercept) -- the AR-only path
 * (S/models/ARIMA.scala:80-90): differencesOfOrderD(ts, d) (S/UnivariateTimeSeries.scala:
 * 438-450, ping-pong buffers) with the first d values dropped, then
 * Autoregression.fitModel(diffed, p, !includeIntercept).  The ARIMAModel's coefficients are
 * [c (if includeIntercept)] ++ coef.  Differencing bit-exact, the fit 1e-10 relative. */
int sts_arima_fit_ar(const double* in, int64_t S, int64_t T, int64_t ld, int p, int d,
                     int include_intercept, double* c, double* coef, int32_t* err_per_series,
                     void* stream);

/* ---- a12 / a13: ARModel.remove/addTimeDependentEffects (S/models/Autoregression.scala:60-88).
 * out == in reproduces the reference's aliasing semantics.  Bit-exact. */
int sts_ar_remove(const double* in, double* out, int64_t S, int64_t T, int64_t ld_in,
                  int64_t ld_out, const double* c, const double* coef, int p, void* stream);
int sts_ar_add(const double* in, double* out, int64_t S, int64_t T, int64_t ld_in,
               int64_t ld_out, const double* c, const double* coef, int p, void* stream);

/* ---- fused mapSeries pipelines (one pass over HBM; each returned output written once) ---- */

/* C1/C3: fill(method) then autocorr(K) of the filled series.  filled may be NULL when
 * method == STS_FILL_NONE. */
int sts_fill_autocorr(const double* in, double* filled, int64_t S, int64_t T, int64_t ld_in,
                      int64_t ld_out, int method, int K, double* acf, int32_t* err_per_series,
                      void* stream);
/* C2: fill(method) -> differencesAtLag(lag) -> EWMAModel(smoothing[s]).addTimeDependentEffects */
int sts_fill_diff_ewma(const double* in, double* out, int64_t S, int64_t T, int64_t ld_in,
                       int64_t ld_out, int method, int lag, const double* smoothing,
                       int32_t* err_per_series, void* stream);
/* C5: fill(method) -> lag(maxLag, includeOriginal); filled may be NULL (not returned). */
int sts_fill_lag_matrix(const double* in, double* filled, double* lagmat, int64_t S, int64_t T,
                        int64_t ld_in, int64_t ld_out, int method, int max_lag,
                        int include_original, int32_t* err_per_series, void* stream);
/* C4: Autoregression.fitModel(ts, p, noIntercept) -> model.removeTimeDependentEffects(ts) */
int sts_ar_fit_remove(const double* in, double* out, int64_t S, int64_t T, int64_t ld_in,
                      int64_t ld_out, int p, int no_intercept, double* c, double* coef,
                      int32_t* err_per_series, void* stream);

/* ---- synthetic panels: counter-based Philox4x32-10, bit-identical
 * to the CPU generator in oracle/, so any shard can be regenerated anywhere. ---- */
int sts_gen_panel(double* out, int64_t s0, int64_t S, int64_t T, int64_t ld, uint64_t seed,
                  double nan_p, void* stream);
int sts_gen_ar_panel(double* out, double* c, double* phi, int64_t s0, int64_t S, int64_t T,
                     int64_t ld, uint64_t seed, int p, void* stream);

/* ---- host-buffer variants (JNI path).  Each call runs a PINNED STAGING PIPELINE: the
 * panel is split by series into chunks of ~64 MB of device traffic, and each chunk's H2D
 * copy, kernel(s) and D2H copy run on one of the FIVE slots (a HIP stream, a 64 MB device
 * buffer and a pinned bounce buffer each) of a slot set, so uploads, compute and downloads of
 * consecutive chunks overlap.  A call borrows one slot set from a process-wide pool for its
 * duration: at most sts_staging_set_limit() sets per device (default 4), so staging memory is
 * bounded by 4 x 5 x 64 MB = 1.25 GiB of HBM plus as much pinned host memory however many
 * executor threads call; a call that finds every set borrowed waits for one.  Nothing is
 * owned by the calling thread, so retired threads leave nothing behind.  Host arrays that are
 * already pinned (sts_host_alloc) move by DMA directly; pageable arrays go through the set's
 * reused pinned bounce buffers.  err_per_series, c, coef, acf, ... are host arrays; with
 * err_per_series NULL the first failing series becomes the return status (the reference's
 * exception), decided after every chunk is back.  Every call returns only after all of its
 * transfers have completed, on success and on error alike.  Reference operators as for the
 * device entry points above. ---- */

/* Pinned host memory for callers that fill it themselves (the JNI shim copies Java arrays
 * into it with GetDoubleArrayRegion, then calls a _host entry point on it: no JVM array is
 * held across device work). */
int sts_host_alloc(size_t bytes, void** out);
int sts_host_free(void* p);
/* Free the idle staging slot sets of every device (they are otherwise kept for reuse). */
int sts_staging_release(void);
/* At most max_sets (>= 1) staging slot sets per device; lowering it frees idle sets now and
 * borrowed ones when their calls end. */
int sts_staging_set_limit(int max_sets);
/* Staging pool of the current device: out8 = {sets alive, idle, borrowed, limit, high-water
 * mark of sets alive, sets abandoned after a device error, calls that had to wait for a set,
 * the bound on an idle set's device bytes (and, alike, its pinned bytes): 5 slots x (64 MB + the
 * per-argument alignment).  A call whose ONE series exceeds a 64 MB chunk grows its set's slots
 * for its own duration; the set is trimmed back to the bound when the call ends}. */
int sts_staging_pool_info(int64_t* out8);
/* Statistics of the calling thread's last _host call: out8 = {wall ms, H2D ms, kernel ms,
 * D2H ms (summed per-chunk event times on the staging streams; they overlap each other),
 * H2D bytes, D2H bytes, chunks, fraction of the bytes moved by direct DMA from / to pinned
 * caller memory}. */
int sts_staging_stats(double* out8);
int sts_fill_autocorr_host(const double* in, double* filled, int64_t S, int64_t T, int64_t ld,
                           int method, int K, double* acf, int32_t* err_per_series);
int sts_fill_diff_ewma_host(const double* in, double* out, int64_t S, int64_t T, int64_t ld,
                            int method, int lag, const double* smoothing, int32_t* err_per_series);
int sts_ar_fit_remove_host(const double* in, double* out, int64_t S, int64_t T, int64_t ld, int p,
                           int no_intercept, double* c, double* coef, int32_t* err_per_series);
int sts_fill_host(const double* in, double* out, int64_t S, int64_t T, int64_t ld, int method,
                  int32_t* err_per_series);
int sts_autocorr_host(const double* in, int64_t S, int64_t T, int64_t ld, int K, double* acf);
int sts_diff_at_lag_host(const double* in, double* out, int64_t S, int64_t T, int64_t ld,
                         int lag, int start);
int sts_lag_matrix_host(const double* in, double* out, int64_t S, int64_t T, int64_t ld,
                        int max_lag, int include_original);
int sts_ewma_add_host(const double* in, double* out, int64_t S, int64_t T, int64_t ld,
                      const double* smoothing);
int sts_ewma_remove_host(const double* in, double* out, int64_t S, int64_t T, int64_t ld,
                         const double* smoothing);
int sts_ewma_fit_host(const double* in, int64_t S, int64_t T, int64_t ld, double* smoothing,
                      int32_t* err_per_series);
int sts_ar_fit_host(const double* in, int64_t S, int64_t T, int64_t ld, int p, int no_intercept,
                    double* c, double* coef, int32_t* err_per_series);
int sts_garch_fit_host(const double* in, int64_t S, int64_t T, int64_t ld, double* params,
                       int32_t* err_per_series);
int sts_argarch_fit_host(const double* in, int64_t S, int64_t T, int64_t ld, double* c,
                         double* phi, double* params, int32_t* err_per_series);
int sts_ar_remove_host(const double* in, double* out, int64_t S, int64_t T, int64_t ld,
                       const double* c, const double* coef, int p);
int sts_ar_add_host(const double* in, double* out, int64_t S, int64_t T, int64_t ld,
                    const double* c, const double* coef, int p);

#ifdef __cplusplus
}
#endif
#endif /* STS_H */
