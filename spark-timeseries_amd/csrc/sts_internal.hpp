// sts_internal.hpp -- shared declarations between the C-ABI layer (sts_api.cpp) and
// the HIP kernel translation units.  Host-side launchers only: no kernel bodies here.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdlib>

#include "sts.h"

namespace sts {

// Tile geometry of the imputation / autocorrelation tile kernel (sts_tile.hip).
// A tile is TW consecutive steps of ONE series plus HB steps of look-back and HA
// steps of look-ahead (ACF pairs reach 16*NT-1 <= 79 steps past the tile).
constexpr int kHB = 64;
constexpr int kHA = 128;
// per-chunk ACF partials: [0, 64) lag products, [64] sum y and [65] sum y^2 over the
// series' middle (sts_acf.hpp), [66] the shift c, [67] pad
constexpr int kPartStride = 68;
constexpr int kPartSum = 64, kPartSq = 65, kPartShift = 66;
// autocorr head / tail length handled per lag by the finalize (sts_acf.hpp); K <= kAcfEdge
// on the fused paths, and series shorter than 2 kAcfEdge take the direct two-pass finalize
constexpr int kAcfEdge = 64;
// short fused fill + ACF: the two-series-per-block form (sts_short.hip short_pair_kernel) by default
constexpr bool kShortPairDefault = false;

struct TileArgs {
    const double* in;
    double* out;          // filled output (may be null when not written)
    double* lagmat;       // lag-matrix output (may be null)
    double* partials;     // ACF partial sums [tiles][kPartStride] (may be null)
    int32_t* err;         // per-series error flags (may be null)
    int64_t S, T, ld_in, ld_out;
    int64_t tiles_per_series;
    int64_t tiles_per_chunk;    // tiles one workgroup walks (register-prefetched pipeline)
    int64_t chunks_per_series;  // = ceil(tiles_per_series / tiles_per_chunk)
    int K;                // ACF lags (0 = no ACF)
    int max_lag;          // lag matrix p
    int include_original; // lag matrix inc
    double* acf_fused;    // seg kernel, one segment per series: final ACF written directly (S x K)
    const double* shift;  // tile kernel with K > 0: per-series ACF shift (launch_acf_shift)
    int err_all;          // seg kernel, one segment per series: err[s] written for every series
};

struct FinalizeArgs {
    const double* F;      // filled series (or raw input when no fill), ld = ldF
    const double* partials;
    double* acf;          // S x K
    int64_t S, T, ldF, parts_per_series;   // ACF partials per series (one per chunk)
    int K;
    int32_t* exact;       // per series, zeroed by the caller: set where rule 3 (sts_acf.hpp) fires,
                          // for launch_acf_exact to recompute that series by the reference's loop
};

// A/B experiment knobs (environment variables) exist only in the -DSTS_AB build
// (build/libsts_hip_ab.so, tools/ and the knob tests); the product libsts_hip.so never reads
// its environment, so a Spark executor's environment cannot change which kernels run.
#ifdef STS_AB
inline const char* ab_knob(const char* name) { return std::getenv(name); }
#else
inline const char* ab_knob(const char*) { return nullptr; }
#endif

// status helpers of the C-ABI layer (sts_api.cpp): the first failing entry of a host copy of
// err_per_series as the reference's exception; a status with a thread-local message
int series_status(const int32_t* h, int64_t S, const char* what);
int set_error(int status, const char* msg);
// Run fn(ctx) -- a call of a device entry point -- in validate-only mode: the entry point
// checks its arguments and returns their status, stopping at its first device action.
// The `_host` entry points validate this way before staging anything.
int validate_call(int (*fn)(void*), void* ctx);
template <class F>
int validate(F&& f) {
    return validate_call([](void* c) { return (*static_cast<F*>(c))(); }, static_cast<void*>(&f));
}

// launchers (return hipError_t of the launch)
hipError_t launch_tile(int method, int tw, const TileArgs& a, hipStream_t st);
hipError_t launch_acf_finalize(const FinalizeArgs& a, hipStream_t st);
// rule 3's fallback for the series flagged in exact[S] (acf_finalize / the wide finalize): every
// lag 1..K by the reference's two-pass loop, F streamed through LDS (sts_acf.hpp acf_exact_stream)
hipError_t launch_acf_exact(const double* F, int64_t S, int64_t T, int64_t ldF, int K, const int32_t* exact,
                            double* acf, hipStream_t st);
// per-series robust ACF shift (sts_acf.hpp) for the tile kernel
// method: the fill the series will take (STS_FILL_PREVIOUS reverses the shift's fallback)
hipError_t launch_acf_shift(const double* in, int64_t S, int64_t T, int64_t ld, int method, double* shift,
                            hipStream_t st);
// numLags above the fused kernels' 63 (sts_acf_wide.hip): partial count for S x T x K, and the
// lag-block MFMA pass + finalize on a filled panel F (shift: launch_acf_shift of F)
constexpr int kFusedMaxLags = 63;
size_t acf_wide_partials(int64_t S, int64_t T, int K);
hipError_t launch_acf_wide(const double* F, int64_t S, int64_t T, int64_t ld, const double* shift, int K, double* part,
                           double* acf, int32_t* exact, hipStream_t st);

// Wave-private segment kernel (sts_seg.hip): tiles of kSegW steps, kSegTiles tiles per
// wave.  TileArgs.tiles_per_series = ceil(T / kSegW), tiles_per_chunk = tiles per
// segment, chunks_per_series = segments per series.  seg_nt(K) < 0: K not supported.
constexpr int kSegW = 512;
constexpr int kSegTiles = 128;
int seg_nt(int K);
hipError_t launch_segment(int method, const TileArgs& a, hipStream_t st);
// fill('linear') + fused ACF with the whole series in one wave's registers (sts_short.hip):
// short_ok() says whether a one-segment, fused-ACF seg call may take it instead
bool short_ok(int method, int64_t T, int K);
hipError_t launch_short(int method, const TileArgs& a, hipStream_t st, bool pair);

// fillts "spline" (sts_spline.hip): series per launch for the (mu, z) scratch rows (16 B per
// step), and the batched launches over S series (scratch: spline_batch(S, T) x T double2)
int64_t spline_batch(int64_t S, int64_t T);
hipError_t launch_spline(const double* in, double* out, int64_t S, int64_t T, int64_t ld_in, int64_t ld_out,
                         int32_t* err, double* scratch, int64_t batch, hipStream_t st);

hipError_t launch_diff(const double* in, double* out, int64_t S, int64_t T, int64_t ld_in,
                       int64_t ld_out, int lag, int start, hipStream_t st);
hipError_t launch_diff_inplace(double* x, int64_t S, int64_t T, int64_t ld, int lag, int start,
                               hipStream_t st);
hipError_t launch_lagmat(const double* in, double* out, int64_t S, int64_t T, int64_t ld_in,
                         int max_lag, int include_original, hipStream_t st);
hipError_t launch_ewma_remove(const double* in, double* out, int64_t S, int64_t T, int64_t ld_in,
                              int64_t ld_out, const double* sm, hipStream_t st);
hipError_t launch_ar_remove(const double* in, double* out, int64_t S, int64_t T, int64_t ld_in,
                            int64_t ld_out, const double* c, const double* coef, int p,
                            hipStream_t st);

// series-per-lane recurrences (sts_recur.hip)
enum RecurOp { kEwmaAdd = 0, kEwmaRemoveInplace = 1, kArAdd = 2, kArRemoveInplace = 3,
               kFillDiffEwma = 4, kDiffInplace = 5 };
struct RecurArgs {
    const double* in;
    double* out;
    int64_t S, T, ld_in, ld_out;
    const double* sm;     // EWMA smoothing per series
    const double* c;      // AR intercept per series
    const double* coef;   // AR coefficients [S][p]
    int p;                // AR order
    int lag, start;       // differencing
    int method;           // fill method for kFillDiffEwma
};
hipError_t launch_recur(RecurOp op, const RecurArgs& a, hipStream_t st);

// AR fit (sts_ar.hip)
struct ArArgs {
    const double* in;
    double* out;          // remove output (null -> fit only)
    double* c;
    double* coef;
    int32_t* err;
    int64_t S, T, ld_in, ld_out;
    int p, no_intercept;
    // AR rule (sts_ar.hip / sts_ar_qr.hip): series the fast fit flags, appended by the fit
    // kernels (set by launch_ar_fit, not by callers)
    int64_t* qr_list;
    uint32_t* qr_count;
};
hipError_t launch_ar_fit(const ArArgs& a, hipStream_t st);
// the fast fit kernels only, flagged series counted into *count (device; AR rule diagnostic)
hipError_t launch_ar_rule_count(const ArArgs& a, uint32_t* count, hipStream_t st);
// the reference's Householder QR on the listed series (list == nullptr: series 0 .. n_direct-1;
// otherwise list[0 .. *count-1]); scratch = slots x ar_qr_wave_slot_elems doubles for p > 8
bool ar_qr_lane_ok(int p);
size_t ar_qr_wave_slot_elems(int64_t T, int p, int no_intercept);
hipError_t launch_ar_qr(const ArArgs& a, const int64_t* list, const uint32_t* count, int64_t n_direct,
                        double* scratch, int slots, bool force_wave, hipStream_t st);

// EWMA.fitModel and EWMAModel.sse / gradient (sts_ewma_fit.hip)
struct EwmaFitArgs {
    const double* in;
    int64_t S, T, ld;
    double* smoothing;    // fit: output; sse / gradient: input (per series)
    double* sse;          // sse / gradient outputs (may be null)
    double* grad;
    int32_t* err;         // fit: per-series status (may be null)
    int32_t* evals;       // fit: objective evaluations commons-math3 counted (may be null)
};
hipError_t launch_ewma_fit(const EwmaFitArgs& a, bool fit, hipStream_t st);

// GARCH.fitModel / GARCHModel.logLikelihood + gradient and the GARCH / ARGARCH
// time-dependent effects (sts_garch.hip)
struct GarchFitArgs {
    const double* in;
    int64_t S, T, ld;
    double* params;       // S x 3 (omega, alpha, beta): fit output / evaluation input
    int32_t* err;         // fit: per-series status (optional)
    int keep_err;         // fit: leave a nonzero err entry as it is (ARGARCH: the AR stage's)
    int32_t* evals;       // fit: commons-math3 evaluation count (optional)
    double* loglik;       // evaluation: S
    double* grad;         // evaluation: S x 3, the reference's (alpha, beta, omega) order
    // fit, MaxEval tail (set by launch_garch_fit): a lane still running after pass_budget
    // passes parks its optimizer state in park[slot] (slot from park_ctr[0], < park_cap)
    // and garch_tail_kernel finishes it, one wave per series (park_ctr[1]: its work queue)
    void* park;           // park_cap x GarchOpt
    int64_t* park_ids;    // series of each slot
    int32_t* park_ctr;
    int park_cap;
    int pass_budget;      // 0: no tail phase
};
hipError_t launch_garch_fit(const GarchFitArgs& a, bool fit, hipStream_t st);
enum GarchOp { kGarchRemove = 0, kGarchAdd = 1, kArgarchRemove = 2, kArgarchRemoveInplace = 3, kArgarchAdd = 4 };
struct GarchEffectsArgs {
    const double* in;
    double* out;
    int64_t S, T, ld_in, ld_out;
    const double *c, *phi, *omega, *alpha, *beta;   // per series (c, phi: ARGARCH only)
};
hipError_t launch_garch_effects(int op, const GarchEffectsArgs& a, hipStream_t st);

// seriesStats / removeInstantsWithNaNs / toInstants (sts_instants.hip)
hipError_t launch_series_stats(const double* in, double* out, int64_t S, int64_t T, int64_t ld, hipStream_t st);
hipError_t launch_nan_instants(const double* in, uint8_t* flags, int64_t S, int64_t T, int64_t ld, hipStream_t st);
int64_t active_scratch_elems(int64_t T);
hipError_t launch_active_instants(const uint8_t* flags, int64_t T, int64_t* active, int64_t* n_active,
                                  int64_t* scratch, hipStream_t st);
hipError_t launch_gather_instants(const double* in, double* out, const int64_t* active, int64_t n_active, int64_t S,
                                  int64_t ld_in, int64_t ld_out, hipStream_t st);
hipError_t launch_transpose(const double* in, double* out, int64_t S, int64_t T, int64_t ld_in, int64_t ld_out,
                            hipStream_t st);

// ingest formats (sts_ingest.hip)
hipError_t launch_wire_decode(const unsigned char* bytes, const int64_t* val_off, double* panel, int64_t S, int64_t T,
                              int64_t ld, hipStream_t st);
hipError_t launch_wire_encode(const double* panel, int64_t S, int64_t T, int64_t ld, const int64_t* val_off,
                              unsigned char* bytes, hipStream_t st);
hipError_t launch_observations(const int32_t* sid, const int64_t* loc, const double* val, int64_t n, double* panel,
                               int64_t S, int64_t T, int64_t ld, unsigned char* win, hipStream_t st);

// generators (sts_gen.hip)
hipError_t launch_gen_panel(double* out, int64_t s0, int64_t S, int64_t T, int64_t ld,
                            uint64_t seed, uint32_t nan_thr, hipStream_t st);
hipError_t launch_gen_ar(double* out, double* c, double* phi, int64_t s0, int64_t S, int64_t T,
                         int64_t ld, uint64_t seed, int p, hipStream_t st);

}  // namespace sts
