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
#include "sts_ewma_opt.hpp"
#include "sts_internal.hpp"

#include <hip/hip_runtime.h>

#include <cstdlib>

namespace sts {
namespace {

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
#pragma unroll 8
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
    static_assert(SPW * CH % 64 == 0 && (CH % 64 == 0 || 64 % CH == 0), "chunk shape: whole load instructions");
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

#ifndef STS_EWMA_SPW
#define STS_EWMA_SPW 32   // series per wave (lanes that run the pass)
#endif
#ifndef STS_EWMA_CH
#define STS_EWMA_CH 64    // steps per LDS chunk
#endif
constexpr int kFitSpw = STS_EWMA_SPW;
constexpr int kFitCh = STS_EWMA_CH;

#ifdef STS_AB
// A/B: the wave's SPW rows held in LDS for the whole fit (one load, every
// optimizer request served from LDS) instead of re-streamed per request.  LDS = SPW x (T + 1)
// doubles per wave (T = 390: 50 KB for 16 rows, 100 KB for 32), so 3 / 1 waves per CU.
template <int SPW>
__global__ __launch_bounds__(64) void ewma_fit_res_kernel(EwmaFitArgs a) {
    extern __shared__ double rows[];
    const int lane = threadIdx.x;
    const int64_t s0 = (int64_t)blockIdx.x * SPW;
    const int64_t sl = s0 + lane;
    const bool live = lane < SPW && sl < a.S;
    const int ns = (a.S - s0 < SPW) ? (int)(a.S - s0) : SPW;
    const int T = (int)a.T;
    const int kRow = T + 1;
    const double* base = a.in + s0 * a.ld;
    for (int r = 0; r < ns; r++)   // each load instruction: 64 consecutive steps of one row
        for (int t = lane; t < T; t += 64) rows[r * kRow + t] = base[r * a.ld + t];
    __syncthreads();
    EwmaOpt o;
    o.pc = 0;
    o.status = -1;
    o.iter = 0;
    o.evals = 0;
    o.have_cur = 0;
    o.cn = 0;
    o.res_f = o.res_g = 0.0;
    if (live) ewma_advance(o);
    const double* myrow = rows + (live ? lane : 0) * kRow;
    bool first = true;
    for (;;) {
        const bool pending = live && o.status < 0;
        if (__ballot(pending) == 0) break;
        if (pending) {
            const double s = o.req, oms = 1.0 - s;
            SseGrad g;
            g.start(myrow[0]);
            g.run(myrow, 1, T, s, oms);
            o.res_f = g.sq;
            o.res_g = 2 * g.dJ;
            if (first && g.bad && T >= 2) {
                o.status = STS_ERR_TOO_MANY_EVALUATIONS;
            } else {
                cache_insert(o);
                ewma_advance(o);
            }
        }
        first = false;
    }
    if (!live) return;
    a.smoothing[sl] = (o.status == STS_OK) ? o.point : __builtin_nan("");
    if (a.err) a.err[sl] = o.status;
    if (a.evals) a.evals[sl] = o.evals;
}
#endif

}  // namespace

hipError_t launch_ewma_fit(const EwmaFitArgs& a, bool fit, hipStream_t st) {
    if (a.S <= 0) return hipSuccess;
#ifdef STS_AB
    if (const char* k = ab_knob("STS_EWMA_RES")) {   // 16 | 32 rows per wave held in LDS
        const int spw = std::atoi(k) == 32 ? 32 : 16;
        const size_t lds = (size_t)spw * (size_t)(a.T + 1) * sizeof(double);
        if (fit && a.T >= 1 && lds <= 160 * 1024) {
            dim3 g((unsigned)((a.S + spw - 1) / spw)), b(64);
            if (spw == 32) hipLaunchKernelGGL(ewma_fit_res_kernel<32>, g, b, lds, st, a);
            else hipLaunchKernelGGL(ewma_fit_res_kernel<16>, g, b, lds, st, a);
            return hipGetLastError();
        }
    }
#endif
    dim3 grid((unsigned)((a.S + kFitSpw - 1) / kFitSpw)), block(64);
    if (fit) hipLaunchKernelGGL((ewma_fit_kernel<kFitSpw, kFitCh, true>), grid, block, 0, st, a);
    else hipLaunchKernelGGL((ewma_fit_kernel<kFitSpw, kFitCh, false>), grid, block, 0, st, a);
    return hipGetLastError();
}

}  // namespace sts
