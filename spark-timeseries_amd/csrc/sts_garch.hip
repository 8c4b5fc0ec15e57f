// sts_garch.hip -- GARCH(1,1) and AR(1)+GARCH(1,1) batched over a panel
// ("ARGARCH reuse of AR fit").
//
// Reference (S/ = src/main/scala/com/cloudera/sparkts/):
//   GARCH.fitModel                    S/models/GARCH.scala:33-53
//   ARGARCH.fitModel                  S/models/GARCH.scala:62-68 (AR(1) fit + remove: the
//                                     existing sts_ar_fit_remove path, then GARCH.fitModel)
//   GARCHModel.logLikelihood          S/models/GARCH.scala:80-86
//   GARCHModel.gradient               S/models/GARCH.scala:94-114
//   iterateWithHAndEta                S/models/GARCH.scala:116-128
//   GARCHModel.remove/add             S/models/GARCH.scala:130-159
//   ARGARCHModel.remove/add           S/models/GARCH.scala:203-234
//
// Fit: one LANE per series runs commons-math3's optimizer as a resumable state machine
// (sts_garch_opt.hpp); a wave owns SPW series and, each round, streams its block of rows
// through LDS once (CH-step chunks, each load instruction = 64 consecutive steps of one
// series) while every lane with a pending request evaluates logLikelihood AND gradient of
// its own series at its own point in one sequential pass, in the reference's operation
// order (-ffp-contract=off; Math.log as fdlibm's e_log.c, see sts_fdlibm.hpp), so every
// evaluation is bit-exact and the optimizer takes the reference's path.  A series holding a
// NaN (T >= 2) makes every logLikelihood NaN; the reference then ends in
// TooManyEvaluationsException after 10000 evaluations, decided here after the first pass.
//
// Effects (remove / add): the same LDS-staged row blocks, one lane per series running the
// recurrence in order and writing its row back through LDS.
#include "sts_fdlibm.hpp"
#include "sts_garch_opt.hpp"
#include "sts_internal.hpp"

#include <hip/hip_runtime.h>

namespace sts {
namespace {

// logLikelihood and gradient of one series in one pass (statement order of :80-86 and
// :94-114 over iterateWithHAndEta :116-128), state carried across chunks.
struct GarchEval {
    double omega, alpha, beta;
    double prevH, prevX, sum, oD, aD, bD, oG, aG, bG;
    bool bad;
    __device__ __forceinline__ void start(double x0) {
        prevH = omega / (1 - alpha - beta);
        prevX = x0;
        sum = oD = aD = bD = oG = aG = bG = 0.0;
        bad = x0 != x0;
    }
    __device__ __forceinline__ void run(const double* row, int c0, int len) {
        for (int c = c0; c < len; c++) {
            const double eta = row[c];
            bad |= eta != eta;
            const double h = omega + alpha * prevX * prevX + beta * prevH;
            sum += -.5 * fdlibm_log(h) - .5 * eta * eta / h;
            oD = 1 + beta * oD;
            aD = prevX * prevX + beta * aD;
            bD = prevH + beta * bD;
            const double multiplier = (eta * eta / (h * h)) - (1 / h);
            oG += multiplier * oD;
            aG += multiplier * aD;
            bG += multiplier * bD;
            prevH = h;
            prevX = eta;
        }
    }
    __device__ __forceinline__ double loglik(int64_t n) const {
        return sum + -.5 * fdlibm_log(2 * 3.141592653589793) * (double)(n - 1);
    }
};

// One wave = SPW series (lanes < SPW), CH-step chunks through LDS.  FIT = false evaluates
// logLikelihood / gradient once at params[s].
template <int SPW, int CH, bool FIT>
__global__ __launch_bounds__(64) void garch_fit_kernel(GarchFitArgs a) {
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

    GarchOpt o;
    garch_init(o);
    if (FIT) {
        if (live) garch_advance(o);
    } else if (live) {
        o.req[0] = a.params[3 * sl];
        o.req[1] = a.params[3 * sl + 1];
        o.req[2] = a.params[3 * sl + 2];
    }
    bool first = true;
    for (;;) {
        const bool pending = live && o.status < 0;
        const unsigned long long want = __ballot(pending);
        if (want == 0) break;
        GarchEval g;
        g.omega = o.req[0];
        g.alpha = o.req[1];
        g.beta = o.req[2];
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
            if (tc + CH < T) fetch(tc + CH);
            __syncthreads();
            if (pending) {
                const double* myrow = tile + lane * kRow;
                if (tc == 0) g.start(myrow[0]);
                g.run(myrow, tc == 0 ? 1 : 0, len);
            }
            __syncthreads();
        }
        if (pending) {
            o.res_f = g.loglik(T);
            o.res_g[0] = g.aG * .5;   // the reference's order: alpha, beta, omega (:113)
            o.res_g[1] = g.bG * .5;
            o.res_g[2] = g.oG * .5;
            if (!FIT) {
                o.status = STS_OK;
            } else if (first && g.bad && T >= 2) {
                o.status = STS_ERR_TOO_MANY_EVALUATIONS;   // every logLikelihood is NaN
            } else {
                garch_cache_insert(o);
                garch_advance(o);
            }
        }
        first = false;
    }
    if (!live) return;
    if (FIT) {
        const bool ok = o.status == STS_OK;
        for (int j = 0; j < 3; j++) a.params[3 * sl + j] = ok ? o.point[j] : __builtin_nan("");
        if (a.err && !(a.keep_err && a.err[sl] != 0)) a.err[sl] = o.status;
        if (a.evals) a.evals[sl] = o.evals;
    } else {
        if (a.loglik) a.loglik[sl] = o.res_f;
        if (a.grad)
            for (int j = 0; j < 3; j++) a.grad[3 * sl + j] = o.res_g[j];
    }
}

// GARCHModel / ARGARCHModel remove / add, one lane per series, rows through LDS in place.
template <int OP, int SPW = 32, int CH = 64>
__global__ __launch_bounds__(64) void garch_effects_kernel(GarchEffectsArgs a) {
    constexpr int kRow = CH + 1;
    constexpr int NLD = SPW * CH / 64;
    __shared__ double tile[SPW * kRow];
    const int lane = threadIdx.x;
    const int64_t s0 = (int64_t)blockIdx.x * SPW;
    const int64_t sl = s0 + lane;
    const bool live = lane < SPW && sl < a.S;
    const int ns = (a.S - s0 < SPW) ? (int)(a.S - s0) : SPW;
    const int64_t T = a.T;
    const bool ar = OP == kArgarchRemove || OP == kArgarchRemoveInplace || OP == kArgarchAdd;
    double c = 0.0, phi = 0.0, omega = 0.0, alpha = 0.0, beta = 0.0;
    if (live) {
        omega = a.omega[sl];
        alpha = a.alpha[sl];
        beta = a.beta[sl];
        if (ar) {
            c = a.c[sl];
            phi = a.phi[sl];
        }
    }
    double prevEta = 0.0, prevVariance = 0.0, prevX = 0.0, prevY = 0.0;
    double pre[NLD];
    auto fetch = [&](int64_t tc) {
        const int len = (T - tc < CH) ? (int)(T - tc) : CH;
#pragma unroll
        for (int i = 0; i < NLD; i++) {
            const int row = (i * 64 + lane) / CH, col = (i * 64 + lane) % CH;
            pre[i] = (row < ns && col < len) ? a.in[(s0 + row) * a.ld_in + tc + col] : 0.0;
        }
    };
    fetch(0);
    for (int64_t tc = 0; tc < T; tc += CH) {
        const int len = (T - tc < CH) ? (int)(T - tc) : CH;
#pragma unroll
        for (int i = 0; i < NLD; i++) {
            const int row = (i * 64 + lane) / CH, col = (i * 64 + lane) % CH;
            if (row < ns && col < len) tile[row * kRow + col] = pre[i];
        }
        if (tc + CH < T) fetch(tc + CH);
        __syncthreads();
        if (live) {
            double* myrow = tile + lane * kRow;
            for (int cc = 0; cc < len; cc++) {
                const double x = myrow[cc];
                double y;
                if (tc + cc == 0) {
                    prevVariance = omega / (1.0 - alpha - beta);
                    if (OP == kGarchRemove) {
                        prevEta = x;
                        y = prevEta / __builtin_sqrt(prevVariance);
                    } else if (OP == kArgarchRemove || OP == kArgarchRemoveInplace) {
                        prevEta = x - c;
                        y = prevEta / __builtin_sqrt(prevVariance);
                    } else {   // add
                        prevEta = x * __builtin_sqrt(prevVariance);
                        y = (OP == kArgarchAdd) ? c + prevEta : prevEta;
                    }
                } else {
                    const double variance = omega + alpha * prevEta * prevEta + beta * prevVariance;
                    if (OP == kGarchRemove) {
                        y = x / __builtin_sqrt(variance);
                        prevEta = x;
                    } else if (OP == kArgarchRemove || OP == kArgarchRemoveInplace) {
                        // ts(i - 1): the input, or (dest eq ts) the value already overwritten
                        const double tsPrev = (OP == kArgarchRemoveInplace) ? prevY : prevX;
                        const double eta = x - c - phi * tsPrev;
                        y = eta / __builtin_sqrt(variance);
                        prevEta = eta;
                    } else {
                        const double eta = x * __builtin_sqrt(variance);
                        y = (OP == kArgarchAdd) ? c + phi * prevY + eta : eta;
                        prevEta = eta;
                    }
                    prevVariance = variance;
                }
                prevX = x;
                prevY = y;
                myrow[cc] = y;
            }
        }
        __syncthreads();
#pragma unroll
        for (int i = 0; i < NLD; i++) {
            const int row = (i * 64 + lane) / CH, col = (i * 64 + lane) % CH;
            if (row < ns && col < len) a.out[(s0 + row) * a.ld_out + tc + col] = tile[row * kRow + col];
        }
        __syncthreads();
    }
}

constexpr int kGSpw = 32;
constexpr int kGCh = 64;

}  // namespace

hipError_t launch_garch_fit(const GarchFitArgs& a, bool fit, hipStream_t st) {
    if (a.S <= 0) return hipSuccess;
    dim3 grid((unsigned)((a.S + kGSpw - 1) / kGSpw)), block(64);
    if (fit) hipLaunchKernelGGL((garch_fit_kernel<kGSpw, kGCh, true>), grid, block, 0, st, a);
    else hipLaunchKernelGGL((garch_fit_kernel<kGSpw, kGCh, false>), grid, block, 0, st, a);
    return hipGetLastError();
}

hipError_t launch_garch_effects(int op, const GarchEffectsArgs& a, hipStream_t st) {
    if (a.S <= 0 || a.T <= 0) return hipSuccess;
    dim3 grid((unsigned)((a.S + 31) / 32)), block(64);
    switch (op) {
    case kGarchRemove: hipLaunchKernelGGL((garch_effects_kernel<kGarchRemove>), grid, block, 0, st, a); break;
    case kGarchAdd: hipLaunchKernelGGL((garch_effects_kernel<kGarchAdd>), grid, block, 0, st, a); break;
    case kArgarchRemove: hipLaunchKernelGGL((garch_effects_kernel<kArgarchRemove>), grid, block, 0, st, a); break;
    case kArgarchRemoveInplace:
        hipLaunchKernelGGL((garch_effects_kernel<kArgarchRemoveInplace>), grid, block, 0, st, a);
        break;
    case kArgarchAdd: hipLaunchKernelGGL((garch_effects_kernel<kArgarchAdd>), grid, block, 0, st, a); break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace sts
