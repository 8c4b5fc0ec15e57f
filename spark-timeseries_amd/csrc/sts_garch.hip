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

#include <cstdlib>
#include <cstring>

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
#pragma unroll 4
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
    bool first = true, parked = false;
    int passes = 0;
    for (;;) {
        const bool pending = live && o.status < 0 && !parked;
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
                // past its pass budget: hand the series to garch_tail_kernel
                if (a.pass_budget > 0 && o.status < 0 && ++passes == a.pass_budget) {
                    const int slot = atomicAdd(a.park_ctr, 1);
                    if (slot < a.park_cap) {
                        static_cast<GarchOpt*>(a.park)[slot] = o;
                        a.park_ids[slot] = sl;
                        parked = true;
                    }
                }
            }
        }
        first = false;
    }
    if (!live || parked) return;
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

// ---- MaxEval tail: one wave per parked series ------------------------------------------
//
// A few series need thousands of optimizer passes (up to MaxEval = 10000 evaluations); in
// garch_fit_kernel each pass is one lane's sequential walk over its series, so those lanes
// set the launch time.  Here a whole wave evaluates one series.  The pass (GarchEval::run)
// is a set of first-order recurrences
//     h_t  = (omega + alpha x_{t-1} x_{t-1}) + beta h_{t-1}
//     oD_t = 1 + beta oD_{t-1}    aD_t = x_{t-1} x_{t-1} + beta aD_{t-1}    bD_t = h_{t-1} + beta bD_{t-1}
//     sum += term_t    oG += m_t oD_t    aG += m_t aD_t    bG += m_t bD_t
// whose costly parts (term_t: fdlibm log + a division, m_t: two divisions) depend only on
// h_t and x_t.  Every chain has the form y = u_t + b y, with b = beta or, for the sums, b = 1
// (1 * y is exact and + commutes, so `sum += term` is u + 1 * y bit for bit).  Lanes 0-7 run
// the eight chains as ONE instruction stream, each from its own u array in LDS, pipelined
// over C-step chunks: in iteration j lanes 0-2 run h / oD / aD of chunk j, lanes 3-4 bD and
// sum of chunk j - 1, lanes 5-7 the gradient sums of chunk j - 2.  Before each chain loop
// all 64 lanes compute the chunk-parallel inputs: u of chunk j, term / m / h_{t-1} of chunk
// j - 1, the products m oD, m aD, m bD of chunk j - 2.  Same operations, same order as
// GarchEval, so the pass is bit-identical and the optimizer path unchanged.
template <int C>
struct TailLds {
    static constexpr int kSlots = 3 * C + 2;   // 3 chunk slots; +2 doubles skews the arrays' banks
    double a[13][kSlots];                       // UH XX ETA H OD AD TERM M UB BD PO PA PB
    double one[C + 2];                          // u of the oD chain
    double negz[C + 2];                         // u of an idle chain: -0 + 1 * y == y for every y
    double sink[C];                             // chain outputs nobody reads (the sums)
};

// LDS hand-offs between lanes of the one wave: the wave's LDS instructions execute in order,
// so only the compiler must not reorder; an LDS-only fence leaves the x prefetch in flight.
__device__ __forceinline__ void tail_wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
}

// y = u_i + b y over one C-step chunk, u read 8 steps ahead (unconditionally, so the reads
// stay ahead of the dependent multiply-add chain).  SEL: steps i >= len are identity steps.
template <int C, bool SEL>
__device__ __forceinline__ void tail_chain(const double* up, double* wp, double b, int len, double& y) {
    double u[8], un[8];
#pragma unroll
    for (int k = 0; k < 8; k++) u[k] = up[k];
    for (int i = 0; i < C; i += 8) {
        if (i + 8 < C) {
#pragma unroll
            for (int k = 0; k < 8; k++) un[k] = up[i + 8 + k];
        }
#pragma unroll
        for (int k = 0; k < 8; k++) {
            if (SEL) {
                const bool on = i + k < len;
                y = (on ? u[k] : -0.0) + (on ? b : 1.0) * y;
            } else {
                y = u[k] + b * y;
            }
            wp[i + k] = y;
        }
#pragma unroll
        for (int k = 0; k < 8; k++) u[k] = un[k];
    }
}

template <int C>
__device__ __forceinline__ void garch_tail_pass(const double* __restrict__ x, int64_t T, GarchOpt& o,
                                                TailLds<C>& L) {
    enum { UH, XX, ETA, H, OD, AD, TERM, M, UB, BD, PO, PA, PB };
    const int lane = threadIdx.x;
    const double omega = o.req[0], alpha = o.req[1], beta = o.req[2];
    const int64_t nsteps = T > 1 ? T - 1 : 0;      // steps t = 1 .. T-1
    const int nc = (int)((nsteps + C - 1) / C);
    const int rem = (int)(nsteps - (int64_t)(nc - 1) * C);   // length of the last chunk
    const double h0 = omega / (1 - alpha - beta);
    // chain roles: lane -> (u array, output array, b, chunk lag)
    const int lag = lane < 3 ? 0 : lane < 5 ? 1 : 2;
    const double b = lane < 4 ? beta : 1.0;
    const int u_arr = lane == 0 ? UH : lane == 1 ? -1 : lane == 2 ? XX : lane == 3 ? UB : lane == 4 ? TERM
                    : lane == 5 ? PO : lane == 6 ? PA : PB;
    const int w_arr = lane == 0 ? H : lane == 1 ? OD : lane == 2 ? AD : lane == 3 ? BD : -1;
    double y = lane == 0 ? h0 : 0.0;
    for (int i = lane; i < C; i += 64) {
        L.one[i] = 1.0;
        L.negz[i] = -0.0;
    }
    // prefetch of chunk 0's x_{t-1}, x_t
    constexpr int NP = C / 64;
    double xp[NP], xe[NP];
    auto fetch = [&](int j) {
#pragma unroll
        for (int k = 0; k < NP; k++) {
            const int64_t t = 1 + (int64_t)j * C + k * 64 + lane;
            xp[k] = (j < nc && t < T) ? x[t - 1] : 0.0;
            xe[k] = (j < nc && t < T) ? x[t] : 0.0;
        }
    };
    fetch(0);
    for (int j = 0; j < nc + 2; j++) {
        const int s0 = (j % 3) * C, s1 = ((j + 2) % 3) * C, s2 = ((j + 1) % 3) * C;   // chunks j, j-1, j-2
        if (j < nc) {   // chunk j: the chain inputs that need only x
#pragma unroll
            for (int k = 0; k < NP; k++) {
                const int i = k * 64 + lane;
                L.a[UH][s0 + i] = omega + alpha * xp[k] * xp[k];
                L.a[XX][s0 + i] = xp[k] * xp[k];
                L.a[ETA][s0 + i] = xe[k];
            }
            fetch(j + 1);
        }
        if (j >= 1 && j - 1 < nc) {   // chunk j - 1: log-likelihood terms, multipliers, h_{t-1}
            const double hprev = j == 1 ? h0 : L.a[H][s2 + C - 1];
            const int len = j - 1 == nc - 1 ? rem : C;
#pragma unroll
            for (int k = 0; k < NP; k++) {
                const int i = k * 64 + lane;
                if (i < len) {
                    const double h = L.a[H][s1 + i], eta = L.a[ETA][s1 + i];
                    L.a[TERM][s1 + i] = -.5 * fdlibm_log(h) - .5 * eta * eta / h;
                    L.a[M][s1 + i] = (eta * eta / (h * h)) - (1 / h);
                    L.a[UB][s1 + i] = i > 0 ? L.a[H][s1 + i - 1] : hprev;
                }
            }
        }
        if (j >= 2) {   // chunk j - 2: gradient products
            const int len = j - 2 == nc - 1 ? rem : C;
#pragma unroll
            for (int k = 0; k < NP; k++) {
                const int i = k * 64 + lane;
                if (i < len) {
                    const double m = L.a[M][s2 + i];
                    L.a[PO][s2 + i] = m * L.a[OD][s2 + i];
                    L.a[PA][s2 + i] = m * L.a[AD][s2 + i];
                    L.a[PB][s2 + i] = m * L.a[BD][s2 + i];
                }
            }
        }
        tail_wave_sync();
        if (lane < 8) {
            const int cj = j - lag;
            const bool act = cj >= 0 && cj < nc;
            const int s = lag == 0 ? s0 : lag == 1 ? s1 : s2;
            // idle chains (chunk out of range) take identity steps from the -0 array
            const double* up = !act ? L.negz : u_arr < 0 ? L.one : &L.a[u_arr][s];
            double* wp = (!act || w_arr < 0) ? L.sink : &L.a[w_arr][s];
            const double bl = act ? b : 1.0;
            const int len = act && cj == nc - 1 ? rem : C;
            // does any chain run a partial chunk in this iteration? (lane-uniform)
            bool partial = false;
            for (int l = 0; l < 3; l++) partial |= j - l == nc - 1 && rem < C;
            if (partial) tail_chain<C, true>(up, wp, bl, len, y);
            else tail_chain<C, false>(up, wp, bl, len, y);
        }
        tail_wave_sync();
    }
    const double sum = __shfl(y, 4), oG = __shfl(y, 5), aG = __shfl(y, 6), bG = __shfl(y, 7);
    o.res_f = sum + -.5 * fdlibm_log(2 * 3.141592653589793) * (double)(T - 1);
    o.res_g[0] = aG * .5;   // the reference's order: alpha, beta, omega (:113)
    o.res_g[1] = bG * .5;
    o.res_g[2] = oG * .5;
}

template <int C>
__global__ __launch_bounds__(64) void garch_tail_kernel(GarchFitArgs a) {
    __shared__ TailLds<C> L;
    const int lane = threadIdx.x;
    const int n_park = a.park_ctr[0] < a.park_cap ? a.park_ctr[0] : a.park_cap;
    for (;;) {   // work queue over the parked series; every wave leaves when it is empty
        int idx = 0;
        if (lane == 0) idx = atomicAdd(a.park_ctr + 1, 1);
        idx = __shfl(idx, 0);
        if (idx >= n_park) return;
        const int64_t sl = a.park_ids[idx];
        GarchOpt o = static_cast<const GarchOpt*>(a.park)[idx];
        while (o.status < 0) {
            garch_tail_pass<C>(a.in + sl * a.ld, a.T, o, L);
            garch_cache_insert(o);
            garch_advance(o);
        }
        if (lane == 0) {
            const bool ok = o.status == STS_OK;
            for (int j = 0; j < 3; j++) a.params[3 * sl + j] = ok ? o.point[j] : __builtin_nan("");
            if (a.err && !(a.keep_err && a.err[sl] != 0)) a.err[sl] = o.status;
            if (a.evals) a.evals[sl] = o.evals;
        }
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

constexpr int kGSpw = 64;   // A/B 64 x 64 vs 32 x 64: phase 1 178 vs 218 ms (100k x 2520)
constexpr int kGCh = 64;
constexpr int kTailC = 64;
constexpr int kTailGrid = 1024;

// Passes a lane runs in garch_fit_kernel before its series moves to the tail kernel;
// STS_GARCH_PASS_BUDGET overrides it in the A/B build (0 = no tail phase; A/B runs and the
// tests).
int garch_pass_budget() {
    const char* e = ab_knob("STS_GARCH_PASS_BUDGET");
    return e ? std::atoi(e) : 64;
}

}  // namespace

hipError_t launch_garch_fit(const GarchFitArgs& a0, bool fit, hipStream_t st) {
    if (a0.S <= 0) return hipSuccess;
    GarchFitArgs a = a0;
    dim3 grid((unsigned)((a.S + kGSpw - 1) / kGSpw)), block(64);
    if (!fit) {
        hipLaunchKernelGGL((garch_fit_kernel<kGSpw, kGCh, false>), grid, block, 0, st, a);
        return hipGetLastError();
    }
    const int budget = garch_pass_budget();
    void* scratch = nullptr;
    if (budget > 0) {
        const int64_t cap = a.S;   // a slot per series (~650 B): every lane past its budget can park
        const size_t state = (size_t)cap * sizeof(GarchOpt);
        hipError_t e = hipMallocAsync(&scratch, state + (size_t)cap * sizeof(int64_t) + 16, st);
        if (e != hipSuccess) return e;
        a.park = scratch;
        a.park_ids = reinterpret_cast<int64_t*>(static_cast<char*>(scratch) + state);
        a.park_ctr = reinterpret_cast<int32_t*>(a.park_ids + cap);
        a.park_cap = (int)cap;
        a.pass_budget = budget;
        e = hipMemsetAsync(a.park_ctr, 0, 2 * sizeof(int32_t), st);
        if (e != hipSuccess) return e;
    }
    const char* shape = ab_knob("STS_GARCH_SHAPE");   // A/B: series per wave x chunk steps
    if (shape && !std::strcmp(shape, "32x64"))
        hipLaunchKernelGGL((garch_fit_kernel<32, 64, true>), dim3((unsigned)((a.S + 31) / 32)), block, 0, st, a);
    else
        hipLaunchKernelGGL((garch_fit_kernel<kGSpw, kGCh, true>), grid, block, 0, st, a);
    hipError_t e = hipGetLastError();
    if (scratch) {
        if (e == hipSuccess) {
            const unsigned tg = (unsigned)(a.park_cap < kTailGrid ? a.park_cap : kTailGrid);
            const char* tc = ab_knob("STS_GARCH_TAIL_C");   // A/B: tail chunk length
            if (tc && std::atoi(tc) == 256)
                hipLaunchKernelGGL((garch_tail_kernel<256>), dim3(tg), block, 0, st, a);
            else if (tc && std::atoi(tc) == 128)
                hipLaunchKernelGGL((garch_tail_kernel<128>), dim3(tg), block, 0, st, a);
            else
                hipLaunchKernelGGL((garch_tail_kernel<kTailC>), dim3(tg), block, 0, st, a);
            e = hipGetLastError();
        }
        const hipError_t ef = hipFreeAsync(scratch, st);
        if (e == hipSuccess) e = ef;
    }
    return e;
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
