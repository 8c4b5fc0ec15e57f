// sts_ar.hip -- batched AR(p) fit (Autoregression.fitModel, S/models/Autoregression.scala:38-53)
// with the lag-matrix Gram on FP64 MFMA, plus the fused removeTimeDependentEffects
// (S/models/Autoregression.scala:60-73) for the C4 pipeline.
//
// The reference builds the (n-p) x p lag matrix (Lag.lagMatTrimBoth, S/Lag.scala:62-77),
// prepends an intercept column and solves OLS by Householder QR (commons-math3 3.4.1
// OLSMultipleLinearRegression).  Here one wave owns one series (staged in LDS when it
// fits).  Every Gram entry of the design [Y | X_1..X_p] is a lag product over a window:
//   G[j][k] = sum_{r<m} y_{r+p-j} y_{r+p-k} = P_d - head - tail,  d = |j - k|,
// with P_d = sum_u y_u y_{u+d} the full lag-d product and head/tail at most p terms at
// the series ends.  P_0..P_p come from v_mfma_f64_16x16x4_f64 rank-4 updates exactly as
// in the autocorrelation tile kernel (rows of 16 steps, U_t = sum_a A_a^T A_{a+t}).
// The data are centred first (y = x - mean, exact algebra for the intercept model), the
// intercept is eliminated (centred normal equations), the p x p system is solved by
// Cholesky in fp64 and one step of iterative refinement against an exact residual pass
// (corrected semi-normal equations) brings the error back to Householder-QR level.
#include "sts_internal.hpp"
#include "sts_dma.hpp"
#include "sts_lanes.hpp"

#include <hip/hip_runtime.h>

#include <cstdlib>

namespace sts {
namespace {

typedef double d4 __attribute__((ext_vector_type(4)));
constexpr int kPMax = 31;
constexpr int kLd = kPMax + 2;   // row stride of the (p+1) x (p+1) Gram in LDS

// ---- AR rule: which series the reference's own arithmetic must fit ----
// commons-math3's Householder QR on the uncentred lag design drifts from the exact least-
// squares solution with the level / spread ratio of the lag columns, with their collinearity,
// and (in c) with how small the intercept is against the level it is the difference of.  The
// fast kernels land ~1e-13 from exact; where the reference may sit farther than ~1e-11 from
// exact the series is flagged and sts_ar_qr.hip recomputes it with the reference's operation
// order (bit-exact to oracle/sts_oracle.c).  Thresholds from tools/ar_flag_study.py (11,240
// series: walks, integrated walks, AR(1), noise, trends, sines at levels 0 .. 1e7, T 300 /
// 2,520 / 6,000, p 1 / 2 / 5 / 8): inside all three bounds the reference is within 7e-14
// (normwise) and 8.8e-12 (elementwise, over coefficients down to 1e-6 of the vector) of exact.
// C4 panels sit at ratio 4.2, kappa 1.1, level 1.4: no C4 series is flagged.
constexpr double kRuleRatio2 = 256.0;   // (|mean| / centred column rms)^2 < 16^2
constexpr double kRuleKappa = 100.0;    // 1 / (scaled Cholesky pivot)^2 < 100
constexpr double kRuleLevel = 100.0;    // |mean| / |c| < 100
// Round 6: the register kernel skips its refinement pass when every scaled Cholesky pivot^2 of
// the centred lag Gram exceeds 1 / kRefineKappa (nearly orthogonal lags, e.g. every C4 series:
// 1 / pivot^2 ~ 1.1).  Calibration (tools/ar_flag_study.py families + the filled ones, 6 488
// intercept fits, numpy emulation of the unrefined centred normal equations): wherever the AR
// rule keeps a series AND 1 / pivot^2 < 4, the unrefined solution is within 8.8e-12
// elementwise of the reference -- the reference's own distance to the exact solution there, the
// refined one's too -- against 1.8e-9 without the pivot bound.
#ifndef STS_AR_SKIP_REFINE
#define STS_AR_SKIP_REFINE 1
#endif
constexpr double kRefineKappa = 4.0;

// the intercept half of the rule on a finished fit
__device__ __forceinline__ bool ar_rule_level(double c, double mu) {
    return !(__builtin_fabs(mu) < kRuleLevel * __builtin_fabs(c));
}

__device__ __forceinline__ void ar_rule_append(const ArArgs& a, int64_t s) {
    const uint32_t i = atomicAdd(a.qr_count, 1u);
    a.qr_list[i] = s;
}

template <bool STAGED, int PB>
__global__ __launch_bounds__(64) void ar_fit_kernel(ArArgs a, int NT) {
    extern __shared__ __attribute__((aligned(16))) double lds[];
    double* scr = lds;                       // 256: one U_t tile
    double* lagp = scr + 256;                // 64: P_d
    double* G = lagp + 64;                   // (p+1) x kLd
    double* cs = G + (kPMax + 1) * kLd;      // p+1 column sums (+1 pad)
    double* sol = cs + kPMax + 2;            // c, coef[p], status
    double* zz = sol + kPMax + 4;            // refinement: gradient (kPMax + 2) | solve (kPMax + 2)
    double* sx = zz + 2 * (kPMax + 2);       // staged series (T doubles)
    const int lane = threadIdx.x;
    const int64_t s = blockIdx.x;
    const int64_t T = a.T;
    const int p = a.p;
    const double* xg = a.in + s * a.ld_in;

    // ---- pass 1: stage + mean ----
    double part = 0.0;
    for (int64_t t0 = 0; t0 < T; t0 += 512) {     // 8 independent loads in flight per lane
        double v[8];
#pragma unroll
        for (int u = 0; u < 8; u++) {
            const int64_t t = t0 + u * 64 + lane;
            v[u] = (t < T) ? xg[t] : 0.0;
        }
#pragma unroll
        for (int u = 0; u < 8; u++) {
            const int64_t t = t0 + u * 64 + lane;
            if (STAGED && t < T) sx[t] = v[u];
            part += v[u];
        }
    }
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) part += __shfl_xor(part, d);
    const double mu = a.no_intercept ? 0.0 : part / (double)T;
    if (STAGED) __syncthreads();
    auto X = [&](int64_t t) -> double { return STAGED ? sx[t] : xg[t]; };
    auto Y = [&](int64_t t) -> double { return (t < T) ? X(t) - mu : 0.0; };

    // ---- pass 2: P_d on MFMA ----
    d4 U0 = {0, 0, 0, 0}, U1 = {0, 0, 0, 0}, U2 = {0, 0, 0, 0};
    double sy = 0.0;
    for (int64_t j0 = 0; j0 < T; j0 += 64) {
        const double av = Y(j0 + lane);
        const double b1 = Y(j0 + 16 + lane);
        U0 = __builtin_amdgcn_mfma_f64_16x16x4f64(av, av, U0, 0, 0, 0);
        U1 = __builtin_amdgcn_mfma_f64_16x16x4f64(av, b1, U1, 0, 0, 0);
        if (NT > 2) {
            const double b2 = Y(j0 + 32 + lane);
            U2 = __builtin_amdgcn_mfma_f64_16x16x4f64(av, b2, U2, 0, 0, 0);
        }
        sy += av;
    }
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) sy += __shfl_xor(sy, d);
    double lagacc = 0.0;   // lane d <-> lag d
    for (int t = 0; t < NT; t++) {
        const d4 U = (t == 0) ? U0 : (t == 1 ? U1 : U2);
#pragma unroll
        for (int r = 0; r < 4; r++) scr[((lane >> 4) + 4 * r) * 16 + (lane & 15)] = U[r];
        __syncthreads();
#pragma unroll
        for (int b = 0; b < 16; b++)
            if (((b + lane) >> 4) == t) lagacc += scr[b * 16 + ((b + lane) & 15)];
        __syncthreads();
    }
    lagp[lane] = lagacc;
    __syncthreads();

    // ---- Gram of [Y | X_1..X_p] and column sums, lanes in parallel ----
    const int64_t m = T - p;
    const int np1 = p + 1;
    const int npair = np1 * (np1 + 1) / 2;
    for (int idx = lane; idx < npair; idx += 64) {
        int j = 0, rem = idx;
        while (rem >= np1 - j) { rem -= np1 - j; j++; }
        const int k = j + rem;                 // j <= k
        const int d = k - j;
        double g = lagp[d];
        for (int64_t u = 0; u < p - k; u++) g -= Y(u) * Y(u + d);          // head
        for (int64_t u = T - k; u <= T - 1 - d; u++) g -= Y(u) * Y(u + d); // tail
        G[j * kLd + k] = g;
        G[k * kLd + j] = g;
    }
    if (lane < np1) {
        const int k = lane;
        double c = sy;
        for (int64_t u = 0; u < p - k; u++) c -= Y(u);
        for (int64_t u = T - k; u < T; u++) c -= Y(u);
        cs[k] = c;
    }
    __syncthreads();

    // ---- centred normal equations + Cholesky (lane 0), then one step of iterative
    //      refinement with an exact residual pass (corrected semi-normal equations:
    //      recovers the Householder-QR accuracy the normal equations lose to cond^2) ----
    const bool intercept = !a.no_intercept;
    const double fm = (double)m;
    const bool bad = __builtin_isnan(sy) || __builtin_isnan(part);
    bool illc = false;   // AR rule, conditioning half (lane 0)
    if (lane == 0 && !bad) {
        int status = STS_OK;
        if (intercept) {
            for (int j = 1; j <= p; j++) {
                for (int k = 1; k <= p; k++) G[j * kLd + k] -= cs[j] * cs[k] / fm;
                G[0 * kLd + j] -= cs[0] * cs[j] / fm;
            }
        }
        const double mu2m = mu * mu * fm;
        // Cholesky in place on the lower triangle of the 1-based p x p block
        for (int j = 1; j <= p && status == STS_OK; j++) {
            const double dg = G[j * kLd + j];   // centred column j's sum of squares
            double d = dg;
            for (int k = 1; k < j; k++) d -= G[j * kLd + k] * G[j * kLd + k];
            illc = illc || !(mu2m < kRuleRatio2 * dg) || !(d * kRuleKappa > dg);
            if (!(d > 0.0)) { status = STS_ERR_SINGULAR; break; }
            const double l = __builtin_sqrt(d);
            G[j * kLd + j] = l;
            for (int i = j + 1; i <= p; i++) {
                double v = G[i * kLd + j];
                for (int k = 1; k < j; k++) v -= G[i * kLd + k] * G[j * kLd + k];
                G[i * kLd + j] = v / l;
            }
        }
        sol[kPMax + 2] = (double)status;
        if (status == STS_OK) {
            // rhs in row 0; solution phi -> sol[1..p], centred intercept -> sol[0]
            for (int i = 1; i <= p; i++) {
                double v = G[0 * kLd + i];
                for (int k = 1; k < i; k++) v -= G[i * kLd + k] * sol[k];
                sol[i] = v / G[i * kLd + i];
            }
            for (int i = p; i >= 1; i--) {
                double v = sol[i];
                for (int k = i + 1; k <= p; k++) v -= G[k * kLd + i] * sol[k];
                sol[i] = v / G[i * kLd + i];
            }
            double sc = cs[0];
            for (int k = 1; k <= p; k++) sc -= sol[k] * cs[k];
            sol[0] = intercept ? sc / fm : 0.0;
        }
    }
    __syncthreads();
    const int status = bad ? STS_OK : (int)sol[kPMax + 2];
    if (!bad && status == STS_OK) {
        // residual pass: e_r = Y_r - c' - sum_k phi_k X_k(r); g = [sum e, sum e X_k]
        double g[PB + 1];
#pragma unroll
        for (int k = 0; k <= PB; k++) g[k] = 0.0;
        const double cpr = sol[0];
        for (int64_t r = lane; r < m; r += 64) {
            double e = Y(r + p) - cpr;
#pragma unroll
            for (int k = 1; k <= PB; k++)
                if (k <= p) e -= sol[k] * Y(r + p - k);
            g[0] += e;
#pragma unroll
            for (int k = 1; k <= PB; k++)
                if (k <= p) g[k] += e * Y(r + p - k);
        }
#pragma unroll
        for (int k = 0; k <= PB; k++) {
            if (k <= p) {
#pragma unroll
                for (int d = 32; d >= 1; d >>= 1) g[k] += __shfl_xor(g[k], d);
            }
        }
#pragma unroll
        for (int k = 0; k <= PB; k++)
            if (lane == 0 && k <= p) zz[k] = g[k];
        if (lane == 0) {
            double* gg = zz;                 // gradient g[0..p]
            double* z = zz + (kPMax + 2);    // correction z[1..p]
            const double g0 = gg[0];
            for (int i = 1; i <= p; i++) {
                double v = gg[i] - (intercept ? cs[i] * g0 / fm : 0.0);
                for (int k = 1; k < i; k++) v -= G[i * kLd + k] * z[k];
                z[i] = v / G[i * kLd + i];
            }
            for (int i = p; i >= 1; i--) {
                double v = z[i];
                for (int k = i + 1; k <= p; k++) v -= G[k * kLd + i] * z[k];
                z[i] = v / G[i * kLd + i];
            }
            double dc = g0;
            for (int k = 1; k <= p; k++) dc -= z[k] * cs[k];
            double sphi = 0.0;
            for (int k = 1; k <= p; k++) {
                sol[k] += z[k];
                sphi += sol[k];
            }
            // un-shift: y = x - mu  =>  c = c' + mu * (1 - sum phi)
            sol[0] = intercept ? (sol[0] + dc / fm) + mu * (1.0 - sphi) : 0.0;
        }
    }
    if (lane == 0 && !bad && a.qr_list) {
        // AR rule: a singular Cholesky, an ill-conditioned design or a fragile coefficient
        // vector -> the reference's QR decides (sts_ar_qr.hip)
        const bool flag = status != STS_OK || illc || ar_rule_level(sol[0], mu);
        if (flag) ar_rule_append(a, s);
    }
    if (lane == 0) {
        if (bad || status != STS_OK) {
            sol[0] = __builtin_nan("");
            for (int j = 1; j <= p; j++) sol[j] = __builtin_nan("");
        }
        a.c[s] = sol[0];
        for (int j = 0; j < p; j++) a.coef[s * p + j] = sol[1 + j];
        if (a.err) a.err[s] = status;
    }
    if (!a.out) return;
    __syncthreads();

    // ---- fused removeTimeDependentEffects with the fitted model (bit-exact order) ----
    const double c = sol[0];
    double* dst = a.out + s * a.ld_out;
    for (int64_t t = lane; t < T; t += 64) {
        double d = X(t) - c;
        for (int j = 0; j < p && t - j - 1 >= 0; j++) d -= X(t - j - 1) * sol[1 + j];
        dst[t] = d;
    }
}


// ---------------------------------------------------------------------------------------
// Register-resident variant for short series and small p (C4: T = 2,520, p = 5): one WAVE
// per series, four independent waves per workgroup.  Lane l owns the contiguous block of
// B steps [lB, lB + B) in registers, so every lagged operand of the three passes (lag
// products, refinement residuals, the fused remove) is a static register index; only the
// first p steps of a block need the previous lane's last p values (one wave shuffle per
// pass).  No LDS beyond the head/tail terms; the block loads/stores are 16 B per lane.
// The lag products P_0..P_p are lane-local FP64 FMAs: for p <= 8 the 16 x 16 MFMA tile
// would compute >= 24 lags to use p + 1 of them, and on MI355X the FP64 VALU and FP64
// MFMA peaks are equal (profiles/r01_ubench_fp64.jsonl).  Measured in round 4 (commit
// history: STS_AR_MFMA): P_d from v_mfma_f64_16x16x4f64 on the LDS block, 2 MFMAs per 64
// steps, parity green, C4 5.51 ms against 4.11 (profiles/r04_v8_ab_c4_ar_mfma.jsonl).  The (p+1) x (p+1) Gram and the
// Cholesky run uniformly in every lane (ar_normal_chol).  Same algebra as ar_fit_kernel: centred
// data, Gram from lag products minus head/tail terms, Cholesky + one step of refinement
// against an exact residual pass (corrected semi-normal equations: Householder-QR accuracy).
constexpr int kRegPB = 8;             // p <= kRegPB
#ifndef STS_AR_NWV
#define STS_AR_NWV 4   // waves (= series) per workgroup of the register kernel
#endif
constexpr int kRegWaves = STS_AR_NWV;

#ifdef STS_STAMPS
__device__ unsigned long long g_ar_stamps[16];
#define AR_STAMP(i)                                                                          \
    do {                                                                                     \
        const unsigned long long now_ = __builtin_amdgcn_s_memtime();                       \
        st_acc[i] += now_ - st_prev;                                                         \
        st_prev = now_;                                                                      \
    } while (0)
#else
#define AR_STAMP(i) \
    do {            \
    } while (0)
#endif

struct ArWaveLds {
    double head[kRegPB];                     // Y(0 .. p-1)
    double tail[kRegPB];                     // Y(T-p .. T-1)
};

#ifndef STS_AR_FMA
#define STS_AR_FMA 1   // explicit FMAs in the fit passes (A/B on C4: 6.26 -> 5.72 ms; remove stays bit-exact)
#endif

#ifndef STS_AR_DMA
#define STS_AR_DMA 1   // series block in by LDS-DMA, residuals out through the same LDS block
#endif

#ifndef STS_AR_WAVES_PER_EU
#define STS_AR_WAVES_PER_EU 2   // 256 VGPRs: the block (2B), windows and Gram rows stay spill-free
#endif
// DMA: the wave's series arrives by LDS-DMA (global_load_lds_dwordx4, 1 KB of consecutive
// steps per instruction, no VGPR staging) into a per-wave LDS block of 64 B doubles that is
// exactly the lanes' blocks back to back; each lane then reads its B steps with 16-B LDS
// reads.  The fit's LDS scratch (ArWaveLds) aliases that block once the series is in
// registers, and the fused residuals go out through it again (16-B LDS writes at the lanes'
// block offsets, then 1-KB coalesced stores).  Without DMA every load / store instruction
// touches one 16-B piece per lane at a B * 8-byte stride: 64 cache lines per instruction.
// The (p+1)^2 normal equations of the register kernels, solved UNIFORMLY: every lane of the
// wave computes the same Gram, centring and Cholesky in its own registers (round 3).  The
// round-2 form gave lane j row j and moved every column through v_readlane, LDS and a wave
// barrier: ~13 k cycles per series of dependent broadcasts and LDS round trips, the largest
// single phase after the block wait (tools/ar_stamps.py, profiles/r03_v7_ar_stamps.jsonl).
// The same algebra as the lane-parallel form, but NOT its bits: centring multiplies by ifm = 1 / m
// (cs_i cs_k ifm, not cs_i cs_k / m) and the solves multiply by reciprocal pivots; the fitted c / phi
// agree with the reference within the fit's 1e-10 tolerance (tests/test_parity_gpu.py, the
// refinement step absorbs the rounding difference), not bit for bit:
//   A[i][k] (k <= i) = P_{i-k} - sum_{u < P-i} y_u y_{u+i-k} - sum_{v = P-i}^{P-1-(i-k)} t_v t_{v+i-k}
// with y_u the head y(0..p-1) and t_v the tail y(T-p..T-1) (T >= 2p + 1: disjoint); column 0
// is Y, rows / columns 1..p the lags; cs = the design's column sums; centring eliminates the
// intercept; the Cholesky factor of the 1..p block overwrites A's lower triangle; phi = the
// centred right-hand side A[1..p][0].  Returns false when a pivot is not positive (or NaN).
// illc: the conditioning half of the AR rule (kRuleRatio2 on mu2m = mean^2 * m against each
// centred column, kRuleKappa on each scaled pivot).
template <int P>
__device__ __forceinline__ bool ar_normal_chol(const double (&Pd)[P + 1], double sy, const double (&hd)[P],
                                               const double (&tl)[P], bool intercept, double ifm,
                                               double (&A)[P + 1][P + 1], double (&cs)[P + 1],
                                               double (&phi)[P + 1], double mu2m, bool& illc, bool& wellc) {
#pragma unroll
    for (int i = 1; i <= P; i++) {
#pragma unroll
        for (int k = 0; k <= i; k++) {
            const int d = i - k;
            double g = Pd[d];
#pragma unroll
            for (int u = 0; u < P - i; u++) g -= hd[u] * hd[u + d];
#pragma unroll
            for (int v = P - i; v <= P - 1 - d; v++) g -= tl[v] * tl[v + d];
            A[i][k] = g;
        }
    }
#pragma unroll
    for (int j = 0; j <= P; j++) {
        double c = sy;
#pragma unroll
        for (int u = 0; u < P - j; u++) c -= hd[u];
#pragma unroll
        for (int v = P - j; v < P; v++) c -= tl[v];
        cs[j] = c;
    }
    if (intercept) {
#pragma unroll
        for (int i = 1; i <= P; i++)
#pragma unroll
            for (int k = 0; k <= i; k++) A[i][k] -= cs[i] * cs[k] * ifm;
    }
    double dg[P + 1];
#pragma unroll
    for (int j = 1; j <= P; j++) dg[j] = A[j][j];
    bool ok = true;
    illc = false;
    wellc = true;
#pragma unroll
    for (int j = 1; j <= P; j++) {
        const double djj = A[j][j];
        ok = ok && (djj > 0.0);
        illc = illc || !(mu2m < kRuleRatio2 * dg[j]) || !(djj * kRuleKappa > dg[j]);
        wellc = wellc && (djj * kRefineKappa > dg[j]);
        const double l = __builtin_sqrt(djj);
        A[j][j] = l;
#pragma unroll
        for (int i = j + 1; i <= P; i++) A[i][j] = A[i][j] / l;
#pragma unroll
        for (int k = j + 1; k <= P; k++) {
            const double lkj = A[k][j];
#pragma unroll
            for (int i = k; i <= P; i++) A[i][k] -= A[i][j] * lkj;
        }
    }
    phi[0] = 0.0;
#pragma unroll
    for (int i = 1; i <= P; i++) phi[i] = A[i][0];
    return ok;
}

template <int P, int B, int NWV = kRegWaves, bool DMA = false>
__global__ __launch_bounds__(64 * NWV, STS_AR_WAVES_PER_EU) void ar_fit_blk_kernel(ArArgs a) {
    constexpr int BUFD = 64 * B;              // doubles per wave block
    static_assert(!DMA || sizeof(ArWaveLds) <= BUFD * sizeof(double), "scratch fits the block");
    __shared__ __attribute__((aligned(16))) double buf_mem[DMA ? NWV * BUFD : 2];
    __shared__ ArWaveLds lds_mem[DMA ? 1 : NWV];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    // XCD x takes one contiguous range of series (C4: 4.039-4.049 vs 4.074 ms, profiles/r04_v10_ab_c4_xcd.jsonl)
    const int64_t s = xcd_remap(blockIdx.x, gridDim.x) * NWV + wave;
    if (s >= a.S) return;
    double* buf = buf_mem + (DMA ? wave * BUFD : 0);
    ArWaveLds& w = DMA ? *reinterpret_cast<ArWaveLds*>(buf) : lds_mem[wave];
    const int T = (int)a.T;
    const int t0 = lane * B;                  // this lane's block [t0, t0 + B)
    const double* xg = a.in + s * a.ld_in;
    const bool intercept = !a.no_intercept;
#ifdef STS_STAMPS
    unsigned long long st_acc[8] = {0};
    unsigned long long st_prev = __builtin_amdgcn_s_memtime();
#endif

    // ---- the block into registers (16 B per lane per load when aligned); mean ----
    double x[B];
    const bool full = (t0 + B <= T);
    const bool al = ((reinterpret_cast<uintptr_t>(xg) & 15) == 0) && (B % 2 == 0);
    // DMA needs whole 16-B pieces inside the row: T even (and a 16-B aligned row)
    const bool dma = DMA && al && !(T & 1);
    // head / tail of y straight from the DMA block instead of per-step LDS writes in the lag
    // pass (p <= 6: at p = 7, 8 the changed schedule spills)
    constexpr bool hd_blk = P <= 6;
    if (dma) {
        const unsigned lb = lds_addr(buf);
#pragma unroll
        for (int i = 0; i < B / 2; i++) {
            const int u = 2 * (i * 64 + lane);   // series position of this lane's 16-B piece
            glds16<true>(xg + (u < T ? u : 0), lb + i * 1024);   // nt loads + nt stores: C4 4.121-4.128 vs 4.149 ms
        }
        dma_wait();
        wave_lds_sync();
#pragma unroll
        for (int j = 0; j < B / 2; j++) {
            const double2 v = *reinterpret_cast<const double2*>(buf + t0 + 2 * j);
            x[2 * j] = (t0 + 2 * j < T) ? v.x : 0.0;
            x[2 * j + 1] = (t0 + 2 * j + 1 < T) ? v.y : 0.0;
        }
        wave_lds_sync();   // the block is in registers: the LDS block becomes the fit's scratch
    } else if (full && al) {
        const double2* s2 = reinterpret_cast<const double2*>(xg + t0);
#pragma unroll
        for (int j = 0; j < B / 2; j++) {
            const double2 v = s2[j];
            x[2 * j] = v.x;
            x[2 * j + 1] = v.y;
        }
    } else {
#pragma unroll
        for (int j = 0; j < B; j++) {
            const int t = t0 + j;
            const double v = xg[t < T ? t : T - 1];
            x[j] = (t < T) ? v : 0.0;
        }
    }
    double part = 0.0;
#pragma unroll
    for (int j = 0; j < B; j++) part += x[j];
    part = wave_sum_dpp(part);
    const double mu = intercept ? part / (double)T : 0.0;
    // positions past the row take the value mu, so y = x - mu is exactly 0 there and no pass
    // needs a per-step mask (round 3: 3 VALU per step in two passes); the remove pass never
    // stores them
#pragma unroll
    for (int j = 0; j < B; j++) x[j] = (t0 + j < T) ? x[j] : mu;
    AR_STAMP(0);
    // the previous lane's last P raw values (0 before the series)
    double xp[P + 1];
#pragma unroll
    for (int k = 1; k <= P; k++) {
        const double v = lane_prev(x[B - k]);
        xp[k] = (lane > 0) ? v : 0.0;
    }
    // y at block offset j - k (k >= 1 may reach into the previous lane's block)
    auto Y = [&](int j) -> double { return x[j] - mu; };
    auto Yprev = [&](int k) -> double { return (lane > 0) ? xp[k] - mu : 0.0; };

    // ---- lag products P_d = sum_t y_t y_{t-d}; head / tail of the series to LDS ----
    double Pd[P + 1];
#pragma unroll
    for (int d = 0; d <= P; d++) Pd[d] = 0.0;
    double sy = 0.0;
    {
        double win[P + 1];                    // win[k] = y_{t-k}: a rolling window, no arrays of B
#pragma unroll
        for (int k = 1; k <= P; k++) win[k] = Yprev(k);
#pragma unroll
        for (int j = 0; j < B; j++) {
            const double yj = Y(j);
            sy += yj;
#if STS_AR_FMA
            // the fit is a 1e-10-tolerance reduction, not a bit-exact path: explicit FMAs
            // (the library is built with -ffp-contract=off for the bit-exact operators)
            Pd[0] = __builtin_fma(yj, yj, Pd[0]);
#pragma unroll
            for (int d = 1; d <= P; d++) Pd[d] = __builtin_fma(yj, win[d], Pd[d]);
#else
            Pd[0] += yj * yj;
#pragma unroll
            for (int d = 1; d <= P; d++) Pd[d] += yj * win[d];
#endif
#pragma unroll
            for (int k = P; k >= 2; k--) win[k] = win[k - 1];
            win[1] = yj;
            if (!(hd_blk && dma)) {   // with DMA the raw series is still in the LDS block
                if (j < P && lane == 0) w.head[j] = yj;
                const int t = t0 + j;
                if (t >= T - P && t < T) w.tail[t - (T - P)] = yj;
            }
        }
    }
    AR_STAMP(1);
    sy = wave_sum_dpp(sy);
#pragma unroll
    for (int d = 0; d <= P; d++) Pd[d] = wave_sum_dpp(Pd[d]);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
    AR_STAMP(2);
    // ---- normal equations, centring, Cholesky: uniform in every lane (ar_normal_chol) ----
    double hd[P], tl[P];
#pragma unroll
    for (int u = 0; u < P; u++) {   // y = x - mu of the head / tail steps (T >= 2P + 1: raw values)
        hd[u] = (hd_blk && dma) ? buf[u] - mu : w.head[u];
        tl[u] = (hd_blk && dma) ? buf[T - P + u] - mu : w.tail[u];
    }
    const int m = T - P;
    const double fm = (double)m;
    const double ifm = 1.0 / fm;   // the fit is a 1e-10-tolerance path: multiply, no division chains
    const bool bad = __builtin_isnan(sy) || __builtin_isnan(part);
    double A[P + 1][P + 1], cs[P + 1], phi[P + 1];
    bool illc, wellc;
    const bool ok = ar_normal_chol<P>(Pd, sy, hd, tl, intercept, ifm, A, cs, phi, mu * mu * fm, illc, wellc);
    auto Lu = [&](int i, int k) -> double { return A[i][k]; };
    // reciprocals of L's diagonal once: the two solves' substitutions are chains of P steps,
    // and a division per step was ~10 instructions of dependent latency
    double rdg[P + 1];
    rdg[0] = 0.0;
#pragma unroll
    for (int i = 1; i <= P; i++) rdg[i] = 1.0 / Lu(i, i);
    auto solve = [&](double (&z)[P + 1]) {
#pragma unroll
        for (int i = 1; i <= P; i++) {
            double v = z[i];
#pragma unroll
            for (int k = 1; k < i; k++) v -= Lu(i, k) * z[k];
            z[i] = v * rdg[i];
        }
#pragma unroll
        for (int i = P; i >= 1; i--) {
            double v = z[i];
#pragma unroll
            for (int k = i + 1; k <= P; k++) v -= Lu(k, i) * z[k];
            z[i] = v * rdg[i];
        }
    };
    const int status = (!bad && !ok) ? STS_ERR_SINGULAR : STS_OK;
    double cpr = 0.0;
    if (!bad && ok) {
        solve(phi);
        double sc = cs[0];
#pragma unroll
        for (int k = 1; k <= P; k++) sc -= phi[k] * cs[k];
        cpr = intercept ? sc * ifm : 0.0;
        AR_STAMP(3);
        if (STS_AR_SKIP_REFINE && wellc && !illc) {
            // nearly orthogonal lags: the unrefined solution already sits at the reference's own
            // distance from the exact one (kRefineKappa); un-shift and skip the residual pass
            double sphi = 0.0;
#pragma unroll
            for (int k = 1; k <= P; k++) sphi += phi[k];
            cpr = intercept ? cpr + mu * (1.0 - sphi) : 0.0;
        } else {

        // ---- refinement: exact residual pass e_t = Y_t - c' - sum_k phi_k Y_{t-k},
        //      rows t = P .. T-1 of the lag design ----
        double g[P + 1];
#pragma unroll
        for (int k = 0; k <= P; k++) g[k] = 0.0;
        {
            // x "changes" here: y_t = x_t - mu is recomputed instead of being kept live
            // from the lag-product pass (2B more VGPRs)
#pragma unroll
            for (int j = 0; j < B; j++) asm volatile("" : "+v"(x[j]));
            double win[P + 1];
#pragma unroll
            for (int k = 1; k <= P; k++) win[k] = Yprev(k);
#pragma unroll
            for (int j = 0; j < B; j++) {
                const double yj = Y(j);
                double e = yj - cpr;
#if STS_AR_FMA
#pragma unroll
                for (int k = 1; k <= P; k++) e = __builtin_fma(-phi[k], win[k], e);
#else
#pragma unroll
                for (int k = 1; k <= P; k++) e -= phi[k] * win[k];
#endif
                const int t = t0 + j;
                e = (t >= P && t < T) ? e : 0.0;
                g[0] += e;
#if STS_AR_FMA
#pragma unroll
                for (int k = 1; k <= P; k++) g[k] = __builtin_fma(e, win[k], g[k]);
#else
#pragma unroll
                for (int k = 1; k <= P; k++) g[k] += e * win[k];
#endif
#pragma unroll
                for (int k = P; k >= 2; k--) win[k] = win[k - 1];
                win[1] = yj;
            }
        }
        AR_STAMP(4);
#pragma unroll
        for (int k = 0; k <= P; k++) g[k] = wave_sum_dpp(g[k]);
        double z[P + 1];
        const double g0 = g[0];
#pragma unroll
        for (int i = 1; i <= P; i++) z[i] = g[i] - (intercept ? cs[i] * g0 * ifm : 0.0);
        z[0] = 0.0;
        solve(z);
        double dc = g0;
#pragma unroll
        for (int k = 1; k <= P; k++) dc -= z[k] * cs[k];
        double sphi = 0.0;
#pragma unroll
        for (int k = 1; k <= P; k++) {
            phi[k] += z[k];
            sphi += phi[k];
        }
        // un-shift: y = x - mu  =>  c = c' + mu * (1 - sum phi)
        cpr = intercept ? (cpr + dc * ifm) + mu * (1.0 - sphi) : 0.0;
        }
        AR_STAMP(5);
    } else {
        cpr = __builtin_nan("");
#pragma unroll
        for (int k = 1; k <= P; k++) phi[k] = __builtin_nan("");
    }
    if (lane == 0) {
        a.c[s] = cpr;
#pragma unroll
        for (int j = 0; j < P; j++) a.coef[s * P + j] = phi[1 + j];
        if (a.err) a.err[s] = status;
        // AR rule (uniform in every lane; lane 0 appends): the reference's QR decides
        if (!bad && a.qr_list &&
            (!ok || illc || ar_rule_level(cpr, mu)))
            ar_rule_append(a, s);
    }
    if (!a.out) return;

    // ---- fused removeTimeDependentEffects with the fitted model, in the reference's order
    //      (S/models/Autoregression.scala:60-73): d = x_t - c; d -= x_{t-j-1} * coef_j ----
    double* dst = a.out + s * a.ld_out;
    const bool dma_out = dma && ((reinterpret_cast<uintptr_t>(dst) & 15) == 0);
    const bool st16 = !dma_out && full && al && ((reinterpret_cast<uintptr_t>(dst) & 15) == 0);
    if (dma_out) wave_lds_sync();   // every read of the block (head / tail) is done before it is rewritten
    double xw[P + 1];                          // xw[k] = x_{t-k}
#pragma unroll
    for (int k = 1; k <= P; k++) xw[k] = xp[k];
    double rprev = 0.0;
    // one step of the remove; j is a constant after unrolling, so only a block's first P steps
    // carry the "t - k >= 0" test (lane 0's look-back before the series)
    auto step = [&](int j) -> double {
        double d = x[j] - cpr;
#pragma unroll
        for (int k = 1; k <= P; k++)
            if (j >= k || t0 + j - k >= 0) d -= xw[k] * phi[k];
#pragma unroll
        for (int k = P; k >= 2; k--) xw[k] = xw[k - 1];
        xw[1] = x[j];
        return d;
    };
    if (dma_out) {   // the LDS-staged form as its own loop: no per-step branch on the form
#pragma unroll
        for (int j = 0; j < B; j++) {
            const double d = step(j);
            if (j & 1) *reinterpret_cast<double2*>(buf + t0 + j - 1) = make_double2(rprev, d);
            rprev = d;
        }
    } else {
#pragma unroll
        for (int j = 0; j < B; j++) {
            const double d = step(j);
            if (st16) {
                if (j & 1) *reinterpret_cast<double2*>(dst + t0 + j - 1) = make_double2(rprev, d);
                rprev = d;
            } else if (t0 + j < T) {
                dst[t0 + j] = d;
            }
        }
    }
    if (dma_out) {   // coalesced 1-KB stores of the staged residuals (T even)
        wave_lds_sync();
#pragma unroll
        for (int i = 0; i < B / 2; i++) {
            const int u = 2 * (i * 64 + lane);
            if (u < T) store_pair16<true>(dst + u, buf + u);
        }
    }
#ifdef STS_STAMPS
    AR_STAMP(6);
    if (lane == 0) {
#pragma unroll
        for (int i = 0; i < 7; i++) atomicAdd(&g_ar_stamps[i], st_acc[i]);
        atomicAdd(&g_ar_stamps[15], 1ull);
    }
#endif
}

}  // namespace

#ifdef STS_STAMPS
extern "C" int sts_debug_ar_stamps(unsigned long long* out16) {
    if (hipMemcpyFromSymbol(out16, HIP_SYMBOL(g_ar_stamps), sizeof(unsigned long long) * 16) != hipSuccess) return 4;
    unsigned long long z[16] = {0};
    return hipMemcpyToSymbol(HIP_SYMBOL(g_ar_stamps), z, sizeof(z)) == hipSuccess ? 0 : 4;
}
#endif

// scratch of the one-wave-per-series QR form (p > 8): slots of m x ldc doubles.  The host cannot
// see how many series the rule flags (normally none), and the wave kernel strides over its list,
// so the slot count is bounded: one per SIMD (1 024), at most 512 MiB (up to 2 048
// slots / 1 GiB were allocated per call before); a failed allocation retries with half the slots
// rather than failing a fit whose QR phase may have nothing to do.
static hipError_t alloc_qr_scratch(const ArArgs& a, int64_t n, double** scr, int* slots, hipStream_t st) {
    const size_t slot = ar_qr_wave_slot_elems(a.T, a.p, a.no_intercept) * sizeof(double);
    int64_t k = (int64_t)((size_t(512) << 20) / (slot ? slot : 1));
    if (k > 1024) k = 1024;
    if (k > n) k = n;
    if (k < 1) k = 1;
    for (;;) {
        const hipError_t e = hipMallocAsync(reinterpret_cast<void**>(scr), (size_t)k * (slot ? slot : 8), st);
        if (e == hipSuccess) {
            *slots = (int)k;
            return e;
        }
        (void)hipGetLastError();   // clear the failed allocation's error
        if (k == 1) return e;
        k /= 2;
    }
}

static hipError_t launch_ar_fast(const ArArgs& a, hipStream_t st);

hipError_t launch_ar_fit(const ArArgs& a0, hipStream_t st) {
    if (a0.S <= 0) return hipSuccess;
    if (a0.p < 1 || a0.p > kPMax) return hipErrorInvalidValue;
    ArArgs a = a0;
    // A/B build only: the one-wave-per-series QR form for every p (its parity tests)
    const bool force_wave = ab_knob("STS_AR_QR_WAVE") != nullptr;
    const bool wave = force_wave || !ar_qr_lane_ok(a.p);
    hipError_t e;
    if (a.no_intercept) {
        // noIntercept: every series through the reference's QR: without the
        // intercept the lag columns keep the level, and no fast basis tracks the reference's
        // rounding closely enough on price levels
        double* scr = nullptr;
        int slots = 0;
        if (wave) {
            e = alloc_qr_scratch(a, a.S, &scr, &slots, st);
            if (e != hipSuccess) return e;
        }
        e = launch_ar_qr(a, nullptr, nullptr, a.S, scr, slots, force_wave, st);
        if (scr) (void)hipFreeAsync(scr, st);
        return e;
    }
    // intercept: the fast fit, the rule's list of flagged series, the reference's QR on the list
    void* buf = nullptr;
    const size_t list_bytes = ((size_t)a.S * sizeof(int64_t) + 255) & ~size_t(255);
    e = hipMallocAsync(&buf, list_bytes + 256, st);
    if (e != hipSuccess) return e;
    a.qr_list = static_cast<int64_t*>(buf);
    a.qr_count = reinterpret_cast<uint32_t*>(static_cast<char*>(buf) + list_bytes);
    e = hipMemsetAsync(a.qr_count, 0, sizeof(uint32_t), st);
    if (e == hipSuccess) e = launch_ar_fast(a, st);
    double* scr = nullptr;
    int slots = 0;
    if (e == hipSuccess && wave) e = alloc_qr_scratch(a, a.S, &scr, &slots, st);
    if (e == hipSuccess) e = launch_ar_qr(a, a.qr_list, a.qr_count, 0, scr, slots, force_wave, st);
    if (scr) (void)hipFreeAsync(scr, st);
    (void)hipFreeAsync(buf, st);
    return e;
}

hipError_t launch_ar_rule_count(const ArArgs& a0, uint32_t* count, hipStream_t st) {
    if (a0.S <= 0 || a0.no_intercept) return hipSuccess;
    if (a0.p < 1 || a0.p > kPMax) return hipErrorInvalidValue;
    ArArgs a = a0;
    a.out = nullptr;
    void* buf = nullptr;
    hipError_t e = hipMallocAsync(&buf, (size_t)a.S * sizeof(int64_t), st);
    if (e != hipSuccess) return e;
    a.qr_list = static_cast<int64_t*>(buf);
    a.qr_count = count;
    e = hipMemsetAsync(count, 0, sizeof(uint32_t), st);
    if (e == hipSuccess) e = launch_ar_fast(a, st);
    (void)hipFreeAsync(buf, st);
    return e;
}

// the fast fit kernels (intercept)
static hipError_t launch_ar_fast(const ArArgs& a, hipStream_t st) {
    // register path: p <= 8, T <= 64 * 40 (lane blocks of B steps, B in {8, 16, 24, 32, 40})
    if (a.p <= kRegPB && a.T <= 64 * 40 && !ab_knob("STS_AR_STAGED")) {
        constexpr int NWV = kRegWaves;
        dim3 g((unsigned)((a.S + NWV - 1) / NWV)), b(64 * NWV);
        const int64_t need = (a.T + 63) / 64;
        const int B = need <= 8 ? 8 : need <= 16 ? 16 : need <= 24 ? 24 : need <= 32 ? 32 : 40;
#define STS_AR_BLK(PP)                                                                          \
        case PP:                                                                                \
            switch (B) {                                                                        \
            case 8: hipLaunchKernelGGL((ar_fit_blk_kernel<PP, 8, NWV, STS_AR_DMA>), g, b, 0, st, a); break;      \
            case 16: hipLaunchKernelGGL((ar_fit_blk_kernel<PP, 16, NWV, STS_AR_DMA>), g, b, 0, st, a); break;    \
            case 24: hipLaunchKernelGGL((ar_fit_blk_kernel<PP, 24, NWV, STS_AR_DMA>), g, b, 0, st, a); break;    \
            case 32: hipLaunchKernelGGL((ar_fit_blk_kernel<PP, 32, NWV, STS_AR_DMA>), g, b, 0, st, a); break;    \
            default: hipLaunchKernelGGL((ar_fit_blk_kernel<PP, 40, NWV, STS_AR_DMA>), g, b, 0, st, a); break;    \
            }                                                                                   \
            break;
        switch (a.p) {
            STS_AR_BLK(1) STS_AR_BLK(2) STS_AR_BLK(3) STS_AR_BLK(4)
            STS_AR_BLK(5) STS_AR_BLK(6) STS_AR_BLK(7) STS_AR_BLK(8)
        default: return hipErrorInvalidValue;
        }
#undef STS_AR_BLK
        return hipGetLastError();
    }
    const int NT = (a.p + 15) / 16 + 1;
    const size_t fixed = (256 + 64 + (kPMax + 1) * kLd + (kPMax + 2) + (kPMax + 4) + 2 * (kPMax + 2)) * sizeof(double);
    dim3 grid((unsigned)a.S), block(64);
    const bool staged = a.T <= 6144;
    const size_t bytes = fixed + (staged ? (size_t)a.T * sizeof(double) : 0);
    if (staged && a.p <= 8) hipLaunchKernelGGL((ar_fit_kernel<true, 8>), grid, block, bytes, st, a, NT);
    else if (staged) hipLaunchKernelGGL((ar_fit_kernel<true, kPMax>), grid, block, bytes, st, a, NT);
    else if (a.p <= 8) hipLaunchKernelGGL((ar_fit_kernel<false, 8>), grid, block, bytes, st, a, NT);
    else hipLaunchKernelGGL((ar_fit_kernel<false, kPMax>), grid, block, bytes, st, a, NT);
    return hipGetLastError();
}

}  // namespace sts
