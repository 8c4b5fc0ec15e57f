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

#include <hip/hip_runtime.h>

namespace sts {
namespace {

typedef double d4 __attribute__((ext_vector_type(4)));
constexpr int kPMax = 31;
constexpr int kLd = kPMax + 2;   // row stride of the (p+1) x (p+1) Gram in LDS

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
    if (lane == 0 && !bad) {
        int status = STS_OK;
        if (intercept) {
            for (int j = 1; j <= p; j++) {
                for (int k = 1; k <= p; k++) G[j * kLd + k] -= cs[j] * cs[k] / fm;
                G[0 * kLd + j] -= cs[0] * cs[j] / fm;
            }
        }
        // Cholesky in place on the lower triangle of the 1-based p x p block
        for (int j = 1; j <= p && status == STS_OK; j++) {
            double d = G[j * kLd + j];
            for (int k = 1; k < j; k++) d -= G[j * kLd + k] * G[j * kLd + k];
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

}  // namespace

hipError_t launch_ar_fit(const ArArgs& a, hipStream_t st) {
    if (a.S <= 0) return hipSuccess;
    if (a.p < 1 || a.p > kPMax) return hipErrorInvalidValue;
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
