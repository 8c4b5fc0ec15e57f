// sts_spline.hip -- a1 fillts(ts, "spline") = UnivariateTimeSeries.fillSpline
// (S/UnivariateTimeSeries.scala:268-297) over commons-math3 3.4.1 SplineInterpolator.interpolate,
// PolynomialSplineFunction.value and PolynomialFunction.value; bit-exact (built with
// -ffp-contract=off: every product and sum rounds as on the JVM).
//
// The natural cubic spline through the knots (the non-NaN steps, x = the step index as a
// double) is a tridiagonal solve: a forward sweep
//     g = 2 (x[i+1] - x[i-1]) - h[i-1] mu[i-1],  mu[i] = h[i] / g,
//     z[i] = (3 (y[i+1] h[i-1] - y[i] (x[i+1] - x[i-1]) + y[i-1] h[i]) / (h[i-1] h[i])
//             - h[i-1] z[i-1]) / g                                   (mu[0] = z[0] = 0)
// and a backward sweep
//     c[j] = z[j] - mu[j] c[j+1],  b[j] = (y[j+1] - y[j]) / h[j] - h[j] (c[j+1] + 2 c[j]) / 3,
//     d[j] = (c[j+1] - c[j]) / (3 h[j])                               (c[n] = 0),
// two first-order recurrences whose every rounding the reference fixes, so one LANE owns one
// series and runs both in the reference's order.  The forward sweep stores (mu[i], z[i]) at the
// knot's step in a per-series scratch row; the backward sweep walks the series from its end in
// 16-step register chunks and writes every output step exactly once: knot j's polynomial
// {y[j], b[j], c[j], d[j]} gives the steps [x[j], x[j+1]) -- the reference evaluates EVERY step
// from the first knot up to (not including) the last one, knots too (:289-294) -- by Horner's
// rule after PolynomialFunction's trailing-zero trim, at (double)t - x[j] as
// PolynomialSplineFunction.value forms it.  Steps before the first knot, from the last knot on,
// and every step of a series with fewer than 3 knots keep their raw value; the latter also gets
// STS_ERR_TOO_FEW_POINTS (SplineInterpolator's NumberIsTooSmallException) in err.
//
// Off the north_star path's data rates by construction: ~20 dependent FP64 operations (six
// IEEE divisions) per knot per lane; the launcher batches series so the scratch stays bounded.
#include <hip/hip_runtime.h>

#include "sts_internal.hpp"

namespace {

constexpr int kCh = 16;          // steps per register chunk
constexpr int kBlock = 256;      // lanes (series) per workgroup

// commons-math3 PolynomialFunction({y, b, c, d}).value(arg): trailing zero coefficients are
// dropped by the constructor, then Horner's rule (no FMA: the build's -ffp-contract=off)
__device__ __forceinline__ double poly_value(double y, double b, double c, double d, double arg) {
    if (d != 0.0) {
        double r = d;
        r = arg * r + c;
        r = arg * r + b;
        return arg * r + y;
    }
    if (c != 0.0) {
        double r = c;
        r = arg * r + b;
        return arg * r + y;
    }
    if (b != 0.0) return arg * b + y;
    return y;
}

__global__ __launch_bounds__(kBlock) void spline_fill_kernel(const double* __restrict__ in,
                                                            double* __restrict__ out,
                                                            double2* __restrict__ scratch,
                                                            int64_t S, int64_t T, int64_t ld_in,
                                                            int64_t ld_out, int32_t* __restrict__ err) {
    const int64_t s = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (s >= S) return;
    const double* x = in + s * ld_in;
    double* o = out + s * ld_out;
    double2* sc = scratch + s * T;

    // ---- forward sweep (SplineInterpolator.interpolate, the mu / z loop) ----
    int64_t cnt = 0;
    int64_t xa = 0, xb = 0;      // knots i-1 and i (steps)
    double ya = 0.0, yb = 0.0;
    int64_t first = 0;
    double mu_prev = 0.0, z_prev = 0.0;
    for (int64_t t0 = 0; t0 < T; t0 += kCh) {
        double v[kCh];
#pragma unroll
        for (int k = 0; k < kCh; k++) v[k] = (t0 + k < T) ? x[t0 + k] : __builtin_nan("");
#pragma unroll
        for (int k = 0; k < kCh; k++) {
            const double yv = v[k];
            if (yv != yv) continue;
            const int64_t t = t0 + k;
            if (cnt == 0) {
                first = t;
                sc[t] = make_double2(0.0, 0.0);   // mu[0] = z[0] = 0
                xb = t;
                yb = yv;
            } else if (cnt == 1) {
                xa = xb;
                ya = yb;
                xb = t;
                yb = yv;
            } else {
                // knot i = xb gets (mu, z) now that knot i + 1 = t is known
                const double xi1 = (double)t, xi = (double)xb, xim1 = (double)xa;
                const double hm1 = xi - xim1;      // h[i-1]
                const double hi = xi1 - xi;        // h[i]
                const double span = xi1 - xim1;    // x[i+1] - x[i-1]
                const double g = 2.0 * span - hm1 * mu_prev;
                const double mu = hi / g;
                const double z = (3.0 * (yv * hm1 - yb * span + ya * hi) / (hm1 * hi) - hm1 * z_prev) / g;
                sc[xb] = make_double2(mu, z);
                mu_prev = mu;
                z_prev = z;
                xa = xb;
                ya = yb;
                xb = t;
                yb = yv;
            }
            cnt++;
        }
    }
    const bool ok = cnt >= 3;
    if (err) err[s] = ok ? STS_OK : STS_ERR_TOO_FEW_POINTS;

    // ---- backward sweep (the c / b / d loop) and the evaluation ----
    const int64_t lo = ok ? first : T;   // steps < lo keep their raw value
    const int64_t hi = ok ? xb : T;      // steps >= hi too (the last knot is not evaluated)
    double c_next = 0.0, y_next = yb;    // c[n] = 0
    int64_t x_next = hi;
    const int64_t tlast = ((T - 1) / kCh) * kCh;
    for (int64_t t0 = tlast; t0 >= 0; t0 -= kCh) {
        double v[kCh];
        double2 q[kCh];
#pragma unroll
        for (int k = 0; k < kCh; k++) v[k] = (t0 + k < T) ? x[t0 + k] : 0.0;
#pragma unroll
        for (int k = 0; k < kCh; k++) q[k] = (t0 + k < hi && t0 + k >= lo) ? sc[t0 + k] : make_double2(0.0, 0.0);
#pragma unroll
        for (int k = kCh - 1; k >= 0; k--) {
            const int64_t t = t0 + k;
            if (t >= T) continue;
            const double yv = v[k];
            if (t >= hi || t < lo) {
                o[t] = yv;
                continue;
            }
            if (yv != yv) continue;   // filled when its left knot is reached
            const double c = q[k].y - q[k].x * c_next;
            const double xt = (double)t;
            const double h = (double)x_next - xt;
            const double b = (y_next - yv) / h - h * (c_next + 2.0 * c) / 3.0;
            const double d = (c_next - c) / (3.0 * h);
            for (int64_t p = t; p < x_next; p++) o[p] = poly_value(yv, b, c, d, (double)p - xt);
            c_next = c;
            y_next = yv;
            x_next = t;
        }
    }
}

}  // namespace

namespace sts {

int64_t spline_batch(int64_t S, int64_t T) {
    // scratch rows of 16 B per step, at most ~2 GiB per launch (and at least one series)
    const int64_t cap = (int64_t(2) << 30) / (16 * (T > 0 ? T : 1));
    return S < cap ? S : (cap > 0 ? cap : 1);
}

hipError_t launch_spline(const double* in, double* out, int64_t S, int64_t T, int64_t ld_in, int64_t ld_out,
                         int32_t* err, double* scratch, int64_t batch, hipStream_t st) {
    if (S <= 0 || T <= 0) return hipSuccess;
    for (int64_t s0 = 0; s0 < S; s0 += batch) {
        const int64_t n = S - s0 < batch ? S - s0 : batch;
        dim3 g((unsigned)((n + kBlock - 1) / kBlock)), b(kBlock);
        hipLaunchKernelGGL(spline_fill_kernel, g, b, 0, st, in + s0 * ld_in, out + s0 * ld_out,
                           reinterpret_cast<double2*>(scratch), n, T, ld_in, ld_out, err ? err + s0 : nullptr);
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

}  // namespace sts
