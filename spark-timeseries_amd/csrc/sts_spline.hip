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

#include "sts_dma.hpp"
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

#ifndef STS_SPLINE_LDS
#define STS_SPLINE_LDS 1   // round 6: the rows' reads and the (mu, z) scratch through LDS (below)
#endif

// Round 6: the same two sweeps, the same arithmetic in the same order (bit-identical), with the
// memory access reorganised.  spline_fill_kernel's lanes read their own rows 8 B at a time --
// each load instruction touches 64 cache lines, one per lane -- and that, not the FP64 chain,
// bounded it (16.6 ms for 1 M x 390 against a chain floor below 1 ms).  Here a one-wave
// workgroup owns 64 series and walks them in chunks of kLc steps: the chunk of all 64 rows
// arrives by coalesced 16-B loads (4 lanes per row: 16 rows per instruction), is written to an
// LDS tile [row][kLc + 1], and each lane reads its row from there; the next chunk's loads are in
// flight meanwhile.  The forward sweep stores knot i's (mu, z) at the step of knot i + 1 (the
// knot being read when they are formed, so always inside the current chunk) into LDS tiles that
// leave as coalesced 16-B stores; the backward sweep reads them back the same way and carries
// them from knot i + 1 to knot i.  The outputs are still written per lane.
#ifndef STS_SPLINE_LC
#define STS_SPLINE_LC 8   // 8: 190 VGPRs, 18 KB of LDS, 8 waves per CU; 4 (122 VGPRs, 10 KB, 16 waves) measured slower
#endif
constexpr int kLc = STS_SPLINE_LC;  // steps per chunk (4 or 8)
constexpr int kRl = kLc / 2;        // lanes per row in a raw chunk move (16 B each)
constexpr int kRi = kRl;            // raw move instructions per chunk (64 / kRl rows each)
constexpr int kSi = kLc;            // scratch move instructions per chunk (kLc lanes per row, 64 / kLc rows each)
static_assert(kLc == 4 || kLc == 8, "chunk");
constexpr int kLp = kLc + 1;       // LDS row pitch in doubles (odd: conflict-free row reads)

__global__ __launch_bounds__(64) void spline_lds_kernel(const double* __restrict__ in, double* __restrict__ out,
                                                        double2* __restrict__ scratch, int64_t S, int64_t T,
                                                        int64_t ld_in, int64_t ld_out, int32_t* __restrict__ err) {
    __shared__ double RB[2 * 64 * kLp];   // raw chunk tiles (the backward sweep's outputs in place)
    double* const R = RB;
    __shared__ double MU[64 * kLp];   // scratch chunk: mu ...
    __shared__ double Z[64 * kLp];    // ... and z
    const int lane = threadIdx.x;
    const int64_t s0 = (int64_t)blockIdx.x * 64;
    const int nrows = (int)(S - s0 < 64 ? S - s0 : 64);
    const int64_t s = s0 + lane;
    const bool live = lane < nrows;
    // coalesced chunk loads: lane L takes row 16 i + L / 4, steps 2 (L % 4) .. + 1 of the chunk
    const int lr = lane / kRl, lp = (lane % kRl) * 2;
    auto load_raw = [&](int64_t t0, double2 (&v)[kRi]) {
#pragma unroll
        for (int i = 0; i < kRi; i++) {
            const int row = (64 / kRl) * i + lr;
            const int64_t t = t0 + lp;
            if (row < nrows && t < T) {
                const double* src = in + (s0 + row) * ld_in + t;
                if (t + 1 < T) v[i] = *reinterpret_cast<const double2*>(src);   // rows 16-B aligned, t even
                else v[i] = make_double2(src[0], 0.0);
            } else {
                v[i] = make_double2(0.0, 0.0);
            }
        }
    };
    auto put_raw = [&](const double2 (&v)[kRi]) {
#pragma unroll
        for (int i = 0; i < kRi; i++) {
            const int row = (64 / kRl) * i + lr;
            R[row * kLp + lp] = v[i].x;
            R[row * kLp + lp + 1] = v[i].y;
        }
    };
    // scratch chunk moves: lane L takes row 8 i + L / 8, step L % 8
    const int sr = lane / kLc, sk = lane % kLc;
    auto sc_at = [&](int row, int64_t t) { return scratch + (s0 + row) * T + t; };

    // ---- forward sweep: per step straight-line code (32-bit step indices, selects instead of
    //      branches; a lane forms (mu, z) at every step and keeps them only at its knots) ----
    const int Ti = (int)T;
    int cnt = 0, xa = 0, xb = 0, first = 0;
    double ya = 0.0, yb = 0.0, mu_prev = 0.0, z_prev = 0.0;
    double2 nv[kRi];
    load_raw(0, nv);
    for (int t0 = 0; t0 < Ti; t0 += kLc) {
        sts::wave_lds_sync();   // the previous chunk's tiles are read / stored
        put_raw(nv);
        sts::wave_lds_sync();
        if (t0 + kLc < Ti) load_raw(t0 + kLc, nv);   // next chunk in flight
#pragma unroll
        for (int k = 0; k < kLc; k++) {
            const double yv = R[lane * kLp + k];
            const int t = t0 + k;
            const bool knot = live && t < Ti && yv == yv;
            const double xi1 = (double)t, xi = (double)xb, xim1 = (double)xa;
            const double hm1 = xi - xim1;
            const double hi = xi1 - xi;
            const double span = xi1 - xim1;
            const double g = 2.0 * span - hm1 * mu_prev;
            const double mu = hi / g;
            const double z = (3.0 * (yv * hm1 - yb * span + ya * hi) / (hm1 * hi) - hm1 * z_prev) / g;
            // knot 1 stores knot 0's (0, 0), knot i + 1 knot i's (mu, z); other steps' slots are never read
            const bool full = cnt >= 2;
            MU[lane * kLp + k] = full ? mu : 0.0;
            Z[lane * kLp + k] = full ? z : 0.0;
            if (knot) {
                if (full) {
                    mu_prev = mu;
                    z_prev = z;
                }
                if (cnt == 0) first = t;
                if (cnt >= 1) {
                    xa = xb;
                    ya = yb;
                }
                xb = t;
                yb = yv;
                cnt++;
            }
        }
        sts::wave_lds_sync();   // the chunk's (mu, z) out
#pragma unroll
        for (int i = 0; i < kSi; i++) {
            const int row = (64 / kLc) * i + sr;
            const int t = t0 + sk;
            if (row < nrows && t < Ti) *sc_at(row, t) = make_double2(MU[row * kLp + sk], Z[row * kLp + sk]);
        }
    }
    const bool ok = cnt >= 3;
    if (live && err) err[s] = ok ? STS_OK : STS_ERR_TOO_FEW_POINTS;

    // ---- backward sweep.  The outputs go into the raw tile in place (a step's raw value is read
    //      before its output is written) and leave as coalesced 16-B stores one chunk late, so a
    //      knot's gap steps in the chunk to its right still land in LDS; gap steps further right
    //      (gaps longer than a chunk) are stored directly, after the earlier stores completed ----
    double* o = out + s * ld_out;
    const int lo = ok ? first : Ti;
    const int hi = ok ? xb : Ti;
    double c_next = 0.0, y_next = yb, mu_p = 0.0, z_p = 0.0;   // (mu, z) of the knot left of x_next
    int x_next = hi;
    const int tlast = ((Ti - 1) / kLc) * kLc;
    double2 ns[kSi];
    auto load_sc = [&](int t0, double2 (&q)[kSi]) {
#pragma unroll
        for (int i = 0; i < kSi; i++) {
            const int row = (64 / kLc) * i + sr;
            const int t = t0 + sk;
            q[i] = (row < nrows && t < Ti) ? *sc_at(row, t) : make_double2(0.0, 0.0);
        }
    };
    auto flush = [&](int tc, const double* tile) {   // chunk [tc, tc + kLc) of the 64 rows out
#pragma unroll
        for (int i = 0; i < kRi; i++) {
            const int row = (64 / kRl) * i + lr;
            const int t = tc + lp;
            if (row < nrows && t < Ti) {
                double* dst = out + (s0 + row) * ld_out + t;
                if (t + 1 < Ti) *reinterpret_cast<double2*>(dst) = make_double2(tile[row * kLp + lp], tile[row * kLp + lp + 1]);
                else dst[0] = tile[row * kLp + lp];
            }
        }
    };
    load_raw(tlast, nv);
    load_sc(tlast, ns);
    for (int t0 = tlast; t0 >= 0; t0 -= kLc) {
        double* Rc = RB + ((t0 / kLc) & 1) * (64 * kLp);         // this chunk's tile
        double* Rr = RB + (((t0 / kLc) & 1) ^ 1) * (64 * kLp);   // the chunk to its right (not yet out)
        sts::wave_lds_sync();
#pragma unroll
        for (int i = 0; i < kRi; i++) {
            const int row = (64 / kRl) * i + lr;
            Rc[row * kLp + lp] = nv[i].x;
            Rc[row * kLp + lp + 1] = nv[i].y;
        }
#pragma unroll
        for (int i = 0; i < kSi; i++) {
            const int row = (64 / kLc) * i + sr;
            MU[row * kLp + sk] = ns[i].x;
            Z[row * kLp + sk] = ns[i].y;
        }
        sts::wave_lds_sync();
        if (t0 > 0) {
            load_raw(t0 - kLc, nv);
            load_sc(t0 - kLc, ns);
        }
#pragma unroll
        for (int k = kLc - 1; k >= 0; k--) {
            const int t = t0 + k;
            const double yv = Rc[lane * kLp + k];
            const double mu_here = MU[lane * kLp + k], z_here = Z[lane * kLp + k];
            const bool in_t = live && t < Ti;
            const bool raw = t >= hi || t < lo;                       // keeps its raw value
            const bool knot = in_t && !raw && yv == yv;
            const double c = z_p - mu_p * c_next;
            const double xt = (double)t;
            const double h = (double)x_next - xt;
            const double b = (y_next - yv) / h - h * (c_next + 2.0 * c) / 3.0;
            const double d = (c_next - c) / (3.0 * h);
            // PolynomialFunction({yv, b, c, d}).value(arg): Horner over the untrimmed coefficients
            // equals the trimmed form (a zero leading coefficient contributes +0.0 exactly), except
            // all-zero b, c, d, where the trimmed form returns yv itself (its sign of zero)
            const bool deg0 = b == 0.0 && c == 0.0 && d == 0.0;
            if (knot) Rc[lane * kLp + k] = deg0 ? yv : ((0.0 * d + c) * 0.0 + b) * 0.0 + yv;
            if (in_t && t == hi) {   // the last knot: its left neighbour's (mu, z)
                mu_p = mu_here;
                z_p = z_here;
            }
            if (knot) {
                // a gap past the right chunk: those chunks are out already -- wait for their stores
                // before storing over them (once per such knot)
                if (x_next > t0 + 2 * kLc) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                for (int p = t + 1; p < x_next; p++) {   // the NaN steps up to the next knot
                    const double arg = (double)p - xt;
                    const double v = deg0 ? yv : ((arg * d + c) * arg + b) * arg + yv;
                    if (p < t0 + kLc) Rc[lane * kLp + (p - t0)] = v;
                    else if (p < t0 + 2 * kLc) Rr[lane * kLp + (p - t0 - kLc)] = v;
                    else o[p] = v;
                }
                c_next = c;
                y_next = yv;
                x_next = t;
                mu_p = mu_here;
                z_p = z_here;
            }
        }
        sts::wave_lds_sync();
        if (t0 + kLc < Ti) flush(t0 + kLc, Rr);   // the right chunk is final now
    }
    flush(0, RB);
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
        if (STS_SPLINE_LDS && !(ld_in & 1) && !(ld_out & 1) && !(reinterpret_cast<uintptr_t>(in) & 15) &&
            !(reinterpret_cast<uintptr_t>(out) & 15) && T < (int64_t(1) << 30)) {   // 16-B row pieces, 32-bit steps
            dim3 g((unsigned)((n + 63) / 64)), b(64);
            hipLaunchKernelGGL(spline_lds_kernel, g, b, 0, st, in + s0 * ld_in, out + s0 * ld_out,
                               reinterpret_cast<double2*>(scratch), n, T, ld_in, ld_out, err ? err + s0 : nullptr);
        } else {
            dim3 g((unsigned)((n + kBlock - 1) / kBlock)), b(kBlock);
            hipLaunchKernelGGL(spline_fill_kernel, g, b, 0, st, in + s0 * ld_in, out + s0 * ld_out,
                               reinterpret_cast<double2*>(scratch), n, T, ld_in, ld_out, err ? err + s0 : nullptr);
        }
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

}  // namespace sts
