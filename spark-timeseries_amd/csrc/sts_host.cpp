// sts_host.cpp -- host-buffer entry points (the JNI path): stage the
// caller's arrays into HBM on the calling thread's stream (hipStreamPerThread), run the
// device entry point, copy the results back and wait.  Scratch is stream-ordered, so
// concurrent executor threads never share buffers.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>

#include "sts.h"

namespace {

hipStream_t kStream = hipStreamPerThread;

struct Dev {
    void* p = nullptr;
    ~Dev() {
        if (p) (void)hipFreeAsync(p, kStream);
    }
    template <class T>
    T* as() { return static_cast<T*>(p); }
};

int up(Dev& d, const void* h, size_t bytes) {
    if (hipMallocAsync(&d.p, bytes ? bytes : 16, kStream) != hipSuccess) return STS_ERR_HIP;
    if (h && bytes && hipMemcpyAsync(d.p, h, bytes, hipMemcpyHostToDevice, kStream) != hipSuccess) return STS_ERR_HIP;
    return STS_OK;
}

int down(void* h, const Dev& d, size_t bytes) {
    if (h && bytes && hipMemcpyAsync(h, d.p, bytes, hipMemcpyDeviceToHost, kStream) != hipSuccess) return STS_ERR_HIP;
    return STS_OK;
}

int finish(int st) {
    hipError_t e = hipStreamSynchronize(kStream);
    if (st == STS_OK && e != hipSuccess) return STS_ERR_HIP;
    return st;
}

size_t panel_bytes(int64_t S, int64_t ld) { return (size_t)(S > 0 ? S : 0) * (size_t)(ld > 0 ? ld : 0) * sizeof(double); }

}  // namespace

extern "C" {

int sts_fill_host(const double* in, double* out, int64_t S, int64_t T, int64_t ld, int method, int32_t* err) {
    Dev di, dout, de;
    int r;
    if ((r = up(di, in, panel_bytes(S, ld))) || (r = up(dout, nullptr, panel_bytes(S, ld))) ||
        (r = up(de, nullptr, (size_t)S * sizeof(int32_t))))
        return finish(r);
    // without a caller error array the device call checks synchronously (exception semantics)
    r = sts_fill(di.as<double>(), dout.as<double>(), S, T, ld, ld, method, err ? de.as<int32_t>() : nullptr, kStream);
    if (r == STS_OK) r = down(out, dout, panel_bytes(S, ld));
    if (r == STS_OK) r = down(err, de, (size_t)S * sizeof(int32_t));
    return finish(r);
}

int sts_autocorr_host(const double* in, int64_t S, int64_t T, int64_t ld, int K, double* acf) {
    Dev di, da;
    int r;
    if ((r = up(di, in, panel_bytes(S, ld))) || (r = up(da, nullptr, (size_t)S * (K > 0 ? K : 0) * sizeof(double))))
        return finish(r);
    r = sts_autocorr(di.as<double>(), S, T, ld, K, da.as<double>(), kStream);
    if (r == STS_OK) r = down(acf, da, (size_t)S * (K > 0 ? K : 0) * sizeof(double));
    return finish(r);
}

int sts_diff_at_lag_host(const double* in, double* out, int64_t S, int64_t T, int64_t ld, int lag, int start) {
    if (!(start >= lag))  // validate before staging, like the reference's require() (:361)
        return sts_diff_at_lag(nullptr, nullptr, 0, 0, 0, 0, lag, start, kStream);
    Dev di, dout;
    int r;
    const bool inplace = (in == out);
    if ((r = up(di, in, panel_bytes(S, ld)))) return finish(r);
    if (!inplace && (r = up(dout, out, panel_bytes(S, ld)))) return finish(r);   // dest contents matter for lag 0
    double* o = inplace ? di.as<double>() : dout.as<double>();
    r = sts_diff_at_lag(di.as<double>(), o, S, T, ld, ld, lag, start, kStream);
    if (r == STS_OK) r = down(out, inplace ? di : dout, panel_bytes(S, ld));
    return finish(r);
}

int sts_lag_matrix_host(const double* in, double* out, int64_t S, int64_t T, int64_t ld, int max_lag, int inc) {
    Dev di, dout;
    int r;
    const int64_t rows = T - max_lag;
    const size_t ob = (size_t)((S > 0 && rows > 0) ? S * rows * (max_lag + (inc ? 1 : 0)) : 0) * sizeof(double);
    if ((r = up(di, in, panel_bytes(S, ld))) || (r = up(dout, nullptr, ob))) return finish(r);
    r = sts_lag_matrix(di.as<double>(), dout.as<double>(), S, T, ld, max_lag, inc, kStream);
    if (r == STS_OK) r = down(out, dout, ob);
    return finish(r);
}

static int ewma_host(bool add, const double* in, double* out, int64_t S, int64_t T, int64_t ld, const double* sm) {
    if (!out) return add ? sts_ewma_add(in, nullptr, S, T, ld, ld, sm, kStream)
                         : sts_ewma_remove(in, nullptr, S, T, ld, ld, sm, kStream);
    Dev di, dout, ds;
    int r;
    const bool inplace = (in == out);
    if ((r = up(di, in, panel_bytes(S, ld))) || (r = up(ds, sm, (size_t)S * sizeof(double)))) return finish(r);
    if (!inplace && (r = up(dout, nullptr, panel_bytes(S, ld)))) return finish(r);
    double* o = inplace ? di.as<double>() : dout.as<double>();
    r = add ? sts_ewma_add(di.as<double>(), o, S, T, ld, ld, ds.as<double>(), kStream)
            : sts_ewma_remove(di.as<double>(), o, S, T, ld, ld, ds.as<double>(), kStream);
    if (r == STS_OK) r = down(out, inplace ? di : dout, panel_bytes(S, ld));
    return finish(r);
}

int sts_ewma_add_host(const double* in, double* out, int64_t S, int64_t T, int64_t ld, const double* sm) {
    return ewma_host(true, in, out, S, T, ld, sm);
}

int sts_ewma_remove_host(const double* in, double* out, int64_t S, int64_t T, int64_t ld, const double* sm) {
    return ewma_host(false, in, out, S, T, ld, sm);
}

int sts_ewma_fit_host(const double* in, int64_t S, int64_t T, int64_t ld, double* smoothing, int32_t* err) {
    Dev di, ds, de;
    int r;
    if ((r = up(di, in, panel_bytes(S, ld))) || (r = up(ds, nullptr, (size_t)S * sizeof(double))) ||
        (r = up(de, nullptr, (size_t)S * sizeof(int32_t))))
        return finish(r);
    r = sts_ewma_fit(di.as<double>(), S, T, ld, ds.as<double>(), err ? de.as<int32_t>() : nullptr, kStream);
    if (r == STS_OK) r = down(smoothing, ds, (size_t)S * sizeof(double));
    if (r == STS_OK) r = down(err, de, (size_t)S * sizeof(int32_t));
    return finish(r);
}

int sts_ar_fit_host(const double* in, int64_t S, int64_t T, int64_t ld, int p, int no_intercept, double* c,
                    double* coef, int32_t* err) {
    Dev di, dc, dk, de;
    int r;
    if ((r = up(di, in, panel_bytes(S, ld))) || (r = up(dc, nullptr, (size_t)S * sizeof(double))) ||
        (r = up(dk, nullptr, (size_t)S * (p > 0 ? p : 0) * sizeof(double))) ||
        (r = up(de, nullptr, (size_t)S * sizeof(int32_t))))
        return finish(r);
    r = sts_ar_fit(di.as<double>(), S, T, ld, p, no_intercept, dc.as<double>(), dk.as<double>(),
                   err ? de.as<int32_t>() : nullptr, kStream);
    if (r == STS_OK) r = down(c, dc, (size_t)S * sizeof(double));
    if (r == STS_OK) r = down(coef, dk, (size_t)S * p * sizeof(double));
    if (r == STS_OK) r = down(err, de, (size_t)S * sizeof(int32_t));
    return finish(r);
}

int sts_garch_fit_host(const double* in, int64_t S, int64_t T, int64_t ld, double* params, int32_t* err) {
    Dev di, dp, de;
    int r;
    if ((r = up(di, in, panel_bytes(S, ld))) || (r = up(dp, nullptr, (size_t)S * 3 * sizeof(double))) ||
        (r = up(de, nullptr, (size_t)S * sizeof(int32_t))))
        return finish(r);
    r = sts_garch_fit(di.as<double>(), S, T, ld, dp.as<double>(), err ? de.as<int32_t>() : nullptr, kStream);
    if (r == STS_OK) r = down(params, dp, (size_t)S * 3 * sizeof(double));
    if (r == STS_OK) r = down(err, de, (size_t)S * sizeof(int32_t));
    return finish(r);
}

int sts_argarch_fit_host(const double* in, int64_t S, int64_t T, int64_t ld, double* c, double* phi,
                         double* params, int32_t* err) {
    Dev di, dc, dphi, dp, de;
    int r;
    if ((r = up(di, in, panel_bytes(S, ld))) || (r = up(dc, nullptr, (size_t)S * sizeof(double))) ||
        (r = up(dphi, nullptr, (size_t)S * sizeof(double))) ||
        (r = up(dp, nullptr, (size_t)S * 3 * sizeof(double))) || (r = up(de, nullptr, (size_t)S * sizeof(int32_t))))
        return finish(r);
    r = sts_argarch_fit(di.as<double>(), S, T, ld, dc.as<double>(), dphi.as<double>(), dp.as<double>(),
                        err ? de.as<int32_t>() : nullptr, kStream);
    if (r == STS_OK) r = down(c, dc, (size_t)S * sizeof(double));
    if (r == STS_OK) r = down(phi, dphi, (size_t)S * sizeof(double));
    if (r == STS_OK) r = down(params, dp, (size_t)S * 3 * sizeof(double));
    if (r == STS_OK) r = down(err, de, (size_t)S * sizeof(int32_t));
    return finish(r);
}

static int ar_host(bool add, const double* in, double* out, int64_t S, int64_t T, int64_t ld, const double* c,
                   const double* coef, int p) {
    Dev di, dout, dc, dk;
    int r;
    const bool inplace = (in == out);
    if ((r = up(di, in, panel_bytes(S, ld))) || (r = up(dc, c, (size_t)S * sizeof(double))) ||
        (r = up(dk, coef, (size_t)S * (p > 0 ? p : 0) * sizeof(double))))
        return finish(r);
    if (!inplace && (r = up(dout, nullptr, panel_bytes(S, ld)))) return finish(r);
    double* o = inplace ? di.as<double>() : dout.as<double>();
    r = add ? sts_ar_add(di.as<double>(), o, S, T, ld, ld, dc.as<double>(), dk.as<double>(), p, kStream)
            : sts_ar_remove(di.as<double>(), o, S, T, ld, ld, dc.as<double>(), dk.as<double>(), p, kStream);
    if (r == STS_OK) r = down(out, inplace ? di : dout, panel_bytes(S, ld));
    return finish(r);
}

int sts_ar_remove_host(const double* in, double* out, int64_t S, int64_t T, int64_t ld, const double* c,
                       const double* coef, int p) {
    return ar_host(false, in, out, S, T, ld, c, coef, p);
}

int sts_ar_add_host(const double* in, double* out, int64_t S, int64_t T, int64_t ld, const double* c,
                    const double* coef, int p) {
    return ar_host(true, in, out, S, T, ld, c, coef, p);
}

}  // extern "C"
