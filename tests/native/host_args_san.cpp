// Sanitizer driver for the C-ABI argument paths (TEST INFRASTRUCTURE ONLY;
// tests/test_sanitizers.py).  csrc/sts_api.cpp and csrc/sts_host.cpp are compiled for the
// host with -fsanitize=address,undefined (the device objects are linked as built) and every
// `_host` / device entry point is called with the invalid arguments the C ABI must reject
// (null panels, ld < T, bad method / order / lag, numLags < 0, aliasing) -- each must return
// its documented status without touching memory it does not own -- and then with valid
// arguments, which on a machine without a gfx950 device must fail cleanly with
// STS_ERR_NO_DEVICE or STS_ERR_HIP.  Prints "ok" and exits 0 when every status matched.
//
// `host_args_san N` runs the whole sequence in N threads at once (the ThreadSanitizer build
// of tests/test_sanitizers.py: Spark's N executor threads calling the ABI concurrently,
// S/TimeSeriesRDD.scala:417-421), and checks that sts_last_error() stays per thread: each
// thread's own failing call leaves its own message, whatever the other threads do meanwhile.
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "sts.h"

static std::atomic<int> failures{0};

static void expect(int got, int want, const char* what) {
    if (got != want) {
        std::printf("FAIL %s: status %d, expected %d (%s)\n", what, got, want, sts_last_error());
        failures++;
    }
}

static void expect_no_device(int got, const char* what) {
    if (got != STS_ERR_NO_DEVICE && got != STS_ERR_HIP) {
        std::printf("FAIL %s: status %d, expected no-device (%s)\n", what, got, sts_last_error());
        failures++;
    }
}

static void run_checks(int tid) {
    const int64_t S = 3, T = 50;
    std::vector<double> in(S * T, 1.0), out(S * T), acf(S * 70), c(S), coef(S * 8), sm(S, 0.2), par(S * 3);
    std::vector<int32_t> err(S);
    for (int64_t i = 0; i < S * T; i++) in[i] = std::sin(0.1 * (double)i) + (i % 7 == 3 ? NAN : 0.0);

    // ---- argument validation (no device needed) ----
    expect(sts_fill_host(nullptr, out.data(), S, T, T, STS_FILL_LINEAR, nullptr), STS_ERR_BAD_ARG, "fill null in");
    expect(sts_fill_host(in.data(), in.data(), S, T, T, STS_FILL_LINEAR, nullptr), STS_ERR_BAD_ARG, "fill alias");
    expect(sts_fill_host(in.data(), out.data(), S, T, T, 99, nullptr), STS_ERR_UNSUPPORTED_METHOD, "fill method");
    expect(sts_fill_host(in.data(), out.data(), S, T, T - 1, STS_FILL_SPLINE, nullptr), STS_ERR_BAD_ARG,
           "fill spline ld < T");
    expect(sts_fill_host(in.data(), out.data(), S, T, T, STS_FILL_SPLINE + 1, nullptr), STS_ERR_UNSUPPORTED_METHOD,
           "fill method past spline");
    expect(sts_fill_host(in.data(), out.data(), S, T, T - 1, STS_FILL_LINEAR, nullptr), STS_ERR_BAD_ARG, "fill ld < T");
    expect(sts_fill_host(in.data(), out.data(), -1, T, T, STS_FILL_LINEAR, nullptr), STS_ERR_BAD_ARG, "fill S < 0");
    expect(sts_autocorr_host(in.data(), S, T, T, -1, acf.data()), STS_ERR_BAD_ARG, "autocorr K < 0");
    expect(sts_autocorr_host(in.data(), S, T, T, 5, nullptr), STS_ERR_BAD_ARG, "autocorr null out");
    expect(sts_fill_autocorr_host(in.data(), out.data(), S, T, T, 42, 5, acf.data(), nullptr),
           STS_ERR_UNSUPPORTED_METHOD, "fill_autocorr method");
    expect(sts_diff_at_lag_host(in.data(), out.data(), S, T, T, 3, 2), STS_ERR_REQUIREMENT, "diff start < lag");
    expect(sts_diff_at_lag_host(in.data(), out.data(), S, T, T, -1, 0), STS_ERR_BAD_ARG, "diff lag < 0");
    expect(sts_lag_matrix_host(in.data(), out.data(), S, T, T, T + 1, 1), STS_ERR_BAD_ARG, "lag maxLag > T");
    expect(sts_ewma_add_host(in.data(), out.data(), S, T, T, nullptr), STS_ERR_BAD_ARG, "ewma null smoothing");
    expect(sts_ewma_remove_host(in.data(), nullptr, S, T, T, sm.data()), STS_ERR_NULL_DEST, "ewma remove null dest");
    expect(sts_ar_fit_host(in.data(), S, T, T, 0, 0, c.data(), coef.data(), nullptr), STS_ERR_BAD_ARG, "ar p = 0");
    expect(sts_ar_fit_host(in.data(), S, T, T, 32, 0, c.data(), coef.data(), nullptr), STS_ERR_BAD_ARG, "ar p = 32");
    expect(sts_ar_fit_host(in.data(), S, 6, 6, 3, 0, c.data(), coef.data(), nullptr), STS_ERR_NOT_ENOUGH_DATA,
           "ar too short");
    expect(sts_ar_fit_remove_host(in.data(), in.data(), S, T, T, 2, 0, c.data(), coef.data(), nullptr),
           STS_ERR_BAD_ARG, "ar_fit_remove alias");
    expect(sts_ar_remove_host(in.data(), out.data(), S, T, T, nullptr, coef.data(), 2), STS_ERR_BAD_ARG,
           "ar remove null model");
    expect(sts_argarch_fit_host(in.data(), S, 2, 2, c.data(), coef.data(), par.data(), nullptr),
           STS_ERR_NOT_ENOUGH_DATA, "argarch T < 3");
    expect(sts_garch_fit_host(in.data(), S, T, T, nullptr, nullptr), STS_ERR_BAD_ARG, "garch null params");
    expect(sts_host_alloc(16, nullptr), STS_ERR_BAD_ARG, "host_alloc null out");
    expect(sts_staging_stats(nullptr), STS_ERR_BAD_ARG, "staging_stats null");
    double st8[8];
    expect(sts_staging_stats(st8), STS_OK, "staging_stats");
    expect(sts_staging_release(), STS_OK, "staging_release");
    // empty panels are no-ops
    expect(sts_fill_host(in.data(), out.data(), 0, T, T, STS_FILL_LINEAR, nullptr), STS_OK, "fill S = 0");
    expect(sts_fill_method_from_name("linear"), STS_FILL_LINEAR, "method name");
    expect(sts_fill_method_from_name("bogus"), -2, "method name bogus");
    expect(sts_fill_method_from_name(nullptr), -2, "method name null");

    // ---- valid calls: no gfx950 device here, so they must fail cleanly ----
    expect_no_device(sts_fill_host(in.data(), out.data(), S, T, T, STS_FILL_LINEAR, err.data()), "fill");
    expect_no_device(sts_fill_autocorr_host(in.data(), out.data(), S, T, T, STS_FILL_LINEAR, 20, acf.data(), nullptr),
                     "fill_autocorr");
    expect_no_device(sts_fill_diff_ewma_host(in.data(), out.data(), S, T, T, STS_FILL_PREVIOUS, 1, sm.data(), nullptr),
                     "fill_diff_ewma");
    expect_no_device(sts_ar_fit_remove_host(in.data(), out.data(), S, T, T, 5, 0, c.data(), coef.data(), nullptr),
                     "ar_fit_remove");
    expect_no_device(sts_init(0), "init");
    // staging pool controls
    expect(sts_staging_set_limit(0), STS_ERR_BAD_ARG, "staging limit 0");
    expect(sts_staging_set_limit(2 + tid % 3), STS_OK, "staging limit");
    expect(sts_staging_pool_info(nullptr), STS_ERR_BAD_ARG, "pool info null");
    // the thread-local error message: this thread's failing call, other threads' calls in
    // between, still this thread's message
    char want[64];
    std::snprintf(want, sizeof want, "S=%d,", -(tid + 1));
    expect(sts_fill_host(in.data(), out.data(), -(tid + 1), T, T, STS_FILL_LINEAR, nullptr), STS_ERR_BAD_ARG,
           "fill S < 0 (per thread)");
    for (int k = 0; k < 200; k++) std::this_thread::yield();
    const std::string msg = sts_last_error();
    if (msg.find(want) == std::string::npos) {
        std::printf("FAIL thread %d: last error \"%s\" is not its own (%s)\n", tid, msg.c_str(), want);
        failures++;
    }
    sts_staging_release();
}

int main(int argc, char** argv) {
    const int nthreads = argc > 1 ? std::atoi(argv[1]) : 0;
    if (nthreads <= 0) {
        run_checks(0);
    } else {
        for (int rep = 0; rep < 3; rep++) {
            std::vector<std::thread> th;
            for (int t = 0; t < nthreads; t++) th.emplace_back(run_checks, t);
            for (auto& t : th) t.join();
        }
    }
    if (failures) return 1;
    std::puts("ok");
    return 0;
}
