/* Sanitizer driver for the CPU oracle (TEST INFRASTRUCTURE ONLY; tests/test_sanitizers.py).
 * Built with -fsanitize=address,undefined -fno-sanitize-recover=all together with
 * oracle/sts_oracle.c and oracle/sts_oracle_garch.c, it runs every restated operator on the
 * edge shapes the parity tests use (n = 0, 1, 2, all-NaN, leading / trailing NaN runs,
 * maxLag = n, AR order at the data limit) so any out-of-bounds access, overflow or
 * undefined conversion aborts the run.  Prints "ok" and exits 0 when clean. */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "sts_oracle.h"

static double* vec(int64_t n) { return (double*)calloc((size_t)(n > 0 ? n : 1), sizeof(double)); }

static void series(double* x, int64_t n, int kind, unsigned seed) {
    double v = 1.0 + (seed % 7);
    for (int64_t i = 0; i < n; i++) {
        seed = seed * 1103515245u + 12345u;
        v += ((seed >> 8) % 2001 - 1000) * 1e-3;
        x[i] = v;
        if (kind == 1 && (seed >> 20) % 5 == 0) x[i] = NAN;                   /* 20 % NaN */
        if (kind == 2) x[i] = NAN;                                             /* all NaN */
        if (kind == 3 && (i < n / 3 || i >= n - n / 4)) x[i] = NAN;            /* NaN head and tail */
        if (kind == 4) x[i] = 3.0;                                             /* constant */
    }
}

int main(void) {
    const int64_t lens[] = {0, 1, 2, 3, 5, 17, 64, 65, 130, 600};
    for (size_t li = 0; li < sizeof lens / sizeof lens[0]; li++) {
        const int64_t n = lens[li];
        for (int kind = 0; kind < 5; kind++) {
            double* x = vec(n);
            double* r = vec(n);
            double* d = vec(n);
            series(x, n, kind, (unsigned)(n * 31 + kind));
            for (int m = 0; m < 4; m++) (void)orc_fillts(x, r, n, m);
            orc_fill_linear(x, r, n);
            for (int K = 0; K <= 70 && n > 0; K += 7) {
                double* acf = vec(K);
                orc_autocorr(r, n, K, acf);
                free(acf);
            }
            for (int lag = 0; lag <= 4 && lag <= n; lag++) {
                double* lm = vec((n - lag + 1) * (lag + 1));
                (void)orc_lag_mat_trim_both(r, n, lag, 1, lm);
                (void)orc_lag_mat_trim_both(r, n, lag, 0, lm);
                free(lm);
                (void)orc_differences_at_lag(r, d, n, lag, lag);
                (void)orc_inverse_differences_at_lag(d, d, n, lag, lag);
            }
            orc_differences_of_order_d(r, d, n, n > 2 ? 2 : 0);
            orc_ewma_add(r, d, n, 0.3);
            orc_ewma_remove(r, d, n, 0.3);
            double c = 0.1, coef[8] = {0.5, -0.2, 0.1, 0, 0, 0, 0, 0};
            orc_ar_add(r, d, n, c, coef, 3);
            orc_ar_remove(r, d, n, c, coef, 3);
            for (int p = 1; p <= 8; p++)
                if (n - p >= p + 1) {
                    (void)orc_ar_fit(r, n, p, 0, &c, coef);
                    (void)orc_ar_fit(r, n, p, 1, &c, coef);
                }
            double st[4];
            orc_stat_counter(x, n, st);
            if (n > 0 && n <= 130) {
                double sm = 0;
                int64_t ev = 0;
                (void)orc_ewma_fit(r, n, &sm, &ev);
                double g[3];
                (void)orc_garch_loglik(r, n, 0.2, 0.2, 0.2);
                orc_garch_gradient(r, n, 0.2, 0.2, 0.2, g);
                orc_garch_remove(r, d, n, 0.2, 0.1, 0.3);
                orc_garch_add(r, d, n, 0.2, 0.1, 0.3);
                orc_argarch_remove(r, d, n, 0.1, 0.5, 0.2, 0.1, 0.3);
                orc_argarch_add(r, d, n, 0.1, 0.5, 0.2, 0.1, 0.3);
            }
            free(x);
            free(r);
            free(d);
        }
    }
    /* panel drivers, padded ld, two threads */
    const int64_t S = 5, T = 300, ld = 311;
    double* in = vec(S * ld);
    double* out = vec(S * ld);
    double* acf = vec(S * 60);
    int32_t err[5];
    orc_gen_panel(3, 0, S, T, ld, 0.1, in);
    for (int m = 0; m < 4; m++) (void)orc_panel_fill(in, out, S, T, ld, m, err, 2);
    (void)orc_panel_fill_autocorr(in, out, S, T, ld, 0, 60, acf, err, 2);
    (void)orc_panel_fill_diff_ewma(in, out, S, T, ld, 0.2, 2);
    double cs[5], co[5 * 5];
    orc_gen_ar_panel(4, 0, S, T, ld, 5, in);
    (void)orc_panel_ar_fit_remove(in, out, S, T, ld, 5, 0, cs, co, 2);
    double* inst = vec(S * T);
    int64_t active[300];
    (void)orc_remove_instants_with_nans(in, S, T, ld, out, active);
    orc_to_instants(in, S, T, ld, inst);
    free(in);
    free(out);
    free(acf);
    free(inst);
    puts("ok");
    return 0;
}
