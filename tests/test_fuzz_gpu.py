"""Randomised parity sweeps through the product library (seeded, deterministic).

Every case draws a panel shape (T log-uniform over 2 .. 40 000, so the short, segment and tile
kernels all run), a fill method, numLags, a NaN rate with or without long runs, a level and a
series family, and checks the fused fill + autocorr against the oracle: the fill bit for bit,
the ACF within the tolerance contract of tests/test_acf_robust.py (1e-10 relative plus the
reference's own rounding-noise floor, computed on the filled series).  A second sweep does the
same for the AR(p) fit (both intercept modes, 1e-10 elementwise against commons-math3's
Householder QR as restated in the oracle).  These complement the hand-picked edge cases of
test_parity_gpu.py with breadth."""
import os
import zlib

import numpy as np
import pytest

import oracle
from test_acf_robust import noise_floor, within

METHODS = ["linear", "previous", "next", "nearest"]
# STS_FUZZ_SCALE=n multiplies the number of cases (a deeper one-off sweep; default 1)
SCALE = int(os.environ.get("STS_FUZZ_SCALE", "1"))


@pytest.fixture(scope="module")
def torch():
    import torch as _t
    if not _t.cuda.is_available():
        pytest.skip("no GPU")
    from sparkts import _native
    _native.ensure_device(0)
    return _t


def fuzz_panel(rng, S, T, family, level, nan_p, runs):
    if family == "walk":
        x = level + np.cumsum(rng.standard_normal((S, T)), axis=1) * 0.1
    elif family == "noise":
        x = level + rng.standard_normal((S, T))
    elif family == "ar1":
        e = rng.standard_normal((S, T))
        x = np.empty((S, T))
        x[:, 0] = e[:, 0]
        for t in range(1, T):
            x[:, t] = 0.95 * x[:, t - 1] + e[:, t]
        x += level
    else:   # steps: piecewise constant with a few jumps
        x = level + np.cumsum((rng.random((S, T)) < 0.01) * rng.standard_normal((S, T)), axis=1)
    x[rng.random((S, T)) < nan_p] = np.nan
    if runs and T > 10:
        for s in range(S):
            a = int(rng.integers(0, T))
            x[s, a: min(T, a + int(rng.integers(1, max(2, T // 4))))] = np.nan
    return x


@pytest.mark.gpu
@pytest.mark.parametrize("case", range(40 * SCALE))
def test_fuzz_fill_autocorr(torch, case):
    from sparkts import TimeSeriesRDD
    rng = np.random.default_rng(zlib.crc32(b"fuzz-acf-%d" % case))
    T = int(np.exp(rng.uniform(np.log(2), np.log(40000))))
    S = int(rng.integers(1, 9))
    method = METHODS[case % 4]
    K = int(rng.integers(1, max(2, min(61, T))))
    family = ["walk", "noise", "ar1", "steps"][int(rng.integers(0, 4))]
    level = float(rng.choice([0.0, 100.0, 1e4, 1e6]))
    x = fuzz_panel(rng, S, T, family, level, float(rng.choice([0.0, 0.02, 0.1, 0.4])), bool(rng.integers(0, 2)))
    if method == "nearest" and T > 1:
        x[:, 1] = level + 1.0   # a valid step after index 0: no "Input is all NaNs!"
    filled, acf = TimeSeriesRDD(None, None, torch.as_tensor(x, device="cuda:0")).fillAndAutocorr(method, K)
    rf, racf, err = oracle.panel_fill_autocorr(x, method, K)
    assert (err == 0).all()
    f = filled.data.cpu().numpy()
    same = (f.view(np.uint64) == rf.view(np.uint64)) | (np.isnan(f) & np.isnan(rf))
    assert same.all(), (case, T, method, int((~same).sum()))
    got = acf.cpu().numpy()
    for s in range(S):
        w = within(got[s], racf[s], noise_floor(rf[s], K))
        assert w <= 1.0, (case, s, T, K, method, family, level, w)


@pytest.mark.gpu
@pytest.mark.parametrize("case", range(24 * SCALE))
def test_fuzz_ar_fit(torch, case):
    from sparkts.models import Autoregression
    rng = np.random.default_rng(zlib.crc32(b"fuzz-ar-%d" % case))
    p = int(rng.integers(1, 9))
    T = int(rng.integers(2 * p + 3, 6001))
    S = int(rng.integers(1, 40))
    no_int = bool(case % 3 == 2)
    family = ["walk", "noise", "ar1"][int(rng.integers(0, 3))]   # (piecewise-constant rows can be singular)
    level = float(rng.choice([0.0, 10.0, 1e3, 1e5, -2e4]))
    x = fuzz_panel(rng, S, T, family, level, 0.0, False)
    m = Autoregression.fitModel(torch.as_tensor(x, device="cuda:0"), p, no_int)
    c = np.atleast_1d(m.c.cpu().numpy()) if hasattr(m.c, "cpu") else np.full(S, m.c)
    coef = m.coefficients.cpu().numpy().reshape(S, p)
    for s in range(S):
        rc, rcoef = oracle.ar_fit(x[s], p, no_int)
        ref = np.r_[rc, rcoef]
        got = np.r_[c[s], coef[s]]
        if no_int:
            ref, got = ref[1:], got[1:]
        if not np.all(np.isfinite(ref)):
            assert np.array_equal(np.isnan(got), np.isnan(ref)), (case, s)
            continue
        big = np.abs(ref) > 1e-6 * np.linalg.norm(ref)
        e = float(np.max(np.abs(got[big] - ref[big]) / np.abs(ref[big])))
        assert e <= 1e-10, (case, s, p, T, no_int, family, level, e)


@pytest.mark.gpu
@pytest.mark.parametrize("case", range(24 * SCALE))
def test_fuzz_fill_diff_ewma(torch, case):
    # C2's fused pipeline: fillPrevious -> differencesAtLag(lag) -> EWMA add, bit for bit
    from sparkts import _native
    rng = np.random.default_rng(zlib.crc32(b"fuzz-c2-%d" % case))
    T = int(np.exp(rng.uniform(np.log(2), np.log(3000))))
    S = int(rng.integers(1, 70))
    lag = int(rng.integers(1, max(2, min(6, T))))
    family = ["walk", "noise", "steps"][int(rng.integers(0, 3))]
    x = fuzz_panel(rng, S, T, family, float(rng.choice([0.0, 100.0, 1e6])), float(rng.choice([0.0, 0.05, 0.3])),
                   bool(rng.integers(0, 2)))
    s = rng.uniform(0.01, 0.99, S)
    xd = torch.as_tensor(x, device="cuda:0")
    out = torch.empty_like(xd)
    sd = torch.as_tensor(s, device="cuda:0")
    assert _native.lib().sts_fill_diff_ewma(xd.data_ptr(), out.data_ptr(), S, T, T, T, 3, lag, sd.data_ptr(),
                                            None, None) == 0
    ref = np.array([oracle.ewma_add(oracle.differences_at_lag(oracle.fill_previous(r), lag), float(si))
                    for r, si in zip(x, s)])
    got = out.cpu().numpy()
    same = (got.view(np.uint64) == ref.view(np.uint64)) | (np.isnan(got) & np.isnan(ref))
    assert same.all(), (case, S, T, lag, int((~same).sum()))


@pytest.mark.gpu
@pytest.mark.parametrize("case", range(16 * SCALE))
def test_fuzz_fill_lag_matrix(torch, case):
    # C5's fused pipeline: fill(method) -> lag(p, includeOriginal), bit for bit
    from sparkts import _native
    from sparkts import UnivariateTimeSeries as uts
    rng = np.random.default_rng(zlib.crc32(b"fuzz-c5-%d" % case))
    T = int(np.exp(rng.uniform(np.log(16), np.log(30000))))
    S = int(rng.integers(1, 6))
    p = int(rng.integers(1, min(12, T - 1)))
    inc = int(rng.integers(0, 2))
    method = METHODS[case % 4]
    x = fuzz_panel(rng, S, T, "walk", 100.0, float(rng.choice([0.0, 0.05, 0.3])), bool(rng.integers(0, 2)))
    x[:, 1] = 100.0   # nearest: a valid step after index 0
    xd = torch.as_tensor(x, device="cuda:0")
    filled = torch.empty_like(xd)
    ncol = p + inc
    lm = torch.empty((S, ncol, T - p), dtype=torch.float64, device="cuda:0")
    assert _native.lib().sts_fill_lag_matrix(xd.data_ptr(), filled.data_ptr(), lm.data_ptr(), S, T, T, T,
                                             uts.fill_method_code(method), p, inc, None, None) == 0
    rf, _ = oracle.panel_fill(x, method)
    f = filled.cpu().numpy()
    assert ((f.view(np.uint64) == rf.view(np.uint64)) | (np.isnan(f) & np.isnan(rf))).all(), (case, "fill")
    ref = np.array([oracle.lag(r, p, bool(inc)) for r in rf])   # (S, rows, cols)
    got = lm.cpu().numpy().transpose(0, 2, 1)
    assert ((got.view(np.uint64) == ref.view(np.uint64)) | (np.isnan(got) & np.isnan(ref))).all(), (case, "lag")


@pytest.mark.gpu
@pytest.mark.parametrize("case", range(12 * SCALE))
def test_fuzz_ewma_fit(torch, case):
    # EWMA.fitModel (commons-math3 nonlinear CG + bracketing + Brent per series): the smoothing
    # parameter bit for bit and the same per-series errors as the restatement
    from sparkts.models import EWMA
    rng = np.random.default_rng(zlib.crc32(b"fuzz-ewma-%d" % case))
    T = int(np.exp(rng.uniform(np.log(2), np.log(1500))))
    S = int(rng.integers(1, 70))
    family = ["walk", "noise", "ar1", "steps"][int(rng.integers(0, 4))]
    x = fuzz_panel(rng, S, T, family, float(rng.choice([0.0, 100.0, 1e4])), 0.0, False)
    err = torch.zeros(S, dtype=torch.int32, device="cuda:0")
    m = EWMA.fitModel(torch.as_tensor(x, device="cuda:0"), errors=err)
    ref_s, ref_err = oracle.panel_ewma_fit(x, threads=8)
    assert np.array_equal(err.cpu().numpy(), ref_err), case
    got = np.asarray(m.smoothing.cpu().numpy(), dtype=np.float64)
    same = (got.view(np.uint64) == ref_s.view(np.uint64)) | (np.isnan(got) & np.isnan(ref_s))
    assert same.all(), (case, S, T, family, int((~same).sum()))


@pytest.mark.gpu
@pytest.mark.parametrize("case", range(6 * SCALE))
def test_fuzz_garch_fit(torch, case):
    # GARCH.fitModel (commons-math3 CG without a GoalType, per series): (omega, alpha, beta) bit for
    # bit and the same per-series errors as the restatement, over random GARCH(1,1) samples
    from sparkts.models import GARCH
    from test_garch import MersenneTwister, garch_sample
    rng = np.random.default_rng(zlib.crc32(b"fuzz-garch-%d" % case))
    T = int(rng.integers(40, 700))
    S = int(rng.integers(1, 12))
    rows = []
    for s in range(S):
        om, al = float(rng.uniform(0.05, 0.5)), float(rng.uniform(0.02, 0.4))
        be = float(rng.uniform(0.0, 0.95 - al))
        rows.append(garch_sample(om, al, be, T, MersenneTwister(int(rng.integers(1, 2**31)))))
    x = np.array(rows)
    err = torch.zeros(S, dtype=torch.int32, device="cuda:0")
    m = GARCH.fitModel(torch.as_tensor(x, device="cuda:0"), errors=err)
    got = np.stack([m.omega.cpu().numpy(), m.alpha.cpu().numpy(), m.beta.cpu().numpy()], axis=1)
    rpar, rerr = oracle.panel_garch_fit(x)
    assert np.array_equal(err.cpu().numpy(), rerr), case
    same = (got.view(np.uint64) == rpar.view(np.uint64)) | (np.isnan(got) & np.isnan(rpar))
    assert same.all(), (case, S, T, int((~same).sum()))


@pytest.mark.gpu
@pytest.mark.parametrize("case", range(12 * SCALE))
def test_fuzz_stats_instants(torch, case):
    # seriesStats (Spark StatCounter per series), removeInstantsWithNaNs and toInstants on random
    # shapes, magnitudes, NaN / inf patterns: bit for bit
    from sparkts.timeseriesrdd import TimeSeriesRDD
    rng = np.random.default_rng(zlib.crc32(b"fuzz-f2-%d" % case))
    S = int(np.exp(rng.uniform(0, np.log(400))))
    T = int(np.exp(rng.uniform(0, np.log(6000))))
    x = rng.standard_normal((S, T)) * 10.0 ** rng.integers(-200, 200, size=(S, 1))
    if rng.random() < 0.5:
        x[rng.random((S, T)) < float(rng.choice([1e-4, 1e-3, 0.02]))] = np.nan
    if rng.random() < 0.3:
        x[rng.random((S, T)) < 1e-3] = np.inf * rng.choice([-1.0, 1.0])
    st = TimeSeriesRDD(None, None, torch.as_tensor(x, device="cuda:0")).seriesStats()
    ref = np.array([oracle.stat_counter(r)[1:] for r in x])
    got = st.stats.cpu().numpy()[:, :4]
    same = (got.view(np.uint64) == ref.view(np.uint64)) | (np.isnan(got) & np.isnan(ref))
    assert same.all(), (case, S, T, "stats", int((~same).sum()))
    r = TimeSeriesRDD(None, None, torch.as_tensor(x, device="cuda:0")).removeInstantsWithNaNs()
    rref, active = oracle.remove_instants_with_nans(x)
    assert np.array_equal(r.index, active), (case, "instants")
    g = r.data.cpu().numpy().reshape(rref.shape)
    assert ((g.view(np.uint64) == rref.view(np.uint64)) | (np.isnan(g) & np.isnan(rref))).all(), (case, "gather")
    _, inst = TimeSeriesRDD(None, None, torch.as_tensor(x, device="cuda:0")).toInstants()
    ti = inst.cpu().numpy()
    tref = oracle.to_instants(x)
    assert ((ti.view(np.uint64) == tref.view(np.uint64)) | (np.isnan(ti) & np.isnan(tref))).all(), (case, "toInstants")


@pytest.mark.gpu
@pytest.mark.parametrize("case", range(12 * SCALE))
def test_fuzz_ar_fit_remove(torch, case):
    # C4's fused fit + removeTimeDependentEffects: the model at 1e-10 elementwise against the
    # reference's QR, the residuals bit for bit given the device's own model
    from sparkts.models import Autoregression
    rng = np.random.default_rng(zlib.crc32(b"fuzz-c4-%d" % case))
    p = int(rng.integers(1, 9))
    T = int(rng.integers(2 * p + 3, 4001))
    S = int(rng.integers(1, 90))
    family = ["walk", "noise", "ar1"][int(rng.integers(0, 3))]
    x = fuzz_panel(rng, S, T, family, float(rng.choice([0.0, 1.0, 1e3, 1e6])), 0.0, False)
    m, resid = Autoregression.fitModelAndRemove(torch.as_tensor(x, device="cuda:0"), p)
    c, coef, res = m.c.cpu().numpy(), m.coefficients.cpu().numpy().reshape(S, p), resid.cpu().numpy()
    for s in range(S):
        rc, rcoef = oracle.ar_fit(x[s], p)
        ref, got = np.r_[rc, rcoef], np.r_[c[s], coef[s]]
        big = np.abs(ref) > 1e-6 * np.linalg.norm(ref)
        assert float(np.max(np.abs(got[big] - ref[big]) / np.abs(ref[big]))) <= 1e-10, (case, s, p, T, family)
        rr = oracle.ar_remove(x[s], c[s], coef[s])
        assert (res[s].view(np.uint64) == rr.view(np.uint64)).all(), (case, s, "residuals")


@pytest.mark.gpu
@pytest.mark.parametrize("case", range(8 * SCALE))
def test_fuzz_host_entry_points(torch, case):
    # the _host entry points: host panels through the pinned staging pipeline (chunked by series,
    # padded row strides), the same bits as the oracle -- fills, the fused fill + ACF (contract),
    # C2's fused pipeline
    import ctypes
    from sparkts import _native
    lib = _native.lib()
    P = lambda a: a.ctypes.data_as(ctypes.c_void_p)   # noqa: E731
    rng = np.random.default_rng(zlib.crc32(b"fuzz-host-%d" % case))
    T = int(np.exp(rng.uniform(np.log(4), np.log(20000))))
    S = int(np.exp(rng.uniform(0, np.log(max(2, 4e7 // (8 * T))))))   # up to ~40 MB panels: several chunks
    pad = int(rng.integers(0, 3))
    ld = T + pad
    method = int(rng.integers(0, 4))   # STS_FILL_LINEAR .. STS_FILL_PREVIOUS
    xb = fuzz_panel(rng, S, ld, "walk", 100.0, float(rng.choice([0.0, 0.05, 0.3])), bool(rng.integers(0, 2)))
    xb[:, 1] = 100.0
    x = np.ascontiguousarray(xb)
    out = np.full((S, ld), -1.0)
    err = np.zeros(S, dtype=np.int32)
    assert lib.sts_fill_host(P(x), P(out), S, T, ld, method, P(err)) == 0, lib.sts_last_error()
    name = {0: "linear", 1: "nearest", 2: "next", 3: "previous"}[method]
    rf, rerr = oracle.panel_fill(x[:, :T].copy(), name)
    assert np.array_equal(err, rerr)
    got = out[:, :T]
    assert ((got.view(np.uint64) == rf.view(np.uint64)) | (np.isnan(got) & np.isnan(rf))).all(), (case, "fill_host")
    if T >= 2:
        K = int(rng.integers(1, min(61, T)))
        acf = np.empty((S, K))
        filled = np.empty((S, ld))
        assert lib.sts_fill_autocorr_host(P(x), P(filled), S, T, ld, method, K, P(acf), P(err)) == 0, lib.sts_last_error()
        _, racf, _ = oracle.panel_fill_autocorr(x[:, :T].copy(), name, K)
        for s in range(0, S, max(1, S // 16)):
            assert within(acf[s], racf[s], noise_floor(rf[s], K)) <= 1.0, (case, s, "fill_autocorr_host")
    sm = rng.uniform(0.05, 0.95, S)
    o2 = np.empty((S, ld))
    assert lib.sts_fill_diff_ewma_host(P(x), P(o2), S, T, ld, 3, 1, P(sm), P(err)) == 0, lib.sts_last_error()
    for s in range(0, S, max(1, S // 16)):
        r = oracle.ewma_add(oracle.differences_at_lag(oracle.fill_previous(x[s, :T]), 1), float(sm[s]))
        g = o2[s, :T]
        assert ((g.view(np.uint64) == r.view(np.uint64)) | (np.isnan(g) & np.isnan(r))).all(), (case, s, "c2_host")


@pytest.mark.gpu
@pytest.mark.parametrize("case", range(24 * SCALE))
def test_fuzz_fill_spline(torch, case):
    """fill("spline") (S/UnivariateTimeSeries.scala:268-297, round 6): random shapes, NaN rates with
    long runs, levels and families -- the filled panel bit for bit against the commons-math3
    restatement, the per-series status (NumberIsTooSmallException on < 3 points) identical, and
    every other case through fill + autocorr (the ACF within the tolerance contract)."""
    from sparkts import TimeSeriesRDD, _native
    rng = np.random.default_rng(zlib.crc32(b"fuzz-spline-%d" % case))
    T = int(np.exp(rng.uniform(np.log(2), np.log(40000))))
    S = int(rng.integers(1, 12))
    family = ["walk", "noise", "ar1", "steps"][int(rng.integers(0, 4))]
    level = float(rng.choice([0.0, 100.0, 1e4, 1e6]))
    x = fuzz_panel(rng, S, T, family, level, float(rng.choice([0.0, 0.02, 0.1, 0.4, 0.95])),
                   bool(rng.integers(0, 2)))
    rf, rerr = oracle.panel_fill(x, "spline")
    xd = torch.as_tensor(x, device="cuda:0")
    out = torch.empty_like(xd)
    err = torch.full((S,), -1, dtype=torch.int32, device="cuda:0")
    assert _native.lib().sts_fill(xd.data_ptr(), out.data_ptr(), S, T, T, T, 4, err.data_ptr(), None) == 0
    torch.cuda.synchronize()
    assert np.array_equal(err.cpu().numpy(), rerr), (case, err.cpu().numpy(), rerr)
    f = out.cpu().numpy()
    same = (f.view(np.uint64) == rf.view(np.uint64)) | (np.isnan(f) & np.isnan(rf))
    assert same.all(), (case, T, family, int((~same).sum()))
    if case % 2 == 0 and (rerr == 0).all() and T > 2:
        K = int(rng.integers(1, max(2, min(61, T))))
        filled, acf = TimeSeriesRDD(None, None, xd).fillAndAutocorr("spline", K)
        rf2, racf, err2 = oracle.panel_fill_autocorr(x, "spline", K)
        assert (err2 == 0).all()
        got = acf.cpu().numpy()
        for s in range(S):
            assert within(got[s], racf[s], noise_floor(rf2[s], K)) <= 1.0, (case, s, T, K)
