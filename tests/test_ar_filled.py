"""Autoregression.fitModel on FILLED series -- the README's own pipeline input.

README.md:57-61 fits `ar(series, 1)` after `tsRdd.fill("linear")`; a fill turns a NaN-riddled
price walk into step series (previous / next / nearest: runs of repeated values) or linear
ramps, families the round-5 AR rule calibration (tools/ar_flag_study.py) did not contain, and
test_fuzz_gpu.py fuzzes AR only at nan_p = 0.  Here:

  * CPU: the calibration on these families (`tools/ar_flag_study.py --families filled`, profiles/
    r06_ar_flag_study_filled.json: 1 728 series, 78-90 % of the intercept fits flagged, the
    unflagged ones' reference within 9.0e-12 elementwise of the exact solution) is re-checked on
    fresh seeds: wherever the rule keeps a filled series on the fast path, the reference is within
    2e-11 elementwise of exact, so the fast path (~1e-13 from exact) meets 1e-10 against it;
  * CPU: series built a hair inside each of the rule's three thresholds (ratio 15.9,
    kappa 97-99.5, level 98-99.9) -- unflagged by the host restatement -- and the same margin;
  * GPU: fill (device, bit-exact) -> Autoregression.fitModel / fitModelAndRemove on the device for
    every fill x p in {1, 5, 8} x both intercept modes x levels 1 .. 1e6 x NaN 5 / 20 / 60 % with
    long gaps: c and phi within 1e-10 ELEMENTWISE of the oracle on every row (elements below
    1e-6 of the coefficient vector's norm are skipped: noise-level coefficients, whose relative
    error says nothing -- the same metric as test_ar_price_levels.py), BIT-IDENTICAL on the rows
    the device's rule flags (they take the reference's Householder order), the residuals
    bit-exact given the device's model; rows the reference cannot fit (a fill that leaves a
    constant series: SingularMatrixException) get the same status; a seeded random sweep.
"""
import ctypes
import zlib

import numpy as np
import pytest

import oracle
from test_ar_price_levels import elementwise, exact_ols

ELEM_TOL = 1e-10
FILLS = ["previous", "next", "nearest", "linear"]
NaN = np.nan


def filled_walk(method, level, sigma, T, nan_p, seed):
    """A price walk with NaN at rate nan_p plus three long gaps (50-300 steps), both ends valid,
    after fill(method) -- the oracle's fill, which the device fill equals bit for bit."""
    rng = np.random.default_rng(seed)
    x = level + np.cumsum(rng.standard_normal(T)) * sigma
    x[rng.random(T) < nan_p] = NaN
    for _ in range(3):
        g = int(rng.integers(50, min(300, T // 3)))
        a = int(rng.integers(1, max(2, T - g - 1)))
        x[a:a + g] = NaN
    x[0] = level
    x[-1] = level + sigma
    return x, oracle.fillts(x, method)


def rule_stats(x, p, c):
    """sts_ar.hip kRule*'s three statistics from the host: |mean| / centred lag-column rms (flag at
    >= 16), 1 / the smallest scaled Cholesky pivot^2 (flag at >= 100), |mean| / |c| (>= 100)."""
    n = x.size
    m = n - p
    X = np.column_stack([x[p - 1 - j: n - 1 - j] for j in range(p)])
    G = (X - X.mean(axis=0)).T @ (X - X.mean(axis=0))
    dg = np.diag(G)
    mu = x.mean()
    d = np.sqrt(dg)
    L = np.linalg.cholesky(G / np.outer(d, d))
    return (abs(mu) / np.sqrt(dg.min() / m), 1.0 / np.min(np.diag(L) ** 2),
            abs(mu) / max(abs(c), 1e-300))


def flagged(stats):
    ratio, kappa, lev = stats
    return ratio >= 16.0 or kappa >= 100.0 or lev >= 100.0


# ---------------- CPU: the calibration on the filled families ----------------

@pytest.mark.parametrize("method", FILLS)
def test_rule_bounds_hold_on_filled_series(method):
    rng = np.random.default_rng(zlib.crc32(method.encode()))
    kept = flagged_n = 0
    for case in range(30):
        T = int(rng.choice([390, 1200]))
        p = int(rng.choice([1, 5, 8]))
        level = float(rng.choice([0.0, 1.0, 10.0, 1e2, 1e4]))
        sigma = float(rng.choice([1.0, 1e-2]))
        _, f = filled_walk(method, level, sigma, T, float(rng.choice([0.05, 0.2, 0.6])), 1000 + case)
        ex = exact_ols(f, p)
        if flagged(rule_stats(f, p, ex[0])):
            flagged_n += 1
            continue
        kept += 1
        c, coef = oracle.ar_fit(f, p)
        assert elementwise(np.r_[c, coef], ex) <= 2e-11, (method, case, T, p, level, sigma)
    assert kept + flagged_n == 30


def near_threshold_series():
    """(name, x, p, stats): one series a hair inside each threshold of the AR rule."""
    out = []
    T = 2520
    rng = np.random.default_rng(77)
    # ratio: AR(0.5) noise shifted so |mean| / rms = 15.9 (the statistic is shift-invariant in rms)
    e = rng.standard_normal(T)
    y = np.empty(T)
    y[0] = e[0]
    for t in range(1, T):
        y[t] = 0.5 * y[t - 1] + e[t]
    p = 5
    n, m = T, T - p
    X = np.column_stack([y[p - 1 - j: n - 1 - j] for j in range(p)])
    rms = np.sqrt(np.min(np.sum((X - X.mean(axis=0)) ** 2, axis=0)) / m)
    x = y + (15.9 * rms - y.mean())
    out.append(("ratio", x, p))
    # kappa: a sine whose lag columns are nearly collinear, period bisected to 1 / pivot^2 ~ 98.5;
    # centred, since around any level a near-unit-root fit has |mean| / |c| = 1 / (1 - sum phi)
    # >= 100 there (the level bound would flag it first)
    t = np.arange(T)
    noise = 1e-2 * rng.standard_normal(T)

    def sine(P):
        z = np.sin(2 * np.pi * t / P) + noise
        return z - z.mean()
    lo, hi = 10.0, 200.0
    for _ in range(60):
        P = 0.5 * (lo + hi)
        if rule_stats(sine(P), 2, 1.0)[1] < 98.5:
            lo = P
        else:
            hi = P
    out.append(("kappa", sine(lo), 2))
    # level: AR(1) around a level, phi bisected so |mean| / |c| ~ 99 (ratio kept small)
    e = rng.standard_normal(T)

    def ar1(phi):
        z = np.empty(T)
        z[0] = e[0]
        for i in range(1, T):
            z[i] = phi * z[i - 1] + e[i]
        return 30.0 + z
    lo, hi = 0.9, 0.995
    for _ in range(40):
        phi = 0.5 * (lo + hi)
        x = ar1(phi)
        c = exact_ols(x, 1)[0]
        if rule_stats(x, 1, c)[2] < 99.0:
            lo = phi
        else:
            hi = phi
    out.append(("level", ar1(lo), 1))
    return [(name, x, p, rule_stats(x, p, exact_ols(x, p)[0])) for name, x, p in out]


def test_near_threshold_series_are_inside_the_bound():
    """the margin at each threshold.  Each series sits just inside its threshold (so the
    fast path keeps it) and the reference there is still within 2e-11 elementwise of exact."""
    for name, x, p, st in near_threshold_series():
        assert not flagged(st), (name, st)
        lim = {"ratio": (15.0, 16.0, 0), "kappa": (95.0, 100.0, 1), "level": (95.0, 100.0, 2)}[name]
        assert lim[0] <= st[lim[2]] < lim[1], (name, st)
        c, coef = oracle.ar_fit(x, p)
        assert elementwise(np.r_[c, coef], exact_ols(x, p)) <= 2e-11, (name, st)


# ---------------- GPU ----------------

@pytest.fixture(scope="module")
def torch():
    import torch as _t
    if not _t.cuda.is_available():
        pytest.skip("no GPU")
    from sparkts import _native
    _native.ensure_device(0)
    return _t


def same_bits(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return bool(np.all((a.view(np.uint64) == b.view(np.uint64)) | (np.isnan(a) & np.isnan(b))))


def device_rule_flags(torch, x, p, no_int):
    """Per row: does the device's AR rule send it to the reference-order QR (sts_ar_rule_count)."""
    from sparkts import _native
    out = []
    for r in x:
        t = torch.as_tensor(np.ascontiguousarray(r[None, :]), device="cuda:0")
        n = ctypes.c_int64(-1)
        assert _native.lib().sts_ar_rule_count(t.data_ptr(), 1, r.size, r.size, p, int(no_int), ctypes.addressof(n),
                                               None) == 0
        out.append(n.value == 1)
    return np.array(out)


def filled_panel(method, T, seed0):
    rows, raw = [], []
    for level in (1.0, 1e2, 1e4, 1e6):
        for sigma in (1.0, 1e-2):
            for nan_p in (0.05, 0.2, 0.6):
                r, f = filled_walk(method, level, sigma, T, nan_p,
                                   zlib.crc32(repr((method, T, level, sigma, nan_p, seed0)).encode()))
                raw.append(r)
                rows.append(f)
    return np.stack(raw), np.stack(rows)


@pytest.mark.gpu
@pytest.mark.parametrize("method", FILLS)
@pytest.mark.parametrize("p", [1, 5, 8])
@pytest.mark.parametrize("no_int", [False, True])
def test_gpu_ar_fit_on_filled_series(torch, method, p, no_int):
    from sparkts import UnivariateTimeSeries as uts
    from sparkts.models import Autoregression
    T = 2520 if p != 8 else 1200
    raw, want_f = filled_panel(method, T, p)
    # the pipeline on the device: fill, then the fit on the device-resident filled panel
    f = uts.fillts(torch.as_tensor(raw, device="cuda:0"), method)
    assert same_bits(f.cpu().numpy(), want_f), "device fill"
    m, resid = Autoregression.fitModelAndRemove(f, p, no_int)
    c, coef, res = m.c.cpu().numpy(), m.coefficients.cpu().numpy(), resid.cpu().numpy()
    m2 = Autoregression.fitModel(f, p, no_int)
    assert same_bits(m2.c.cpu().numpy(), c) and same_bits(m2.coefficients.cpu().numpy(), coef)
    flags = device_rule_flags(torch, want_f, p, no_int)
    worst = 0.0
    for s in range(want_f.shape[0]):
        rc, rcoef = oracle.ar_fit(want_f[s], p, no_int)
        got, ref = np.r_[c[s], coef[s]], np.r_[rc, rcoef]
        if no_int:
            got, ref = got[1:], ref[1:]
        if flags[s]:
            assert same_bits(got, ref), ("flagged row not the reference's bits", method, p, s)
        e = elementwise(got, ref)
        worst = max(worst, e)
        assert e <= ELEM_TOL, (method, p, no_int, s, e)
        assert same_bits(res[s], oracle.ar_remove(want_f[s], c[s], coef[s])), ("residuals", s)
    if no_int:
        assert flags.all()


@pytest.mark.gpu
@pytest.mark.parametrize("method", FILLS)
def test_gpu_ar_fit_on_fills_that_leave_flat_series(torch, method):
    """A fill that leaves a constant or two-level series: the reference's QR decides (throws
    SingularMatrixException or returns finite numbers); the device returns the same status, and
    the reference's bits where it fits."""
    from sparkts import _native
    T, p = 400, 2
    rows = []
    x = np.full(T, NaN); x[0] = 3.7; x[-1] = 3.7; rows.append(x)                    # constant after the fill
    x = np.full(T, NaN); x[0] = 100.1; x[200] = 100.1; x[-1] = 100.1; rows.append(x)
    x = np.full(T, NaN); x[0] = 1.0; x[150] = 2.0; x[-1] = 2.0; rows.append(x)      # two levels
    x = np.full(T, NaN); x[0] = 1e6; x[1] = 1e6 + 0.01; x[-1] = 1e6; rows.append(x)
    x = np.full(T, NaN); x[::97] = np.arange(len(x[::97])) * 1.5; x[-1] = 9.0; rows.append(x)
    for raw in rows:
        f = oracle.fillts(raw, method)
        t = torch.as_tensor(np.ascontiguousarray(f[None, :]), device="cuda:0")
        c = torch.empty(1, dtype=torch.float64, device="cuda:0")
        coef = torch.empty((1, p), dtype=torch.float64, device="cuda:0")
        err = torch.full((1,), -1, dtype=torch.int32, device="cuda:0")
        assert _native.lib().sts_ar_fit(t.data_ptr(), 1, T, T, p, 0, c.data_ptr(), coef.data_ptr(), err.data_ptr(),
                                        None) == 0
        try:
            rc, rcoef = oracle.ar_fit(f, p)
        except oracle.OracleError as e:
            assert int(err.item()) == e.code, (method, raw[:3], int(err.item()), e.code)
            continue
        assert int(err.item()) == 0, (method, raw[:3], int(err.item()))
        got, ref = np.r_[c.item(), coef.cpu().numpy()[0]], np.r_[rc, rcoef]
        assert same_bits(got, ref) or elementwise(got, ref) <= ELEM_TOL, (method, got, ref)


@pytest.mark.gpu
def test_gpu_ar_fit_near_rule_thresholds(torch):
    """the series a hair inside each threshold, on the device: <= 1e-10 elementwise
    against the oracle whichever path the device's own statistics choose."""
    from sparkts.models import Autoregression
    for name, x, p, st in near_threshold_series():
        m = Autoregression.fitModel(torch.as_tensor(np.ascontiguousarray(x[None, :]), device="cuda:0"), p)
        got = np.r_[m.c.cpu().numpy()[0], m.coefficients.cpu().numpy()[0]]
        rc, rcoef = oracle.ar_fit(x, p)
        assert elementwise(got, np.r_[rc, rcoef]) <= ELEM_TOL, (name, st)


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(4))
def test_gpu_ar_fit_filled_fuzz(torch, seed):
    """Seeded sweep: random fill, NaN rate, level, spread, length, p and intercept mode."""
    from sparkts import UnivariateTimeSeries as uts
    from sparkts.models import Autoregression
    rng = np.random.default_rng(900 + seed)
    for case in range(6):
        method = FILLS[int(rng.integers(4))]
        T = int(rng.choice([300, 700, 2520, 4000]))
        p = int(rng.choice([1, 2, 3, 5, 8, 12]))
        no_int = bool(rng.integers(2))
        S = 24
        raw = np.stack([filled_walk(method, float(rng.choice([0.0, 1.0, 1e2, 1e4, 1e6])),
                                    float(rng.choice([1.0, 1e-2])), T, float(rng.uniform(0.05, 0.6)),
                                    int(rng.integers(1 << 30)))[0] for _ in range(S)])
        want_f = np.stack([oracle.fillts(r, method) for r in raw])
        f = uts.fillts(torch.as_tensor(raw, device="cuda:0"), method)
        m = Autoregression.fitModel(f, p, no_int)
        c, coef = m.c.cpu().numpy(), m.coefficients.cpu().numpy()
        for s in range(S):
            rc, rcoef = oracle.ar_fit(want_f[s], p, no_int)
            got, ref = np.r_[c[s], coef[s]], np.r_[rc, rcoef]
            if no_int:
                got, ref = got[1:], ref[1:]
            assert elementwise(got, ref) <= ELEM_TOL, (seed, case, method, T, p, no_int, s)


@pytest.mark.gpu
@pytest.mark.parametrize("p", [2, 5, 8])
def test_gpu_ar_fit_around_the_refinement_bound(torch, p):
    """Round 6: the register AR kernel skips its refinement pass when every scaled Cholesky pivot^2
    exceeds 1 / 4 (sts_ar.hip kRefineKappa).  AR(1) series at phi around sqrt(3) / 2 put
    1 / pivot^2 = 1 / (1 - rho^2) on both sides of 4 (the lags of an AR(1) have no partial
    correlation past the first); levels keep the AR rule quiet.  Device vs oracle <= 1e-10
    elementwise on both sides, fit and fused residuals."""
    from sparkts.models import Autoregression
    T = 2520
    rows = []
    for phi in (0.80, 0.85, 0.86, 0.866, 0.87, 0.88, 0.90):
        for seed in range(3):
            rng = np.random.default_rng(seed * 100 + int(phi * 1000))
            e = rng.standard_normal(T)
            y = np.empty(T)
            y[0] = e[0]
            for t in range(1, T):
                y[t] = phi * y[t - 1] + e[t]
            rows.append(10.0 + y)
    x = np.array(rows)
    m, resid = Autoregression.fitModelAndRemove(torch.as_tensor(x, device="cuda:0"), p)
    c, coef, res = m.c.cpu().numpy(), m.coefficients.cpu().numpy(), resid.cpu().numpy()
    kappas = []
    for s in range(x.shape[0]):
        rc, rcoef = oracle.ar_fit(x[s], p)
        assert elementwise(np.r_[c[s], coef[s]], np.r_[rc, rcoef]) <= ELEM_TOL, (p, s)
        assert same_bits(res[s], oracle.ar_remove(x[s], c[s], coef[s])), ("residuals", s)
        kappas.append(rule_stats(x[s], p, rc)[1])
    assert min(kappas) < 4.0 < max(kappas)   # both sides of the bound are exercised
