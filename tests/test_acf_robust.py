"""autocorr on series whose level is far from their spread (VERDICT r1 "What's weak" #1).

The device kernels accumulate one-pass moments of y = x - c and centre at the end
(spark-timeseries_amd/csrc/sts_acf.hpp).  The reference (S/UnivariateTimeSeries.scala:68-93)
centres first, so it is accurate whatever the level; a one-pass form is accurate only when
(mean - c)^2 / sigma^2 stays O(1) and no head/tail outlier is subtracted back out.

CPU tests (no GPU): a numpy emulation of the kernels' finalize on the cases that broke the
round-1 formula (c = x[0], sums as total - head), against the oracle -- the old formula
misses 1e-10 by orders of magnitude on the outlier / far-level rows (0.27 relative at level
1e6 with x[0] = 0), the new one (median shift, middle sums + explicit head / tail) meets it
on every well-conditioned row.  GPU tests: the HIP path (both imputation kernels by length, all four fills,
K in {20, 60}) against the oracle on the same kinds of series, 1e-10 relative, identical NaN
pattern; for the one row whose correlations are themselves at the reference's rounding-noise
level (~1e-10 .. 1e-6, variance dominated by two outliers) the bar is 1e-10 relative plus that
noise level (noise_floor).
"""
import numpy as np
import pytest

import oracle

RTOL = 1e-10
EDGE = 64    # kAcfEdge


def ar1(rng, T, phi=0.99):
    """Stationary AR(1) noise with unit innovations: well-conditioned correlations (phi^i)."""
    return oracle.ar_add(rng.standard_normal(T), 0.0, [phi])


def hard_rows(T, seed):
    """Series whose level is far from x[0] or from their own spread."""
    rng = np.random.default_rng(seed)
    rows = []
    r = 100.0 + 1e-3 * ar1(rng, T); r[0] = 0.0; rows.append(r)              # x[0] outlier
    rows.append(1e4 + 1.0 * ar1(rng, T))                                     # level 1e4, sigma 1
    rows.append(1e4 + 1e-2 * ar1(rng, T))                                    # level 1e4, sigma 1e-2
    r = 1e-2 * ar1(rng, T); r[T // 3:] += 100.0; rows.append(r)              # step change
    r = 1e6 + 1e-2 * ar1(rng, T); r[0] = 0.0; rows.append(r)                 # level 1e6, x[0] = 0
    rows.append(1e4 + np.cumsum(1e-2 * rng.standard_normal(T)))              # random walk at 1e4
    r = 100.0 + 1e-3 * ar1(rng, T); r[-1] = 0.0; rows.append(r)              # tail outlier
    r = 100.0 + 1e-3 * ar1(rng, T); r[3] = 95.0; r[T - 5] = 107.0; rows.append(r)   # outliers inside both edges
    # outliers that dominate the variance: the correlations are ~1e-10 .. 1e-6, i.e. at the
    # level of the reference's own rounding noise (see noise_floor)
    r = 100.0 + 1e-3 * ar1(rng, T); r[3] = -5e3; r[T - 5] = 7e3; rows.append(r)
    return np.array(rows)


def noise_floor(x, K):
    """Per-lag rounding-noise level of the reference's own result: 64 eps sqrt(N) *
    sum|d1 d2| / sqrt(v1 v2) (S/UnivariateTimeSeries.scala:80-89, centred sums of N terms).
    Where |acf| is far above it (every well-conditioned lag) the parity check below is the
    plain 1e-10 relative bar; it only matters for correlations that are themselves a
    cancellation of much larger terms."""
    x = np.asarray(x, dtype=np.float64)
    T = x.size
    out = np.zeros(K)
    for i in range(1, K + 1):
        if i >= T:
            continue
        a, b = x[i:], x[:T - i]
        d1, d2 = a - a.mean(), b - b.mean()
        den = np.sqrt((d1 * d1).sum()) * np.sqrt((d2 * d2).sum())
        out[i - 1] = 64 * np.finfo(float).eps * np.sqrt(T - i) * np.abs(d1 * d2).sum() / den if den > 0 else 0.0
    return out


def within(got, ref, floor, rtol=RTOL):
    """|got - ref| <= rtol |ref| + floor, identical NaN pattern; returns the worst ratio."""
    got, ref = np.asarray(got), np.asarray(ref)
    assert np.array_equal(np.isnan(got), np.isnan(ref)), "NaN pattern differs"
    fin = ~np.isnan(ref)
    if not fin.any():
        return 0.0
    diff = np.abs(got[fin] - ref[fin])
    den = rtol * np.abs(ref[fin]) + floor[fin]
    # an exact match passes whatever the bound (ref = 0 with a zero floor: a constant slice whose
    # numpy mean is exact while the reference's left-to-right mean is not)
    with np.errstate(divide="ignore", invalid="ignore"):
        return float(np.where(diff == 0.0, 0.0, diff / den).max())


def with_nans(x, rng, p=0.05):
    x = x.copy()
    m = rng.random(x.shape) < p
    m[:, :2] = False       # x[0] and x[1] valid: every fill leaves a finite series (nearest: index 0 quirk)
    m[:, -1] = False
    x[m] = np.nan
    return x


def rel_err(got, ref):
    got, ref = np.asarray(got), np.asarray(ref)
    assert np.array_equal(np.isnan(got), np.isnan(ref)), "NaN pattern differs"
    fin = ~np.isnan(ref)
    return float((np.abs(got[fin] - ref[fin]) / np.abs(ref[fin])).max()) if fin.any() else 0.0


# ---------------- CPU: the finalize algebra, emulated in numpy ----------------

def lag_products(y, K):
    T = y.size
    return np.array([np.dot(y[:T - i], y[i:]) for i in range(K + 1)])


def acf_round1(x, K):
    """Round-1 finalize: c = x[0], slice sums as total minus head / tail."""
    T = x.size
    y = x - x[0]
    P = lag_products(y, K)
    Sy, P0 = y.sum(), P[0]
    out = []
    for i in range(1, K + 1):
        N = T - i
        s1, s2 = Sy - y[:i].sum(), Sy - y[T - i:].sum()
        q1, q2 = P0 - (y[:i] ** 2).sum(), P0 - (y[T - i:] ** 2).sum()
        v1, v2, cv = q1 - s1 * s1 / N, q2 - s2 * s2 / N, P[i] - s1 * s2 / N
        out.append(cv / (np.sqrt(v1) * np.sqrt(v2)))
    return np.array(out)


def robust_shift(x, prev=False):
    """sts_acf.hpp robust_shift (round 3): lane l owns [l T / 64, (l + 1) T / 64) and samples its
    first valid step; a lane whose range has none takes the next sampled lane's value (F(t) of
    fillNext), else the last one before it -- under fillPrevious (prev) the last one before it,
    else the next; c = the lower median of the 64 samples."""
    T = x.size
    samp = [None] * 64
    for lane in range(64):
        seg = x[lane * T // 64:(lane + 1) * T // 64]
        ok = np.flatnonzero(~np.isnan(seg))
        if ok.size:
            samp[lane] = seg[ok[0]]
    have = [l for l in range(64) if samp[l] is not None]
    if not have:
        return 0.0
    vals = []
    for lane in range(64):
        if samp[lane] is None:
            above = [h for h in have if h > lane]
            below = [h for h in have if h < lane]
            if prev:
                src = below[-1] if below else above[0]
            else:
                src = above[0] if above else below[-1]
        else:
            src = lane
        vals.append(samp[src])
    return sorted(vals)[31]


def robust_shift_r2(x, seg=False):
    """The round-2 shift, kept to show what it missed: the lower median of the VALID RAW samples
    x[l T / 64] (or the step after; tile kernel) or x[128 (l & 3) + 2 l] (or +1) of the first
    512-step tile (segment kernel); 0.0 when no sample is valid."""
    T = x.size
    vals = []
    for lane in range(64):
        t = 128 * (lane & 3) + 2 * lane if seg else lane * T // 64
        v = x[t] if t < T else np.nan
        if np.isnan(v) and t + 1 < T:
            v = x[t + 1]
        if not np.isnan(v):
            vals.append(v)
    return 0.0 if not vals else sorted(vals)[(len(vals) - 1) // 2]


def acf_robust(x, K, c=None):
    """sts_acf.hpp acf_combine: median shift, middle sums, explicit head / tail per lag.  x is
    the series the lag products run over (the FILLED one); c defaults to its robust shift."""
    T = x.size
    if c is None:
        c = robust_shift(x)
    y = x - c
    P = lag_products(y, K)
    mid = y[EDGE:T - EDGE]
    Sm, Qm = mid.sum(), (mid * mid).sum()
    out = []
    for i in range(1, K + 1):
        s1 = Sm + y[i:EDGE].sum() + y[T - EDGE:].sum()
        q1 = Qm + (y[i:EDGE] ** 2).sum() + (y[T - EDGE:] ** 2).sum()
        s2 = Sm + y[:EDGE].sum() + y[T - EDGE:T - i].sum()
        q2 = Qm + (y[:EDGE] ** 2).sum() + (y[T - EDGE:T - i] ** 2).sum()
        N = T - i
        v1, v2, cv = q1 - s1 * s1 / N, q2 - s2 * s2 / N, P[i] - s1 * s2 / N
        out.append(cv / (np.sqrt(v1) * np.sqrt(v2)))
    return np.array(out)


EPS = np.finfo(float).eps


def acf_suspect(r, s1, q1, s2, q2, v1, v2, N, c):
    """sts_acf.hpp acf_suspect (rule 3), statement for statement: may the one-pass value r
    differ from the reference's two-pass result by more than the tolerance?"""
    if not np.isfinite([s1, q1, s2, q2]).all():
        return False
    if not (v1 > 0.0 and v2 > 0.0) or not np.isfinite(r):
        return True
    R1, R2, ar, rn = q1 / v1, q2 / v2, abs(r), np.sqrt(N)
    G = max(rn * 0.125, 16.0)
    e_ours = EPS * G * (np.sqrt(R1 * R2) + ar * 0.5 * (R1 + R2))
    d1 = 2.0 ** -55 * N * (abs(c) + np.sqrt(q1 / N))
    d2 = 2.0 ** -55 * N * (abs(c) + np.sqrt(q2 / N))
    e_ref = N * d1 * d2 / np.sqrt(v1 * v2) + ar * 0.5 * (N * d1 * d1 / v1 + N * d2 * d2 / v2)
    return e_ours + e_ref > max(1e-11 * ar, EPS * rn)


def suspect_lags(x, K, c=None):
    """Rule 3's verdict per lag on the emulated one-pass sums of acf_robust."""
    T = x.size
    if c is None:
        c = robust_shift(x)
    y = x - c
    P = lag_products(y, K)
    mid = y[EDGE:T - EDGE]
    Sm, Qm = mid.sum(), (mid * mid).sum()
    out = []
    with np.errstate(all="ignore"):
        for i in range(1, K + 1):
            s1 = Sm + y[i:EDGE].sum() + y[T - EDGE:].sum()
            q1 = Qm + (y[i:EDGE] ** 2).sum() + (y[T - EDGE:] ** 2).sum()
            s2 = Sm + y[:EDGE].sum() + y[T - EDGE:T - i].sum()
            q2 = Qm + (y[:EDGE] ** 2).sum() + (y[T - EDGE:T - i] ** 2).sum()
            N = T - i
            v1, v2, cv = q1 - s1 * s1 / N, q2 - s2 * s2 / N, P[i] - s1 * s2 / N
            out.append(acf_suspect(cv / (np.sqrt(v1) * np.sqrt(v2)), s1, q1, s2, q2, v1, v2, N, c))
    return np.array(out)


def ill_rows(T, seed):
    """(raw row, note) -- the round-3 verdict's ill-conditioned autocorr inputs: constants at
    non-dyadic levels (the reference returns 1.0 from its rounded means, not 0/0), a dyadic
    constant (NaN both ways), constant-but-one-end series (the reference's values are tiny and
    deterministic), and a spike train on the 64 positions the shift samples (moves the median
    shift off the bulk of the series)."""
    rng = np.random.default_rng(seed)
    rows = [np.full(T, 100.1), np.full(T, 1234.567), np.full(T, 5.0)]
    r = np.full(T, 100.1); r[-1] = 100.2; rows.append(r)
    r = np.full(T, 100.1); r[0] = 100.2; rows.append(r)
    r = 100.0 + 1e-3 * ar1(rng, T); r[np.arange(64) * T // 64] += 1e4; rows.append(r)
    r = np.full(T, np.nan); r[0] = 100.1; r[-1] = 100.2; rows.append(r)   # x0, NaN .. T-2, x_{T-1}
    r = 1e4 + 1e-2 * ar1(rng, T); r[200:T - 3] = np.nan; r[T - 3:] += 50.0; rows.append(r)
    return np.array(rows)


def nan_heavy_rows(T, seed):
    """(raw row, fill method) pairs whose RAW samples say little about the FILLED series (VERDICT
    r2 "What's weak" #1): long leading NaN runs under fillNext, an outlier x[0] followed by 511
    NaNs under fillNearest, a 98 %-NaN row under fillLinear, a long trailing run under
    fillPrevious.  Levels far from the spread, so a bad shift shows."""
    rng = np.random.default_rng(seed)
    rows = []
    for run in (600, 5000):
        if run < T - 600:
            r = 1e4 + 1e-2 * ar1(rng, T); r[:run] = np.nan; rows.append((r, "next"))
            r = 100.0 + 1e-3 * ar1(rng, T); r[:run] = np.nan; rows.append((r, "next"))
            r = 1e4 + 1e-2 * ar1(rng, T); r[T - run:] = np.nan; rows.append((r, "previous"))
            r = 1e4 + 1e-2 * ar1(rng, T); r[1:run] = np.nan; rows.append((r, "linear"))
    # (not at the C3 length, where that near-constant filled series is ill-conditioned in the
    # relative sense whatever the shift: 1.8e-6 with it, 3e-2 without)
    # an interior run under fillPrevious followed by a level change: the run holds the value
    # before it, so a shift taken from after the change sits far from the filled bulk
    r = 1e4 + 1e-2 * ar1(rng, T)
    r[200:T - 3] = np.nan
    r[T - 3:] += 50.0
    rows.append((r, "previous"))
    r = 100.0 + 1e-3 * ar1(rng, T); r[0] = 0.0; r[1:512] = np.nan; rows.append((r, "nearest"))
    r = 1e4 + 1e-2 * ar1(rng, T); r[1:512] = np.nan; rows.append((r, "nearest"))
    r = 1e4 + 1e-2 * ar1(rng, T)
    m = rng.random(T) < 0.98
    m[0] = m[-1] = False
    r[m] = np.nan
    for meth in ("linear", "next", "nearest", "previous"):
        rows.append((r, meth))
    # 99.5 % NaN, x[0] among them, and NaN at every step the round-2 tile kernel sampled (l T / 64
    # and the step after): it then had no valid sample and used c = 0
    r = 1e4 + 1e-2 * ar1(rng, T)
    m = rng.random(T) < 0.995
    t = np.arange(64) * T // 64
    m[t] = True
    m[np.minimum(t + 1, T - 1)] = True
    m[-1] = False
    r[m] = np.nan
    rows.append((r, "next"))
    return rows


@pytest.mark.parametrize("T", [2520, 16384 + 77])
def test_round1_formula_fails_and_robust_formula_holds(T):
    K = 60
    x = hard_rows(T, T)
    worst_old, worst_new = [], []
    for r in x[:-1]:
        ref = oracle.autocorr(r, K)
        worst_old.append(rel_err(acf_round1(r, K), ref))
        worst_new.append(rel_err(acf_robust(r, K), ref))
    # the cases are discriminating: the round-1 finalize misses 1e-10 on the outlier and
    # far-level rows ...
    assert max(worst_old[0], worst_old[2], worst_old[4]) > 1e-8, worst_old
    # ... and the robust finalize meets it on every row
    assert max(worst_new) <= RTOL, worst_new


def test_robust_shift_is_the_median_of_valid_samples():
    x = np.arange(1000.0)
    x[::7] = np.nan
    s = robust_shift(x)
    assert not np.isnan(s) and abs(s - 500) < 20
    assert robust_shift(np.full(100, np.nan)) == 0.0
    y = np.full(500, 3.0); y[0] = -1e9
    assert robust_shift(y) == 3.0
    # a NaN-only range takes the next sampled value (F(t) of fillNext), a trailing one the last
    z = np.full(6400, np.nan); z[5000] = 7.0; z[6000:] = 9.0
    assert robust_shift(z) == 7.0          # 50 lanes -> 7 (lanes 0..50 up to z[5000]), 13 -> 9
    z = np.full(6400, np.nan); z[10] = -3.0
    assert robust_shift(z) == -3.0         # one valid step stands for the whole series
    # fillPrevious fills a run with the value BEFORE it: the run's lanes take the lane before
    z = np.full(6400, np.nan); z[10] = 7.0; z[5000:] = 9.0
    assert robust_shift(z) == 9.0 and robust_shift(z, prev=True) == 7.0


@pytest.mark.parametrize("T", [2520, 16384 + 77, 982_800])
def test_round2_shift_fails_and_filled_shift_holds_on_nan_heavy_rows(T):
    """The round-2 shift from raw samples (0.0 when none is valid, x[0] when only it is) misses
    1e-10 by orders of magnitude on the nan_heavy_rows; the round-3 shift meets it on all."""
    K = 60
    rows = nan_heavy_rows(T, T + 1) if T < 100_000 else nan_heavy_rows(T, T + 1)[-5:]
    worst_old, worst_new = [], []
    for raw, meth in rows:
        F = oracle.fillts(raw, meth)
        ref = oracle.autocorr(F, K)
        assert not np.isnan(ref).all(), meth
        kernels = (True, False) if T < 100_000 else (False,)   # segment / tile kernel's round-2 shift
        worst_old.append(max(rel_err(acf_robust(F, K, robust_shift_r2(raw, seg)), ref) for seg in kernels))
        worst_new.append(rel_err(acf_robust(F, K, robust_shift(raw, meth == "previous")), ref))
    assert max(worst_old) > 1e-7, worst_old
    assert max(worst_new) <= RTOL, worst_new


@pytest.mark.parametrize("T", [2520, 16384 + 77, 982_800])
def test_rule3_flags_the_ill_conditioned_rows(T):
    """sts_acf.hpp rule 3 on the verdict's rows: every row whose one-pass value misses the
    reference (NaN for its 1.0, NaN for its tiny constant-but-one-end values, the spike train's
    1e-9 .. 1e-7 relative error at T >= 2e5) is flagged; a row it leaves alone meets 1e-10."""
    K = 60
    np.seterr(invalid="ignore", divide="ignore")
    for j, raw in enumerate(ill_rows(T, T)):
        F = oracle.fillts(raw, "previous") if np.isnan(raw).any() else raw
        ref = oracle.autocorr(F, K)
        c = robust_shift(raw, prev=True)
        flagged = suspect_lags(F, K, c).any()
        if not flagged:
            e = rel_err(acf_robust(F, K, c), ref)
            assert e <= RTOL, (j, T, e)
        if j in (0, 1, 3, 4, 6):      # constants and constant-but-one-end: one-pass gives NaN
            assert flagged, (j, T)
            assert not np.isnan(ref).any() and np.isnan(acf_robust(F, K, c)).any(), j
        if j == 2:                    # dyadic constant: NaN both ways (the exact path keeps it)
            assert np.isnan(ref).all()
        if j == 5 and T > 10_000:     # the spike train: flagged where one-pass loses digits
            assert flagged


@pytest.mark.parametrize("T", [2520, 982_800])
def test_rule3_is_quiet_on_well_conditioned_panels(T):
    """No lag of the bench generator's panels (filled linear: trend + noise at level ~100),
    random walks, white noise or the far-level rows is flagged: the one-pass path stands and
    the bench does not pay for rule 3."""
    K = 60
    rng = np.random.default_rng(T + 5)
    x = oracle.gen_panel(11, 3, T, 0.05)
    rows = [oracle.fillts(r, "linear") for r in x]
    rows.append(100.0 + rng.standard_normal(T).cumsum() * 0.1 + rng.random(T))
    rows.append(rng.standard_normal(T))
    rows.append(1e4 + 1.0 * ar1(rng, T))
    for r in rows:
        assert not suspect_lags(r, K).any()


# ---------------- GPU: the HIP path ----------------

@pytest.fixture(scope="module")
def torch():
    import torch as _t
    if not _t.cuda.is_available():
        pytest.skip("no GPU")
    from sparkts import _native
    _native.ensure_device(0)
    return _t


def run_fill_acf(torch, x, method, K):
    from sparkts import _native
    from sparkts import UnivariateTimeSeries as uts
    S, T = x.shape
    xd = torch.as_tensor(np.ascontiguousarray(x), device="cuda:0")
    acf = torch.empty((S, K), dtype=torch.float64, device="cuda:0")
    if method is None:
        st = _native.lib().sts_autocorr(xd.data_ptr(), S, T, T, K, acf.data_ptr(), None)
        filled = None
    else:
        filled = torch.empty_like(xd)
        st = _native.lib().sts_fill_autocorr(xd.data_ptr(), filled.data_ptr(), S, T, T, T,
                                             uts.fill_method_code(method), K, acf.data_ptr(), None, None)
    assert st == 0, _native.lib().sts_last_error()
    torch.cuda.synchronize()
    return (None if filled is None else filled.cpu().numpy()), acf.cpu().numpy()


@pytest.mark.gpu
@pytest.mark.parametrize("T", [2520, 16384 + 77, 982_800])
@pytest.mark.parametrize("K", [20, 60])
@pytest.mark.parametrize("method", ["linear", "previous", "next", "nearest", None])
def test_gpu_autocorr_far_level_series(torch, T, K, method):
    # T = 2520 runs the segment kernel (fused finalize), the others the tile kernel (chunk
    # partials + acf_finalize_kernel); method None is sts_autocorr on the raw panel
    rng = np.random.default_rng(T * 7 + K)
    x = hard_rows(T, T + K)
    if method is not None:
        x = with_nans(x, rng)
    filled, got = run_fill_acf(torch, x, method, K)
    if method is None:
        ref = np.array([oracle.autocorr(r, K) for r in x])
    else:
        rf, ref, err = oracle.panel_fill_autocorr(x, method, K, threads=4)
        assert (err == 0).all()
        assert np.array_equal(filled.view(np.uint64), rf.view(np.uint64)), "fill not bit-exact"
    src = x if method is None else rf
    floor = np.array([noise_floor(r, K) for r in src])
    e = within(got, ref, floor)
    assert e <= 1.0, "error %.3g x (1e-10 rel + noise floor) (T=%d K=%d %s); plain rel err %g" % (
        e, T, K, method, rel_err(got, ref))
    # every row but the last (variance dominated by two outliers) is well conditioned: the
    # plain 1e-10 relative bar holds there
    assert rel_err(got[:-1], ref[:-1]) <= RTOL


@pytest.mark.gpu
@pytest.mark.parametrize("T", [2520, 16384 + 77, 982_800])
@pytest.mark.parametrize("K", [20, 60])
@pytest.mark.parametrize("kernel", ["product", "seg", "tile"])
def test_gpu_autocorr_nan_heavy_series(torch, request, T, K, kernel):
    """the ACF shift must stand for the FILLED series -- fillNext over
    leading NaN runs of 600 / 5 000, fillNearest with an outlier x[0] before 511 NaNs, 98 % /
    99.5 %-NaN rows at the C3 length -- on both imputation kernels (forced through the A/B
    build) and the product dispatch: 1e-10 relative, identical NaN pattern."""
    if kernel != "product":   # the product library picks by length (short / seg for T <= 16 384)
        request.getfixturevalue("ab_lib")(STS_TILE_KERNEL=kernel, STS_NO_SHORT="1")
    rows = nan_heavy_rows(T, 7 * T + K)
    if T > 100_000:
        rows = rows[-5:]
    by_method = {}
    for raw, meth in rows:
        by_method.setdefault(meth, []).append(raw)
    for meth, rs in sorted(by_method.items()):
        x = np.array(rs)
        filled, got = run_fill_acf(torch, x, meth, K)
        rf, ref, err = oracle.panel_fill_autocorr(x, meth, K, threads=4)
        assert (err == 0).all()
        assert np.array_equal(filled.view(np.uint64), rf.view(np.uint64)), "fill not bit-exact"
        assert not np.isnan(ref).all()
        e = rel_err(got, ref)
        assert e <= RTOL, "rel err %.3g (T=%d K=%d %s %s)" % (e, T, K, meth, kernel)


_ILL_REF = {}


def _ill_ref(T, K, method, x):
    key = (T, K, method)
    if key not in _ILL_REF:
        if method is None:
            _ILL_REF[key] = (None, np.array([oracle.autocorr(r, K) for r in x]))
        else:
            rf, ref, err = oracle.panel_fill_autocorr(x, method, K, threads=8)
            assert (err == 0).all()
            _ILL_REF[key] = (rf, ref)
    return _ILL_REF[key]


@pytest.mark.gpu
@pytest.mark.parametrize("T", [2520, 16384 + 77, 982_800])
@pytest.mark.parametrize("K", [20, 60, 100])
@pytest.mark.parametrize("kernel", ["product", "seg", "tile"])
def test_gpu_autocorr_ill_conditioned(torch, request, T, K, kernel):
    """non-dyadic constants (the reference's 1.0), a dyadic constant (NaN),
    constant-but-one-end rows (the reference's tiny deterministic values), the spike train on the
    shift's 64 sample positions and the interior fillPrevious run before a level change, through
    every ACF path -- the short-series kernel (product, T = 2 520, K = 20 with a fill), the
    segment kernel, the tile kernel + acf_finalize_kernel, the wide path (K = 100) -- and all four
    fills plus the raw panel: identical NaN pattern and 1e-10 relative to the oracle, no noise
    floor, no masked rows (sts_acf.hpp rule 3)."""
    if kernel != "product":
        if K > 63 or (kernel == "seg" and T > 100_000):
            pytest.skip("the wide path and the multi-segment finalize run on the product dispatch only")
        request.getfixturevalue("ab_lib")(STS_TILE_KERNEL=kernel, STS_NO_SHORT="1")
    if K > 63 and T > 100_000:
        pytest.skip("K = 100 at the C3 length: covered by tests/test_acf_wide.py's far-level rows")
    x = ill_rows(T, T)
    methods = ["linear", "previous", "next", "nearest", None] if T < 100_000 else ["previous", None]
    for method in methods:
        xs = x if method is not None else x[~np.isnan(x).any(axis=1)]
        filled, got = run_fill_acf(torch, xs, method, K)
        rf, ref = _ill_ref(T, K, method, xs)
        if method is not None:
            assert np.array_equal(filled.view(np.uint64), rf.view(np.uint64)), "fill not bit-exact"
        e = rel_err(got, ref)
        assert e <= RTOL, "rel err %.3g (T=%d K=%d %s %s)" % (e, T, K, method, kernel)


def returns_rows(T, seed):
    """White noise and differenced random walks (returns): every correlation is O(1 / sqrt(T))
    and some lags land near 0 -- below the reference's own rounding noise."""
    rng = np.random.default_rng(seed)
    walk = 100.0 + np.cumsum(rng.standard_normal(T + 1) * 0.01)
    return np.array([rng.standard_normal(T), 1e-3 * rng.standard_normal(T) + 5e-4,
                     np.diff(walk), np.diff(np.log(np.abs(walk)))])


@pytest.mark.gpu
@pytest.mark.parametrize("T,K", [(2520, 20), (16384 + 77, 60), (982_800, 60)])
@pytest.mark.parametrize("method", ["linear", None])
def test_gpu_autocorr_returns_tolerance_contract(torch, T, K, method):
    """rule 3 does not flag a lag whose one-pass error is below the
    reference's own rounding noise (eps sqrt(N), sts_acf.hpp acf_suspect), so on returns-like
    rows -- white noise, differenced random walks, log returns -- the contract is explicit:
    |acf - ref| <= 1e-10 |ref| + noise_floor(lag) (64 eps sqrt(N) sum|d1 d2| / sqrt(v1 v2), the
    reference's own rounding level); every lag with |ref| above 100x that floor meets the plain
    1e-10 relative bar.  T = 2 520 / K = 20 runs the short kernel (fill linear), 16 461 the
    segment kernel, 982 800 the tile kernel."""
    x = returns_rows(T, T + K)
    if method is not None:
        x = with_nans(x, np.random.default_rng(T))
    filled, got = run_fill_acf(torch, x, method, K)
    if method is None:
        src, ref = x, np.array([oracle.autocorr(r, K) for r in x])
    else:
        src, ref, err = oracle.panel_fill_autocorr(x, method, K, threads=8)
        assert (err == 0).all()
        assert np.array_equal(filled.view(np.uint64), src.view(np.uint64)), "fill not bit-exact"
    floor = np.array([noise_floor(r, K) for r in src])
    e = within(got, ref, floor)
    assert e <= 1.0, "error %.3g x (1e-10 rel + noise floor)" % e
    big = np.abs(ref) > 100.0 * floor
    assert big.mean() > 0.5
    assert rel_err(got[big], ref[big]) <= RTOL, rel_err(got[big], ref[big])


@pytest.mark.gpu
@pytest.mark.parametrize("T,K", [(300, 20), (2520, 20), (2520, 24), (5000, 60), (16384 + 77, 60), (70_001, 63),
                                 (70_001, 1), (5000, 100), (70_001, 130), (982_800, 60)])
def test_gpu_rule3_fallback_is_the_reference_bits(torch, T, K):
    """Round 6: rule 3's fallback streams the series through LDS (sts_acf.hpp acf_exact_stream:
    the short kernel's block, the segment kernel's ring, acf_exact_kernel after the tile and wide
    finalizes).  On rows where it fires for the whole series -- non-dyadic constants with NaN
    gaps, constant-but-one-end rows -- every lag is the reference's two-pass loop, so the result
    must be the oracle's BITS (not merely 1e-10), across chunk boundaries (T = 70 001: 68 full
    1 024-step chunks plus a masked tail), lag blocks (K = 100, 130: two and three 64-lag waves)
    and every kernel the product dispatch picks."""
    rng = np.random.default_rng(T + K)
    rows = []
    for c in (100.1, 1234.567, -0.3):
        r = np.full(T, c)
        r[rng.random(T) < 0.05] = np.nan
        r[0] = c
        r[-1] = c
        rows.append(r)
    r = np.full(T, 7.7)
    r[-1] = 7.7 + 1e-9
    rows.append(r)
    x = np.array(rows)
    filled, got = run_fill_acf(torch, x, "linear", K)
    rf, ref, err = oracle.panel_fill_autocorr(x, "linear", K, threads=4)
    assert (err == 0).all()
    assert np.array_equal(filled.view(np.uint64), rf.view(np.uint64)), "fill not bit-exact"
    same = (got.view(np.uint64) == ref.view(np.uint64)) | (np.isnan(got) & np.isnan(ref))
    assert same.all(), "T=%d K=%d: %d lags differ from the reference's bits, first %s: %r vs %r" % (
        T, K, (~same).sum(), np.argwhere(~same)[0], got[~same][0], ref[~same][0])
