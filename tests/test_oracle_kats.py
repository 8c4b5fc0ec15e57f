"""Pin the CPU oracle against the reference's own known-answer tests.

Each test mirrors a reference ScalaTest case (T/ = /root/reference/src/test/
scala/com/cloudera/sparkts/).  Exact KATs are checked bit for bit; statistical
ones with the reference's own tolerances on inputs regenerated with the
commons-math3 MersenneTwister restatement (oracle/mt19937.py).
"""
import math

import numpy as np
import pytest

import oracle
from mt19937 import MersenneTwister

NaN = float("nan")


def same(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    return a.shape == b.shape and np.array_equal(a.view(np.uint64), b.view(np.uint64))


# ---- T/FillSuite.scala:35-61 (exact) ----

def test_fill_previous_kat():  # T/FillSuite.scala:35-42
    assert same(oracle.fill_previous([1.0]), [1.0])
    assert same(oracle.fill_previous([1.0, 1.0, 2.0]), [1.0, 1.0, 2.0])
    assert same(oracle.fill_previous([1.0, NaN, 2.0]), [1.0, 1.0, 2.0])
    assert same(oracle.fill_previous([1.0, NaN, NaN, 2.0]), [1.0, 1.0, 1.0, 2.0])
    assert same(oracle.fill_previous([1.0, NaN, NaN, NaN, 2.0]), [1.0, 1.0, 1.0, 1.0, 2.0])
    assert same(oracle.fill_previous([1.0, NaN, 3.0, NaN, 2.0]), [1.0, 1.0, 3.0, 3.0, 2.0])


def test_fill_next_kat():  # T/FillSuite.scala:44-51
    assert same(oracle.fill_next([1.0]), [1.0])
    assert same(oracle.fill_next([1.0, 1.0, 2.0]), [1.0, 1.0, 2.0])
    assert same(oracle.fill_next([1.0, NaN, 2.0]), [1.0, 2.0, 2.0])
    assert same(oracle.fill_next([1.0, NaN, NaN, 2.0]), [1.0, 2.0, 2.0, 2.0])
    assert same(oracle.fill_next([1.0, NaN, NaN, NaN, 2.0]), [1.0, 2.0, 2.0, 2.0, 2.0])
    assert same(oracle.fill_next([1.0, NaN, 3.0, NaN, 2.0]), [1.0, 3.0, 3.0, 2.0, 2.0])


def test_fill_linear_kat():  # T/FillSuite.scala:53-61
    assert same(oracle.fill_linear([1.0]), [1.0])
    assert same(oracle.fill_linear([1.0, 1.0, 2.0]), [1.0, 1.0, 2.0])
    assert same(oracle.fill_linear([1.0, NaN, 2.0]), [1.0, 1.5, 2.0])
    assert same(oracle.fill_linear([2.0, NaN, 1.0]), [2.0, 1.5, 1.0])
    assert same(oracle.fill_linear([1.0, NaN, NaN, 4.0]), [1.0, 2.0, 3.0, 4.0])
    assert same(oracle.fill_linear([1.0, NaN, NaN, NaN, 5.0]), [1.0, 2.0, 3.0, 4.0, 5.0])
    assert same(oracle.fill_linear([1.0, NaN, 3.0, NaN, 2.0]), [1.0, 2.0, 3.0, 2.5, 2.0])


def test_fill_nearest_follows_code_not_ignored_suite():
    # T/FillSuite.scala:25-33 is `ignore`d because S/UnivariateTimeSeries.scala:156-184
    # does not satisfy it; the oracle restates the CODE.
    assert same(oracle.fill_nearest([1.0]), [1.0])
    assert same(oracle.fill_nearest([1.0, NaN, 2.0]), [1.0, 2.0, 2.0])  # tie -> next
    assert same(oracle.fill_nearest([1.0, NaN, NaN, NaN, 2.0]), [1.0, 2.0, 2.0, 2.0, 2.0])
    # index 0 is never a "previous" source, so [1, NaN, NaN, 3, NaN, NaN, NaN, 9]:
    assert same(oracle.fill_nearest([1.0, NaN, NaN, 3.0, NaN, NaN, NaN, 9.0]),
                [1.0, 3.0, 3.0, 3.0, 3.0, 9.0, 9.0, 9.0])
    # a genuine previous source at i >= 1 wins when strictly closer
    assert same(oracle.fill_nearest([0.0, 5.0, NaN, NaN, NaN, NaN, 7.0]),
                [0.0, 5.0, 5.0, 5.0, 7.0, 7.0, 7.0])
    assert same(oracle.fill_nearest([NaN, 4.0, NaN]), [NaN, 4.0, 4.0])
    with pytest.raises(oracle.OracleError, match="Input is all NaNs!"):
        oracle.fill_nearest([5.0, NaN])
    with pytest.raises(oracle.OracleError):
        oracle.fill_nearest([NaN, NaN, NaN])
    assert same(oracle.fill_nearest([NaN]), [NaN])


def test_fillts_dispatch():  # S/UnivariateTimeSeries.scala:141-150
    with pytest.raises(oracle.OracleError):
        oracle.fillts([1.0, NaN], "cubic")
    assert same(oracle.fillts([1.0, NaN, 3.0], "linear"), [1.0, 2.0, 3.0])


def test_fill_linear_is_sequential_accumulation():
    # SURVEY.md hard part: r[j] = r[j-1] + inc, not before + k*inc.
    a, b = 26.872848822480243, 169.48674738744654
    x = np.array([a] + [NaN] * 9 + [b])
    got = oracle.fill_linear(x)
    inc = (b - a) / 10
    seq = [a]
    for _ in range(9):
        seq.append(seq[-1] + inc)
    assert same(got[:10], seq)
    direct = [a + k * inc for k in range(10)]
    assert not same(got[:10], direct)  # the two orders really differ here


def test_fill_linear_edges_stay_nan():
    assert same(oracle.fill_linear([NaN, NaN, 2.0, NaN, 4.0, NaN]), [NaN, NaN, 2.0, 3.0, 4.0, NaN])
    assert same(oracle.fill_linear([]), [])


# ---- T/UnivariateTimeSeriesSuite.scala ----

def test_lag_matrices_kat():  # :31-39
    assert same(oracle.lag([1.0, 2.0, 3.0, 4.0, 5.0], 2, True),
                [[3.0, 2.0, 1.0], [4.0, 3.0, 2.0], [5.0, 4.0, 3.0]])
    assert same(oracle.lag([1.0, 2.0, 3.0, 4.0, 5.0], 2, False),
                [[2.0, 1.0], [3.0, 2.0], [4.0, 3.0]])


def test_panel_lags_kat():  # T/TimeSeriesSuite.scala:42-70 (series a, b side by side)
    a = [1.0, 2.0, 3.0, 4.0, 5.0]
    b = [6.0, 7.0, 8.0, 9.0, 10.0]
    m = np.hstack([oracle.lag(a, 2, True), oracle.lag(b, 2, True)])
    assert same(m, [[3, 2, 1, 8, 7, 6], [4, 3, 2, 9, 8, 7], [5, 4, 3, 10, 9, 8]])
    m = np.hstack([oracle.lag(a, 2, False), oracle.lag(b, 2, False)])
    assert same(m, [[2, 1, 7, 6], [3, 2, 8, 7], [4, 3, 9, 8]])


def test_autocorr_statistical():  # :47-60
    rand = MersenneTwister(5)
    iid = [rand.next_double() * 5.0 for _ in range(10000)]
    for r in oracle.autocorr(iid, 3):
        assert abs(r) < 0.03
    # ARModel(1.5, [.2]).sample(10000, rand) = addTimeDependentEffects(vec, vec)
    g = np.array([rand.next_gaussian() for _ in range(10000)])
    ar = oracle.ar_add(g, 1.5, [0.2], inplace=True)
    acf = oracle.autocorr(ar, 3)
    assert abs(0.2 - acf[0]) < 0.02
    assert 0.0 < acf[1] < 0.06
    assert 0.0 < acf[2] < 0.06


def test_differencing_at_lag():  # :112-126
    rand = MersenneTwister(10)
    s = np.array([rand.next_gaussian() for _ in range(100)])
    d = oracle.differences_at_lag(s, 5)
    inv = oracle.inverse_differences_at_lag(d, 5)
    assert np.all(np.abs(s - inv) <= 1e-6)
    assert d[10] == s[10] - s[5]
    assert d[99] == s[99] - s[94]


def test_differencing_of_order_d():  # :128-156
    rand = MersenneTwister(10)
    s = np.array([rand.next_gaussian() for _ in range(100)])
    o1 = oracle.differences_of_order_d(s, 1)
    assert np.all(np.abs(oracle.differences_at_lag(s, 1) - o1) <= 1e-6)
    o5 = oracle.differences_of_order_d(s, 5)
    inv = o5.copy()
    for i in range(5, 0, -1):  # inverseDifferencesOfOrderD, :459-465
        out = inv.copy()
        for k in range(inv.size):
            out[k] = inv[k] if k < i else inv[k] + out[k - 1]
        inv = out
    assert np.all(np.abs(inv - s) <= 1e-6)
    o6 = oracle.differences_of_order_d(s, 6)
    more = oracle.differences_of_order_d(o5, 1)
    assert np.all(np.abs(o6[6:] - more[6:]) <= 1e-6)


def test_differences_requirement():  # :361 require(startIndex >= lag)
    with pytest.raises(oracle.OracleError, match="starting index cannot be less than lag"):
        oracle.differences_at_lag([1.0, 2.0, 3.0], 2, start=1)


def test_differences_in_place_aliasing():
    # dest eq ts: reads overwritten values
    x = np.array([1.0, 3.0, 6.0, 10.0])
    out = oracle.differences_at_lag(x, 1, inplace=True)
    assert same(out, [1.0, 2.0, 4.0, 6.0])  # 3-1=2, 6-2=4, 10-4=6


# ---- T/models/EWMASuite.scala:22-51 ----

def round2(x):
    return math.floor(x * 100 + 0.5) / 100.0  # Scala Double.round = Math.round


def test_ewma_add_kat():
    orig = np.arange(1, 11, dtype=np.float64)
    for s, last in ((0.2, 6.54), (0.6, 9.33)):
        sm = oracle.ewma_add(orig, s)
        assert sm[0] == orig[0]
        assert sm[1] == s * orig[1] + (1 - s) * sm[0]
        assert round2(sm[-1]) == last


def test_ewma_remove_kat():
    smoothed = np.array([1.0, 1.2, 1.56, 2.05, 2.64, 3.31, 4.05, 4.84, 5.67, 6.54])
    orig = oracle.ewma_remove(smoothed, 0.2)
    assert round2(orig[0]) == 1.0
    assert int(orig[-1]) == 10


# ---- T/models/EWMASuite.scala:54-63 (fitting EWMA model) ----

OIL = [446.7, 454.5, 455.7, 423.6, 456.3, 440.6, 425.3, 485.1, 506.0, 526.8, 514.3, 494.2]


def test_ewma_fit_oil_kat():
    # the reference's only pin of the commons-math3 optimizer restatement: (s * 100).toInt == 89
    st, s, evals = oracle.ewma_fit(OIL)
    assert st == oracle.OK
    assert int(s * 100.0) == 89
    assert evals > 0


def test_ewma_sse_gradient_consistent():
    # EWMAModel.gradient (:102-123) is MINUS the derivative of EWMAModel.sse (:80-95):
    # d(error^2)/ds = -2 * error * dS/ds, and the reference accumulates +error * dSda.
    # Restated as the reference has it (the line search then walks backwards along the
    # search direction: BracketFinder accepts negative steps).
    rng = np.random.default_rng(3)
    x = np.cumsum(rng.standard_normal(300)) + 50
    for s in (0.1, 0.5, 0.9, 1.2):
        h = 1e-6
        fd = (oracle.ewma_sse(x, s + h) - oracle.ewma_sse(x, s - h)) / (2 * h)
        g = oracle.ewma_gradient(x, s)
        assert abs(fd + g) <= 1e-5 * max(1.0, abs(g))


def test_ewma_fit_nan_series_never_converges():
    # a NaN makes every sse NaN: commons-math3 ends in TooManyEvaluationsException
    x = np.ones(10)
    x[3] = np.nan
    st, s, evals = oracle.ewma_fit(x)
    assert st == oracle.ERR_TOO_MANY_EVALUATIONS and math.isnan(s) and evals == 10001


def test_ewma_fit_is_a_minimum():
    rng = np.random.default_rng(4)
    for T in (50, 390):
        x = np.cumsum(rng.standard_normal(T)) + 100
        st, s, _ = oracle.ewma_fit(x)
        assert st == oracle.OK
        grid = np.linspace(0.01, 2.0, 400)
        best = grid[int(np.argmin([oracle.ewma_sse(x, g) for g in grid]))]
        assert abs(s - best) < 0.02   # SimpleValueChecker(1e-6, 1e-6) stops near, not at, the minimum


# ---- T/models/AutoregressionSuite.scala:25-51 ----

def test_ar1_fit():
    rand = MersenneTwister(10)
    ts = oracle.ar_add(np.array([rand.next_gaussian() for _ in range(5000)]), 1.5, [0.2], inplace=True)
    c, coef = oracle.ar_fit(ts, 1)
    assert coef.size == 1
    assert abs(c - 1.5) < 0.07
    assert abs(coef[0] - 0.2) < 0.03


def test_ar2_fit():
    rand = MersenneTwister(10)
    ts = oracle.ar_add(np.array([rand.next_gaussian() for _ in range(5000)]), 1.5, [0.2, 0.3], inplace=True)
    c, coef = oracle.ar_fit(ts, 2)
    assert coef.size == 2
    assert abs(c - 1.5) < 0.15
    assert abs(coef[0] - 0.2) < 0.03
    assert abs(coef[1] - 0.3) < 0.03


def test_ar_add_remove_round_trip():
    ts = np.random.default_rng(0).random(1000)
    added = oracle.ar_add(ts, 1.5, [0.2, 0.3])
    removed = oracle.ar_remove(added, 1.5, [0.2, 0.3])
    assert np.all(np.abs(ts - removed) < 1e-3)


def test_ols_matches_lstsq():
    # the Householder restatement agrees with LAPACK least squares
    rng = np.random.default_rng(3)
    ts = oracle.ar_add(rng.standard_normal(3000), 0.7, [0.5, -0.25, 0.1])
    c, coef = oracle.ar_fit(ts, 3)
    X = np.column_stack([np.ones(2997)] + [ts[3 - k:3000 - k] for k in range(1, 4)])
    beta = np.linalg.lstsq(X, ts[3:], rcond=None)[0]
    assert np.allclose([c, *coef], beta, rtol=1e-12, atol=1e-12)


def test_ar_fit_not_enough_data():
    with pytest.raises(oracle.OracleError):
        oracle.ar_fit([1.0, 2.0, 3.0, 4.0], 2)  # 2 rows < 3 predictors


# ---- generator ----

def test_generator_deterministic_and_nan_rate():
    a = oracle.gen_panel(7, 4, 1000, 0.05)
    b = oracle.gen_panel(7, 4, 1000, 0.05)
    assert same(a, b)
    frac = np.isnan(a).mean()
    assert 0.03 < frac < 0.07
    c = oracle.gen_panel(7, 2, 1000, 0.05, s0=2)
    assert same(a[2:], c)
    v = a[~np.isnan(a)]
    assert v.min() > 99.0 and v.max() < 112.0


# ---- T/TimeSeriesRDDSuite.scala:210-231 (removeInstantsWithNaNs), :71-89 (toInstants) ----

def test_remove_instants_with_nans_kat():
    x = np.array([[1.0, 2.0, 3.0, 4.0], [5.0, np.nan, 7.0, 8.0], [9.0, 10.0, 11.0, np.nan]])
    out, active = oracle.remove_instants_with_nans(x)
    assert active.tolist() == [0, 2]          # index irregular(2015-4-9, 2015-4-11)
    assert same(out, [[1.0, 3.0], [5.0, 7.0], [9.0, 11.0]])


def test_to_instants_kat():
    series = np.array([np.arange(x, x + 4, dtype=np.float64) for x in range(0, 20, 4)])   # a..e
    inst = oracle.to_instants(series)
    for t in range(4):
        assert same(inst[t], np.arange(t, 20, 4, dtype=np.float64))


def test_stat_counter():
    # Spark StatCounter: count 4, mean 2.5, variance m2 / n = 1.25
    n, mu, m2, mx, mn = oracle.stat_counter([1.0, 2.0, 3.0, 4.0])
    assert (n, mu, m2 / n, mx, mn) == (4, 2.5, 1.25, 4.0, 1.0)
    # NaN propagates through mean, m2, max and min (java.lang.Math.max / min)
    _, mu, m2, mx, mn = oracle.stat_counter([1.0, np.nan, 3.0])
    assert all(math.isnan(v) for v in (mu, m2, mx, mn))
    # signed zeros: max(-0.0, 0.0) = 0.0, min(0.0, -0.0) = -0.0
    _, _, _, mx, mn = oracle.stat_counter([-0.0, 0.0])
    assert mx == 0.0 and not math.copysign(1.0, mx) < 0 and math.copysign(1.0, mn) < 0
    _, mu, m2, mx, mn = oracle.stat_counter([])
    assert (mu, m2, mx, mn) == (0.0, 0.0, -math.inf, math.inf)
