"""TimeSeriesRDD.fill / mapSeries (S/TimeSeriesRDD.scala:180-199): keys and their order
are preserved, per-series closures keep the reference's semantics, batched closures run
once on the panel, and the fused pipelines (README.md:61's AR closure, the C2 chain) equal
the per-series composition of the primitives (GPU, vs the oracle)."""
import numpy as np
import pytest

import oracle
from sparkts import TimeSeriesRDD
from sparkts.pipelines import apply_per_series, batched, is_batched

KEYS = ["k%03d" % i for i in (7, 3, 11, 0, 5)]


def test_per_series_closure_semantics_and_key_order():
    x = np.arange(5 * 6, dtype=np.float64).reshape(5, 6)
    rdd = TimeSeriesRDD(None, KEYS, x)
    seen = []

    def f(series):                       # a closure that only makes sense per series
        seen.append(float(series[0]))
        return series - series.mean()

    out = rdd.mapSeries(f)
    assert out.keys == KEYS                                  # same keys, same order
    assert seen == [float(r[0]) for r in x]                  # called once per series, in key order
    assert np.array_equal(out.data, x - x.mean(axis=1, keepdims=True))
    assert out.index is None and rdd.mapSeries(f, index="idx").index == "idx"


def test_batched_closure_runs_once_on_the_panel():
    x = np.random.default_rng(1).standard_normal((5, 9))
    calls = []

    @batched
    def g(panel):
        calls.append(panel.shape)
        return panel * 2.0

    assert is_batched(g) and not is_batched(lambda s: s)
    out = TimeSeriesRDD(None, KEYS, x).mapSeries(g)
    assert calls == [(5, 9)]
    assert out.keys == KEYS and np.array_equal(out.data, 2.0 * x)


def test_apply_per_series_empty_and_stacking():
    assert apply_per_series(lambda s: s, np.zeros((0, 4))).shape == (0, 4)
    got = apply_per_series(lambda s: s[:2], np.arange(12.0).reshape(3, 4))
    assert got.tolist() == [[0, 1], [4, 5], [8, 9]]


# ---------------- GPU: fused pipelines through mapSeries ----------------

@pytest.fixture(scope="module")
def torch():
    import torch as _t
    if not _t.cuda.is_available():
        pytest.skip("no GPU")
    from sparkts import _native
    _native.ensure_device(0)
    return _t


@pytest.mark.gpu
def test_readme_ar_closure_fused_vs_per_series(torch):
    # filled.mapSeries(series => ar(series, 1).removeTimeDependentEffects(series)) (README.md:61)
    from sparkts import UnivariateTimeSeries as uts
    from sparkts.pipelines import ar_remove
    S, T = 6, 700
    x = oracle.gen_panel(21, S, T, 0.05)
    keys = ["s%d" % i for i in range(S)][::-1]
    rdd = TimeSeriesRDD(None, keys, torch.as_tensor(x, device="cuda:0")).fill("linear")
    fused = rdd.mapSeries(ar_remove(1))
    per = rdd.mapSeries(lambda s: uts.ar(s, 1).removeTimeDependentEffects(s))
    assert fused.keys == keys and per.keys == keys
    f = fused.data.cpu().numpy()
    p = per.data.cpu().numpy()
    rf, _ = oracle.panel_fill(x, "linear")
    # residuals depend on the fitted (c, phi): within the AR-fit tolerance of the oracle's
    for s in range(S):
        c, coef = oracle.ar_fit(rf[s], 1)
        want = oracle.ar_remove(rf[s], c, coef)
        fin = ~np.isnan(want)
        assert np.array_equal(np.isnan(f[s]), ~fin)
        assert np.allclose(f[s][fin], want[fin], rtol=1e-9, atol=1e-9 * np.abs(want[fin]).max())
    assert np.array_equal(np.isnan(f), np.isnan(p))
    assert np.allclose(np.nan_to_num(f), np.nan_to_num(p), rtol=1e-12, atol=1e-12)


@pytest.mark.gpu
def test_fill_diff_ewma_pipeline_bit_exact(torch):
    from sparkts.pipelines import fill_diff_ewma
    S, T = 9, 390
    x = oracle.gen_panel(22, S, T, 0.05)
    keys = ["k%d" % (S - i) for i in range(S)]
    rdd = TimeSeriesRDD(None, keys, torch.as_tensor(x, device="cuda:0"))
    out = rdd.mapSeries(fill_diff_ewma("previous", 1, 0.2))
    assert out.keys == keys
    want = oracle.panel_fill_diff_ewma(x, 0.2)
    got = out.data.cpu().numpy()
    assert np.array_equal(np.isnan(got), np.isnan(want))
    assert np.array_equal(np.nan_to_num(got).view(np.uint64), np.nan_to_num(want).view(np.uint64))
    # the host (JNI-equivalent) path gives the same bits
    host = TimeSeriesRDD(None, keys, x).mapSeries(fill_diff_ewma("previous", 1, 0.2)).data
    assert np.array_equal(np.nan_to_num(host).view(np.uint64), np.nan_to_num(want).view(np.uint64))
