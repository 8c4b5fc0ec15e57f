"""Committed golden fixtures (tests/golden/, made by tests/golden/make_golden.py).

CPU: the oracle reproduces the reference's own KAT vectors (kats.json) and its frozen
outputs on the seeded edge-case panels (panels.npz) -- a change in the restatement shows
up here before it can move the GPU parity bar.
GPU: the HIP path, through the C ABI and the sparkts mirror, reproduces the same frozen
outputs: bit-exact for fills, differencing, lag matrices, EWMA and AR remove; ACF and AR
coefficients within RTOL = 1e-10 relative (BASELINE.json north_star).
"""
import json
import os
import sys

import numpy as np
import pytest

import oracle

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden")
sys.path.insert(0, GOLD)
import make_golden  # noqa: E402

RTOL = 1e-10
METHODS = ("linear", "previous", "next", "nearest")


def _nan(v):
    if isinstance(v, list):
        return [_nan(u) for u in v]
    return float("nan") if v == "NaN" else v


@pytest.fixture(scope="module")
def kats():
    with open(os.path.join(GOLD, "kats.json")) as f:
        return json.load(f)


@pytest.fixture(scope="module")
def gold():
    with np.load(os.path.join(GOLD, "panels.npz"), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def bits_equal(got, ref):
    got = np.ascontiguousarray(got, dtype=np.float64)
    ref = np.ascontiguousarray(ref, dtype=np.float64)
    if got.shape != ref.shape:
        return False
    return bool(((got.view(np.uint64) == ref.view(np.uint64)) | (np.isnan(got) & np.isnan(ref))).all())


def rel_ok(got, ref, rtol=RTOL):
    got, ref = np.asarray(got), np.asarray(ref)
    if got.shape != ref.shape or not np.array_equal(np.isnan(got), np.isnan(ref)):
        return False
    fin = ~np.isnan(ref)
    if not fin.any():
        return True
    return float((np.abs(got[fin] - ref[fin]) / np.maximum(np.abs(ref[fin]), 1e-300)).max()) <= rtol


# ---------------- CPU: oracle vs the fixtures ----------------

def test_oracle_fill_kats(kats):
    for k in kats["fill"]:
        assert bits_equal(oracle.fillts(_nan(k["x"]), k["method"]), _nan(k["want"])), k["src"]


def test_oracle_lag_kats(kats):
    for k in kats["lag"]:
        assert bits_equal(oracle.lag(k["x"], k["max_lag"], k["include_original"]), k["want"]), k["src"]


def test_oracle_ewma_kats(kats):
    for k in kats["ewma_add_rounded_last"]:
        assert round(oracle.ewma_add(k["x"], k["smoothing"])[-1] * 100) / 100 == k["last_2dp"], k["src"]
    for k in kats["ewma_remove_int_last"]:
        assert int(oracle.ewma_remove(k["x"], k["smoothing"])[-1]) == k["int_last"], k["src"]


def test_oracle_remove_instants_kat(kats):
    for k in kats["remove_instants_with_nans"]:
        out, active = oracle.remove_instants_with_nans(np.array(_nan(k["x"])))
        assert bits_equal(out, k["want"]) and list(active) == k["active"], k["src"]


def test_oracle_reproduces_frozen_panels(gold):
    x = gold["short_x"]
    for m in METHODS:
        f, a, err = oracle.panel_fill_autocorr(x, m, int(gold["short_K"]))
        assert bits_equal(f, gold["short_fill_%s" % m]), m
        assert bits_equal(a, gold["short_acf_%s" % m]), m
    xd = gold["dense_x"]
    assert bits_equal([oracle.differences_at_lag(r, 3) for r in xd], gold["diff_lag3"])
    assert bits_equal([oracle.lag(r, 10, False) for r in xd], gold["lag10_false"])
    assert bits_equal([oracle.ewma_add(r, s) for r, s in zip(xd, gold["ewma_s"])], gold["ewma_add"])
    for s, r in enumerate(gold["ar_x"]):
        c, coef = oracle.ar_fit(r, 5, False)
        assert c == gold["ar5_c"][s] and bits_equal(coef, gold["ar5_coef"][s])


def test_long_case_regenerates(gold):
    # the tile-kernel case is regenerated from the counter-based generator, not stored
    assert make_golden.digest(make_golden.long_panel()) == str(gold["long_x_sha256"])


# ---------------- GPU: HIP path vs the fixtures ----------------

@pytest.fixture(scope="module")
def torch():
    import torch as _t
    if not _t.cuda.is_available():
        pytest.skip("no GPU")
    from sparkts import _native
    _native.ensure_device(0)
    return _t


def dev(torch, a):
    return torch.as_tensor(np.ascontiguousarray(a, dtype=np.float64), device="cuda:0")


def host(t):
    return t.detach().cpu().numpy()


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["short", "long"])
@pytest.mark.parametrize("method", METHODS)
def test_gpu_fill_autocorr_golden(torch, gold, case, method):
    from sparkts import TimeSeriesRDD
    from sparkts import UnivariateTimeSeries as uts
    x = gold["short_x"] if case == "short" else make_golden.long_panel()
    K = int(gold["%s_K" % case])
    filled, acf = TimeSeriesRDD(None, None, dev(torch, x)).fillAndAutocorr(method, K)
    fill_only = host(uts.fillts(dev(torch, x), method))
    if case == "short":
        assert bits_equal(host(filled.data), gold["short_fill_%s" % method])
        assert bits_equal(fill_only, gold["short_fill_%s" % method])
    else:
        want = str(gold["long_fill_%s_sha256" % method])
        assert make_golden.digest(host(filled.data)) == want
        assert make_golden.digest(fill_only) == want
    assert rel_ok(host(acf), gold["%s_acf_%s" % (case, method)])


@pytest.mark.gpu
def test_gpu_elementwise_golden(torch, gold):
    from sparkts import UnivariateTimeSeries as uts
    from sparkts.models import EWMAModel
    x = gold["dense_x"]
    assert bits_equal(host(uts.differencesAtLag(dev(torch, x), 3)), gold["diff_lag3"])
    xd = dev(torch, x)
    uts.differencesAtLag(xd, 3, destTs=xd)
    assert bits_equal(host(xd), gold["diff_lag3_inplace"])
    assert bits_equal(host(uts.lag(dev(torch, x), 10, False)), gold["lag10_false"])
    assert bits_equal(host(uts.lag(dev(torch, x), 4, True)), gold["lag4_true"])
    sm = dev(torch, gold["ewma_s"])
    out = torch.empty_like(dev(torch, x))
    EWMAModel(sm).addTimeDependentEffects(dev(torch, x), out)
    assert bits_equal(host(out), gold["ewma_add"])
    EWMAModel(sm).removeTimeDependentEffects(dev(torch, x), out)
    assert bits_equal(host(out), gold["ewma_remove"])


@pytest.mark.gpu
def test_gpu_ar_golden(torch, gold):
    from sparkts.models import ARModel, Autoregression
    xa = dev(torch, gold["ar_x"])
    m = Autoregression.fitModel(xa, 5, False)
    assert rel_ok(host(m.c), gold["ar5_c"]) and rel_ok(host(m.coefficients), gold["ar5_coef"])
    # remove is bit-exact given (c, coef): feed the frozen model
    rm = ARModel(dev(torch, gold["ar5_c"]), dev(torch, gold["ar5_coef"]))
    assert bits_equal(host(rm.removeTimeDependentEffects(xa)), gold["ar5_remove"])
