"""The persistent, double-buffered AR(p) fit kernel (round 3, csrc/sts_ar.hip PERS form).

It is an A/B form (STS_AR_PERS on libsts_hip_ab.so; measured slower than the
one-series-per-wave kernel) for aligned panels with at least 4 x (CUs x 4)
series: two 4-wave workgroups per CU whose waves each walk every (2 CUs x 4)-th series,
streaming series k + 1's block into their LDS block as soon as series k is in registers.  Reference:
S/models/Autoregression.scala:38-53 (fit), :60-73 (removeTimeDependentEffects).

Checks, on panels big enough to take that path (S >= 2048 on a 256-CU MI355X) and with a
series count that leaves the waves uneven trip counts:
* coefficients within 1e-10 of the oracle's Householder restatement, residuals bit-exact
  given the fitted model (the reference's remove loop), fused and fit-only entry points;
* bit-identical results to the one-series-per-wave kernel (the product library);
* a NaN series gives the NaN model without disturbing its neighbours in the pipeline.
"""
import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu

RTOL = 1e-10


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


@pytest.fixture
def pers(monkeypatch):
    from sparkts import _native
    monkeypatch.setattr(_native, "_lib", _native.load_variant(_native.AB_LIB_PATH))
    monkeypatch.setenv("STS_AR_PERS", "1")


def rel_ok(got, ref, what):
    assert np.array_equal(np.isnan(got), np.isnan(ref)), "%s: NaN pattern differs" % what
    fin = ~np.isnan(ref)
    err = np.abs(got[fin] - ref[fin]) / np.maximum(np.abs(ref[fin]), 1e-300)
    assert err.size == 0 or err.max() <= RTOL, "%s: max rel err %g" % (what, err.max())


def bits_equal(a, b):
    a = np.ascontiguousarray(a, dtype=np.float64)
    b = np.ascontiguousarray(b, dtype=np.float64)
    return bool(np.all((a.view(np.uint64) == b.view(np.uint64)) | (np.isnan(a) & np.isnan(b))))


@pytest.mark.parametrize("p,T", [(5, 2520), (1, 2520), (4, 1000), (3, 200), (8, 2520)])
def test_persistent_fit_remove_matches_oracle(torch, pers, p, T):
    from sparkts.models import Autoregression
    S = 4300
    x = oracle.gen_ar_panel(12, S, T, min(p, 5))
    x[17, T // 3] = np.nan                     # one NaN series in the middle of a wave's walk
    m, resid = Autoregression.fitModelAndRemove(dev(torch, x), p)
    c, coef = host(m.c), host(m.coefficients)
    _, rc, rcoef = oracle.panel_ar_fit_remove(x, p, threads=8)
    rel_ok(coef, rcoef, "coef p=%d T=%d" % (p, T))
    rel_ok(c, rc, "c p=%d T=%d" % (p, T))
    assert np.isnan(c[17]) and not np.isnan(c[16]) and not np.isnan(c[18])
    sample = [0, 1, 17, 1023, 1024, 2047, 2048, 4095, 4096, S - 2, S - 1]
    ref = np.array([oracle.ar_remove(x[s], c[s], coef[s]) for s in sample])
    assert bits_equal(host(resid)[sample], ref), "fused remove not bit-exact given the model"
    m2 = Autoregression.fitModel(dev(torch, x), p)          # fit-only entry point (no residuals)
    assert bits_equal(host(m2.c), c) and bits_equal(host(m2.coefficients), coef)


def test_persistent_equals_one_series_per_wave(torch, monkeypatch):
    from sparkts import _native
    from sparkts.models import Autoregression
    S, T, p = 4300, 2520, 5
    x = oracle.gen_ar_panel(13, S, T, p)
    m1, resid1 = Autoregression.fitModelAndRemove(dev(torch, x), p)      # product: one series per wave
    monkeypatch.setattr(_native, "_lib", _native.load_variant(_native.AB_LIB_PATH))
    monkeypatch.setenv("STS_AR_PERS", "1")
    m, resid = Autoregression.fitModelAndRemove(dev(torch, x), p)
    assert bits_equal(host(m.c), host(m1.c))
    assert bits_equal(host(m.coefficients), host(m1.coefficients))
    assert bits_equal(host(resid), host(resid1))


def test_persistent_many_series_per_wave(torch, monkeypatch):
    """~15 series per wave (S = 30 000, a 605 MB panel): every wave's DMA / store pipeline
    runs through many iterations, over row addresses past 2^31 bytes from the panel's start;
    results bit-identical to the one-series-per-wave kernel."""
    from sparkts import _native
    from sparkts.models import Autoregression
    S, T, p = 30000, 2520, 5
    x = torch.empty((S, T), dtype=torch.float64, device="cuda:0")
    cg = torch.empty(S, dtype=torch.float64, device="cuda:0")
    pg = torch.empty((S, p), dtype=torch.float64, device="cuda:0")
    sp = torch.cuda.current_stream().cuda_stream
    assert _native.lib().sts_gen_ar_panel(x.data_ptr(), cg.data_ptr(), pg.data_ptr(), 0, S, T, T, 4, p, sp) == 0
    m1, resid1 = Autoregression.fitModelAndRemove(x, p)
    monkeypatch.setattr(_native, "_lib", _native.load_variant(_native.AB_LIB_PATH))
    monkeypatch.setenv("STS_AR_PERS", "1")
    m, resid = Autoregression.fitModelAndRemove(x, p)
    assert bits_equal(host(m.c), host(m1.c))
    assert bits_equal(host(m.coefficients), host(m1.coefficients))
    assert torch.equal(resid.view(torch.int64), resid1.view(torch.int64))
