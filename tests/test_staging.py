"""The `_host` entry points' pinned staging pipeline (spark-timeseries_amd/csrc/sts_host.cpp):
panels larger than one ~64 MB chunk, pageable and pinned (sts_host_alloc) host arrays,
padded leading dimensions, in-place calls and per-series errors in late chunks -- every
result bit-identical to the same entry point on HBM-resident data (and to the oracle)."""
import ctypes

import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch():
    import torch as _t
    if not _t.cuda.is_available():
        pytest.skip("no GPU")
    from sparkts import _native
    _native.ensure_device(0)
    return _t


def lib():
    from sparkts import _native
    return _native.lib()


def P(a):
    return a.ctypes.data


class Pinned:
    """A numpy view of pinned host memory from sts_host_alloc."""

    def __init__(self, shape, dtype=np.float64):
        n = int(np.prod(shape)) * np.dtype(dtype).itemsize
        self.p = ctypes.c_void_p()
        assert lib().sts_host_alloc(n, ctypes.byref(self.p)) == 0
        buf = (ctypes.c_char * n).from_address(self.p.value)
        self.a = np.frombuffer(buf, dtype=dtype).reshape(shape)

    def __del__(self):
        if getattr(self, "p", None) and self.p.value:
            lib().sts_host_free(self.p)


def stats():
    s = np.zeros(8)
    assert lib().sts_staging_stats(P(s)) == 0
    return dict(zip(["wall_ms", "h2d_ms", "kernel_ms", "d2h_ms", "h2d_bytes", "d2h_bytes", "chunks", "direct"], s))


def bits(a, b):
    a, b = np.ascontiguousarray(a), np.ascontiguousarray(b)
    return a.shape == b.shape and bool(((a.view(np.uint64) == b.view(np.uint64)) | (np.isnan(a) & np.isnan(b))).all())


@pytest.mark.parametrize("pinned", [False, True])
def test_fill_diff_ewma_host_multi_chunk(torch, pinned):
    S, T = 30000, 390                       # 94 MB in + 94 MB out: three chunks
    x = oracle.gen_panel(2, S, T, 0.05)
    x[3, :40] = np.nan
    sm = np.full(S, 0.2)
    if pinned:
        hx, hout = Pinned((S, T)), Pinned((S, T))
        hx.a[:] = x
        xin, out = hx.a, hout.a
    else:
        xin, out = x, np.empty_like(x)
    assert lib().sts_fill_diff_ewma_host(P(xin), P(out), S, T, T, 3, 1, P(sm), None) == 0
    st = stats()
    assert st["chunks"] >= 2
    assert (st["direct"] > 0.99) if pinned else (st["direct"] == 0.0)
    assert st["h2d_bytes"] == S * T * 8 + S * 8 + 0 * S and st["d2h_bytes"] == S * T * 8 + S * 4
    xd = torch.as_tensor(x, device="cuda:0")
    od = torch.empty_like(xd)
    smd = torch.as_tensor(sm, device="cuda:0")
    assert lib().sts_fill_diff_ewma(xd.data_ptr(), od.data_ptr(), S, T, T, T, 3, 1, smd.data_ptr(), None, None) == 0
    assert bits(out, od.cpu().numpy())
    ref = oracle.panel_fill_diff_ewma(x[:50], 0.2)
    assert bits(out[:50], ref)


@pytest.mark.parametrize("pinned", [False, True])
def test_fill_autocorr_host_padded_ld_and_late_error(torch, pinned):
    S, T, ld, K = 2600, 9000, 9003, 20      # ~190 MB in + out: several chunks, padded rows
    x = np.full((S, ld), 7.0)
    x[:, :T] = oracle.gen_panel(3, S, T, 0.05)
    if pinned:
        hx = Pinned((S, ld)); hx.a[:] = x; xin = hx.a
        hf = Pinned((S, ld)); hf.a[:] = -1.0; filled = hf.a
    else:
        xin, filled = x, np.full((S, ld), -1.0)
    acf = np.empty((S, K))
    err = np.zeros(S, np.int32)
    assert lib().sts_fill_autocorr_host(P(xin), P(filled), S, T, ld, 0, K, P(acf), P(err)) == 0
    assert (err == 0).all() and stats()["chunks"] >= 2
    rf, racf, _ = oracle.panel_fill_autocorr(np.ascontiguousarray(x[-20:, :T]), "linear", K)
    assert bits(filled[-20:, :T], rf)
    assert (filled[:, T:] == -1.0).all()   # padding untouched
    ok = ~np.isnan(racf)
    assert np.array_equal(np.isnan(acf[-20:]), ~ok)
    assert np.max(np.abs(acf[-20:][ok] - racf[ok]) / np.abs(racf[ok])) <= 1e-10
    # nearest on a series whose only valid value is index 0, in the LAST chunk: with a NULL
    # err array the call fails with the reference's exception after all chunks are back
    x2 = np.ascontiguousarray(x[:, :T])
    x2[-3, 1:] = np.nan
    f2 = np.empty_like(x2)
    st = lib().sts_fill_autocorr_host(P(x2), P(f2), S, T, T, 1, K, P(acf), None)
    assert st == 2 and b"Input is all NaNs!" in lib().sts_last_error()
    e2 = np.zeros(S, np.int32)
    assert lib().sts_fill_autocorr_host(P(x2), P(f2), S, T, T, 1, K, P(acf), P(e2)) == 0
    assert list(np.flatnonzero(e2)) == [S - 3] and e2[S - 3] == 2


def test_in_place_host_paths_match_device(torch):
    S, T = 20000, 1000                      # 160 MB: three chunks, in place
    rng = np.random.default_rng(4)
    x = rng.standard_normal((S, T)) + 5
    sm = rng.uniform(0.1, 0.9, S)
    # differencesAtLag with dest eq ts (the reference's in-place recurrence)
    h = x.copy()
    assert lib().sts_diff_at_lag_host(P(h), P(h), S, T, T, 3, 5) == 0
    assert bits(h[:30], np.array([oracle.differences_at_lag(r, 3, start=5, inplace=True) for r in x[:30]]))
    # EWMA remove in place reads overwritten values
    h = x.copy()
    assert lib().sts_ewma_remove_host(P(h), P(h), S, T, T, P(sm)) == 0
    ref = []
    for r, v in zip(x[-30:], sm[-30:]):
        rr = r.copy(); oracle.ewma_remove(rr, v, dest=rr); ref.append(rr)
    assert bits(h[-30:], np.array(ref))
    # AR(5) fit + remove through the staged path = the device path
    xa = oracle.gen_ar_panel(4, 4000, 2520, 5)
    out = np.empty_like(xa); c = np.empty(4000); coef = np.empty((4000, 5))
    assert lib().sts_ar_fit_remove_host(P(xa), P(out), 4000, 2520, 2520, 5, 0, P(c), P(coef), None) == 0
    xd = torch.as_tensor(xa, device="cuda:0")
    od = torch.empty_like(xd)
    cd = torch.empty(4000, dtype=torch.float64, device="cuda:0")
    kd = torch.empty((4000, 5), dtype=torch.float64, device="cuda:0")
    assert lib().sts_ar_fit_remove(xd.data_ptr(), od.data_ptr(), 4000, 2520, 2520, 2520, 5, 0, cd.data_ptr(),
                                   kd.data_ptr(), None, None) == 0
    assert bits(out, od.cpu().numpy()) and bits(c, cd.cpu().numpy()) and bits(coef, kd.cpu().numpy())


def test_staging_release_and_reuse(torch):
    x = oracle.gen_panel(1, 10, 100, 0.1)
    out = np.empty_like(x)
    assert lib().sts_fill_host(P(x), P(out), 10, 100, 100, 3, None) == 0
    assert lib().sts_staging_release() == 0
    out2 = np.empty_like(x)
    assert lib().sts_fill_host(P(x), P(out2), 10, 100, 100, 3, None) == 0
    assert bits(out, out2) and bits(out, oracle.panel_fill(x, "previous")[0])
