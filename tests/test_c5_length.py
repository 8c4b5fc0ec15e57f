"""C5 at its real series length under -m gpu (VERDICT r2 "What's weak" #8): the fused
fill(nearest | next) + lag(10, includeOriginal = false) on 2 series x 10,000,000 steps at 30 %
NaN (BASELINE.json configs[4]; Lag.lagMatTrimBoth, S/Lag.scala:62-77; fills
S/UnivariateTimeSeries.scala:156-184 / :206-224).

The filled panel is compared in full, bit for bit, with the oracle.  The lag matrix (1.6 GB on
the device) is compared on every row within 80 of a 4096-step tile edge of the tile kernel
(4096 k +- 80: where the look-back / look-ahead halos and the carried last-valid index change
hands) and on the last 20 000 rows, each window against oracle.lag of the same filled slice:
bit-exact (index-driven copies)."""
import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu

T = 10_000_000
P = 10
TILE = 4096


@pytest.fixture(scope="module")
def torch():
    import torch as _t
    if not _t.cuda.is_available():
        pytest.skip("no GPU")
    from sparkts import _native
    _native.ensure_device(0)
    return _t


def rows_to_check():
    edges = np.arange(TILE, T, TILE)
    win = (edges[:, None] + np.arange(-80, 80)[None, :]).ravel()
    tail = np.arange(T - P - 20_000, T - P)
    rows = np.unique(np.concatenate([np.arange(0, 200), win, tail]))
    return rows[(rows >= 0) & (rows < T - P)]


def windows(rows):
    """Maximal runs of consecutive row indices: [(a, b), ...] with rows a..b-1."""
    br = np.flatnonzero(np.diff(rows) != 1) + 1
    starts = np.concatenate([[0], br])
    ends = np.concatenate([br, [rows.size]])
    return [(int(rows[s]), int(rows[e - 1]) + 1) for s, e in zip(starts, ends)]


@pytest.mark.parametrize("method", ["nearest", "next"])
def test_c5_fill_lag_at_ten_million_steps(torch, method):
    from sparkts import _native
    from sparkts import UnivariateTimeSeries as uts
    S = 2
    x = oracle.gen_panel(5, S, T, 0.3)
    x[1, 5_000_000:5_300_000] = np.nan            # a 300 k-step gap across ~73 tiles
    xd = torch.as_tensor(x, device="cuda:0")
    filled = torch.empty_like(xd)
    lm = torch.empty((S, P, T - P), dtype=torch.float64, device="cuda:0")
    st = _native.lib().sts_fill_lag_matrix(xd.data_ptr(), filled.data_ptr(), lm.data_ptr(), S, T, T, T,
                                           uts.fill_method_code(method), P, 0, None, None)
    assert st == 0, _native.lib().sts_last_error()
    torch.cuda.synchronize()
    rf, err = oracle.panel_fill(x, method, threads=4)
    assert (err == 0).all()
    got_f = filled.cpu().numpy()
    same = (got_f.view(np.uint64) == rf.view(np.uint64)) | (np.isnan(got_f) & np.isnan(rf))
    assert same.all(), "filled panel differs at %s" % np.argwhere(~same)[:5].tolist()
    rows = rows_to_check()
    idx = torch.as_tensor(rows, device="cuda:0")
    got = lm.index_select(2, idx).cpu().numpy()    # (S, P, n_rows)
    del lm
    for s in range(S):
        ref = np.empty((rows.size, P))
        k = 0
        for a, b in windows(rows):
            ref[k:k + b - a] = oracle.lag(rf[s, a:b + P], P, False)   # rows a..b-1 of the full lag matrix
            k += b - a
        g = got[s].T
        ok = (g.view(np.uint64) == ref.view(np.uint64)) | (np.isnan(g) & np.isnan(ref))
        assert ok.all(), "series %d: lag rows differ at %s" % (s, rows[np.argwhere(~ok)[:5, 0]].tolist())
