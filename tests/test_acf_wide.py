"""autocorr for any numLags (VERDICT r1 "What's missing" #2): the reference has no bound on
numLags (S/UnivariateTimeSeries.scala:68-93; lbtest and acfPlot pass user-chosen lags).

numLags <= 63 runs fused in the imputation kernels; larger numLags runs the lag-block path
of spark-timeseries_amd/csrc/sts_acf_wide.hip: 61-lag blocks of the shifted-window MFMA
decomposition with the B operand offset by L0 = 1 + 61 b, edge E = K in the robust finalize,
and the reference's own two-pass loop when T <= 2K (so lags >= T come out NaN like the
reference's empty slices).

CPU: a numpy emulation of the shifted-window lag map with a lag offset (every (position,
lag) pair counted exactly once over the chunk bases {-64, 0, 64, ...}) against direct dot
products.  GPU: the HIP path against the oracle, 1e-10 relative with identical NaN pattern,
K in {64, 100, 250} on short / multi-range / C3-length series, far-level rows, K >= T.
"""
import numpy as np
import pytest

import oracle
from test_acf_robust import hard_rows, noise_floor, rel_err, run_fill_acf, with_nans, within

QS, NT, LAGS = 4, 4, 61


def h(j):
    return 16 * (j // QS) + (16 - QS) + j % QS


def shifted_window_lag_products(y, L0):
    """P[d] = sum_p y_p y_{p + L0 + d}, d = 0..60, accumulated exactly as acf_wide_kernel's
    MFMAs: chunk bases -64, 0, 64, ... < T; MFMA t, row i, column j, k-group k; y = 0
    outside [0, T)."""
    T = y.size

    def Y(p):
        return y[p] if 0 <= p < T else 0.0

    P = np.zeros(64)
    for base in range(-64, T, 64):
        for t in range(NT):
            for k in range(4):
                for i in range(16):
                    a = Y(base + QS * t + i + 16 * k)
                    if a == 0.0:
                        continue
                    for j in range(16):
                        d = h(j) - i
                        if 0 <= d < LAGS:
                            P[d] += a * Y(base + QS * t + 16 * k + h(j) + L0)
    return P[:LAGS]


@pytest.mark.parametrize("T,L0", [(200, 1), (333, 62), (150, 123), (64, 1)])
def test_lag_block_decomposition_counts_every_pair_once(T, L0):
    y = np.random.default_rng(T + L0).standard_normal(T)
    got = shifted_window_lag_products(y, L0)
    want = np.array([np.dot(y[:max(T - L0 - d, 0)], y[L0 + d:]) if L0 + d < T else 0.0 for d in range(LAGS)])
    assert np.allclose(got, want, rtol=1e-12, atol=1e-12)


# ---------------- GPU ----------------

@pytest.fixture(scope="module")
def torch():
    import torch as _t
    if not _t.cuda.is_available():
        pytest.skip("no GPU")
    from sparkts import _native
    _native.ensure_device(0)
    return _t


def walks(S, T, seed):
    rng = np.random.default_rng(seed)
    return np.cumsum(rng.standard_normal((S, T)), axis=1)


@pytest.mark.gpu
@pytest.mark.parametrize("K", [64, 100, 250])
@pytest.mark.parametrize("T,S", [(2520, 6), (16384 + 77, 3), (70_000, 2)])
@pytest.mark.parametrize("method", ["linear", None])
def test_gpu_autocorr_many_lags(torch, K, T, S, method):
    x = walks(S, T, K * 3 + T)
    if method is not None:
        x = with_nans(x, np.random.default_rng(K + T))
    filled, got = run_fill_acf(torch, x, method, K)
    if method is None:
        ref = np.array([oracle.autocorr(r, K) for r in x])
    else:
        rf, ref, err = oracle.panel_fill_autocorr(x, method, K, threads=4)
        assert (err == 0).all()
        assert np.array_equal(filled.view(np.uint64), rf.view(np.uint64)), "fill not bit-exact"
    assert rel_err(got, ref) <= 1e-10


@pytest.mark.gpu
@pytest.mark.parametrize("K", [64, 120])
def test_gpu_autocorr_many_lags_far_level(torch, K):
    T = 16384 + 77
    x = hard_rows(T, T + K)
    filled, got = run_fill_acf(torch, x, None, K)
    ref = np.array([oracle.autocorr(r, K) for r in x])
    floor = np.array([noise_floor(r, K) for r in x])
    assert within(got, ref, floor) <= 1.0
    assert rel_err(got[:-1], ref[:-1]) <= 1e-10


@pytest.mark.gpu
def test_gpu_autocorr_many_lags_c3_length(torch):
    T, K = 982_800, 100
    x = oracle.gen_panel(3, 2, T, 0.05)
    filled, got = run_fill_acf(torch, x, "linear", K)
    rf, ref, _ = oracle.panel_fill_autocorr(x, "linear", K, threads=2)
    assert np.array_equal(filled.view(np.uint64), rf.view(np.uint64))
    assert rel_err(got, ref) <= 1e-10


@pytest.mark.gpu
@pytest.mark.parametrize("T,K", [(100, 150), (300, 200), (129, 64), (1, 70), (2, 70)])
def test_gpu_autocorr_lags_at_or_past_the_length(torch, T, K):
    # T <= 2K: the reference's two-pass loop; lags >= T are NaN (empty slices), lag T-1 is a
    # one-element slice (0 / 0 = NaN)
    x = walks(4, T, T + K)
    x[1, T // 2] = np.nan                     # interior NaN: only lags whose slices miss it are finite
    _, got = run_fill_acf(torch, x, None, K)
    ref = np.array([oracle.autocorr(r, K) for r in x])
    assert np.isnan(got[:, T - 1:]).all() if T - 1 < K else True
    assert rel_err(got, ref) <= 1e-10


@pytest.mark.gpu
def test_gpu_autocorr_many_lags_host_path(torch):
    from sparkts import UnivariateTimeSeries as uts
    x = walks(5, 3000, 9)
    got = uts.autocorr(x, 90)                 # numpy -> the _host staging path
    ref = np.array([oracle.autocorr(r, 90) for r in x])
    assert rel_err(got, ref) <= 1e-10
