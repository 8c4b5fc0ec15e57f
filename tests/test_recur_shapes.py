"""Bit-exact parity of the recurrence kernels (recur_kernel: one lane per series, 16 series x
128-step chunks through LDS with 16-B accesses when rows are 16-B aligned, 64 x 32 with 8-B
accesses otherwise; recur_row_kernel for EWMA add and the fused C2 pipeline on 16-B aligned rows
of T <= 1 024: one wave per series) with the oracle, through the C ABI.  Shapes cover partial chunks and
partial series groups (S, T not multiples of 16 / 128), padded row strides (ld > T, different
in and out strides, odd padding that forces the 8-B kernel) and the in-place operators
(reference aliasing).  Needs an MI355X.
"""
import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu
NaN = np.nan

SHAPES = [(37, 2), (37, 8), (33, 14), (33, 64), (65, 390), (9, 512), (41, 100), (70, 16), (1, 390), (17, 510),
          (19, 129), (21, 1000)]


@pytest.fixture(scope="module")
def torch():
    import torch as _t
    if not _t.cuda.is_available():
        pytest.skip("no GPU")
    from sparkts import _native
    _native.ensure_device(0)
    return _t


def padded(torch, x, ld):
    S, T = x.shape
    t = torch.full((S, ld), 7.0, dtype=torch.float64, device="cuda:0")
    t[:, :T] = torch.as_tensor(x, device="cuda:0")
    return t


def host(t, T):
    return t.detach().cpu().numpy()[:, :T]


def assert_bits(got, ref, what=""):
    got = np.ascontiguousarray(got, dtype=np.float64)
    ref = np.ascontiguousarray(ref, dtype=np.float64)
    assert got.shape == ref.shape, (what, got.shape, ref.shape)
    same = (got.view(np.uint64) == ref.view(np.uint64)) | (np.isnan(got) & np.isnan(ref))
    if not same.all():
        idx = np.argwhere(~same)[:5]
        raise AssertionError("%s: %d mismatches, first %s" % (what, (~same).sum(), idx.tolist()))


def dvec(torch, v):
    return torch.as_tensor(np.ascontiguousarray(v, dtype=np.float64), device="cuda:0")


@pytest.mark.parametrize("S,T", SHAPES)
@pytest.mark.parametrize("pad", [0, 6, 3])
def test_recur_ewma(torch, S, T, pad):
    from sparkts import _native
    lib = _native.lib()
    rng = np.random.default_rng(S * 1000 + T + pad)
    x = rng.standard_normal((S, T)) + 10
    s = rng.uniform(0.05, 0.95, S)
    sd = dvec(torch, s)
    xi = padded(torch, x, T + pad)
    out = padded(torch, np.zeros((S, T)), T + 2 * pad)
    assert lib.sts_ewma_add(xi.data_ptr(), out.data_ptr(), S, T, T + pad, T + 2 * pad, sd.data_ptr(), None) == 0
    assert_bits(host(out, T), np.array([oracle.ewma_add(r, v) for r, v in zip(x, s)]), "ewma add")
    assert (out[:, T:].cpu().numpy() == 7.0).all(), "wrote into the row padding"
    ip = padded(torch, x, T + pad)
    assert lib.sts_ewma_remove(ip.data_ptr(), ip.data_ptr(), S, T, T + pad, T + pad, sd.data_ptr(), None) == 0
    ref = []
    for r, v in zip(x, s):
        rr = r.copy()
        oracle.ewma_remove(rr, v, dest=rr)
        ref.append(rr)
    assert_bits(host(ip, T), np.array(ref), "ewma remove in place")


@pytest.mark.parametrize("S,T", SHAPES)
@pytest.mark.parametrize("p", [1, 3, 8])
def test_recur_ar(torch, S, T, p):
    from sparkts import _native
    lib = _native.lib()
    rng = np.random.default_rng(S * 7 + T + p)
    x = rng.standard_normal((S, T))
    c = rng.standard_normal(S)
    coef = rng.uniform(-0.3, 0.3, (S, p))
    cd, fd = dvec(torch, c), dvec(torch, coef)
    xi = padded(torch, x, T + 4)
    out = padded(torch, np.zeros((S, T)), T)
    assert lib.sts_ar_add(xi.data_ptr(), out.data_ptr(), S, T, T + 4, T, cd.data_ptr(), fd.data_ptr(), p, None) == 0
    assert_bits(host(out, T), np.array([oracle.ar_add(x[s], c[s], coef[s]) for s in range(S)]), "ar add")
    ip = padded(torch, x, T + 4)
    assert lib.sts_ar_remove(ip.data_ptr(), ip.data_ptr(), S, T, T + 4, T + 4, cd.data_ptr(), fd.data_ptr(), p,
                             None) == 0
    ref = []
    for s in range(S):
        r = x[s].copy()
        for i in range(T):
            v = r[i] - c[s]
            for j in range(min(p, i)):
                v -= r[i - j - 1] * coef[s, j]
            r[i] = v
        ref.append(r)
    assert_bits(host(ip, T), np.array(ref), "ar remove in place")


@pytest.mark.parametrize("S,T", SHAPES)
@pytest.mark.parametrize("lag,start", [(1, 1), (3, 3), (2, 5), (8, 8)])
def test_recur_diff_in_place(torch, S, T, lag, start):
    from sparkts import _native
    lib = _native.lib()
    if start > T:
        pytest.skip("start beyond the series")
    x = np.random.default_rng(S + T + lag).standard_normal((S, T))
    ip = padded(torch, x, T + 2)
    assert lib.sts_diff_at_lag(ip.data_ptr(), ip.data_ptr(), S, T, T + 2, T + 2, lag, start, None) == 0
    ref = np.array([oracle.differences_at_lag(r, lag, start=start, inplace=True) for r in x])
    assert_bits(host(ip, T), ref, "diff in place")


@pytest.mark.parametrize("S,T", SHAPES)
@pytest.mark.parametrize("lag", [1, 2, 8])
def test_recur_fill_diff_ewma(torch, S, T, lag):
    from sparkts import _native
    lib = _native.lib()
    rng = np.random.default_rng(S + 3 * T + lag)
    x = 100 + rng.standard_normal((S, T)).cumsum(axis=1)
    x[rng.random((S, T)) < 0.2] = NaN
    x[0, : min(T, 5)] = NaN          # leading NaN run (fillPrevious leaves it NaN)
    if S > 2:
        x[2, :] = NaN                # all-NaN series
    s = rng.uniform(0.05, 0.95, S)
    xi = padded(torch, x, T + 6)
    out = padded(torch, np.zeros((S, T)), T + 2)
    assert lib.sts_fill_diff_ewma(xi.data_ptr(), out.data_ptr(), S, T, T + 6, T + 2, 3, lag,
                                  dvec(torch, s).data_ptr(), None, None) == 0
    ref = []
    for r, v in zip(x, s):
        f = oracle.fill_previous(r)
        d = oracle.differences_at_lag(f, lag)
        ref.append(oracle.ewma_add(d, v))
    assert_bits(host(out, T), np.array(ref), "fill_diff_ewma")


# Row-contiguous panels (ld == T, 16-B aligned rows): the shapes of the round-4 whole-row batch
# variant (batch edges, T = 2 .. 1202, more batches than CUs); with T <= 1 024 they now take
# recur_row_kernel (32 lanes per series, two series per wave, lane blocks of up to 32 steps
# (kRowLps = 32), bit-exact affine-scan guess verified lane by lane), T = 1 200 / 1 202 the chunk
# kernel.
@pytest.mark.parametrize("S,T", [(1, 2), (5, 2), (300, 390), (301, 390), (24, 390), (25, 390), (17, 1200),
                                 (9, 1202), (20_000, 390), (777, 64)])
@pytest.mark.parametrize("lag", [1, 8])
def test_recur_fill_diff_ewma_rows(torch, S, T, lag):
    from sparkts import _native
    lib = _native.lib()
    rng = np.random.default_rng(7 * S + T + lag)
    x = 100 + rng.standard_normal((S, T)).cumsum(axis=1)
    x[rng.random((S, T)) < 0.1] = NaN
    x[0, : min(T, 5)] = NaN
    if S > 3:
        x[3, :] = NaN
    s = rng.uniform(0.05, 0.95, S)             # a different smoothing per series
    xd = torch.as_tensor(x, device="cuda:0")
    out = torch.full_like(xd, 7.0)
    assert lib.sts_fill_diff_ewma(xd.data_ptr(), out.data_ptr(), S, T, T, T, 3, lag,
                                  dvec(torch, s).data_ptr(), None, None) == 0
    ref = []
    for r, v in zip(x, s):
        ref.append(oracle.ewma_add(oracle.differences_at_lag(oracle.fill_previous(r), lag), v))
    assert_bits(out.cpu().numpy(), np.array(ref), "fill_diff_ewma rows")


# recur_row_kernel edges: lane-block boundaries (T around 64 x 8 and 64 x 16, odd T: the scalar
# tail), smoothing extremes (s = 1: every map constant; s = 1e-6: a block contracts by only
# 1 - 8e-6, so the scan's guess is verified over more rounds), NaN runs across many lane blocks,
# infinities, and series whose EWMA crosses zero (cancellation in the guess, not in the result).
@pytest.mark.parametrize("T", [1, 2, 3, 7, 9, 15, 63, 64, 65, 390, 511, 512, 513, 1023, 1024, 1025])
@pytest.mark.parametrize("lag", [1, 3, 5, 8])
def test_recur_row_scan_edges(torch, T, lag):
    from sparkts import _native
    lib = _native.lib()
    S = 11
    rng = np.random.default_rng(31 * T + lag)
    x = 100 + rng.standard_normal((S, T)).cumsum(axis=1)
    x[rng.random((S, T)) < 0.1] = NaN
    x[1, T // 8: T // 2 + 1] = NaN                  # a run over many lane blocks
    x[2, :] = NaN
    x[3, : T - 1] = NaN                             # only the last step valid
    x[4] = rng.standard_normal(T) * 1e-3            # zero-mean: the EWMA of its diffs crosses 0
    x[5, T // 3:T // 3 + 2] = np.inf
    x[6, T // 2] = -np.inf
    s = np.array([1.0, 1e-6, 0.999999, 0.5, 0.2, 0.2, 0.2, 1e-3, 0.97, 0.3, 0.05])
    xd = torch.as_tensor(x, device="cuda:0")
    out = torch.full_like(xd, 7.0)
    assert lib.sts_fill_diff_ewma(xd.data_ptr(), out.data_ptr(), S, T, T, T, 3, lag,
                                  dvec(torch, s).data_ptr(), None, None) == 0
    ref = np.array([oracle.ewma_add(oracle.differences_at_lag(oracle.fill_previous(r), lag), v) for r, v in zip(x, s)])
    assert_bits(out.cpu().numpy(), ref, "fill_diff_ewma row kernel")
    # EWMA add alone, raw values (NaN / inf in the chain)
    out2 = torch.full_like(xd, 7.0)
    assert lib.sts_ewma_add(xd.data_ptr(), out2.data_ptr(), S, T, T, T, dvec(torch, s).data_ptr(), None) == 0
    assert_bits(out2.cpu().numpy(), np.array([oracle.ewma_add(r, v) for r, v in zip(x, s)]), "ewma add row kernel")
    # in place (the reference's dest eq ts is safe for add)
    ip = torch.as_tensor(x, device="cuda:0").clone()
    assert lib.sts_ewma_add(ip.data_ptr(), ip.data_ptr(), S, T, T, T, dvec(torch, s).data_ptr(), None) == 0
    assert_bits(ip.cpu().numpy(), np.array([oracle.ewma_add(r, v) for r, v in zip(x, s)]), "ewma add in place")


# recur_row_kernel's direct-access form on odd T (16-B aligned rows need an even stride: ld = T + 1
# or T + 3), where the last pair of a row is a single step (8-B loads from clamped addresses).
@pytest.mark.parametrize("T", [1, 3, 9, 65, 391, 1023])
@pytest.mark.parametrize("extra", [1, 3])
def test_recur_row_scan_odd_rows(torch, T, extra):
    from sparkts import _native
    lib = _native.lib()
    S = 9
    ld = T + extra
    rng = np.random.default_rng(17 * T + extra)
    x = 100 + rng.standard_normal((S, T)).cumsum(axis=1)
    x[rng.random((S, T)) < 0.15] = NaN
    x[1, :] = NaN
    s = rng.uniform(0.05, 0.95, S)
    xi = padded(torch, x, ld)
    out = padded(torch, np.zeros((S, T)), ld)
    assert lib.sts_fill_diff_ewma(xi.data_ptr(), out.data_ptr(), S, T, ld, ld, 3, 1,
                                  dvec(torch, s).data_ptr(), None, None) == 0
    ref = np.array([oracle.ewma_add(oracle.differences_at_lag(oracle.fill_previous(r), 1), v) for r, v in zip(x, s)])
    assert_bits(host(out, T), ref, "fill_diff_ewma odd rows")
    assert (out[:, T:].cpu().numpy() == 7.0).all(), "wrote into the row padding"
    out2 = padded(torch, np.zeros((S, T)), ld)
    assert lib.sts_ewma_add(xi.data_ptr(), out2.data_ptr(), S, T, ld, ld, dvec(torch, s).data_ptr(), None) == 0
    assert_bits(host(out2, T), np.array([oracle.ewma_add(r, v) for r, v in zip(x, s)]), "ewma add odd rows")
    assert (out2[:, T:].cpu().numpy() == 7.0).all(), "wrote into the row padding"
