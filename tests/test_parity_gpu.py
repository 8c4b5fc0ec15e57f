"""Parity of the HIP path (through the C ABI) with the CPU oracle.  Needs an MI355X.

Tolerances (BASELINE.json north_star): index-driven work (lag, differencing,
previous/next/nearest fill) and the recurrences restated in the reference's own
order (linear fill, EWMA add/remove, AR add/remove) are BIT-EXACT; autocorrelation
and AR coefficients within 1e-10 relative (RTOL below), NaN patterns identical.
"""
import zlib

import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu

RTOL = 1e-10
NaN = np.nan


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


def assert_bits(got, ref, what=""):
    got = np.ascontiguousarray(got, dtype=np.float64)
    ref = np.ascontiguousarray(ref, dtype=np.float64)
    assert got.shape == ref.shape, (what, got.shape, ref.shape)
    gb, rb = got.view(np.uint64), ref.view(np.uint64)
    # all NaNs compare equal regardless of payload
    same = (gb == rb) | (np.isnan(got) & np.isnan(ref))
    if not same.all():
        idx = np.argwhere(~same)[:5]
        raise AssertionError("%s: %d mismatches, first %s got %s ref %s" % (
            what, (~same).sum(), idx.tolist(), [got[tuple(i)] for i in idx], [ref[tuple(i)] for i in idx]))


def assert_rel(got, ref, rtol=RTOL, what=""):
    got = np.asarray(got)
    ref = np.asarray(ref)
    assert got.shape == ref.shape
    assert np.array_equal(np.isnan(got), np.isnan(ref)), "%s: NaN pattern differs" % what
    fin = ~np.isnan(ref)
    if fin.any():
        err = np.abs(got[fin] - ref[fin]) / np.maximum(np.abs(ref[fin]), 1e-300)
        assert err.max() <= rtol, "%s: max rel err %g > %g" % (what, err.max(), rtol)


def random_panel(rng, S, T, nan_p, runs=False):
    x = 100.0 + rng.standard_normal((S, T)).cumsum(axis=1) * 0.1 + rng.random((S, T))
    x[rng.random((S, T)) < nan_p] = NaN
    if runs and T > 10:
        for s in range(S):
            a = rng.integers(0, T)
            b = min(T, a + rng.integers(1, max(2, T // 3)))
            x[s, a:b] = NaN
    return x


SHAPES = [(3, 1), (4, 2), (5, 3), (7, 5), (9, 63), (9, 64), (9, 65), (16, 390), (5, 511), (5, 512), (5, 513),
          (11, 2520), (3, 4096), (3, 4097), (4, 4159), (4, 4161), (3, 9000), (2, 20000)]


# ---------------- fills (a1-a5): bit-exact ----------------

FILL_KATS = [  # T/FillSuite.scala:35-61
    ("previous", [1.0, NaN, 3.0, NaN, 2.0], [1.0, 1.0, 3.0, 3.0, 2.0]),
    ("next", [1.0, NaN, 3.0, NaN, 2.0], [1.0, 3.0, 3.0, 2.0, 2.0]),
    ("linear", [1.0, NaN, 3.0, NaN, 2.0], [1.0, 2.0, 3.0, 2.5, 2.0]),
    ("linear", [1.0, NaN, NaN, NaN, 5.0], [1.0, 2.0, 3.0, 4.0, 5.0]),
    ("linear", [2.0, NaN, 1.0], [2.0, 1.5, 1.0]),
    ("nearest", [1.0, NaN, 2.0], [1.0, 2.0, 2.0]),
]


@pytest.mark.parametrize("method,x,want", FILL_KATS)
def test_fill_kats_device_and_host(torch, method, x, want):
    from sparkts import UnivariateTimeSeries as uts
    assert_bits(host(uts.fillts(dev(torch, x), method)), want, method)
    assert_bits(uts.fillts(np.array(x), method), want, method + " host path")


@pytest.mark.parametrize("method", ["linear", "previous", "next", "nearest"])
@pytest.mark.parametrize("nan_p", [0.0, 0.05, 0.3, 0.9])
def test_fill_panels(torch, method, nan_p):
    from sparkts import UnivariateTimeSeries as uts
    from sparkts import _native
    rng = np.random.default_rng(zlib.crc32(("%s%g" % (method, nan_p)).encode()))
    lib = _native.lib()
    code = uts.fill_method_code(method)
    for S, T in SHAPES:
        x = random_panel(rng, S, T, nan_p, runs=True)
        ref, err = oracle.panel_fill(x, method)
        xd = dev(torch, x)
        out = torch.empty_like(xd)
        e = torch.zeros(S, dtype=torch.int32, device="cuda:0")
        st = lib.sts_fill(xd.data_ptr(), out.data_ptr(), S, T, T, T, code, e.data_ptr(), None)
        assert st == 0
        torch.cuda.synchronize()
        ge = host(e)
        assert np.array_equal(ge != 0, err != 0), (method, S, T, ge, err)
        ok = err == 0
        assert_bits(host(out)[ok], ref[ok], "%s S=%d T=%d" % (method, S, T))


@pytest.mark.parametrize("method", ["linear", "previous", "next", "nearest"])
def test_fill_long_runs_and_edges(torch, method):
    from sparkts import UnivariateTimeSeries as uts
    T = 30000
    rows = []
    x = np.arange(T, dtype=np.float64) * 0.37 + 1.0
    a = x.copy(); a[100:25000] = NaN; rows.append(a)          # run across many tiles (slow path both ways)
    a = x.copy(); a[:9000] = NaN; rows.append(a)              # long leading run
    a = x.copy(); a[-9000:] = NaN; rows.append(a)             # long trailing run
    a = x.copy(); a[1:] = NaN; rows.append(a)                 # only x[0] valid (nearest throws)
    a = x.copy(); a[4090:4200] = NaN; rows.append(a)          # run straddling a tile edge
    a = x.copy(); a[::2] = NaN; rows.append(a)                # alternating
    a = np.full(T, NaN); rows.append(a)                       # all NaN
    a = x.copy(); a[4096 - 64 - 70:4096 + 200] = NaN; rows.append(a)  # run longer than the look-back halo
    a = x.copy(); a[0] = NaN; a[8191:8192 + 130] = NaN; rows.append(a)
    P = np.array(rows)
    ref, err = oracle.panel_fill(P, method)
    from sparkts import _native
    lib = _native.lib()
    xd = dev(torch, P)
    out = torch.empty_like(xd)
    e = torch.zeros(P.shape[0], dtype=torch.int32, device="cuda:0")
    assert lib.sts_fill(xd.data_ptr(), out.data_ptr(), P.shape[0], T, T, T, uts.fill_method_code(method),
                        e.data_ptr(), None) == 0
    torch.cuda.synchronize()
    assert np.array_equal(host(e) != 0, err != 0)
    ok = err == 0
    assert_bits(host(out)[ok], ref[ok], method)


def _gap_rows(T, gaps, seed):
    rng = np.random.default_rng(seed)
    rows = []
    for a, b in gaps:
        x = 1e4 + np.cumsum(rng.standard_normal(T) * 0.01)
        x[rng.random(T) < 0.05] = NaN
        x[0] = x[-1] = 1e4                                    # interior gaps only: linear fills them
        x[a:b] = NaN
        rows.append(x)
    return np.array(rows)


@pytest.mark.parametrize("method", ["linear", "previous", "next", "nearest"])
def test_fill_long_gaps_bit_exact(torch, method):
    # NaN runs around the chain-pass threshold (kLongRun = 32), across tile (4096) and
    # workgroup (16 tiles) boundaries, starting / ending at tile edges, and longer than a
    # workgroup: the chain pass (carried across tiles) and the cached global scans
    from sparkts import _native
    from sparkts import UnivariateTimeSeries as uts
    T = 200_000
    gaps = [(100, 133), (100, 134), (4063, 4097), (4096, 4096 + 33), (4000, 12300), (8192, 8192 + 4096),
            (60000, 70000), (65536 - 7, 65536 + 40), (30000, 190000), (4096 * 5 - 1, 4096 * 21 + 1),
            (2, T - 2), (17, 99)]
    x = _gap_rows(T, gaps, 7)
    ref, err = oracle.panel_fill(x, method, threads=4)
    xd = dev(torch, x)
    out = torch.empty_like(xd)
    e = torch.zeros(x.shape[0], dtype=torch.int32, device="cuda:0")
    assert _native.lib().sts_fill(xd.data_ptr(), out.data_ptr(), x.shape[0], T, T, T, uts.fill_method_code(method),
                                  e.data_ptr(), None) == 0
    torch.cuda.synchronize()
    assert np.array_equal(host(e), err)
    assert_bits(host(out), ref, method)
    # the same through the fused fill + ACF path (tile kernel with MFMA) and the segment kernel
    K = 60
    filled, acf = __import__("sparkts").TimeSeriesRDD(None, None, xd).fillAndAutocorr(method, K)
    assert_bits(host(filled.data), ref, method + " fused")
    xs = _gap_rows(16000, [(40, 15950), (100, 133), (511, 545), (1000, 9000)], 8)
    rs, es = oracle.panel_fill(xs, method)
    assert_bits(host(uts.fillts(dev(torch, xs), method)), rs, method + " segment kernel")


@pytest.mark.parametrize("T,gap", [(982_800, (200_000, 700_000)), (16_384, (30, 16_300))])
def test_fill_linear_long_gap_is_linear_time(torch, T, gap):
    # a G-step interior gap used to cost O(G^2) sequential adds (each NaN
    # replayed its whole chain from L); the chain pass makes it O(G).  Bit-exact, and the
    # gap panel must fill in about the time of a gap-free one.
    from sparkts import _native
    S = 4
    x = _gap_rows(T, [gap] * S, 9)
    xd = dev(torch, x)
    out = torch.empty_like(xd)
    acf = torch.empty((S, 60), dtype=torch.float64, device="cuda:0")
    lib = _native.lib()

    def run(src):
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev0.record()
        assert lib.sts_fill_autocorr(src.data_ptr(), out.data_ptr(), S, T, T, T, 0, 60, acf.data_ptr(), None,
                                     torch.cuda.current_stream().cuda_stream) == 0
        ev1.record()
        torch.cuda.synchronize()
        return ev0.elapsed_time(ev1)

    run(xd)
    t_gap = min(run(xd) for _ in range(3))
    ref, racf, _ = oracle.panel_fill_autocorr(x, "linear", 60, threads=4)
    assert_bits(host(out), ref, "linear gap")
    assert_rel(host(acf), racf, what="acf after a long gap")
    base = dev(torch, _gap_rows(T, [(10, 11)] * S, 9))
    run(base)
    t_base = min(run(base) for _ in range(3))
    print("T=%d gap=%d: %.3f ms with the gap, %.3f ms without" % (T, gap[1] - gap[0], t_gap, t_base))
    # the floor is the reference's own serial chain (bit-exactness forbids reassociating the
    # G additions): ~G dependent FP64 adds in the workgroup deepest in the gap.  The O(G^2)
    # replay took on the order of a second for G = 500k.
    assert t_gap < t_base + 50.0, (t_gap, t_base)


def test_fill_nearest_raises(torch):
    from sparkts import UnivariateTimeSeries as uts
    from sparkts.errors import IllegalArgumentException
    with pytest.raises(IllegalArgumentException, match="Input is all NaNs!"):
        uts.fillNearest(dev(torch, [5.0, NaN]))
    with pytest.raises(IllegalArgumentException):
        uts.fillNearest(np.array([[1.0, 2.0, 3.0], [NaN, NaN, NaN]]))


def test_fill_unsupported(torch):
    # only an unknown method throws (:148); "spline" is a working method (tests/test_spline.py)
    from sparkts import UnivariateTimeSeries as uts
    from sparkts.errors import UnsupportedOperationException
    with pytest.raises(UnsupportedOperationException):
        uts.fillts(dev(torch, [1.0, NaN, 2.0]), "cubic")
    with pytest.raises(UnsupportedOperationException):
        uts.fillts(dev(torch, [1.0, NaN, 2.0]), "Spline")
    got = uts.fillts(dev(torch, [1.0, NaN, 2.0, 5.0]), "spline")
    assert_bits(host(got), oracle.fill_spline([1.0, NaN, 2.0, 5.0]), "spline")


def test_fill_padded_leading_dimension(torch):
    from sparkts import _native
    rng = np.random.default_rng(5)
    S, T, ld = 6, 5000, 5003
    x = random_panel(rng, S, T, 0.2)
    buf = np.full((S, ld), 7.0); buf[:, :T] = x
    ref, _ = oracle.panel_fill(x, "linear")
    xd = dev(torch, buf)
    out = torch.full((S, ld + 1), -1.0, dtype=torch.float64, device="cuda:0")
    assert _native.lib().sts_fill(xd.data_ptr(), out.data_ptr(), S, T, ld, ld + 1, 0, None, None) == 0
    o = host(out)
    assert_bits(o[:, :T], ref)
    assert (o[:, T:] == -1.0).all()


# ---------------- autocorr (a8): 1e-10 relative ----------------

@pytest.mark.parametrize("K", [1, 5, 16, 17, 20, 33, 48, 49, 60, 63])
def test_autocorr_panels(torch, K):
    from sparkts import UnivariateTimeSeries as uts
    rng = np.random.default_rng(K)
    for S, T in [(5, 1), (5, 2), (7, 40), (7, 121), (6, 130), (9, 390), (5, 2520), (3, 4096), (3, 4097), (2, 12345)]:
        x = 50.0 + rng.standard_normal((S, T)).cumsum(axis=1) * 0.5 + rng.standard_normal((S, T))
        got = host(uts.autocorr(dev(torch, x), K))
        ref = np.array([oracle.autocorr(r, K) for r in x])
        assert_rel(got, ref, what="K=%d T=%d" % (K, T))


def test_autocorr_nan_and_constant(torch):
    from sparkts import UnivariateTimeSeries as uts
    K = 20
    rows = [np.full(100, 5.0), np.r_[np.full(50, 1.0), np.full(50, 3.0)], np.arange(100.0)]
    a = np.arange(100.0); a[40] = NaN; rows.append(a)
    b = np.arange(30.0); b[15] = NaN; rows.append(b[:30])   # short series: NaN only in the middle
    # non-dyadic constants: the reference's rounded mean makes every diff the same d != 0, so
    # it returns 1.0 (not NaN) -- sts_acf.hpp rule 3 takes its loop
    rows += [np.full(100, 100.1), np.full(3000, 1234.567), np.full(20000, 0.3)]
    c = np.full(5000, 100.1); c[-1] = 100.2; rows.append(c)   # constant but one end
    got = [host(uts.autocorr(dev(torch, r), K)) for r in rows]
    ref = [oracle.autocorr(r, K) for r in rows]
    for g, r in zip(got, ref):
        assert_rel(g, r)


def test_autocorr_reference_statistics(torch):
    # T/UnivariateTimeSeriesSuite.scala:47-60 through the device path
    from mt19937 import MersenneTwister
    from sparkts import UnivariateTimeSeries as uts
    rand = MersenneTwister(5)
    iid = np.array([rand.next_double() * 5.0 for _ in range(10000)])
    for r in host(uts.autocorr(dev(torch, iid), 3)):
        assert abs(r) < 0.03
    g = np.array([rand.next_gaussian() for _ in range(10000)])
    ar = oracle.ar_add(g, 1.5, [0.2], inplace=True)
    acf = host(uts.autocorr(dev(torch, ar), 3))
    assert abs(0.2 - acf[0]) < 0.02 and 0.0 < acf[1] < 0.06 and 0.0 < acf[2] < 0.06


@pytest.mark.parametrize("method", ["linear", "previous", "next", "nearest"])
def test_fill_autocorr_fused(torch, method):
    from sparkts import TimeSeriesRDD
    for seed, (S, T, K) in enumerate([(50, 2520, 20), (6, 9000, 60), (3, 4096 * 3 + 17, 63)]):
        x = oracle.gen_panel(seed + 3, S, T, 0.05)
        if method == "nearest":
            x[:, 1] = 100.0  # keep every series valid for nearest
        rdd = TimeSeriesRDD(None, None, dev(torch, x))
        filled, acf = rdd.fillAndAutocorr(method, K)
        rf, racf, err = oracle.panel_fill_autocorr(x, method, K)
        assert (err == 0).all()
        assert_bits(host(filled.data), rf, method)
        assert_rel(host(acf), racf, what=method)


# Both imputation kernels on every length, whatever the product dispatch picks, and the A/B
# knob settings that change the decomposition -- all through the A/B build
# (libsts_hip_ab.so); each must stay parity-green.
KNOB_VARIANTS = {
    "tile": {"STS_TILE_KERNEL": "tile"},
    "seg": {"STS_TILE_KERNEL": "seg", "STS_NO_SHORT": "1"},
    "short": {"STS_TILE_KERNEL": "seg"},                              # linear, K <= 24, T <= 2560: sts_short.hip
    "short1": {"STS_TILE_KERNEL": "seg", "STS_SHORT_PAIR": "0"},      # its one-series-per-block form
    "short2": {"STS_TILE_KERNEL": "seg", "STS_SHORT_PAIR": "1"},      # two series per block (round 6)
    "tile2048": {"STS_TILE_KERNEL": "tile", "STS_TILE_W": "2048"},    # 2-wave workgroups, 2048-step tiles
    "tilec4": {"STS_TILE_KERNEL": "tile", "STS_TILES_PER_CHUNK": "4"},  # 4 tiles per workgroup
    "seg3": {"STS_TILE_KERNEL": "seg", "STS_SEG_TILES": "3"},          # multi-segment partials + finalize
}


@pytest.mark.parametrize("kernel", sorted(KNOB_VARIANTS))
@pytest.mark.parametrize("method", ["linear", "previous", "next", "nearest"])
def test_fill_autocorr_both_kernels(torch, ab_lib, kernel, method):
    from sparkts import TimeSeriesRDD
    from sparkts import UnivariateTimeSeries as uts
    ab_lib(**KNOB_VARIANTS[kernel])
    rng = np.random.default_rng(zlib.crc32(("both%s%s" % (kernel, method)).encode()))
    for S, T, K in [(7, 600, 20), (5, 2520, 60), (3, 16384 + 77, 24), (2, 70000, 60), (2, 513, 0)]:
        x = random_panel(rng, S, T, 0.07, runs=True)
        if method == "nearest":
            x[:, 1] = 100.0
        if K > 0:
            filled, acf = TimeSeriesRDD(None, None, dev(torch, x)).fillAndAutocorr(method, K)
            rf, racf, err = oracle.panel_fill_autocorr(x, method, K)
            assert (err == 0).all()
            assert_bits(host(filled.data), rf, "%s %s T=%d" % (kernel, method, T))
            assert_rel(host(acf), racf, what="%s %s T=%d K=%d" % (kernel, method, T, K))
        else:
            got = host(uts.fillts(dev(torch, x), method))
            ref, _ = oracle.panel_fill(x, method)
            assert_bits(got, ref, "%s %s T=%d" % (kernel, method, T))


@pytest.mark.parametrize("T", [121, 128, 512, 575, 576, 1000, 1024, 2520, 4097, 16384])
def test_fused_acf_finalize_matches_two_kernel_path(torch, monkeypatch, T):
    # one segment per series: the segment kernel finalizes the ACF itself (no partials, no
    # second launch) when T > 2K, T >= 128 and its last tile holds >= 64 steps; bit-identical
    # to the separate acf_finalize_kernel (forced with STS_NO_FUSED_ACF on the A/B build), and
    # err is written for every series without a memset.  Both sides on the A/B build with the
    # short-series kernel off (STS_NO_SHORT), which the product takes for linear fills with
    # K <= 24 and even T <= 2560 (test_short_fill_acf covers it)
    from sparkts import TimeSeriesRDD
    from sparkts import _native
    rng = np.random.default_rng(T)
    monkeypatch.setenv("STS_NO_SHORT", "1")
    x = random_panel(rng, 9, T, 0.05, runs=True)
    x[4] = 7.0                                            # constant: 0/0 = NaN
    x[5, 0] = NaN                                         # head NaN -> all-NaN ACF
    prod = _native.load_variant(_native.AB_LIB_PATH)
    ab = prod
    monkeypatch.setattr(_native, "_lib", prod)
    for K in (1, 20, 60):
        if T <= 2 * K:
            continue
        f1, a1 = TimeSeriesRDD(None, None, dev(torch, x)).fillAndAutocorr("linear", K)
        monkeypatch.setattr(_native, "_lib", ab)
        monkeypatch.setenv("STS_NO_FUSED_ACF", "1")
        f2, a2 = TimeSeriesRDD(None, None, dev(torch, x)).fillAndAutocorr("linear", K)
        monkeypatch.delenv("STS_NO_FUSED_ACF")
        monkeypatch.setattr(_native, "_lib", prod)
        assert_bits(host(a1), host(a2), "fused vs separate finalize T=%d K=%d" % (T, K))
        assert_bits(host(f1.data), host(f2.data), "filled")
        _, racf, _ = oracle.panel_fill_autocorr(x, "linear", K)
        assert_rel(host(a1), racf, what="fused T=%d K=%d" % (T, K))
    # err written for every series (stale values in the caller's array are overwritten)
    xn = x.copy()
    xn[2, 1:] = NaN
    xd = dev(torch, xn)
    out = torch.empty_like(xd)
    acf = torch.empty((9, 20), dtype=torch.float64, device="cuda:0")
    err = torch.full((9,), 99, dtype=torch.int32, device="cuda:0")
    st = prod.sts_fill_autocorr(xd.data_ptr(), out.data_ptr(), 9, T, T, T, 1, 20, acf.data_ptr(),
                                err.data_ptr(), torch.cuda.current_stream().cuda_stream)
    assert st == 0
    want = np.zeros(9, np.int32)
    want[2] = 2                                            # nearest on [x0, NaN, ...]: "Input is all NaNs!"
    assert np.array_equal(host(err), want)


@pytest.mark.parametrize("method,K", [("linear", 1), ("linear", 8), ("linear", 9), ("linear", 20), ("linear", 24),
                                      ("previous", 20), ("previous", 5), ("next", 20), ("next", 13),
                                      ("nearest", 20), ("nearest", 7)])
def test_short_fill_acf(torch, monkeypatch, method, K):
    # sts_short.hip: fillts + ACF with the whole series in one wave (K <= 24, even T in
    # [128, 2560], aligned rows).  Fill bit-exact and ACF 1e-10 against the oracle, on NaN
    # patterns that cross lane blocks (B = 8..40 steps): runs entering a block from the left,
    # runs spanning many blocks, leading / trailing / t = 0 / t = T-1 NaNs, all-NaN (nearest:
    # "Input is all NaNs!" in err), constant, one valid step, alternating; err written for every
    # series; the segment kernel (STS_NO_SHORT on the A/B build) agrees to 1e-10
    from sparkts import _native
    from sparkts import UnivariateTimeSeries as uts
    code = uts.fill_method_code(method)
    rng = np.random.default_rng(1000 + K + 100 * code)

    def run(lib, x, T):
        S = x.shape[0]
        xd = dev(torch, x)
        out = torch.empty_like(xd)
        acf = torch.empty((S, K), dtype=torch.float64, device="cuda:0")
        e = torch.full((S,), 99, dtype=torch.int32, device="cuda:0")
        assert lib.sts_fill_autocorr(xd.data_ptr(), out.data_ptr(), S, T, T, T, code, K, acf.data_ptr(),
                                     e.data_ptr(), torch.cuda.current_stream().cuda_stream) == 0
        torch.cuda.synchronize()
        return host(out), host(acf), host(e)

    for T in (128, 130, 512, 514, 1000, 1024, 1536, 2048, 2520, 2560):
        if T <= 2 * K:
            continue
        x = random_panel(rng, 16, T, 0.05, runs=True)
        x[1, : T // 3] = NaN                                  # leading run over many blocks
        x[2, T // 4: 3 * T // 4] = NaN                        # interior run over many blocks
        x[3, -(T // 5):] = NaN                                # trailing run
        x[4, 0] = NaN; x[4, T - 1] = NaN                      # the ends
        x[5] = NaN                                            # all NaN
        x[6] = 3.25                                           # constant: 0/0
        x[7] = NaN; x[7, T // 2] = 1.0                        # one valid step
        x[8, 1::2] = NaN                                      # alternating
        x[9, 7:9] = NaN; x[9, 39:41] = NaN; x[9, 79:81] = NaN  # runs across 8 / 40-step block edges
        x[10, 1:T - 1] = NaN                                  # one run from 1 to T-2
        x[11] = 1e6 + rng.standard_normal(T)                  # high level, no NaN
        x[12, 22:200] = NaN                                   # run across several small blocks
        x[13, 1:] = NaN                                       # only x[0] (nearest: all NaN)
        x[14, 1:T // 2] = NaN; x[14, 0] = 5.0                 # nearest: x[0] is never an end
        x[15] = 100.1; x[15, 3:T // 2] = NaN                  # constant at a non-dyadic level: the
        #                                                       reference's rounded means give 1.0
        rf, racf, err = oracle.panel_fill_autocorr(x, method, K)
        got_f, got_a, got_e = run(_native.lib(), x, T)
        assert np.array_equal(got_e, err), (method, T, got_e, err)
        ok = err == 0
        assert_bits(got_f[ok], rf[ok], "fill %s T=%d K=%d" % (method, T, K))
        # every row, including the (near-)constant lag slices (rows 6, 10, 15: the reference's
        # own two-pass values, taken by sts_acf.hpp rule 3)
        assert_rel(got_a[ok], racf[ok], what="acf %s T=%d K=%d" % (method, T, K))
        monkeypatch.setenv("STS_NO_SHORT", "1")
        seg_f, seg_a, seg_e = run(_native.load_variant(_native.AB_LIB_PATH), x, T)
        monkeypatch.delenv("STS_NO_SHORT")
        assert np.array_equal(seg_e, err)
        assert_bits(seg_f[ok], rf[ok], "seg fill T=%d" % T)
        assert_rel(got_a[ok], seg_a[ok], what="short vs seg %s T=%d K=%d" % (method, T, K))
        # both forms of the short kernel (one series per LDS block / two per block: round 6),
        # also on an odd panel (the second wave of the last pair has no series)
        for pair in ("0", "1"):
            monkeypatch.setenv("STS_SHORT_PAIR", pair)
            for rows in (slice(0, 16), slice(0, 15), slice(15, 16)):
                pf, pa, pe = run(_native.load_variant(_native.AB_LIB_PATH), x[rows], T)
                okr = ok[rows]
                assert np.array_equal(pe, err[rows]), (pair, rows)
                assert_bits(pf[okr], rf[rows][okr], "pair=%s fill T=%d" % (pair, T))
                assert_rel(pa[okr], racf[rows][okr], what="pair=%s acf %s T=%d K=%d" % (pair, method, T, K))
            monkeypatch.delenv("STS_SHORT_PAIR")


def test_fill_autocorr_c3_length(torch):
    # C3 series length (982,800 minute bars), a few series: fused fill("linear") + ACF(60)
    S, T, K = 3, 982_800, 60
    x = oracle.gen_panel(3, S, T, 0.05)
    from sparkts import TimeSeriesRDD
    filled, acf = TimeSeriesRDD(None, None, dev(torch, x)).fillAndAutocorr("linear", K)
    rf, racf, _ = oracle.panel_fill_autocorr(x, "linear", K, threads=3)
    assert_bits(host(filled.data), rf)
    assert_rel(host(acf), racf)


# ---------------- differencing (a6), lag (a7): bit-exact ----------------

@pytest.mark.parametrize("lag,start", [(1, 1), (5, 5), (3, 7), (40, 40), (0, 0), (0, 3)])
def test_diff_at_lag(torch, lag, start):
    from sparkts import UnivariateTimeSeries as uts
    rng = np.random.default_rng(lag * 10 + start)
    x = rng.standard_normal((13, 777))
    got = host(uts.differencesAtLag(dev(torch, x), lag, startIndex=start))
    ref = np.array([oracle.differences_at_lag(r, lag, start=start) for r in x])
    assert_bits(got, ref)
    # in place (dest eq ts): the reference's aliasing semantics
    xd = dev(torch, x)
    uts.differencesAtLag(xd, lag, destTs=xd, startIndex=start)
    ref2 = np.array([oracle.differences_at_lag(r, lag, start=start, inplace=True) for r in x])
    assert_bits(host(xd), ref2, "in place")


def test_diff_dest_checks(torch):
    # destTs must match ts: a smaller dest is refused instead of overrun; a
    # strided dest receives the result (the kernel writes a unit-stride copy, copied back)
    from sparkts import UnivariateTimeSeries as uts
    rng = np.random.default_rng(5)
    x = rng.standard_normal((6, 300))
    ref = np.array([oracle.differences_at_lag(r, 2) for r in x])
    with pytest.raises(ValueError, match="same kind and shape"):
        uts.differencesAtLag(dev(torch, x), 2, destTs=dev(torch, x[:5]))
    wide = torch.zeros((6, 600), dtype=torch.float64, device="cuda:0")
    dst = wide[:, ::2]                       # time stride 2
    out = uts.differencesAtLag(dev(torch, x), 2, destTs=dst)
    assert out is dst
    assert_bits(host(dst.contiguous()), ref, "strided dest")
    # strided ts updated in place (dest is ts)
    xs = torch.zeros((6, 600), dtype=torch.float64, device="cuda:0")
    xs[:, ::2] = dev(torch, x)
    v = xs[:, ::2]
    uts.differencesAtLag(v, 2, destTs=v)
    ref2 = np.array([oracle.differences_at_lag(r, 2, start=2, inplace=True) for r in x])
    assert_bits(host(xs[:, ::2].contiguous()), ref2, "strided in place")


def test_diff_requirement(torch):
    from sparkts import UnivariateTimeSeries as uts
    from sparkts.errors import IllegalArgumentException
    with pytest.raises(IllegalArgumentException, match="starting index cannot be less than lag"):
        uts.differencesAtLag(dev(torch, np.arange(10.0)), 3, startIndex=2)


def test_diff_reference_kat(torch):
    # T/UnivariateTimeSeriesSuite.scala:112-126
    from mt19937 import MersenneTwister
    from sparkts import UnivariateTimeSeries as uts
    rand = MersenneTwister(10)
    s = np.array([rand.next_gaussian() for _ in range(100)])
    d = host(uts.differencesAtLag(dev(torch, s), 5))
    assert d[10] == s[10] - s[5] and d[99] == s[99] - s[94]


@pytest.mark.parametrize("p,inc", [(0, True), (1, False), (2, True), (2, False), (10, False), (10, True)])
def test_lag_matrix(torch, p, inc):
    from sparkts import UnivariateTimeSeries as uts
    rng = np.random.default_rng(p)
    x = rng.standard_normal((7, 300))
    got = host(uts.lag(dev(torch, x), p, inc))
    ref = np.array([oracle.lag(r, p, inc) for r in x])
    assert_bits(got, ref)


def test_lag_kat(torch):
    from sparkts import UnivariateTimeSeries as uts
    v = dev(torch, [1.0, 2.0, 3.0, 4.0, 5.0])
    assert_bits(host(uts.lag(v, 2, True)), [[3.0, 2.0, 1.0], [4.0, 3.0, 2.0], [5.0, 4.0, 3.0]])
    assert_bits(host(uts.lag(v, 2, False)), [[2.0, 1.0], [3.0, 2.0], [4.0, 3.0]])


@pytest.mark.parametrize("method", ["nearest", "next"])
def test_fill_lag_matrix_fused(torch, method):
    from sparkts import _native
    S, T, p = 5, 9000, 10
    x = oracle.gen_panel(5, S, T, 0.3)
    x[:, 1] = 1.0
    xd = dev(torch, x)
    filled = torch.empty_like(xd)
    lm = torch.empty((S, p, T - p), dtype=torch.float64, device="cuda:0")
    from sparkts import UnivariateTimeSeries as uts
    assert _native.lib().sts_fill_lag_matrix(xd.data_ptr(), filled.data_ptr(), lm.data_ptr(), S, T, T, T,
                                             uts.fill_method_code(method), p, 0, None, None) == 0
    rf, _ = oracle.panel_fill(x, method)
    assert_bits(host(filled), rf)
    ref = np.array([oracle.lag(r, p, False) for r in rf])      # (S, rows, cols)
    assert_bits(host(lm).transpose(0, 2, 1), ref)


# ---------------- EWMA (a9, a10): bit-exact ----------------

def test_ewma_kats(torch):
    # T/models/EWMASuite.scala:22-51
    from sparkts.models import EWMAModel
    orig = dev(torch, np.arange(1, 11, dtype=np.float64))
    for s, last in ((0.2, 6.54), (0.6, 9.33)):
        out = torch.zeros_like(orig)
        EWMAModel(s).addTimeDependentEffects(orig, out)
        o = host(out)
        assert o[0] == 1.0 and o[1] == s * 2.0 + (1 - s) * o[0]
        assert round(o[-1] * 100) / 100 == last
    sm = dev(torch, [1.0, 1.2, 1.56, 2.05, 2.64, 3.31, 4.05, 4.84, 5.67, 6.54])
    o = torch.zeros_like(sm)
    EWMAModel(0.2).removeTimeDependentEffects(sm, o)
    assert int(host(o)[-1]) == 10


def test_ewma_panels(torch):
    from sparkts.models import EWMAModel
    from sparkts.errors import NullPointerException
    rng = np.random.default_rng(7)
    for S, T in [(1, 1), (3, 31), (64, 33), (130, 390), (5, 4000)]:
        x = rng.standard_normal((S, T)) + 10
        s = rng.uniform(0.05, 0.95, S)
        xd = dev(torch, x)
        out = torch.empty_like(xd)
        EWMAModel(dev(torch, s)).addTimeDependentEffects(xd, out)
        assert_bits(host(out), np.array([oracle.ewma_add(r, v) for r, v in zip(x, s)]), "add")
        EWMAModel(dev(torch, s)).removeTimeDependentEffects(xd, out)
        assert_bits(host(out), np.array([oracle.ewma_remove(r, v) for r, v in zip(x, s)]), "remove")
        # in place: add is safe; remove reads overwritten values (reference aliasing)
        ip = dev(torch, x)
        EWMAModel(dev(torch, s)).removeTimeDependentEffects(ip, ip)
        ref = []
        for r, v in zip(x, s):
            rr = r.copy(); oracle.ewma_remove(rr, v, dest=rr); ref.append(rr)
        assert_bits(host(ip), np.array(ref), "remove in place")
    with pytest.raises(NullPointerException):
        EWMAModel(0.2).removeTimeDependentEffects(dev(torch, [1.0, 2.0]))


# ---------------- EWMA.fitModel: bit-exact ----------------
# Every sse / gradient evaluation is the reference's sequential loop, so the device
# optimizer takes the oracle's (commons-math3 restatement's) exact path: smoothing values
# and statuses are compared BIT-EXACT.

OIL = [446.7, 454.5, 455.7, 423.6, 456.3, 440.6, 425.3, 485.1, 506.0, 526.8, 514.3, 494.2]


def test_ewma_fit_oil_kat(torch):
    # T/models/EWMASuite.scala:54-63
    from sparkts.models import EWMA
    m = EWMA.fitModel(dev(torch, OIL))
    assert int(m.smoothing * 100.0) == 89
    st, ref, _ = oracle.ewma_fit(OIL)
    assert_bits(np.array([m.smoothing]), np.array([ref]), "oil")
    mh = EWMA.fitModel(np.array(OIL))          # host-staging (JNI) path
    assert_bits(np.array([mh.smoothing]), np.array([ref]), "oil host")


@pytest.mark.parametrize("T", [2, 3, 12, 63, 64, 65, 390, 1000])
def test_ewma_fit_panels(torch, T):
    from sparkts.models import EWMA
    rng = np.random.default_rng(T)
    S = 70   # three waves of 32 series, the last one partial
    x = np.cumsum(rng.standard_normal((S, T)), axis=1) + 100 + rng.uniform(-5, 5, (S, 1))
    x[5] = 3.0                                  # constant series
    x[6] = rng.standard_normal(T)               # white noise
    err = torch.zeros(S, dtype=torch.int32, device="cuda:0")
    m = EWMA.fitModel(dev(torch, x), errors=err)
    ref_s, ref_err = oracle.panel_ewma_fit(x, threads=8)
    assert np.array_equal(host(err), ref_err)
    assert_bits(host(m.smoothing), ref_s, "EWMA.fitModel T=%d" % T)


def test_ewma_fit_nan_and_short(torch):
    from sparkts.models import EWMA
    from sparkts.errors import TooManyEvaluationsException
    x = np.cumsum(np.random.default_rng(1).standard_normal((40, 50)), axis=1)
    x[3, 0] = NaN
    x[17, 49] = NaN
    x[20, 25] = NaN
    err = torch.zeros(40, dtype=torch.int32, device="cuda:0")
    m = EWMA.fitModel(dev(torch, x), errors=err)
    ref_s, ref_err = oracle.panel_ewma_fit(x, threads=8)
    assert np.array_equal(host(err), ref_err)
    assert set(np.flatnonzero(ref_err)) == {3, 17, 20}
    assert_bits(host(m.smoothing), ref_s, "nan panel")
    with pytest.raises(TooManyEvaluationsException):
        EWMA.fitModel(dev(torch, x))
    # T = 1: sse = 0 everywhere, the optimizer stops at its start point
    one = EWMA.fitModel(dev(torch, [5.0]))
    assert one.smoothing == oracle.ewma_fit([5.0])[1]


def test_ewma_sse_gradient(torch):
    from sparkts.models import EWMAModel
    from sparkts.models.EWMA import gradient, sse
    rng = np.random.default_rng(11)
    for S, T in [(1, 1), (33, 2), (64, 390), (5, 3000)]:
        x = rng.standard_normal((S, T)) + 10
        s = rng.uniform(0.05, 1.5, S)
        xd = dev(torch, x)
        f = host(sse(EWMAModel(dev(torch, s)), xd))
        g = host(gradient(EWMAModel(dev(torch, s)), xd))
        assert_bits(f, np.array([oracle.ewma_sse(r, v) for r, v in zip(x, s)]), "sse")
        assert_bits(g, np.array([oracle.ewma_gradient(r, v) for r, v in zip(x, s)]), "gradient")


# ---------------- AR (a11-a13) ----------------

def test_ar_fit_reference_suite(torch):
    # T/models/AutoregressionSuite.scala:25-42, inputs from MersenneTwister(10)
    from mt19937 import MersenneTwister
    from sparkts.models import Autoregression
    for coefs, tol_c in (([0.2], 0.07), ([0.2, 0.3], 0.15)):
        rand = MersenneTwister(10)
        ts = oracle.ar_add(np.array([rand.next_gaussian() for _ in range(5000)]), 1.5, coefs, inplace=True)
        m = Autoregression.fitModel(dev(torch, ts), len(coefs))
        rc, rcoef = oracle.ar_fit(ts, len(coefs))
        assert abs(m.c - 1.5) < tol_c
        got = host(m.coefficients)
        for g, want in zip(got, coefs):
            assert abs(g - want) < 0.03
        assert_rel([m.c, *got], [rc, *rcoef])


@pytest.mark.parametrize("p", [1, 2, 5, 8, 16, 17, 31])
@pytest.mark.parametrize("no_intercept", [False, True])
def test_ar_fit_panels(torch, p, no_intercept):
    from sparkts.models import Autoregression
    S, T = 24, 2520
    x = oracle.gen_ar_panel(4, S, T, min(p, 5))
    if p > 5:
        x = x + 0.01 * np.sin(np.arange(T))[None, :]
    m = Autoregression.fitModel(dev(torch, x), p, no_intercept)
    rc = np.empty(S); rcoef = np.empty((S, p))
    for s in range(S):
        rc[s], rcoef[s] = oracle.ar_fit(x[s], p, no_intercept)
    assert_rel(host(m.coefficients), rcoef, what="coef")
    if not no_intercept:
        assert_rel(host(m.c), rc, what="c")


@pytest.mark.parametrize("p", [1, 3, 8])
def test_ar_fit_register_path_shapes(torch, p):
    # the register-resident kernel (p <= 8, T <= 2560): ragged last chunk, T at the chunk
    # edges, both intercept modes, fused remove bit-exact given the fitted model
    from sparkts.models import Autoregression
    for T in (2 * p + 1, 64, 65, 127, 1000, 2559, 2560):
        x = oracle.gen_ar_panel(7, 6, T, min(p, 5)) + 0.01 * np.sin(np.arange(T))[None, :]
        for no_int in (False, True):
            m = Autoregression.fitModel(dev(torch, x), p, no_int)
            rc = np.empty(6); rcoef = np.empty((6, p))
            for s in range(6):
                rc[s], rcoef[s] = oracle.ar_fit(x[s], p, no_int)
            assert_rel(host(m.coefficients), rcoef, what="coef T=%d p=%d" % (T, p))
            if not no_int:
                assert_rel(host(m.c), rc, what="c T=%d p=%d" % (T, p))
        m, resid = Autoregression.fitModelAndRemove(dev(torch, x), p)
        c, coef = host(m.c), host(m.coefficients)
        assert_bits(host(resid), np.array([oracle.ar_remove(x[s], c[s], coef[s]) for s in range(6)]),
                    "fused remove T=%d p=%d" % (T, p))


@pytest.mark.parametrize("p", [1, 5, 8])
def test_ar_fit_register_path_edges(torch, p):
    # the register kernel at lane-block edges (B = 8 .. 40), an odd series count, NaN in
    # the first and the last lane blocks (NaN model, the others unaffected), the fused remove
    # bit-exact given the fitted model
    from sparkts.models import Autoregression
    S = 7
    for T in (514, 1024, 1026, 1536, 1538, 2048, 2050, 2520, 2558, 2560):
        x = oracle.gen_ar_panel(12, S, T, min(p, 5)) + 0.01 * np.sin(np.arange(T))[None, :]
        x[2, T - 3] = NaN
        x[4, 5] = NaN
        m, resid = Autoregression.fitModelAndRemove(dev(torch, x), p)
        c, coef = host(m.c), host(m.coefficients)
        ok = [0, 1, 3, 5, 6]
        rc = np.empty(S); rcoef = np.empty((S, p))
        for s in ok:
            rc[s], rcoef[s] = oracle.ar_fit(x[s], p)
        assert_rel(coef[ok], rcoef[ok], what="coef T=%d p=%d" % (T, p))
        assert_rel(c[ok], rc[ok], what="c T=%d p=%d" % (T, p))
        assert np.all(np.isnan(c[[2, 4]])) and np.all(np.isnan(coef[[2, 4]]))
        assert_bits(host(resid)[ok], np.array([oracle.ar_remove(x[s], c[s], coef[s]) for s in ok]),
                    "fused remove T=%d p=%d" % (T, p))


def test_ar_fit_register_path_matches_staged_on_nan(torch, monkeypatch):
    # NaN anywhere -> NaN model, same as the LDS-staged kernel (forced on the A/B build)
    from sparkts import _native
    from sparkts.models import Autoregression
    x = oracle.gen_ar_panel(8, 4, 2520, 5)
    x[1, 700] = NaN
    got = Autoregression.fitModel(dev(torch, x), 5)
    monkeypatch.setattr(_native, "_lib", _native.load_variant(_native.AB_LIB_PATH))
    monkeypatch.setenv("STS_AR_STAGED", "1")
    ref = Autoregression.fitModel(dev(torch, x), 5)
    assert np.isnan(host(got.c)[1]) and np.isnan(host(ref.c)[1])
    assert np.array_equal(np.isnan(host(got.coefficients)), np.isnan(host(ref.coefficients)))
    ok = [0, 2, 3]
    assert_rel(host(got.coefficients)[ok], host(ref.coefficients)[ok])


def test_ar_fit_long_series_unstaged(torch):
    from sparkts.models import Autoregression
    x = oracle.gen_ar_panel(9, 4, 10000, 5)
    m = Autoregression.fitModel(dev(torch, x), 5)
    for s in range(4):
        rc, rcoef = oracle.ar_fit(x[s], 5)
        assert_rel(host(m.coefficients)[s], rcoef)
        assert_rel(host(m.c)[s], rc)


def test_ar_not_enough_data(torch):
    from sparkts.models import Autoregression
    from sparkts.errors import MathIllegalArgumentException
    with pytest.raises(MathIllegalArgumentException):
        Autoregression.fitModel(dev(torch, [1.0, 2.0, 3.0, 4.0]), 2)


def test_ar_remove_add_bit_exact(torch):
    from sparkts.models import ARModel
    rng = np.random.default_rng(11)
    for p in (1, 2, 5, 16, 33):
        S, T = 9, 1000
        x = rng.standard_normal((S, T))
        c = rng.standard_normal(S)
        coef = rng.uniform(-0.3, 0.3, (S, p))
        m = ARModel(dev(torch, c), dev(torch, coef))
        xd = dev(torch, x)
        rem = host(m.removeTimeDependentEffects(xd))
        add = host(m.addTimeDependentEffects(xd))
        assert_bits(rem, np.array([oracle.ar_remove(x[s], c[s], coef[s]) for s in range(S)]), "remove p=%d" % p)
        assert_bits(add, np.array([oracle.ar_add(x[s], c[s], coef[s]) for s in range(S)]), "add p=%d" % p)
        # in-place remove reads overwritten values; in-place add equals out-of-place
        ip = dev(torch, x)
        m.removeTimeDependentEffects(ip, ip)
        ref = []
        for s in range(S):
            r = x[s].copy()
            for i in range(T):
                v = r[i] - c[s]
                for j in range(min(p, i)):
                    v -= r[i - j - 1] * coef[s, j]
                r[i] = v
            ref.append(r)
        assert_bits(host(ip), np.array(ref), "remove in place p=%d" % p)


def test_ar_add_remove_round_trip(torch):
    # T/models/AutoregressionSuite.scala:44-51
    from sparkts.models import ARModel
    ts = np.random.default_rng(0).random(1000)
    m = ARModel(1.5, [0.2, 0.3])
    added = m.addTimeDependentEffects(dev(torch, ts))
    removed = host(m.removeTimeDependentEffects(added))
    assert np.all(np.abs(ts - removed) < 1e-3)


def test_ar_fit_remove_fused(torch):
    from sparkts.models import Autoregression
    S, T, p = 40, 2520, 5
    x = oracle.gen_ar_panel(4, S, T, p)
    m, resid = Autoregression.fitModelAndRemove(dev(torch, x), p)
    c, coef = host(m.c), host(m.coefficients)
    ref_resid = np.array([oracle.ar_remove(x[s], c[s], coef[s]) for s in range(S)])
    assert_bits(host(resid), ref_resid)   # bit-exact given the fitted model
    _, rc, rcoef = oracle.panel_ar_fit_remove(x, p)
    assert_rel(coef, rcoef)
    assert_rel(c, rc)


# ---------------- C2 fused pipeline: bit-exact ----------------

@pytest.mark.parametrize("lag", [1, 3])
def test_fill_diff_ewma(torch, lag):
    from sparkts import _native
    S, T = 300, 390
    x = oracle.gen_panel(2, S, T, 0.05)
    x[3, :40] = NaN
    s = np.full(S, 0.2)
    xd = dev(torch, x)
    out = torch.empty_like(xd)
    assert _native.lib().sts_fill_diff_ewma(xd.data_ptr(), out.data_ptr(), S, T, T, T, 3, lag,
                                            dev(torch, s).data_ptr(), None, None) == 0
    ref = []
    for r in x:
        f = oracle.fill_previous(r)
        d = oracle.differences_at_lag(f, lag)
        ref.append(oracle.ewma_add(d, 0.2))
    assert_bits(host(out), np.array(ref))


# ---------------- generator ----------------

def test_generator_matches_cpu(torch):
    from sparkts import _native
    lib = _native.lib()
    S, T = 37, 1001
    out = torch.empty((S, T), dtype=torch.float64, device="cuda:0")
    assert lib.sts_gen_panel(out.data_ptr(), 5, S, T, T, 123, 0.3, None) == 0
    assert_bits(host(out), oracle.gen_panel(123, S, T, 0.3, s0=5))
    c = torch.empty(S, dtype=torch.float64, device="cuda:0")
    phi = torch.empty((S, 5), dtype=torch.float64, device="cuda:0")
    assert lib.sts_gen_ar_panel(out.data_ptr(), c.data_ptr(), phi.data_ptr(), 5, S, T, T, 77, 5, None) == 0
    assert_bits(host(out), oracle.gen_ar_panel(77, S, T, 5, s0=5))


# ---------------- seriesStats / removeInstantsWithNaNs / toInstants ----------------

def test_series_stats(torch):
    from sparkts.timeseriesrdd import TimeSeriesRDD
    rng = np.random.default_rng(21)
    for S, T in [(1, 1), (3, 2), (33, 64), (70, 390), (5, 5000)]:
        x = rng.standard_normal((S, T)) * 10 + 3
        if S > 2:
            x[1, T // 2] = NaN
            x[2, :] = -0.0
            x[2, 0] = 0.0
        if S > 10 and T > 3:
            x[7, 1] = np.inf
            x[8, 2] = -np.inf
        st = TimeSeriesRDD(None, None, dev(torch, x)).seriesStats()
        ref = np.array([oracle.stat_counter(r)[1:] for r in x])
        assert st.count() == T
        assert_bits(host(st.mean()), ref[:, 0], "mean")
        assert_bits(host(st.stats[:, 1]), ref[:, 1], "m2")
        assert_bits(host(st.max()), ref[:, 2], "max")
        assert_bits(host(st.min()), ref[:, 3], "min")


def test_series_stats_extremes(torch):
    # the fast Welford division (stats_fast_kernel) against the oracle where its range check
    # sends lanes to the library division: huge / tiny / subnormal deltas, zeros, infinities
    from sparkts.timeseriesrdd import TimeSeriesRDD
    rng = np.random.default_rng(22)
    S, T = 130, 300
    x = rng.standard_normal((S, T)) * 10.0 ** rng.integers(-300, 300, size=(S, 1))
    x[0] = 1e-310 * rng.standard_normal(T)                     # subnormals
    x[1] = 7.0                                                 # delta = 0 from step 2 on
    x[2] = rng.choice([1e300, -1e300, 1e-300, 0.0, -0.0], T)   # mixed extreme magnitudes
    x[3, ::7] = np.inf
    x[4, 5] = -np.inf
    x[5, 9] = NaN
    x[6] = rng.standard_normal(T) * 1e200
    x[6, ::3] *= 1e-250
    x[7] = 2.0 ** 700 * (1 + rng.random(T))                    # at the range bound
    x[8] = 2.0 ** -900 * (1 + rng.random(T))
    st = TimeSeriesRDD(None, None, dev(torch, x)).seriesStats()
    ref = np.array([oracle.stat_counter(r)[1:] for r in x])
    for c, name in enumerate(["mean", "m2", "max", "min"]):
        assert_bits(host(st.stats[:, c]), ref[:, c], name)


@pytest.mark.parametrize("T", [1, 2, 15, 16, 17, 63, 64, 65, 390])
def test_stats_and_ewma_row_alignments(torch, T):
    # the line-aligned chunks of stats_fast_kernel / ewma_fit_kernel (a row's chunks start on
    # the 128-B lines of its own addresses): strided views whose rows start at every offset
    # within a line, NaN in the padding (a staged pad step would show), and the last row ending
    # on the allocation's last element -- bit for bit against the restatements
    from sparkts.timeseriesrdd import TimeSeriesRDD
    from sparkts.models import EWMA, EWMAModel
    from sparkts.models.EWMA import gradient, sse
    rng = np.random.default_rng(1000 + T)
    S = 70   # three EWMA waves of 32 series (the last partial), two seriesStats waves of 64
    for pad in [0, 1, 3, 7, 13, 16, 29]:
        ld = T + pad
        x = np.cumsum(rng.standard_normal((S, T)), axis=1) + 50 + rng.uniform(-5, 5, (S, 1))
        flat = torch.full((S * ld,), NaN, dtype=torch.float64, device="cuda:0")
        v = flat.view(S, ld)[:, pad:]
        v.copy_(torch.as_tensor(x))
        st = TimeSeriesRDD(None, None, v).seriesStats()
        ref = np.array([oracle.stat_counter(r)[1:] for r in x])
        for c, name in enumerate(["mean", "m2", "max", "min"]):
            assert_bits(host(st.stats[:, c]), ref[:, c], "stats %s T=%d pad=%d" % (name, T, pad))
        err = torch.zeros(S, dtype=torch.int32, device="cuda:0")
        m = EWMA.fitModel(v, errors=err)
        ref_s, ref_err = oracle.panel_ewma_fit(x, threads=8)
        assert np.array_equal(host(err), ref_err)
        assert_bits(host(m.smoothing), ref_s, "EWMA.fitModel T=%d pad=%d" % (T, pad))
        sm = rng.uniform(0.05, 1.5, S)
        f = host(sse(EWMAModel(dev(torch, sm)), v))
        g = host(gradient(EWMAModel(dev(torch, sm)), v))
        assert_bits(f, np.array([oracle.ewma_sse(r, q) for r, q in zip(x, sm)]), "sse T=%d pad=%d" % (T, pad))
        assert_bits(g, np.array([oracle.ewma_gradient(r, q) for r, q in zip(x, sm)]), "gradient T=%d pad=%d" % (T, pad))


def test_remove_instants_with_nans_kat(torch):
    # T/TimeSeriesRDDSuite.scala:210-231
    from sparkts.timeseriesrdd import TimeSeriesRDD
    x = np.array([[1.0, 2.0, 3.0, 4.0], [5.0, NaN, 7.0, 8.0], [9.0, 10.0, 11.0, NaN]])
    idx = np.array(["2015-04-09", "2015-04-10", "2015-04-11", "2015-04-12"])
    r = TimeSeriesRDD(idx, ["1.0", "5.0", "9.0"], dev(torch, x)).removeInstantsWithNaNs()
    assert list(r.index) == ["2015-04-09", "2015-04-11"]
    assert_bits(host(r.data), np.array([[1.0, 3.0], [5.0, 7.0], [9.0, 11.0]]), "kat")


@pytest.mark.parametrize("S,T,p", [(1, 1, 0.0), (5, 100, 0.01), (64, 5000, 0.0005), (300, 20000, 0.00005),
                                   (4, 9000, 1.0), (1, 2, 0.3), (130, 390, 0.001), (65, 1023, 0.002),
                                   (3, 514, 0.05)])
def test_remove_instants_with_nans_panels(torch, S, T, p):
    from sparkts.timeseriesrdd import TimeSeriesRDD
    rng = np.random.default_rng(S * 7 + T)
    x = rng.standard_normal((S, T))
    x[rng.random((S, T)) < p] = NaN
    r = TimeSeriesRDD(None, None, dev(torch, x)).removeInstantsWithNaNs()
    ref, active = oracle.remove_instants_with_nans(x)
    assert np.array_equal(r.index, active)
    assert_bits(host(r.data).reshape(ref.shape), ref, "removeInstantsWithNaNs")


def test_to_instants(torch):
    # T/TimeSeriesRDDSuite.scala:71-89
    from sparkts.timeseriesrdd import TimeSeriesRDD
    series = np.array([np.arange(v, v + 4, dtype=np.float64) for v in range(0, 20, 4)])
    _, inst = TimeSeriesRDD(None, list("abcde"), dev(torch, series)).toInstants()
    for t in range(4):
        assert_bits(host(inst[t]), np.arange(t, 20, 4, dtype=np.float64), "kat")
    rng = np.random.default_rng(5)
    # odd shapes take the 8-B kernel; even ones the 16-B kernel (ragged last tiles both ways)
    for S, T in [(1, 7), (65, 63), (130, 1000), (3, 70000), (2, 2), (64, 64), (128, 390), (66, 130), (200, 4098)]:
        x = rng.standard_normal((S, T))
        _, inst = TimeSeriesRDD(None, None, dev(torch, x)).toInstants()
        assert_bits(host(inst), oracle.to_instants(x), "toInstants %dx%d" % (S, T))


def test_to_row_matrices(torch):
    # S/TimeSeriesRDD.scala:385-414: toInstants rows; IndexedRowMatrix row i = instant i
    from sparkts.errors import UnsupportedOperationException
    from sparkts.timeseriesrdd import TimeSeriesRDD
    x = np.random.default_rng(6).standard_normal((9, 33))
    days = np.datetime64("2015-04-09") + np.arange(33)
    rdd = TimeSeriesRDD(days.astype(str), None, dev(torch, x))
    assert_bits(host(rdd.toRowMatrix()), x.T, "toRowMatrix")
    ri, rows = rdd.toIndexedRowMatrix()
    assert np.array_equal(host(ri), np.arange(33)) and np.array_equal(host(rows), x.T)
    days = np.array(["2015-04-09", "2015-04-10", "2015-04-12"])
    with pytest.raises(UnsupportedOperationException, match="only supported for uniform indices"):
        TimeSeriesRDD(days, None, dev(torch, x[:, :3])).toIndexedRowMatrix()


# ---------------- ingest / egress formats: bit-exact ----------------

def test_wire_decode_encode_round_trip(torch):
    from sparkts import io as sio
    rng = np.random.default_rng(31)
    for S, T, aligned in [(1, 1, False), (3, 7, False), (40, 390, False), (5, 5000, False), (70, 390, True),
                          (9, 4096, True), (6, 4097, True), (65, 33, False)]:
        keys = ["k%07d" % i for i in range(S)] if aligned else ["k%d" % i + "é" * (i % 3) for i in range(S)]
        x = rng.standard_normal((S, T)) * 1e3
        x.ravel()[rng.random(S * T) < 0.05] = NaN
        if T > 2:
            x[0, 1] = -0.0
            x[0, 2] = np.inf
        data = oracle.wire_records(keys, x)
        rdd = sio.timeSeriesRDDFromWire(None, data)
        assert rdd.keys == keys
        assert_bits(host(rdd.data), x, "wire decode %dx%d" % (S, T))
        assert sio.toWire(rdd) == data                       # KeyAndSeriesToBytes, byte for byte


@pytest.mark.parametrize("parts", [1, 4, 13])
def test_observations_to_panel(torch, parts):
    # S/TimeSeriesRDD.scala:493-542 with the input RDD in `parts` partitions: records in the
    # reference's order (hash partition of the key, then String.compareTo)
    from sparkts import io as sio
    rng = np.random.default_rng(8)
    idx = np.arange(0, 5000, 5, dtype=np.int64)             # 1000 instants
    n = 20000
    keys = ["s%03d" % k for k in rng.integers(0, 150, n)]
    keys[::97] = ["\U0001F600x", "\uffffy", "\u00e9"] * (len(keys[::97]) // 3) + ["z"] * (len(keys[::97]) % 3)
    ts = rng.integers(0, 5100, n).astype(np.int64)          # some off-grid / past the end: dropped
    ts[::3] = ts[::3] // 5 * 5                              # many on the grid, duplicates included
    vals = rng.standard_normal(n)
    rdd = sio.timeSeriesRDDFromObservations(idx, keys, ts, vals, numPartitions=parts)
    ref_keys, ref = oracle.observations_to_panel(idx, keys, ts, vals, num_partitions=parts)
    assert rdd.keys == ref_keys
    assert_bits(host(rdd.data), ref, "observations")


def test_csv_round_trip(torch, tmp_path):
    from sparkts import io as sio
    from sparkts.timeseriesrdd import TimeSeriesRDD
    rng = np.random.default_rng(9)
    x = rng.standard_normal((12, 50)) * 10.0 ** rng.integers(-8, 9, (12, 50))
    x[3, 4] = NaN
    x[5, 6] = -np.inf
    rdd = TimeSeriesRDD("uniform(2015-04-09,50,1 day)", ["key%d" % i for i in range(12)], dev(torch, x))
    sio.saveAsCsv(rdd, str(tmp_path / "ts"))
    back = sio.timeSeriesRDDFromCsv(str(tmp_path / "ts"))
    assert back.keys == rdd.keys and back.index == rdd.index
    assert_bits(host(back.data), x, "csv round trip")


# ---------------- ARIMA(p, d, 0): differencesOfOrderD + AR fit ----------------

@pytest.mark.parametrize("p,d,inc", [(1, 1, True), (2, 1, False), (3, 2, True), (5, 3, True), (9, 1, True)])
def test_arima_ar_path(torch, p, d, inc):
    from sparkts.models import ARIMA
    rng = np.random.default_rng(p * 10 + d)
    S, T = 37, 800
    x = np.empty((S, T))
    for s in range(S):
        e = rng.standard_normal(T)
        y = oracle.ar_add(e, 0.3, [0.5 / p] * p, inplace=True)   # stationary AR(p)
        for _ in range(d):
            y = np.cumsum(y)                                     # integrate d times
        x[s] = y + 50.0
    m = ARIMA.fitModel(p, d, 0, dev(torch, x), includeIntercept=inc)
    got = host(m.coefficients)
    ref = []
    for row in x:
        diffed = oracle.differences_of_order_d(row, d)[d:]
        c, coef = oracle.ar_fit(diffed, p, no_intercept=not inc)
        ref.append(([c] if inc else []) + list(coef))
    assert_rel(got, np.array(ref), what="ARIMA(%d,%d,0)" % (p, d))
    from sparkts.errors import UnsupportedOperationException
    with pytest.raises(UnsupportedOperationException):
        ARIMA.fitModel(1, 1, 2, dev(torch, x))
