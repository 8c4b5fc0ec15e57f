"""CPU check of the EWMA.fitModel optimizer state machine.

The device kernel (spark-timeseries_amd/csrc/sts_ewma_fit.hip) runs the commons-math3
optimizer as a resumable per-series state machine (csrc/sts_ewma_opt.hpp).  Here the SAME
header is compiled for the host (tests/native/ewma_sm_harness.cpp) and driven with the
oracle's sse / gradient; status, smoothing bits and commons-math3's evaluation count must
equal the oracle's straight-line restatement (orc_ewma_fit) for every series.  The GPU
parity tests then only have to show that the device evaluations are bit-exact.
"""
import os
import shutil
import subprocess

import numpy as np
import pytest

import oracle

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HARNESS = os.path.join(ROOT, "tests", "native", "ewma_sm_harness.cpp")
OIL = [446.7, 454.5, 455.7, 423.6, 456.3, 440.6, 425.3, 485.1, 506.0, 526.8, 514.3, 494.2]


@pytest.fixture(scope="module")
def harness(tmp_path_factory):
    gxx = shutil.which("g++")
    if gxx is None:
        pytest.skip("g++ not available")
    oracle.lib()
    out = str(tmp_path_factory.mktemp("ewma") / "ewma_sm")
    lib_dir = os.path.join(ROOT, "oracle", "_build")
    subprocess.check_call([gxx, "-O2", "-std=c++17", "-ffp-contract=off",
                           "-I", os.path.join(ROOT, "include"),
                           "-I", os.path.join(ROOT, "spark-timeseries_amd", "csrc"),
                           HARNESS, "-L", lib_dir, "-lsts_oracle", "-Wl,-rpath," + lib_dir, "-o", out])
    return out


def run(harness, x):
    x = np.ascontiguousarray(x, dtype=np.float64)
    inp = "%d %d\n" % x.shape + " ".join("%x" % v for v in x.view(np.uint64).ravel())
    out = subprocess.run([harness], input=inp, capture_output=True, text=True, check=True).stdout.split()
    rows = np.array(out, dtype=object).reshape(-1, 4)
    st = rows[:, 0].astype(int)
    sm = np.array([int(b, 16) for b in rows[:, 1]], dtype=np.uint64).view(np.float64)
    return st, sm, rows[:, 2].astype(int), rows[:, 3].astype(int)


def check_against_oracle(harness, x):
    st, sm, ev, passes = run(harness, x)
    for i in range(x.shape[0]):
        rst, rsm, rev = oracle.ewma_fit(x[i])
        assert st[i] == rst, (i, st[i], rst)
        assert ev[i] == rev, (i, ev[i], rev)
        if rst == oracle.OK:
            assert sm[i].view(np.uint64) == np.float64(rsm).view(np.uint64), (i, sm[i], rsm)
    return passes


def test_oil(harness):
    passes = check_against_oracle(harness, np.array([OIL]))
    st, s, ev = oracle.ewma_fit(OIL)
    assert int(s * 100.0) == 89 and passes[0] <= ev


@pytest.mark.parametrize("T", [1, 2, 3, 12, 50, 390])
def test_random_walks(harness, T):
    rng = np.random.default_rng(T)
    x = np.cumsum(rng.standard_normal((60, T)), axis=1) + 100
    x[1] = 3.0                                       # constant
    x[2] = rng.standard_normal(T) * 1e-3             # tiny white noise
    x[3] = np.arange(T, dtype=np.float64) * 1e6      # trend, large values
    passes = check_against_oracle(harness, x)
    assert passes.max() < 1000


def test_nan_series_exhausts_evaluations(harness):
    x = np.ones((1, 20))
    x[0, 7] = np.nan
    st, _, ev, _ = run(harness, x)
    assert st[0] == oracle.ERR_TOO_MANY_EVALUATIONS and ev[0] == 10001
    assert oracle.ewma_fit(x[0])[0] == oracle.ERR_TOO_MANY_EVALUATIONS
