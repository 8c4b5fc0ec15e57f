"""GARCH(1,1) and AR(1)+GARCH(1,1) (S/models/GARCH.scala).

CPU (no GPU):
* the oracle against the reference's own GARCHSuite (T/models/GARCHSuite.scala), on inputs
  regenerated with the commons-math3 MersenneTwister restatement;
* fdlibm's log (StrictMath.log, used by oracle and device) within 1 ulp of math.log;
* the device optimizer state machine (csrc/sts_garch_opt.hpp compiled for the host) against
  the oracle's straight-line restatement: status, parameter bits, evaluation count.
GPU: the HIP path through the C ABI against the oracle -- logLikelihood / gradient, the
fitted parameters and the remove / add effects bit-exact; ARGARCH's AR stage within 1e-10
(the Householder-QR bar of a11) and its GARCH stage bit-exact given the residuals.
"""
import math
import os
import shutil
import subprocess

import numpy as np
import pytest

import oracle
from mt19937 import MersenneTwister

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HARNESS = os.path.join(ROOT, "tests", "native", "garch_sm_harness.cpp")
RTOL = 1e-10


def garch_sample(omega, alpha, beta, n, rand):
    """GARCHModel.sampleWithVariances (S/models/GARCH.scala:161-173)."""
    ts = np.zeros(n)
    v = omega / (1 - alpha - beta)
    eta = math.sqrt(v) * rand.next_gaussian()
    for i in range(1, n):
        v = omega + beta * v + alpha * eta * eta
        eta = math.sqrt(v) * rand.next_gaussian()
        ts[i] = eta
    return ts


def argarch_sample(c, phi, omega, alpha, beta, n, rand):
    """ARGARCHModel.sampleWithVariances (S/models/GARCH.scala:236-248)."""
    ts = np.zeros(n)
    v = omega / (1 - alpha - beta)
    eta = math.sqrt(v) * rand.next_gaussian()
    for i in range(1, n):
        v = omega + beta * v + alpha * eta * eta
        eta = math.sqrt(v) * rand.next_gaussian()
        ts[i] = c + phi * ts[i - 1] + eta
    return ts


# T/models/GARCHSuite.scala:73-94 ("fit model 2"): 39 repetitions of an 8-value pattern
FIT2 = np.tile([0.1, -0.2, -0.1, 0.1, 0.0, -0.01, 0.00, -0.1], 39)


def garch_panel(S, n, seed):
    rows = []
    for s in range(S):
        rand = MersenneTwister(seed + s)
        om, al, be = 0.1 + 0.02 * (s % 5), 0.1 + 0.05 * (s % 4), 0.3 + 0.05 * (s % 3)
        rows.append(garch_sample(om, al, be, n, rand))
    return np.array(rows)


# ---------------- CPU: oracle vs the reference's GARCHSuite ----------------

def test_loglikelihood_kat():
    # T/models/GARCHSuite.scala:23-39
    ts = garch_sample(.2, .3, .4, 10000, MersenneTwister(5))
    right = oracle.garch_loglik(ts, .2, .3, .4)
    w1 = oracle.garch_loglik(ts, .3, .4, .5)
    w2 = oracle.garch_loglik(ts, .25, .35, .45)
    w3 = oracle.garch_loglik(ts, .1, .2, .3)
    assert right > w1 and right > w2 and right > w3 and w2 > w1


def test_gradient_kat():
    # T/models/GARCHSuite.scala:41-55
    ts = garch_sample(.2, .3, .4, 10000, MersenneTwister(5))
    assert (oracle.garch_gradient(ts, .2 + .1, .3 + .05, .4 + .1) < 0).all()
    assert (oracle.garch_gradient(ts, .2 - .1, .3 - .05, .4 - .1) > 0).all()


def test_fit_model_kat():
    # T/models/GARCHSuite.scala:57-72 (one-sided bounds, as written in the suite)
    ts = argarch_sample(0.0, 0.0, 0.3, 0.5, 0.2, 10000, MersenneTwister(5))
    st, (om, al, be), _ = oracle.garch_fit(ts)
    assert st == oracle.OK
    assert om - 0.2 < .1 and al - 0.3 < .02 and be - 0.5 < .02


def test_fit_model_2_runs():
    # T/models/GARCHSuite.scala:73-94 only prints the fitted ARGARCH model
    st, par, ev = oracle.argarch_fit(FIT2)
    assert st == oracle.OK and np.isfinite(par).all() and ev > 0


def test_standardize_and_filter_kat():
    # T/models/GARCHSuite.scala:96-109
    c, phi, om, al, be = 40.0, .4, .2, .3, .4
    ts = argarch_sample(c, phi, om, al, be, 10000, MersenneTwister(5))
    std = oracle.argarch_remove(ts, c, phi, om, al, be)
    filt = oracle.argarch_add(std, c, phi, om, al, be)
    assert (np.abs(filt - ts) < .001).all()


def test_fdlibm_log_within_one_ulp():
    rng = np.random.default_rng(3)
    xs = np.concatenate([rng.random(20000) * 10, np.exp(rng.uniform(-700, 700, 20000)), [1.0, 0.5, 2.0, 1e-310]])
    got = np.array([oracle.fdlibm_log(x) for x in xs])
    ref = np.log(xs)
    ulp = np.abs(got.view(np.int64) - ref.view(np.int64))
    assert ulp.max() <= 1
    assert math.isnan(oracle.fdlibm_log(-1.0)) and oracle.fdlibm_log(0.0) == -math.inf


# ---------------- CPU: device state machine vs oracle ----------------

@pytest.fixture(scope="module")
def harness(tmp_path_factory):
    gxx = shutil.which("g++")
    if gxx is None:
        pytest.skip("g++ not available")
    oracle.lib()
    out = str(tmp_path_factory.mktemp("garch") / "garch_sm")
    lib_dir = os.path.join(ROOT, "oracle", "_build")
    subprocess.check_call([gxx, "-O2", "-std=c++17", "-ffp-contract=off",
                           "-I", os.path.join(ROOT, "include"),
                           "-I", os.path.join(ROOT, "spark-timeseries_amd", "csrc"),
                           HARNESS, "-L", lib_dir, "-lsts_oracle", "-Wl,-rpath," + lib_dir, "-o", out])
    return out


def run_harness(harness, x):
    x = np.ascontiguousarray(x, dtype=np.float64)
    inp = "%d %d\n" % x.shape + " ".join("%x" % v for v in x.view(np.uint64).ravel())
    out = subprocess.run([harness], input=inp, capture_output=True, text=True, check=True).stdout.split()
    rows = np.array(out, dtype=object).reshape(-1, 6)
    st = rows[:, 0].astype(int)
    par = np.array([[int(b, 16) for b in r] for r in rows[:, 1:4]], dtype=np.uint64).view(np.float64)
    return st, par, rows[:, 4].astype(int)


def check_machine(harness, x):
    st, par, ev = run_harness(harness, x)
    for i in range(x.shape[0]):
        rst, rpar, rev = oracle.garch_fit(x[i])
        assert st[i] == rst, (i, st[i], rst)
        assert ev[i] == rev, (i, ev[i], rev)
        if rst == oracle.OK:
            assert np.array_equal(par[i].view(np.uint64), rpar.view(np.uint64)), (i, par[i], rpar)


def test_state_machine_matches_oracle(harness):
    check_machine(harness, garch_panel(12, 600, 100))


def test_state_machine_edge_series(harness):
    x = garch_panel(6, 40, 7)
    x[1, 17] = np.nan                 # NaN: TooManyEvaluations after 10000 evaluations
    x[2] = 0.0                        # constant zero
    x[3] = 1.5                        # constant
    x[4, ::2] *= 50                   # heavy tails
    check_machine(harness, x)
    check_machine(harness, FIT2[None, :])
    check_machine(harness, np.array([[0.3]]))      # n = 1: the initial guess converges


# ---------------- GPU: HIP path vs oracle ----------------

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


def bits_equal(got, ref):
    got = np.ascontiguousarray(got, dtype=np.float64)
    ref = np.ascontiguousarray(ref, dtype=np.float64)
    return got.shape == ref.shape and bool(
        ((got.view(np.uint64) == ref.view(np.uint64)) | (np.isnan(got) & np.isnan(ref))).all())


@pytest.mark.gpu
def test_gpu_loglik_gradient(torch):
    from sparkts.models import GARCHModel
    x = garch_panel(40, 777, 11)
    rng = np.random.default_rng(5)
    om, al, be = rng.uniform(0.05, 0.4, 40), rng.uniform(0.05, 0.4, 40), rng.uniform(0.1, 0.5, 40)
    m = GARCHModel(dev(torch, om), dev(torch, al), dev(torch, be))
    ll = host(m.logLikelihood(dev(torch, x)))
    g = host(m.gradient(dev(torch, x)))
    assert bits_equal(ll, [oracle.garch_loglik(x[s], om[s], al[s], be[s]) for s in range(40)])
    assert bits_equal(g, np.array([oracle.garch_gradient(x[s], om[s], al[s], be[s]) for s in range(40)]))


@pytest.fixture(params=["default", "1", "0"])
def pass_budget(request, monkeypatch):
    """Passes a series runs in garch_fit_kernel before garch_tail_kernel (one wave per series)
    takes it over: 1 sends every series past its first pass to the tail kernel, 0 disables
    the tail phase.  The overrides run on the A/B build (libsts_hip_ab.so); "default" is the
    product library."""
    if request.param != "default":
        ab = request.getfixturevalue("ab_lib")
        ab(STS_GARCH_PASS_BUDGET=request.param)
    return request.param


@pytest.mark.gpu
@pytest.mark.parametrize("S,T", [(1, 10000), (70, 600), (33, 65), (5, 2), (3, 1), (40, 129), (40, 257)])
def test_gpu_garch_fit(torch, S, T, pass_budget):
    from sparkts.models import GARCH
    if S == 1:
        x = argarch_sample(0.0, 0.0, 0.3, 0.5, 0.2, T, MersenneTwister(5))[None, :]   # GARCHSuite "fit model"
    else:
        x = garch_panel(S, T, 21 + S)
    if S == 70:
        x[3, 100] = np.nan
        x[4] = 0.0
    err = torch.zeros(S, dtype=torch.int32, device="cuda:0")
    m = GARCH.fitModel(dev(torch, x), errors=err)
    got = np.stack([host(m.omega), host(m.alpha), host(m.beta)], axis=1)
    rpar, rerr = oracle.panel_garch_fit(x)
    assert np.array_equal(host(err), rerr)
    assert bits_equal(got, rpar)


@pytest.mark.gpu
def test_gpu_garch_fit_raises_like_reference(torch):
    from sparkts.errors import TooManyEvaluationsException
    from sparkts.models import GARCH
    x = garch_panel(3, 100, 1)
    x[1, 5] = np.nan
    with pytest.raises(TooManyEvaluationsException):
        GARCH.fitModel(dev(torch, x))


@pytest.mark.gpu
def test_gpu_argarch_fit(torch, pass_budget):
    from sparkts.models import ARGARCH
    rows = [argarch_sample(1.0 + 0.1 * s, 0.3 - 0.05 * (s % 5), 0.2, 0.3, 0.4, 1500, MersenneTwister(40 + s))
            for s in range(24)]
    x = np.vstack(rows)
    m = ARGARCH.fitModel(dev(torch, x))
    c, phi = host(m.c), host(m.phi)
    rc = np.empty(x.shape[0]); rphi = np.empty(x.shape[0])
    for s in range(x.shape[0]):
        rc[s], co = oracle.ar_fit(x[s], 1, False)
        rphi[s] = co[0]
    assert np.allclose(c, rc, rtol=RTOL, atol=0) and np.allclose(phi, rphi, rtol=RTOL, atol=0)
    # GARCH stage: bit-exact given the device's own (c, phi) residuals
    resid = np.array([oracle.ar_remove(x[s], c[s], [phi[s]]) for s in range(x.shape[0])])
    rpar, rerr = oracle.panel_garch_fit(resid)
    got = np.stack([host(m.omega), host(m.alpha), host(m.beta)], axis=1)
    assert (rerr == 0).all() and bits_equal(got, rpar)


@pytest.mark.gpu
def test_gpu_effects_bit_exact(torch):
    from sparkts.models import ARGARCHModel, GARCHModel
    S, T = 37, 300
    rng = np.random.default_rng(9)
    x = rng.standard_normal((S, T))
    c, phi = rng.uniform(-1, 1, S), rng.uniform(-0.5, 0.5, S)
    om, al, be = rng.uniform(0.05, 0.4, S), rng.uniform(0.05, 0.3, S), rng.uniform(0.1, 0.5, S)
    D = lambda a: dev(torch, a)  # noqa: E731
    g = GARCHModel(D(om), D(al), D(be))
    a = ARGARCHModel(D(c), D(phi), D(om), D(al), D(be))
    out = torch.empty((S, T), dtype=torch.float64, device="cuda:0")
    g.removeTimeDependentEffects(D(x), out)
    assert bits_equal(host(out), [oracle.garch_remove(x[s], om[s], al[s], be[s]) for s in range(S)])
    g.addTimeDependentEffects(D(x), out)
    assert bits_equal(host(out), [oracle.garch_add(x[s], om[s], al[s], be[s]) for s in range(S)])
    a.removeTimeDependentEffects(D(x), out)
    assert bits_equal(host(out), [oracle.argarch_remove(x[s], c[s], phi[s], om[s], al[s], be[s]) for s in range(S)])
    a.addTimeDependentEffects(D(x), out)
    assert bits_equal(host(out), [oracle.argarch_add(x[s], c[s], phi[s], om[s], al[s], be[s]) for s in range(S)])
    # dest eq ts: ARGARCH remove reads the overwritten ts(i - 1), as on the JVM
    ip = D(x)
    a.removeTimeDependentEffects(ip, ip)
    ref = [oracle.argarch_remove(x[s].copy(), c[s], phi[s], om[s], al[s], be[s], inplace=True) for s in range(S)]
    assert bits_equal(host(ip), ref)


@pytest.mark.gpu
def test_gpu_argarch_fit_model_2(torch):
    # T/models/GARCHSuite.scala:73-94 on one series (312 steps)
    from sparkts.models import ARGARCH
    m = ARGARCH.fitModel(dev(torch, FIT2))
    st, ref, ev = oracle.argarch_fit(FIT2)
    assert st == oracle.OK
    got = np.array([m.c, m.phi, m.omega, m.alpha, m.beta])
    assert np.allclose(got[:2], ref[:2], rtol=RTOL, atol=0)
    resid = oracle.ar_remove(FIT2, m.c, [m.phi])
    st2, rpar, _ = oracle.garch_fit(resid)
    assert st2 == oracle.OK and bits_equal(got[2:], rpar)
