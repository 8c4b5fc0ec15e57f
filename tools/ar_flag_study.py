"""Calibration study for the AR-fit QR rule (DESIGN.md §3 "AR rule"): how far the reference's
Householder QR (oracle.ar_fit = commons-math3 3.4.1 as restated in oracle/sts_oracle.c) lands
from the EXACT least-squares solution, against per-series features the device fit kernels hold.

CPU only; writes one JSON line per case to stdout (or --out).  Test infrastructure, not product.
"""
import argparse
import json
import os
import sys
from fractions import Fraction
from multiprocessing import Pool

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "oracle"))
import oracle  # noqa: E402


def exact_ols(x, p, no_intercept=False):
    x = np.asarray(x, dtype=np.float64)
    n = x.size
    _, e = np.frexp(x[x != 0]) if np.any(x != 0) else (None, np.array([0]))
    E = int(53 - e.min())
    xi = [int(Fraction(float(v)) * (1 << E)) if E >= 0 else int(Fraction(float(v)) / (1 << -E)) for v in x]
    Y = xi[p:]
    cols = [[xi[r + p - 1 - j] for r in range(n - p)] for j in range(p)]
    if not no_intercept:
        cols = [[1 << E] * (n - p)] + cols
    k = len(cols)
    A = [[Fraction(sum(a * b for a, b in zip(cols[i], cols[j]))) for j in range(k)] +
         [Fraction(sum(a * y for a, y in zip(cols[i], Y)))] for i in range(k)]
    for c in range(k):
        piv = max(range(c, k), key=lambda r: abs(A[r][c]))
        A[c], A[piv] = A[piv], A[c]
        for r in range(k):
            if r != c and A[r][c] != 0:
                f = A[r][c] / A[c][c]
                A[r] = [a - f * bb for a, bb in zip(A[r], A[c])]
    beta = [float(A[i][k] / A[i][i]) for i in range(k)]
    return np.array(([0.0] if no_intercept else []) + beta)


def elementwise(a, b):
    big = np.abs(b) > 1e-6 * np.linalg.norm(b)
    return float(np.max(np.abs(a[big] - b[big]) / np.abs(b[big])))


def amplification(b):
    """||b|| / min |b_i| over the elements `elementwise` compares: how much a normwise error
    can grow in the elementwise metric."""
    nb = np.linalg.norm(b)
    big = np.abs(b) > 1e-6 * nb
    return float(nb / np.min(np.abs(b[big])))


def features(x, p, no_int):
    """What the device kernels hold per series: mean, centred lag-column Gram, its Cholesky."""
    n = x.size
    m = n - p
    X = np.column_stack([x[p - 1 - j: n - 1 - j] for j in range(p)])
    mu = x.mean()
    sd = x.std()
    Xc = X - X.mean(axis=0)
    G = Xc.T @ Xc
    d = np.sqrt(np.diag(G))
    C = G / np.outer(d, d)
    try:
        L = np.linalg.cholesky(C)
        ldmin = float(np.min(np.diag(L)))
    except np.linalg.LinAlgError:
        ldmin = 0.0
    colrms = d / np.sqrt(m)
    ev = np.linalg.eigvalsh(C)
    # the noIntercept kernel's own quantities: column x_{t-1} centred, and the scaled Gram of
    # the difference basis [x_{t-1}, d_{t-1}, .., d_{t-p+1}] (uncentred)
    c1 = x[p - 1: n - 1]
    r_ni = abs(c1.mean()) / max(c1.std(), 1e-300)
    dd = np.diff(x, prepend=np.nan)
    V = np.column_stack([c1] + [dd[p - k: n - k] for k in range(1, p)])
    Gd = V.T @ V
    sd_ = np.sqrt(np.diag(Gd))
    try:
        ld_ni = float(np.min(np.diag(np.linalg.cholesky(Gd / np.outer(sd_, sd_)))))
    except np.linalg.LinAlgError:
        ld_ni = 0.0
    return dict(mu=float(mu), sd=float(sd), rms_min=float(colrms.min()), ldmin=ldmin,
                kappa_c=float(ev.max() / max(ev.min(), 1e-300)),
                absmax=float(np.max(np.abs(x))), r_ni=float(r_ni), ld_ni=ld_ni)


def _ne_refine(V, y, iters):
    """Normal equations on the columns V (Cholesky) + `iters` steps of refinement against
    exact residuals: the fast path's algebra (spark-timeseries_amd/csrc/sts_ar.hip), in numpy."""
    G = V.T @ V
    L = np.linalg.cholesky(G)
    sol = np.linalg.solve(L.T, np.linalg.solve(L, V.T @ y))
    for _ in range(iters):
        e = y - V @ sol
        sol = sol + np.linalg.solve(L.T, np.linalg.solve(L, V.T @ e))
    return sol


def dev_emul(x, p, no_int):
    """Magnitude model of the device fit (not its bits): intercept = centred normal equations +
    one refinement; noIntercept = the difference basis + two refinements."""
    n = x.size
    if not no_int:
        mu = x.mean()
        y = x - mu
        X = np.column_stack([y[p - 1 - j: n - 1 - j] for j in range(p)])
        Y = y[p:]
        cm = X.mean(axis=0)
        ym = Y.mean()
        phi = _ne_refine(X - cm, Y - ym, 1)
        c = (ym - cm @ phi) + mu * (1.0 - phi.sum())
        return np.r_[c, phi]
    d = np.diff(x, prepend=np.nan)
    cols = [x[p - 1: n - 1]] + [d[p - k: n - k] for k in range(1, p)]
    sol = _ne_refine(np.column_stack(cols), d[p:], 2)
    beta = np.empty(p)
    if p == 1:
        beta[0] = 1.0 + sol[0]
    else:
        beta[0] = (1.0 + sol[0]) + sol[1]
        for j in range(2, p):
            beta[j - 1] = sol[j] - sol[j - 1]
        beta[p - 1] = -sol[p - 1]
    return np.r_[0.0, beta]


def series(kind, level, sigma, T, seed):
    rng = np.random.default_rng(seed)
    if kind == "walk":
        return level + np.cumsum(rng.standard_normal(T)) * sigma
    if kind == "walk2":   # integrated random walk: nearly collinear lags without a level
        return level + np.cumsum(np.cumsum(rng.standard_normal(T))) * sigma
    if kind == "sine":    # smooth: collinear lags
        t = np.arange(T)
        return level + sigma * (np.sin(2 * np.pi * t / 500.0) + 1e-3 * rng.standard_normal(T))
    if kind == "ar1":   # stationary AR(1) phi = 0.9 around level
        e = rng.standard_normal(T) * sigma
        y = np.empty(T)
        y[0] = e[0]
        for t in range(1, T):
            y[t] = 0.9 * y[t - 1] + e[t]
        return level + y
    if kind == "noise":
        return level + rng.standard_normal(T) * sigma
    if kind == "trend":
        return level + sigma * (np.arange(T) / T * 10 + rng.uniform(-0.5, 0.5, T))
    if kind == "c4":
        return oracle.gen_ar_panel(seed, 1, T, 5)[0] * sigma + level
    if kind.startswith("filled_"):
        # README.md:57-61's own input: a NaN-riddled price walk after fill(method).
        # NaN rate 5 / 20 / 60 % by seed, plus three long gaps (50-300 steps); step series for
        # previous / next / nearest, linear ramps for linear
        method = {"filled_prev": "previous", "filled_next": "next", "filled_near": "nearest",
                  "filled_lin": "linear"}[kind]
        x = level + np.cumsum(rng.standard_normal(T)) * sigma
        x[rng.random(T) < (0.05, 0.2, 0.6)[seed % 3]] = np.nan
        for _ in range(3):
            g = int(rng.integers(50, 300))
            a = int(rng.integers(1, max(2, T - g - 1)))
            x[a:a + g] = np.nan
        x[0] = level            # keep both ends valid: fills leave leading / trailing NaNs,
        x[-1] = level + sigma   # and an AR fit of a NaN series is NaN
        return oracle.fillts(x, method)
    raise ValueError(kind)


def run(case):
    kind, level, sigma, T, p, no_int, seed = case
    x = series(kind, level, sigma, T, seed)
    c, coef = oracle.ar_fit(x, p, no_int)
    ref = np.r_[c, coef]
    ex = exact_ols(x, p, no_int)
    try:
        dv = dev_emul(x, p, no_int)
    except np.linalg.LinAlgError:
        dv = np.full_like(ex, np.nan)
    if no_int:
        ref, ex, dv = ref[1:], ex[1:], dv[1:]
    f = features(x, p, no_int)
    return dict(kind=kind, level=level, sigma=sigma, T=T, p=p, no_int=no_int, seed=seed,
                e_norm=float(np.linalg.norm(ref - ex) / np.linalg.norm(ex)), e_elem=elementwise(ref, ex),
                d_elem=elementwise(dv, ex), dr_elem=elementwise(dv, ref), amp=amplification(ex), c_ex=float(ex[0]) if not no_int else 0.0,
                bmin=float(np.min(np.abs(ex[1:] if not no_int else ex))), **f)


def cases(quick, families="all"):
    out = []
    if families == "filled":
        for kind in ["filled_prev", "filled_next", "filled_near", "filled_lin"]:
            for L in [0.0, 1.0, 1e1, 1e2, 1e4, 1e6]:
                for sg in [1.0, 1e-2]:
                    for T in ([390] if quick else [390, 2520]):
                        for p in [1, 5, 8]:
                            for ni in (False, True):
                                for sd in (0, 1, 2):
                                    out.append((kind, L, sg, T, p, ni, sd))
        return out
    levels = [0.0, 1.0, 3.0, 1e1, 3e1, 1e2, 3e2, 1e3, 3e3, 1e4, 1e5, 1e6, 1e7]
    sigmas = [1.0, 1e-2]
    Ts = [300, 2520] if quick else [300, 2520, 6000]
    ps = [1, 2, 5, 8]
    seeds = [1, 2] if quick else [1, 2, 3]
    for kind in ["walk", "ar1", "noise", "trend", "walk2", "sine"]:
        for L in levels:
            for sg in sigmas:
                for T in Ts:
                    for p in ps:
                        for ni in (False, True):
                            for sd in seeds:
                                out.append((kind, L, sg, T, p, ni, sd))
    for sd in range(8):
        out.append(("c4", 0.0, 1.0, 2520, 5, False, sd))
    return out


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--quick", action="store_true")
    ap.add_argument("--out", default="-")
    ap.add_argument("--procs", type=int, default=7)
    ap.add_argument("--families", default="all", choices=["all", "filled"])
    args = ap.parse_args()
    cs = cases(args.quick, args.families)
    f = sys.stdout if args.out == "-" else open(args.out, "w")
    with Pool(args.procs) as pool:
        for r in pool.imap_unordered(run, cs, chunksize=2):
            f.write(json.dumps(r) + "\n")
            f.flush()
