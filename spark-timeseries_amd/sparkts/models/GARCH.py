"""Host mirror of com.cloudera.sparkts.models.{GARCH, ARGARCH, GARCHModel, ARGARCHModel}
(S/models/GARCH.scala:26-258), SURVEY.md §8(f) rank 1.

GARCH.fitModel (:33-53) fits every series of a panel in one device call: each lane runs
commons-math3's nonlinear-CG / bracket / Brent optimizer (no GoalType: its maximising
branches) for its series, and every logLikelihood / gradient evaluation is the reference's
sequential loop (bit-exact, with Math.log evaluated as StrictMath.log).  ARGARCH.fitModel
(:62-68) reuses the AR fit: Autoregression.fitModel(ts) (AR(1) with intercept) and its
residuals on the device, then GARCH.fitModel of the residuals.

Note GARCHModel.gradient (:94-114) returns its components in the order (alpha, beta,
omega) while the optimizer's point is (omega, alpha, beta); that is the reference's code
and it is reproduced, since it decides the optimizer's path.
"""
from __future__ import annotations

from .. import _native
from .._panel import Panel, check, ptr
from ..errors import NullPointerException
from .TimeSeriesModel import TimeSeriesModel


def _alloc(p, shape):
    if p.device:
        import torch
        return torch.empty(shape, dtype=torch.float64, device=p.t.device)
    import numpy as np
    return np.empty(shape, dtype=np.float64)


def _col(a, j):
    return a[:, j].contiguous() if hasattr(a, "contiguous") else a[:, j].copy()


def _scalar_or(vals, squeeze):
    return float(vals[0]) if squeeze else vals


class GARCHModel(TimeSeriesModel):
    """omega, alpha, beta: floats, or one value per series of a panel."""

    def __init__(self, omega, alpha, beta):
        self.omega, self.alpha, self.beta = omega, alpha, beta

    def _effects(self, add: bool, ts, dest):
        if dest is None:   # the reference writes into dest (:133, :147): NPE
            raise NullPointerException("GARCHModel.%sTimeDependentEffects: dest is null" % ("add" if add else "remove"))
        p = Panel(ts)
        d = Panel(dest, "dest")
        if not p.device or not d.device:
            raise TypeError("GARCHModel effects: device panels only")
        om, al, be = (p.vec(v, p.S, n) for v, n in ((self.omega, "omega"), (self.alpha, "alpha"), (self.beta, "beta")))
        fn = _native.lib().sts_garch_add if add else _native.lib().sts_garch_remove
        check(fn(ptr(p.t), ptr(d.t), p.S, p.T, p.ld, d.ld, ptr(om), ptr(al), ptr(be), p.stream), "GARCHModel")
        return dest

    def removeTimeDependentEffects(self, ts, dest=None):
        """S/models/GARCH.scala:130-142 (bit-exact); dest may be ts."""
        return self._effects(False, ts, dest)

    def addTimeDependentEffects(self, ts, dest=None):
        """S/models/GARCH.scala:144-159 (bit-exact); dest may be ts."""
        return self._effects(True, ts, dest)

    def _loglik_grad(self, ts):
        import torch
        p = Panel(ts)
        if not p.device:
            raise TypeError("logLikelihood / gradient: device panels only")
        params = torch.stack([p.vec(v, p.S, n) for v, n in
                              ((self.omega, "omega"), (self.alpha, "alpha"), (self.beta, "beta"))], dim=1).contiguous()
        ll = torch.empty((p.S,), dtype=torch.float64, device=p.t.device)
        g = torch.empty((p.S, 3), dtype=torch.float64, device=p.t.device)
        check(_native.lib().sts_garch_loglik_gradient(ptr(p.t), p.S, p.T, p.ld, ptr(params), ptr(ll), ptr(g),
                                                      p.stream), "GARCHModel.logLikelihood/gradient")
        return (p.out(ll), g[0] if p.squeeze else g)

    def logLikelihood(self, ts):
        """S/models/GARCH.scala:80-86, per series."""
        return self._loglik_grad(ts)[0]

    def gradient(self, ts):
        """S/models/GARCH.scala:94-114 (private[sparkts]): [alpha, beta, omega] components."""
        return self._loglik_grad(ts)[1]


class ARGARCHModel(TimeSeriesModel):
    """y(i) = c + phi * y(i - 1) + eta(i), eta's variance GARCH(1, 1) (:169-180)."""

    def __init__(self, c, phi, omega, alpha, beta):
        self.c, self.phi, self.omega, self.alpha, self.beta = c, phi, omega, alpha, beta

    def _effects(self, add: bool, ts, dest):
        if dest is None:
            raise NullPointerException("ARGARCHModel.%sTimeDependentEffects: dest is null"
                                       % ("add" if add else "remove"))
        p = Panel(ts)
        d = Panel(dest, "dest")
        if not p.device or not d.device:
            raise TypeError("ARGARCHModel effects: device panels only")
        vs = [p.vec(v, p.S, n) for v, n in ((self.c, "c"), (self.phi, "phi"), (self.omega, "omega"),
                                             (self.alpha, "alpha"), (self.beta, "beta"))]
        fn = _native.lib().sts_argarch_add if add else _native.lib().sts_argarch_remove
        check(fn(ptr(p.t), ptr(d.t), p.S, p.T, p.ld, d.ld, *[ptr(v) for v in vs], p.stream), "ARGARCHModel")
        return dest

    def removeTimeDependentEffects(self, ts, dest=None):
        """S/models/GARCH.scala:203-217 (bit-exact); dest eq ts reads the overwritten ts(i - 1)."""
        return self._effects(False, ts, dest)

    def addTimeDependentEffects(self, ts, dest=None):
        """S/models/GARCH.scala:219-234 (bit-exact)."""
        return self._effects(True, ts, dest)


class GARCH:
    @staticmethod
    def fitModel(ts, errors=None):
        """S/models/GARCH.scala:33-53.  A single series -> GARCHModel(floats); a panel ->
        GARCHModel(per-series tensors).  A series the optimizer cannot fit raises the
        reference's exception (TooManyEvaluationsException ...), unless `errors` (S int32) is
        given: then it receives the per-series status and that series' parameters are NaN."""
        p = Panel(ts)
        lib = _native.lib()
        par = _alloc(p, (p.S, 3))
        if p.device:
            check(lib.sts_garch_fit(ptr(p.t), p.S, p.T, p.ld, ptr(par), ptr(errors), p.stream), "GARCH.fitModel")
        else:
            check(lib.sts_garch_fit_host(ptr(p.t), p.S, p.T, p.ld, ptr(par), ptr(errors)), "GARCH.fitModel")
        om, al, be = (_scalar_or(_col(par, j), p.squeeze) for j in range(3))
        return GARCHModel(om, al, be)


class ARGARCH:
    @staticmethod
    def fitModel(ts, errors=None):
        """S/models/GARCH.scala:62-68: AR(1) fit + residuals (the a11 / a12 kernels), then
        GARCH.fitModel of the residuals -> ARGARCHModel(c, phi, omega, alpha, beta)."""
        p = Panel(ts)
        lib = _native.lib()
        par = _alloc(p, (p.S, 3))
        c = _alloc(p, (p.S,))
        phi = _alloc(p, (p.S,))
        if p.device:
            check(lib.sts_argarch_fit(ptr(p.t), p.S, p.T, p.ld, ptr(c), ptr(phi), ptr(par), ptr(errors), p.stream),
                  "ARGARCH.fitModel")
        else:
            check(lib.sts_argarch_fit_host(ptr(p.t), p.S, p.T, p.ld, ptr(c), ptr(phi), ptr(par), ptr(errors)),
                  "ARGARCH.fitModel")
        om, al, be = (_scalar_or(_col(par, j), p.squeeze) for j in range(3))
        return ARGARCHModel(_scalar_or(c, p.squeeze), _scalar_or(phi, p.squeeze), om, al, be)
