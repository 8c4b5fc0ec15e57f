"""Host mirror of com.cloudera.sparkts.models.EWMAModel (S/models/EWMA.scala:71-143).

Note the reference's recurrence puts the smoothing weight on the NEW observation,
dest(i) = s*ts(i) + (1 - s)*dest(i-1) (:141), not the docstring's (1-a)X + aS.
EWMA.fitModel (S/models/EWMA.scala:44-68) fits every series of a panel in one device call:
each lane runs commons-math3's nonlinear-CG / bracket / Brent optimizer for its series and
every sse / gradient evaluation is the reference's sequential loop (bit-exact).
"""
from __future__ import annotations

from .. import _native
from .._panel import Panel, check, ptr
from ..errors import NullPointerException
from .TimeSeriesModel import TimeSeriesModel


class EWMAModel(TimeSeriesModel):
    """smoothing: a float, or one value per series of a panel."""

    def __init__(self, smoothing):
        self.smoothing = smoothing

    def _run(self, add: bool, ts, dest):
        if dest is None:  # the reference dereferences dest: NPE (EWMA.scala:132, :141)
            raise NullPointerException("EWMAModel.%sTimeDependentEffects: dest is null"
                                       % ("add" if add else "remove"))
        p = Panel(ts)
        d = Panel(dest, "dest")
        if (d.S, d.T) != (p.S, p.T):
            raise ValueError("dest shape %s != ts shape %s" % ((d.S, d.T), (p.S, p.T)))
        sm = p.vec(self.smoothing, p.S, "smoothing")
        lib = _native.lib()
        if p.device:
            fn = lib.sts_ewma_add if add else lib.sts_ewma_remove
            check(fn(ptr(p.t), ptr(d.t), p.S, p.T, p.ld, d.ld, ptr(sm), p.stream), "ewma")
        else:
            fn = lib.sts_ewma_add_host if add else lib.sts_ewma_remove_host
            inplace = d.t.ctypes.data == p.t.ctypes.data
            check(fn(ptr(p.t), ptr(p.t) if inplace else ptr(d.t), p.S, p.T, p.ld, ptr(sm)), "ewma")
            import numpy as np
            if d.t is not dest and not inplace:
                np.copyto(np.asarray(dest).reshape(d.t.shape), d.t)
            elif inplace and p.t is not ts:
                np.copyto(np.asarray(dest).reshape(p.t.shape), p.t)
        return dest

    def addTimeDependentEffects(self, ts, dest=None):
        """S/models/EWMA.scala:135-142 (bit-exact); dest may be ts (safe)."""
        return self._run(True, ts, dest)

    def removeTimeDependentEffects(self, ts, dest=None):
        """S/models/EWMA.scala:125-133 (bit-exact); dest may be ts (reference aliasing)."""
        return self._run(False, ts, dest)


class EWMA:
    @staticmethod
    def fitModel(ts, errors=None):
        """S/models/EWMA.scala:44-68.  A single series -> EWMAModel(float); a panel ->
        EWMAModel(per-series smoothing).  A series the optimizer cannot fit raises the
        reference's TooManyEvaluationsException, unless `errors` (an int32 array / tensor of
        S elements) is given: then it receives the per-series status and that series' smoothing
        is NaN (the batched form of a failing Spark task)."""
        p = Panel(ts)
        lib = _native.lib()
        if p.device:
            import torch
            sm = torch.empty((p.S,), dtype=torch.float64, device=p.t.device)
            check(lib.sts_ewma_fit(ptr(p.t), p.S, p.T, p.ld, ptr(sm), ptr(errors), p.stream), "EWMA.fitModel")
        else:
            import numpy as np
            sm = np.empty((p.S,), dtype=np.float64)
            check(lib.sts_ewma_fit_host(ptr(p.t), p.S, p.T, p.ld, ptr(sm), ptr(errors)), "EWMA.fitModel")
        if p.squeeze:
            return EWMAModel(float(sm[0]))
        return EWMAModel(sm)


def sse(model: EWMAModel, ts):
    """EWMAModel.sse (private[sparkts], :80-95) per series (device panels only)."""
    return _sse_grad(model, ts)[0]


def gradient(model: EWMAModel, ts):
    """EWMAModel.gradient (private[sparkts], :102-123) per series (device panels only)."""
    return _sse_grad(model, ts)[1]


def _sse_grad(model: EWMAModel, ts):
    import torch
    p = Panel(ts)
    if not p.device:
        raise TypeError("sse / gradient: device panels only")
    sm = p.vec(model.smoothing, p.S, "smoothing")
    f = torch.empty((p.S,), dtype=torch.float64, device=p.t.device)
    g = torch.empty((p.S,), dtype=torch.float64, device=p.t.device)
    check(_native.lib().sts_ewma_sse_gradient(ptr(p.t), p.S, p.T, p.ld, ptr(sm), ptr(f), ptr(g), p.stream),
          "EWMAModel.sse/gradient")
    return (p.out(f), p.out(g))
