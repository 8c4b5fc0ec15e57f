"""Host mirror of com.cloudera.sparkts.models.EWMAModel (S/models/EWMA.scala:71-143).

Note the reference's recurrence puts the smoothing weight on the NEW observation,
dest(i) = s*ts(i) + (1 - s)*dest(i-1) (:141), not the docstring's (1-a)X + aS.
EWMA.fitModel (commons-math3 nonlinear CG) is a "next" row.
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
