"""Host mirror of com.cloudera.sparkts.models.{Autoregression, ARModel}
(S/models/Autoregression.scala:24-94).

Autoregression.fitModel(ts, maxLag, noIntercept) fits every series of a panel in one
batched device call (one wave per series; lag-matrix Gram on FP64 MFMA).  The
returned ARModel holds c / coefficients per series (scalars for a single series).
"""
from __future__ import annotations

import numpy as np

from .. import _native
from .._panel import Panel, check, is_torch, ptr
from .TimeSeriesModel import TimeSeriesModel


class ARModel(TimeSeriesModel):
    """ARModel(c, coefficients): c scalar or (S,), coefficients (p,) or (S, p)."""

    def __init__(self, c, coefficients):
        self.c = c
        self.coefficients = coefficients

    def _params(self, p: Panel):
        coef = self.coefficients
        if is_torch(coef):
            coef = coef.detach()
        arr = coef.cpu().numpy() if is_torch(coef) else np.asarray(coef, dtype=np.float64)
        order = arr.shape[-1] if arr.ndim else 1
        arr = np.broadcast_to(arr.reshape(-1, order), (p.S, order))
        c = p.vec(self.c, p.S, "c")
        if p.device:
            import torch
            coef_t = torch.as_tensor(np.array(arr, dtype=np.float64, order="C"), device=p.t.device)
        else:
            coef_t = np.ascontiguousarray(arr)
        return c, coef_t, order

    def _run(self, add: bool, ts, destTs):
        p = Panel(ts)
        c, coef, order = self._params(p)
        lib = _native.lib()
        if destTs is None:
            out = p.empty()   # DenseVector.zeros (:61, :76) fully overwritten
            dptr, dld, inplace = out, p.T, False
        else:
            d = Panel(destTs, "destTs")
            out = destTs
            dptr, dld = d.t, d.ld
            inplace = (d.t.data_ptr() == p.t.data_ptr()) if p.device else (d.t.ctypes.data == p.t.ctypes.data)
        if p.device:
            fn = lib.sts_ar_add if add else lib.sts_ar_remove
            check(fn(ptr(p.t), ptr(dptr), p.S, p.T, p.ld, dld, ptr(c), ptr(coef), order, p.stream), "ar")
        else:
            fn = lib.sts_ar_add_host if add else lib.sts_ar_remove_host
            check(fn(ptr(p.t), ptr(p.t) if inplace else ptr(dptr), p.S, p.T, p.ld, ptr(c), ptr(coef), order), "ar")
        if destTs is None:
            return p.out(out)
        return destTs

    def removeTimeDependentEffects(self, ts, destTs=None):
        """S/models/Autoregression.scala:60-73 (bit-exact given c / coefficients)."""
        return self._run(False, ts, destTs)

    def addTimeDependentEffects(self, ts, destTs=None):
        """S/models/Autoregression.scala:75-88 (IIR, bit-exact)."""
        return self._run(True, ts, destTs)


class Autoregression:
    @staticmethod
    def fitModel(ts, maxLag: int = 1, noIntercept: bool = False) -> ARModel:
        """S/models/Autoregression.scala:38-53 (OLS with intercept unless noIntercept)."""
        p = Panel(ts)
        lib = _native.lib()
        if p.device:
            import torch
            c = torch.empty((p.S,), dtype=torch.float64, device=p.t.device)
            coef = torch.empty((p.S, maxLag), dtype=torch.float64, device=p.t.device)
            check(lib.sts_ar_fit(ptr(p.t), p.S, p.T, p.ld, maxLag, int(noIntercept), ptr(c), ptr(coef), None,
                                 p.stream), "Autoregression.fitModel")
        else:
            c = np.empty((p.S,), dtype=np.float64)
            coef = np.empty((p.S, maxLag), dtype=np.float64)
            check(lib.sts_ar_fit_host(ptr(p.t), p.S, p.T, p.ld, maxLag, int(noIntercept), ptr(c), ptr(coef), None),
                  "Autoregression.fitModel")
        if p.squeeze:
            return ARModel(float(c[0]), coef[0])
        return ARModel(c, coef)

    @staticmethod
    def fitModelAndRemove(ts, maxLag: int = 1, noIntercept: bool = False):
        """The C4 mapSeries closure `series => ar(series, p).removeTimeDependentEffects(series)`
        (README.md:61) fused into one device pass: returns (model, residuals)."""
        p = Panel(ts)
        lib = _native.lib()
        if not p.device:
            out = p.empty()
            c = np.empty((p.S,), dtype=np.float64)
            coef = np.empty((p.S, maxLag), dtype=np.float64)
            check(lib.sts_ar_fit_remove_host(ptr(p.t), ptr(out), p.S, p.T, p.ld, maxLag, int(noIntercept), ptr(c),
                                             ptr(coef), None), "ar_fit_remove")
            if p.squeeze:
                return ARModel(float(c[0]), coef[0]), out[0]
            return ARModel(c, coef), out
        import torch
        out = p.empty()
        c = torch.empty((p.S,), dtype=torch.float64, device=p.t.device)
        coef = torch.empty((p.S, maxLag), dtype=torch.float64, device=p.t.device)
        check(lib.sts_ar_fit_remove(ptr(p.t), ptr(out), p.S, p.T, p.ld, p.T, maxLag, int(noIntercept), ptr(c),
                                    ptr(coef), None, p.stream), "ar_fit_remove")
        if p.squeeze:
            return ARModel(float(c[0]), coef[0]), out[0]
        return ARModel(c, coef), out
