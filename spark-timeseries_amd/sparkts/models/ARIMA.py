"""Host mirror of com.cloudera.sparkts.models.ARIMA -- the AR-only path (SURVEY.md §8(f)
rank 1: "ARIMA(p,d,0) reuse of the AR fit", S/models/ARIMA.scala:80-90).

ARIMA.fitModel(p, d, 0, ts) is differencesOfOrderD(ts, d).drop(d) followed by
Autoregression.fitModel(diffed, p, !includeIntercept); both run batched on the device
(sts_arima_fit_ar).  Models with MA terms (q > 0) or p = 0 need the reference's CSS
optimizers (BOBYQA / conjugate gradient over the CSS likelihood), which are out of scope.
"""
from __future__ import annotations

import numpy as np

from .. import _native
from .._panel import Panel, check, ptr
from ..errors import UnsupportedOperationException


class ARIMAModel:
    """ARIMAModel(p, d, q, coefficients, hasIntercept) (S/models/ARIMA.scala:251-256):
    coefficients = [intercept] ++ AR ++ MA, per series ((S, n) for a panel)."""

    def __init__(self, p, d, q, coefficients, hasIntercept=True):
        self.p, self.d, self.q = p, d, q
        self.coefficients = coefficients
        self.hasIntercept = hasIntercept


class ARIMA:
    @staticmethod
    def fitModel(p: int, d: int, q: int, ts, includeIntercept: bool = True, method: str = "css-cgd",
                 userInitParams=None) -> ARIMAModel:
        if not (p > 0 and q == 0):
            raise UnsupportedOperationException(
                "ARIMA.fitModel(p=%d, d=%d, q=%d): only the AR path (p > 0, q = 0) runs on the device; "
                "the CSS optimizers for MA terms are out of scope" % (p, d, q))
        pn = Panel(ts)
        if not pn.device:
            raise TypeError("ARIMA.fitModel runs on device-resident series (torch GPU tensors)")
        import torch
        c = torch.empty((pn.S,), dtype=torch.float64, device=pn.t.device)
        coef = torch.empty((pn.S, p), dtype=torch.float64, device=pn.t.device)
        check(_native.lib().sts_arima_fit_ar(ptr(pn.t), pn.S, pn.T, pn.ld, p, d, int(includeIntercept), ptr(c),
                                             ptr(coef), None, pn.stream), "ARIMA.fitModel")
        params = torch.cat([c[:, None], coef], dim=1) if includeIntercept else coef
        if pn.squeeze:
            params = params[0]
        return ARIMAModel(p, d, q, params, includeIntercept)
