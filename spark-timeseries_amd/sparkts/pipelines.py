"""Batched series operators for TimeSeriesRDD.mapSeries (S/TimeSeriesRDD.scala:188-199).

The reference's mapSeries applies a per-series closure, one record at a time.  Here a
closure marked `batched` is applied to the whole partition panel in ONE device call (every
function of UnivariateTimeSeries and the models accepts a panel (S, T) and treats its rows
independently), and an unmarked closure keeps the reference's per-series semantics (one
call per series; correct for any closure, launch-bound).  The two mapSeries pipelines the
reference's own documentation and configs use are provided as fused single-pass operators:

  ar_remove(p)              series => ar(series, p).removeTimeDependentEffects(series)
                            (README.md:61, BASELINE config C4) -> sts_ar_fit_remove
  fill_diff_ewma(m, lag, s) fill(m) -> differencesAtLag(lag) -> EWMAModel(s).add
                            (BASELINE config C2) -> sts_fill_diff_ewma
"""
from __future__ import annotations

import numpy as np

from . import _native
from ._panel import Panel, check, ptr


def batched(f):
    """Mark f as a panel operator: f(panel) must equal the row-wise stack of f(series).
    mapSeries then applies it to the whole partition in one call."""
    f.batched = True
    return f


def is_batched(f) -> bool:
    return bool(getattr(f, "batched", False))


def ar_remove(maxLag: int = 1, noIntercept: bool = False):
    """`series => ar(series, maxLag).removeTimeDependentEffects(series)` as one fused device
    pass over the panel (fit + residuals; the fitted models are not kept)."""
    from .models.Autoregression import Autoregression

    @batched
    def op(panel):
        return Autoregression.fitModelAndRemove(panel, maxLag, noIntercept)[1]
    return op


def fill_diff_ewma(method: str, lag: int, smoothing):
    """fill(method) -> differencesAtLag(lag) -> EWMAModel(smoothing).addTimeDependentEffects,
    one fused pass (smoothing: scalar or one value per series)."""
    from .UnivariateTimeSeries import fill_method_code
    code = fill_method_code(method)

    @batched
    def op(panel):
        p = Panel(panel)
        out = p.empty()
        sm = p.vec(smoothing, p.S, "smoothing")
        lib = _native.lib()
        if p.device:
            check(lib.sts_fill_diff_ewma(ptr(p.t), ptr(out), p.S, p.T, p.ld, p.T, code, lag, ptr(sm), None,
                                         p.stream), "fill_diff_ewma")
        else:
            check(lib.sts_fill_diff_ewma_host(ptr(p.t), ptr(out), p.S, p.T, p.ld, code, lag, ptr(sm), None),
                  "fill_diff_ewma")
        return p.out(out)
    return op


def apply_per_series(f, data):
    """The reference's semantics for an arbitrary closure: f on every series (row), in key
    order; the results (equal lengths) stacked into a new panel of the same kind."""
    rows = [f(data[i]) for i in range(int(data.shape[0]))]
    if not rows:
        return data[:0]
    try:
        import torch
        if isinstance(rows[0], torch.Tensor):
            return torch.stack(rows)
    except ImportError:  # pragma: no cover
        pass
    return np.stack([np.asarray(r) for r in rows])
