"""Host mirror of com.cloudera.sparkts.UnivariateTimeSeries (S/UnivariateTimeSeries.scala).

Same function names, argument meaning and exceptions as the Scala object; every
function accepts one series (T,) or a whole panel (S, T) and dispatches ONE batched
C-ABI call (include/sts.h) -- torch GPU tensors take the device path on torch's
current stream, numpy arrays take the host-staging (`_host`) path.  Results are
always fresh arrays, as in the reference.
"""
from __future__ import annotations

import numpy as np

from . import _native
from ._panel import Panel, check, ptr
from .errors import UnsupportedOperationException

__all__ = ["fillts", "fillLinear", "fillNearest", "fillNext", "fillPrevious", "fillSpline", "autocorr", "lag",
           "differencesAtLag", "ar", "fill_method_code"]


def fill_method_code(method: str) -> int:
    """fillts's string dispatch (S/UnivariateTimeSeries.scala:141-150)."""
    code = _native.lib().sts_fill_method_from_name(method.encode() if isinstance(method, str) else method)
    if code == -2:
        raise UnsupportedOperationException("unsupported fill method %r" % (method,))
    return code


def _fill(ts, code: int):
    p = Panel(ts)
    out = p.empty()
    lib = _native.lib()
    if p.device:
        check(lib.sts_fill(ptr(p.t), ptr(out), p.S, p.T, p.ld, p.T, code, None, p.stream), "fill")
    else:
        check(lib.sts_fill_host(ptr(p.t), ptr(out), p.S, p.T, p.ld, code, None), "fill")
    return p.out(out)


def fillts(ts, fillMethod: str):
    """S/UnivariateTimeSeries.scala:141-150: "linear" | "nearest" | "next" | "previous" |
    "spline"; anything else raises UnsupportedOperationException."""
    return _fill(ts, fill_method_code(fillMethod))


def fillLinear(values):
    """S/UnivariateTimeSeries.scala:247-266 (bit-exact, sequential accumulation)."""
    return _fill(values, 0)


def fillNearest(values):
    """S/UnivariateTimeSeries.scala:156-184; raises IllegalArgumentException("Input is all NaNs!")."""
    return _fill(values, 1)


def fillNext(values):
    """S/UnivariateTimeSeries.scala:214-224."""
    return _fill(values, 2)


def fillPrevious(values):
    """S/UnivariateTimeSeries.scala:194-204."""
    return _fill(values, 3)


def fillSpline(values):
    """S/UnivariateTimeSeries.scala:268-297: natural cubic spline through the non-NaN steps
    (commons-math3 3.4.1 SplineInterpolator), evaluated at every step from the first valid one
    up to the last; bit-exact.  Fewer than 3 non-NaN values raises NumberIsTooSmallException."""
    return _fill(values, 4)


def autocorr(ts, numLags: int):
    """S/UnivariateTimeSeries.scala:68-93; (K,) for a series, (S, K) for a panel."""
    p = Panel(ts)
    out = p.empty(T=numLags)
    lib = _native.lib()
    if p.device:
        check(lib.sts_autocorr(ptr(p.t), p.S, p.T, p.ld, numLags, ptr(out), p.stream), "autocorr")
    else:
        check(lib.sts_autocorr_host(ptr(p.t), p.S, p.T, p.ld, numLags, ptr(out)), "autocorr")
    return p.out(out)


def lag(ts, maxLag: int, includeOriginal: bool):
    """S/UnivariateTimeSeries.scala:37-39 -> Lag.lagMatTrimBoth (S/Lag.scala:62-77).

    Returns the Breeze DenseMatrix as a (rows, cols) array -- (S, rows, cols) for a
    panel -- whose storage is column-major per series, exactly like Breeze's."""
    p = Panel(ts)
    ncols = maxLag + (1 if includeOriginal else 0)
    rows = p.T - maxLag
    lib = _native.lib()
    if rows < 0 or maxLag < 0:
        from .errors import IllegalArgumentException
        raise IllegalArgumentException("lag: maxLag %d outside [0, %d]" % (maxLag, p.T))
    if p.device:
        import torch
        buf = torch.empty((p.S, ncols, rows), dtype=torch.float64, device=p.t.device)
        check(lib.sts_lag_matrix(ptr(p.t), ptr(buf), p.S, p.T, p.ld, maxLag, int(includeOriginal), p.stream), "lag")
        mat = buf.transpose(1, 2)
    else:
        buf = np.empty((p.S, ncols, rows), dtype=np.float64)
        check(lib.sts_lag_matrix_host(ptr(p.t), ptr(buf), p.S, p.T, p.ld, maxLag, int(includeOriginal)), "lag")
        mat = buf.transpose(0, 2, 1)
    return mat[0] if p.squeeze else mat


def differencesAtLag(ts, lag: int, destTs=None, startIndex=None):
    """S/UnivariateTimeSeries.scala:356-386.

    differencesAtLag(ts, lag) returns a differenced copy (startIndex = lag).  With
    destTs given the result is written there and returned; destTs may be ts itself,
    which reproduces the reference's in-place semantics (later elements see already
    differenced values)."""
    start = lag if startIndex is None else startIndex
    p = Panel(ts)
    lib = _native.lib()
    if destTs is None:
        dest = p.t.clone() if p.device else p.t.copy()   # ts.copy (:363)
        dview = dest
        in_place_ptr = False
        dld = (int(dview.stride(0)) if p.S > 1 else p.T) if p.device else p.T
    else:
        dp = Panel(destTs, "destTs")
        if dp.device != p.device or (dp.S, dp.T) != (p.S, p.T):
            raise ValueError("differencesAtLag: destTs must be the same kind and shape as ts: (%d, %d) %s vs "
                             "(%d, %d) %s" % (dp.S, dp.T, "device" if dp.device else "host", p.S, p.T,
                                              "device" if p.device else "host"))
        dview = p.t if destTs is ts else dp.t     # ts may have been made unit-stride: stay in place
        in_place_ptr = dview.data_ptr() == p.t.data_ptr() if p.device else dview.ctypes.data == p.t.ctypes.data
        dld = dp.ld
        dest = dview
    if p.device:
        check(lib.sts_diff_at_lag(ptr(p.t), ptr(dview), p.S, p.T, p.ld,
                                  p.ld if in_place_ptr else dld,
                                  lag, start, p.stream), "differencesAtLag")
    else:
        src = p.t
        check(lib.sts_diff_at_lag_host(ptr(src), ptr(dview), p.S, p.T, p.ld, lag, start), "differencesAtLag")
    if destTs is not None and p.device and dview.data_ptr() != destTs.data_ptr():
        # Panel made a unit-stride copy of a strided destTs: write the result back
        destTs.copy_(dview[0] if dp.squeeze else dview)
        return destTs
    if destTs is not None and not p.device and dview is not destTs:
        np.copyto(np.asarray(destTs).reshape(dview.shape), dview)
        return destTs
    if destTs is not None:
        return destTs
    return p.out(dest)


def ar(values, maxLag: int):
    """S/UnivariateTimeSeries.scala:299 -> Autoregression.fitModel(values, maxLag)."""
    from .models.Autoregression import Autoregression
    return Autoregression.fitModel(values, maxLag)
