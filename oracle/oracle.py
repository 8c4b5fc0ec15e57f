"""ctypes wrapper around the CPU oracle (oracle/_build/libsts_oracle.so).

TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg may import this module, and only as the checker or the CPU
baseline.  The product path (spark-timeseries_amd/sparkts -> libsts_hip.so)
never imports it.

Every wrapped function restates a reference loop; see sts_oracle.c for the
file:line citations (S/ = /root/reference/src/main/scala/com/cloudera/sparkts/).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_build", "libsts_oracle.so")

OK, ERR_BAD_ARG, ERR_ALL_NAN, ERR_UNSUPPORTED_METHOD = 0, 1, 2, 3
ERR_REQUIREMENT, ERR_NOT_ENOUGH_DATA, ERR_SINGULAR = 5, 7, 8
ERR_TOO_MANY_EVALUATIONS, ERR_TOO_MANY_ITERATIONS, ERR_TOO_FEW_POINTS = 10, 11, 12
FILL_METHODS = {"linear": 0, "nearest": 1, "next": 2, "previous": 3, "spline": 4}

_lib = None
_dp = ctypes.POINTER(ctypes.c_double)
_i64 = ctypes.c_int64


def build() -> None:
    subprocess.check_call(["make", "-s", "-C", HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        i32p = ctypes.POINTER(ctypes.c_int32)
        sig = {
            "orc_fill_previous": (None, [_dp, _dp, _i64]),
            "orc_fill_next": (None, [_dp, _dp, _i64]),
            "orc_fill_nearest": (ctypes.c_int, [_dp, _dp, _i64]),
            "orc_fill_linear": (None, [_dp, _dp, _i64]),
            "orc_fill_spline": (ctypes.c_int, [_dp, _dp, _i64]),
            "orc_time_fill": (ctypes.c_double, [_dp, _dp, _i64, ctypes.c_int, ctypes.c_int]),
            "orc_time_autocorr": (ctypes.c_double, [_dp, _i64, ctypes.c_int, _dp, ctypes.c_int]),
            "orc_fillts": (ctypes.c_int, [_dp, _dp, _i64, ctypes.c_int]),
            "orc_autocorr": (None, [_dp, _i64, ctypes.c_int, _dp]),
            "orc_lag_mat_trim_both": (ctypes.c_int, [_dp, _i64, ctypes.c_int, ctypes.c_int, _dp]),
            "orc_differences_at_lag": (ctypes.c_int, [_dp, _dp, _i64, ctypes.c_int, ctypes.c_int]),
            "orc_inverse_differences_at_lag": (ctypes.c_int, [_dp, _dp, _i64, ctypes.c_int, ctypes.c_int]),
            "orc_differences_of_order_d": (None, [_dp, _dp, _i64, ctypes.c_int]),
            "orc_ewma_add": (None, [_dp, _dp, _i64, ctypes.c_double]),
            "orc_ewma_remove": (None, [_dp, _dp, _i64, ctypes.c_double]),
            "orc_ar_remove": (None, [_dp, _dp, _i64, ctypes.c_double, _dp, ctypes.c_int]),
            "orc_ar_add": (None, [_dp, _dp, _i64, ctypes.c_double, _dp, ctypes.c_int]),
            "orc_ar_fit": (ctypes.c_int, [_dp, _i64, ctypes.c_int, ctypes.c_int, _dp, _dp]),
            "orc_panel_fill": (ctypes.c_int, [_dp, _dp, _i64, _i64, _i64, ctypes.c_int, i32p, ctypes.c_int]),
            "orc_panel_fill_autocorr": (ctypes.c_int, [_dp, _dp, _i64, _i64, _i64, ctypes.c_int, ctypes.c_int, _dp, i32p, ctypes.c_int]),
            "orc_panel_fill_diff_ewma": (ctypes.c_int, [_dp, _dp, _i64, _i64, _i64, ctypes.c_double, ctypes.c_int]),
            "orc_panel_ar_fit_remove": (ctypes.c_int, [_dp, _dp, _i64, _i64, _i64, ctypes.c_int, ctypes.c_int, _dp, _dp, ctypes.c_int]),
            "orc_ewma_sse": (ctypes.c_double, [_dp, _i64, ctypes.c_double]),
            "orc_ewma_gradient": (ctypes.c_double, [_dp, _i64, ctypes.c_double]),
            "orc_ewma_fit": (ctypes.c_int, [_dp, _i64, _dp, ctypes.POINTER(ctypes.c_int64)]),
            "orc_panel_ewma_fit": (ctypes.c_int, [_dp, _i64, _i64, _i64, _dp, i32p, ctypes.c_int]),
            "orc_fdlibm_log": (ctypes.c_double, [ctypes.c_double]),
            "orc_garch_loglik": (ctypes.c_double, [_dp, _i64, ctypes.c_double, ctypes.c_double, ctypes.c_double]),
            "orc_garch_gradient": (None, [_dp, _i64, ctypes.c_double, ctypes.c_double, ctypes.c_double, _dp]),
            "orc_garch_fit": (ctypes.c_int, [_dp, _i64, _dp, ctypes.POINTER(ctypes.c_int64)]),
            "orc_argarch_fit": (ctypes.c_int, [_dp, _i64, _dp, ctypes.POINTER(ctypes.c_int64)]),
            "orc_garch_remove": (None, [_dp, _dp, _i64, ctypes.c_double, ctypes.c_double, ctypes.c_double]),
            "orc_garch_add": (None, [_dp, _dp, _i64, ctypes.c_double, ctypes.c_double, ctypes.c_double]),
            "orc_argarch_remove": (None, [_dp, _dp, _i64] + [ctypes.c_double] * 5),
            "orc_argarch_add": (None, [_dp, _dp, _i64] + [ctypes.c_double] * 5),
            "orc_panel_garch_fit": (ctypes.c_int, [_dp, _i64, _i64, _i64, _dp, i32p, ctypes.c_int]),
            "orc_panel_argarch_fit": (ctypes.c_int, [_dp, _i64, _i64, _i64, _dp, i32p, ctypes.c_int]),
            "orc_stat_counter": (None, [_dp, _i64, _dp]),
            "orc_remove_instants_with_nans": (_i64, [_dp, _i64, _i64, _i64, _dp, ctypes.POINTER(ctypes.c_int64)]),
            "orc_to_instants": (None, [_dp, _i64, _i64, _i64, _dp]),
            "orc_gen_value": (ctypes.c_double, [ctypes.c_uint64, _i64, _i64, _i64]),
            "orc_nan_threshold": (ctypes.c_uint32, [ctypes.c_double]),
            "orc_gen_panel": (None, [ctypes.c_uint64, _i64, _i64, _i64, _i64, ctypes.c_double, _dp]),
            "orc_gen_ar_panel": (None, [ctypes.c_uint64, _i64, _i64, _i64, _i64, ctypes.c_int, _dp]),
            "orc_gen_ar_params": (None, [ctypes.c_uint64, _i64, ctypes.c_int, _dp, _dp]),
        }
        for name, (res, args) in sig.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def _p(a: np.ndarray):
    assert a.dtype == np.float64 and a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(_dp)


def _vec(x) -> np.ndarray:
    return np.ascontiguousarray(np.asarray(x, dtype=np.float64))


class OracleError(Exception):
    def __init__(self, code: int, msg: str):
        super().__init__(msg)
        self.code = code


# ---------------- single-series restatements ----------------

def fill_previous(x):
    x = _vec(x); r = np.empty_like(x); lib().orc_fill_previous(_p(x), _p(r), x.size); return r


def fill_next(x):
    x = _vec(x); r = np.empty_like(x); lib().orc_fill_next(_p(x), _p(r), x.size); return r


def fill_nearest(x):
    x = _vec(x); r = np.empty_like(x)
    st = lib().orc_fill_nearest(_p(x), _p(r), x.size)
    if st == ERR_ALL_NAN:
        raise OracleError(st, "Input is all NaNs!")
    return r


def fill_linear(x):
    x = _vec(x); r = np.empty_like(x); lib().orc_fill_linear(_p(x), _p(r), x.size); return r


def fill_spline(x):
    """S/UnivariateTimeSeries.scala:268-297 over commons-math3 3.4.1 SplineInterpolator."""
    x = _vec(x); r = np.empty_like(x)
    st = lib().orc_fill_spline(_p(x), _p(r), x.size)
    if st == ERR_TOO_FEW_POINTS:
        raise OracleError(st, "number of points (%d)" % int(np.count_nonzero(~np.isnan(x))))
    return r


def fillts(x, method: str):
    if method not in FILL_METHODS:
        raise OracleError(ERR_UNSUPPORTED_METHOD, "unsupported fill method %r" % method)
    return {"linear": fill_linear, "nearest": fill_nearest, "next": fill_next,
            "previous": fill_previous, "spline": fill_spline}[method](x)


def time_fill_ns(x, method: str, reps: int = 50) -> float:
    """Best-of-reps ns of one fillts call on one core (timed inside C)."""
    x = _vec(x); r = np.empty_like(x)
    return lib().orc_time_fill(_p(x), _p(r), x.size, FILL_METHODS[method], reps)


def time_autocorr_ns(x, num_lags: int, reps: int = 50) -> float:
    x = _vec(x); out = np.empty(max(num_lags, 1))
    return lib().orc_time_autocorr(_p(x), x.size, num_lags, _p(out), reps)


def autocorr(x, num_lags: int):
    x = _vec(x); out = np.empty(num_lags); lib().orc_autocorr(_p(x), x.size, num_lags, _p(out)); return out


def lag(x, max_lag: int, include_original: bool):
    """Breeze DenseMatrix (n - max_lag) x ncols, returned as a 2-D numpy array
    (rows, cols); the column-major buffer is out.T.ravel()."""
    x = _vec(x)
    ncols = max_lag + (1 if include_original else 0)
    rows = x.size - max_lag
    buf = np.empty(max(rows, 0) * ncols)
    st = lib().orc_lag_mat_trim_both(_p(x), x.size, max_lag, int(include_original), _p(buf))
    if st != OK:
        raise OracleError(st, "bad lag arguments")
    return buf.reshape(ncols, rows).T.copy()


def differences_at_lag(ts, lag_: int, dest=None, start=None, inplace=False):
    ts = _vec(ts)
    start = lag_ if start is None else start
    if inplace:
        d = ts
    else:
        d = ts.copy() if dest is None else _vec(dest).copy()
    st = lib().orc_differences_at_lag(_p(ts), _p(d), ts.size, lag_, start)
    if st != OK:
        raise OracleError(st, "requirement failed: starting index cannot be less than lag")
    return d


def inverse_differences_at_lag(d, lag_: int, start=None):
    d = _vec(d); out = d.copy()
    start = lag_ if start is None else start
    st = lib().orc_inverse_differences_at_lag(_p(d), _p(out), d.size, lag_, start)
    if st != OK:
        raise OracleError(st, "requirement failed: starting index cannot be less than lag")
    return out


def differences_of_order_d(ts, d: int):
    ts = _vec(ts); out = np.empty_like(ts); lib().orc_differences_of_order_d(_p(ts), _p(out), ts.size, d); return out


def ewma_add(ts, s: float, dest=None):
    ts = _vec(ts); out = np.empty_like(ts) if dest is None else dest
    lib().orc_ewma_add(_p(ts), _p(out), ts.size, s); return out


def ewma_remove(ts, s: float, dest=None):
    ts = _vec(ts); out = np.empty_like(ts) if dest is None else dest
    lib().orc_ewma_remove(_p(ts), _p(out), ts.size, s); return out


def ar_remove(ts, c: float, coef):
    ts = _vec(ts); coef = _vec(coef); out = np.empty_like(ts)
    lib().orc_ar_remove(_p(ts), _p(out), ts.size, c, _p(coef), coef.size); return out


def ar_add(ts, c: float, coef, inplace=False):
    ts = _vec(ts); coef = _vec(coef); out = ts if inplace else np.empty_like(ts)
    lib().orc_ar_add(_p(ts), _p(out), ts.size, c, _p(coef), coef.size); return out


def ar_fit(ts, p: int, no_intercept: bool = False):
    ts = _vec(ts); c = np.zeros(1); coef = np.zeros(p)
    st = lib().orc_ar_fit(_p(ts), ts.size, p, int(no_intercept), _p(c), _p(coef))
    if st != OK:
        raise OracleError(st, "AR fit failed (status %d)" % st)
    return float(c[0]), coef


def ewma_sse(ts, s: float) -> float:
    ts = _vec(ts); return lib().orc_ewma_sse(_p(ts), ts.size, s)


def ewma_gradient(ts, s: float) -> float:
    ts = _vec(ts); return lib().orc_ewma_gradient(_p(ts), ts.size, s)


def ewma_fit(ts):
    """EWMA.fitModel (S/models/EWMA.scala:44-68) -> (status, smoothing, evaluations)."""
    ts = _vec(ts); sm = np.zeros(1); ev = ctypes.c_int64(0)
    st = lib().orc_ewma_fit(_p(ts), ts.size, _p(sm), ctypes.byref(ev))
    return st, float(sm[0]), int(ev.value)


def fdlibm_log(x: float) -> float:
    return lib().orc_fdlibm_log(float(x))


def garch_loglik(ts, omega: float, alpha: float, beta: float) -> float:
    """GARCHModel.logLikelihood (S/models/GARCH.scala:80-86)."""
    ts = _vec(ts); return lib().orc_garch_loglik(_p(ts), ts.size, omega, alpha, beta)


def garch_gradient(ts, omega: float, alpha: float, beta: float):
    """GARCHModel.gradient (:94-114) -> [alpha, beta, omega] components (the reference's order)."""
    ts = _vec(ts); g = np.zeros(3); lib().orc_garch_gradient(_p(ts), ts.size, omega, alpha, beta, _p(g))
    return g


def garch_fit(ts):
    """GARCH.fitModel (:33-53) -> (status, (omega, alpha, beta), evaluations)."""
    ts = _vec(ts); out = np.zeros(3); ev = ctypes.c_int64(0)
    st = lib().orc_garch_fit(_p(ts), ts.size, _p(out), ctypes.byref(ev))
    return st, out, int(ev.value)


def argarch_fit(ts):
    """ARGARCH.fitModel (:62-68) -> (status, (c, phi, omega, alpha, beta), evaluations)."""
    ts = _vec(ts); out = np.zeros(5); ev = ctypes.c_int64(0)
    st = lib().orc_argarch_fit(_p(ts), ts.size, _p(out), ctypes.byref(ev))
    return st, out, int(ev.value)


def garch_remove(ts, omega, alpha, beta):
    ts = _vec(ts); out = np.empty_like(ts); lib().orc_garch_remove(_p(ts), _p(out), ts.size, omega, alpha, beta)
    return out


def garch_add(ts, omega, alpha, beta):
    ts = _vec(ts); out = np.empty_like(ts); lib().orc_garch_add(_p(ts), _p(out), ts.size, omega, alpha, beta)
    return out


def argarch_remove(ts, c, phi, omega, alpha, beta, inplace=False):
    ts = _vec(ts); out = ts if inplace else np.empty_like(ts)
    lib().orc_argarch_remove(_p(ts), _p(out), ts.size, c, phi, omega, alpha, beta)
    return out


def argarch_add(ts, c, phi, omega, alpha, beta):
    ts = _vec(ts); out = np.empty_like(ts)
    lib().orc_argarch_add(_p(ts), _p(out), ts.size, c, phi, omega, alpha, beta)
    return out


def stat_counter(ts):
    """Spark StatCounter over the series values -> (count, mean, m2, max, min)."""
    ts = _vec(ts); out = np.zeros(4); lib().orc_stat_counter(_p(ts), ts.size, _p(out))
    return (ts.size,) + tuple(float(v) for v in out)


def remove_instants_with_nans(x):
    """TimeSeriesRDD.removeInstantsWithNaNs over one panel -> (out (S, n), active (n,))."""
    x = np.ascontiguousarray(x, dtype=np.float64); S, T = x.shape
    out = np.empty(S * T); active = np.empty(max(T, 1), np.int64)
    n = lib().orc_remove_instants_with_nans(_p(x), S, T, T, _p(out),
                                            active.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)))
    return out[: S * n].reshape(S, n), active[:n]


def to_instants(x):
    x = np.ascontiguousarray(x, dtype=np.float64); S, T = x.shape
    out = np.empty((T, S)); lib().orc_to_instants(_p(x), S, T, T, _p(out)); return out


def _java_hash(key):
    """java.lang.String.hashCode restated with numpy int32 arithmetic (wraps like Java's int)."""
    units = np.frombuffer(key.encode("utf-16-be", "surrogatepass"), dtype=">u2").astype(np.int64)
    h = np.int64(0)
    for u in units:
        h = np.int64(((h * 31 + u + 2**31) % 2**32) - 2**31)
    return int(h)


def observations_to_panel(target_index, keys, timestamps, values, num_partitions=1):
    """S/TimeSeriesRDD.scala:493-542 restated in Python (small cases): the observations go to
    partition nonNegativeMod(key.hashCode, numPartitions) (HashPartitioner, :509-513) and are
    sorted there by (key, timestamp) with String.compareTo -- UTF-16 code units -- (:502-507;
    a stable sort, so equal (key, timestamp) pairs keep input order); then per key, in that
    order, a NaN series with series(locAtDateTime(ts)) = value for every sample whose
    timestamp is in the index (:517-537).  Returns (keys in record order, (S, T) panel)."""
    idx = {int(t): i for i, t in enumerate(target_index)}

    def part(k):
        h = _java_hash(k)
        m = int(np.fmod(h, num_partitions))           # Java %: truncates toward zero
        return m + num_partitions if m < 0 else m

    def u16(k):
        return k.encode("utf-16-be", "surrogatepass")   # big-endian code units: bytewise = unitwise order
    obs = sorted(range(len(keys)), key=lambda i: (part(keys[i]), u16(keys[i]), int(timestamps[i])))
    out = {}
    order = []
    for i in obs:
        if keys[i] not in out:
            out[keys[i]] = np.full(len(target_index), np.nan)
            order.append(keys[i])
        loc = idx.get(int(timestamps[i]), -1)
        if loc >= 0:
            out[keys[i]][loc] = values[i]
    return order, np.array([out[k] for k in order]).reshape(len(order), len(target_index))


def wire_records(keys, panel) -> bytes:
    """KeyAndSeriesToBytes / python _TimeSeriesSerializer.dumps (python/sparkts/timeseriesrdd.py:
    244-256): int32 BE keyLen, UTF-8 key, int32 BE n, n x '!d'."""
    import struct
    parts = []
    for k, row in zip(keys, panel):
        kb = k.encode("utf-8")
        row = np.asarray(row, dtype=np.float64)
        parts.append(struct.pack("!i", len(kb)) + kb + struct.pack("!i", row.size) + row.astype(">f8").tobytes())
    return b"".join(parts)


# ---------------- panel drivers ----------------

def _panel(x):
    x = np.ascontiguousarray(x, dtype=np.float64)
    assert x.ndim == 2
    return x


def panel_fill(x, method: str, threads: int = 1):
    x = _panel(x); S, T = x.shape; out = np.empty_like(x); err = np.zeros(S, np.int32)
    lib().orc_panel_fill(_p(x), _p(out), S, T, T, FILL_METHODS[method],
                         err.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), threads)
    return out, err


def panel_fill_autocorr(x, method, K: int, threads: int = 1):
    x = _panel(x); S, T = x.shape; filled = np.empty_like(x); acf = np.empty((S, K))
    err = np.zeros(S, np.int32)
    m = -1 if method is None else FILL_METHODS[method]
    lib().orc_panel_fill_autocorr(_p(x), _p(filled), S, T, T, m, K, _p(acf),
                                  err.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), threads)
    return filled, acf, err


def panel_fill_diff_ewma(x, s: float, threads: int = 1):
    x = _panel(x); S, T = x.shape; out = np.empty_like(x)
    lib().orc_panel_fill_diff_ewma(_p(x), _p(out), S, T, T, s, threads); return out


def panel_ar_fit_remove(x, p: int, no_intercept=False, threads: int = 1):
    x = _panel(x); S, T = x.shape; out = np.empty_like(x); c = np.empty(S); coef = np.empty((S, p))
    lib().orc_panel_ar_fit_remove(_p(x), _p(out), S, T, T, p, int(no_intercept), _p(c), _p(coef), threads)
    return out, c, coef


def panel_ewma_fit(x, threads: int = 1):
    x = _panel(x); S, T = x.shape; sm = np.empty(S); err = np.zeros(S, np.int32)
    lib().orc_panel_ewma_fit(_p(x), S, T, T, _p(sm), err.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), threads)
    return sm, err


def panel_garch_fit(x, threads: int = 1):
    x = _panel(x); S, T = x.shape; par = np.empty((S, 3)); err = np.zeros(S, np.int32)
    lib().orc_panel_garch_fit(_p(x), S, T, T, _p(par), err.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), threads)
    return par, err


def panel_argarch_fit(x, threads: int = 1):
    x = _panel(x); S, T = x.shape; par = np.empty((S, 5)); err = np.zeros(S, np.int32)
    lib().orc_panel_argarch_fit(_p(x), S, T, T, _p(par), err.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), threads)
    return par, err


# ---------------- generator ----------------

def gen_panel(seed: int, S: int, T: int, nan_p: float, s0: int = 0):
    out = np.empty((S, T)); lib().orc_gen_panel(seed, s0, S, T, T, nan_p, _p(out)); return out


def gen_ar_panel(seed: int, S: int, T: int, p: int, s0: int = 0):
    out = np.empty((S, T)); lib().orc_gen_ar_panel(seed, s0, S, T, T, p, _p(out)); return out


def gen_ar_params(seed: int, s: int, p: int):
    c = np.zeros(1); phi = np.zeros(p); lib().orc_gen_ar_params(seed, s, p, _p(c), _p(phi))
    return float(c[0]), phi
