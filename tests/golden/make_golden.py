"""Generate the committed golden fixtures under tests/golden/ (test infrastructure only).

    python tests/golden/make_golden.py        # rewrites kats.json and panels.npz

kats.json  -- the reference's own known-answer vectors, transcribed as DATA (inputs and
              expected outputs) with the ScalaTest file:line each comes from
              (T/ = /root/reference/src/test/scala/com/cloudera/sparkts/).  The reference is
              Scala/JVM and cannot run here, so these vectors are the pins.
panels.npz -- seeded small panels with edge cases (leading / trailing / interior NaN runs,
              constant, alternating, runs longer than a tile halo) and the CPU
              oracle's outputs for every hot-path operator (oracle/sts_oracle.c, which follows
              S/UnivariateTimeSeries.scala, S/Lag.scala, S/models/EWMA.scala and
              S/models/Autoregression.scala loop for loop).  The oracle is itself pinned by
              kats.json (tests/test_golden.py); the GPU tests compare the HIP path with these
              frozen outputs, so a regression in either side shows up against the fixture.

Nothing here imports or reads /root/reference at run time.
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

NaN = float("nan")

# (file:line, method, input, expected) -- T/FillSuite.scala:35-61 (the :25-33 nearest suite
# is `ignore`d in the reference and contradicts the code; it is deliberately absent).
FILL = [
    ("T/FillSuite.scala:36", "previous", [1.0], [1.0]),
    ("T/FillSuite.scala:37", "previous", [1.0, 1.0, 2.0], [1.0, 1.0, 2.0]),
    ("T/FillSuite.scala:38", "previous", [1.0, NaN, 2.0], [1.0, 1.0, 2.0]),
    ("T/FillSuite.scala:39", "previous", [1.0, NaN, NaN, 2.0], [1.0, 1.0, 1.0, 2.0]),
    ("T/FillSuite.scala:40", "previous", [1.0, NaN, NaN, NaN, 2.0], [1.0, 1.0, 1.0, 1.0, 2.0]),
    ("T/FillSuite.scala:41", "previous", [1.0, NaN, 3.0, NaN, 2.0], [1.0, 1.0, 3.0, 3.0, 2.0]),
    ("T/FillSuite.scala:45", "next", [1.0], [1.0]),
    ("T/FillSuite.scala:46", "next", [1.0, 1.0, 2.0], [1.0, 1.0, 2.0]),
    ("T/FillSuite.scala:47", "next", [1.0, NaN, 2.0], [1.0, 2.0, 2.0]),
    ("T/FillSuite.scala:48", "next", [1.0, NaN, NaN, 2.0], [1.0, 2.0, 2.0, 2.0]),
    ("T/FillSuite.scala:49", "next", [1.0, NaN, NaN, NaN, 2.0], [1.0, 2.0, 2.0, 2.0, 2.0]),
    ("T/FillSuite.scala:50", "next", [1.0, NaN, 3.0, NaN, 2.0], [1.0, 3.0, 3.0, 2.0, 2.0]),
    ("T/FillSuite.scala:54", "linear", [1.0], [1.0]),
    ("T/FillSuite.scala:55", "linear", [1.0, 1.0, 2.0], [1.0, 1.0, 2.0]),
    ("T/FillSuite.scala:56", "linear", [1.0, NaN, 2.0], [1.0, 1.5, 2.0]),
    ("T/FillSuite.scala:57", "linear", [2.0, NaN, 1.0], [2.0, 1.5, 1.0]),
    ("T/FillSuite.scala:58", "linear", [1.0, NaN, NaN, 4.0], [1.0, 2.0, 3.0, 4.0]),
    ("T/FillSuite.scala:59", "linear", [1.0, NaN, NaN, NaN, 5.0], [1.0, 2.0, 3.0, 4.0, 5.0]),
    ("T/FillSuite.scala:60", "linear", [1.0, NaN, 3.0, NaN, 2.0], [1.0, 2.0, 3.0, 2.5, 2.0]),
]

# T/UnivariateTimeSeriesSuite.scala:31-39: lag(v, 2, includeOriginal) as row-major rows
LAG = [
    ("T/UnivariateTimeSeriesSuite.scala:31-34", [1.0, 2.0, 3.0, 4.0, 5.0], 2, True,
     [[3.0, 2.0, 1.0], [4.0, 3.0, 2.0], [5.0, 4.0, 3.0]]),
    ("T/UnivariateTimeSeriesSuite.scala:36-39", [1.0, 2.0, 3.0, 4.0, 5.0], 2, False,
     [[2.0, 1.0], [3.0, 2.0], [4.0, 3.0]]),
]

# T/models/EWMASuite.scala:21-50: addTimeDependentEffects of 1..10, last value rounded to
# 2 decimals; removeTimeDependentEffects of the rounded smoothed series, int of the last
EWMA_ADD = [
    ("T/models/EWMASuite.scala:21-30", list(range(1, 11)), 0.2, 6.54),
    ("T/models/EWMASuite.scala:32-38", list(range(1, 11)), 0.6, 9.33),
]
EWMA_REMOVE = [
    ("T/models/EWMASuite.scala:41-50", [1.0, 1.2, 1.56, 2.05, 2.64, 3.31, 4.05, 4.84, 5.67, 6.54], 0.2, 10),
]

# T/TimeSeriesRDDSuite.scala:210-229 removeInstantsWithNaNs: 3 series x 4 instants
REMOVE_INSTANTS = [
    ("T/TimeSeriesRDDSuite.scala:210-229",
     [[1.0, 2.0, 3.0, 4.0], [5.0, NaN, 7.0, 8.0], [9.0, 10.0, 11.0, NaN]],
     [[1.0, 3.0], [5.0, 7.0], [9.0, 11.0]], [0, 2]),
]


def _jsonable(v):
    if isinstance(v, float) and v != v:
        return "NaN"
    if isinstance(v, (list, tuple)):
        return [_jsonable(u) for u in v]
    return v


def edge_panel(seed, T):
    """Series exercising every imputation branch, derived from the counter-based generator
    (oracle.gen_panel == sts_gen_panel on the device) with fixed masks, so the long case
    can be regenerated bit for bit instead of stored.  Index 1 stays valid (nearest)."""
    import oracle
    x = oracle.gen_panel(seed, 1, T, 0.0)[0]
    rows = [x.copy()]                                                        # dense
    y = oracle.gen_panel(seed + 100, 1, T, 0.3)[0]; y[1] = 3.0; rows.append(y)  # 30 % NaN
    y = x.copy(); y[:7] = NaN; y[-5:] = NaN; y[1] = 4.0; rows.append(y)      # head / tail runs
    y = x.copy(); y[T // 3: T // 3 + 200] = NaN; rows.append(y)              # run > tile halo
    rows.append(np.full(T, 2.5))                                             # constant
    y = x.copy(); y[0] = NaN; y[2::2] = NaN; rows.append(y)                  # alternating
    return np.array(rows)


def digest(a):
    """sha256 of the float64 bytes with every NaN canonicalised (NaN payloads are not part
    of the contract); used where storing the array would bloat the fixture."""
    import hashlib
    a = np.ascontiguousarray(a, dtype=np.float64).copy()
    a[np.isnan(a)] = np.nan
    return hashlib.sha256(a.tobytes()).hexdigest()


def long_panel():
    """Tile-kernel case (T > 16384), regenerated rather than stored."""
    import oracle
    x = np.vstack([oracle.gen_panel(12, 2, 16400, 0.05), edge_panel(12, 16400)])
    x[:, 1] = np.where(np.isnan(x[:, 1]), 1.0, x[:, 1])
    return x


def main():
    import oracle

    kats = {
        "_doc": "Reference known-answer vectors (data only); NaN encoded as the string 'NaN'.",
        "fill": [dict(src=a, method=m, x=_jsonable(x), want=_jsonable(w)) for a, m, x, w in FILL],
        "lag": [dict(src=a, x=x, max_lag=p, include_original=inc, want=w) for a, x, p, inc, w in LAG],
        "ewma_add_rounded_last": [dict(src=a, x=x, smoothing=s, last_2dp=l) for a, x, s, l in EWMA_ADD],
        "ewma_remove_int_last": [dict(src=a, x=x, smoothing=s, int_last=l) for a, x, s, l in EWMA_REMOVE],
        "remove_instants_with_nans": [dict(src=a, x=_jsonable(x), want=w, active=act)
                                      for a, x, w, act in REMOVE_INSTANTS],
    }
    with open(os.path.join(HERE, "kats.json"), "w") as f:
        json.dump(kats, f, indent=1)

    out = {}
    # short (segment kernel, T <= 16384): inputs and outputs stored in full
    x = np.vstack([oracle.gen_panel(11, 4, 1000, 0.05), edge_panel(11, 1000)])
    x[:, 1] = np.where(np.isnan(x[:, 1]), 1.0, x[:, 1])   # nearest: never all-NaN
    out["short_x"] = x
    out["short_K"] = np.int64(20)
    for m in ("linear", "previous", "next", "nearest"):
        f, a, err = oracle.panel_fill_autocorr(x, m, 20)
        assert (err == 0).all()
        out["short_fill_%s" % m] = f
        out["short_acf_%s" % m] = a
    # long (tile kernel): input regenerated (digest pins it), fills as digests, ACF in full
    x = long_panel()
    out["long_x_sha256"] = np.array(digest(x))
    out["long_K"] = np.int64(60)
    for m in ("linear", "previous", "next", "nearest"):
        f, a, err = oracle.panel_fill_autocorr(x, m, 60)
        assert (err == 0).all()
        out["long_fill_%s_sha256" % m] = np.array(digest(f))
        out["long_acf_%s" % m] = a
    # differencing, lag matrix, EWMA, AR on a NaN-free panel
    x = oracle.gen_panel(13, 8, 777, 0.0)
    out["dense_x"] = x
    out["diff_lag3"] = np.array([oracle.differences_at_lag(r, 3) for r in x])
    out["diff_lag3_inplace"] = np.array([oracle.differences_at_lag(r, 3, inplace=True) for r in x.copy()])
    out["lag10_false"] = np.array([oracle.lag(r, 10, False) for r in x])
    out["lag4_true"] = np.array([oracle.lag(r, 4, True) for r in x])
    sm = np.linspace(0.1, 0.9, x.shape[0])
    out["ewma_s"] = sm
    out["ewma_add"] = np.array([oracle.ewma_add(r, s) for r, s in zip(x, sm)])
    out["ewma_remove"] = np.array([oracle.ewma_remove(r, s) for r, s in zip(x, sm)])
    xa = oracle.gen_ar_panel(14, 4, 2520, 5)
    out["ar_x"] = xa
    c = np.empty(4); coef = np.empty((4, 5))
    for s in range(4):
        c[s], coef[s] = oracle.ar_fit(xa[s], 5, False)
    out["ar5_c"] = c
    out["ar5_coef"] = coef
    out["ar5_remove"] = np.array([oracle.ar_remove(r, cc, ph) for r, cc, ph in zip(xa, c, coef)])
    np.savez_compressed(os.path.join(HERE, "panels.npz"), **out)
    print("wrote kats.json and panels.npz (%d arrays)" % len(out))


if __name__ == "__main__":
    main()
