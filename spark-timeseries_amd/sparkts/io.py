"""Ingest / egress formats of com.cloudera.sparkts: the step before
the hot path, staging a partition's records into the HBM panel, and the way back.

  timeSeriesRDDFromWire / TimeSeriesRDD.toWire  -- the Python wire format
      (S/PythonConnector.scala:47-90 BytesToKeyAndSeries / KeyAndSeriesToBytes,
      python/sparkts/timeseriesrdd.py:239-290): int32 BE keyLen | UTF-8 key | int32 BE n |
      n x float64 BE, records back to back.  Headers are walked on the host (O(S)); the value
      blocks are byte-swapped into the panel on the device.
  timeSeriesRDDFromObservations  -- S/TimeSeriesRDD.scala:493-542: (key, timestamp, value)
      observations scattered into a NaN panel on the device.
  timeSeriesRDDFromCsv / saveAsCsv  -- S/TimeSeriesRDD.scala:427-438, 547-561.
"""
from __future__ import annotations

import ctypes
import os
import struct

import numpy as np

from . import _native
from ._panel import Panel, check, ptr


def _torch():
    import torch
    return torch


def _device(device):
    torch = _torch()
    if device is None:
        device = torch.device("cuda", torch.cuda.current_device())
    device = torch.device(device)
    _native.ensure_device(device.index if device.index is not None else torch.cuda.current_device())
    return device


def _stream(device):
    return ctypes.c_void_p(_torch().cuda.current_stream(device).cuda_stream)


def wire_scan(data: bytes):
    """Walk the record headers -> (keys, T, val_off int64 array)."""
    buf = np.frombuffer(data, dtype=np.uint8)
    lib = _native.lib()
    n = ctypes.c_int64(0)
    T = ctypes.c_int64(0)
    # counting pass (capacity 0: the count comes back with a capacity error when > 0)
    st = lib.sts_wire_scan(buf.ctypes.data, buf.size, 0, ctypes.byref(n), ctypes.byref(T), None, None, None)
    if st != 0 and n.value == 0:
        check(st, "wire_scan")
    S = n.value
    key_off = np.empty(S, np.int64)
    key_len = np.empty(S, np.int32)
    val_off = np.empty(S, np.int64)
    check(lib.sts_wire_scan(buf.ctypes.data, buf.size, S, ctypes.byref(n), ctypes.byref(T), key_off.ctypes.data,
                            key_len.ctypes.data, val_off.ctypes.data), "wire_scan")
    keys = [bytes(buf[o: o + k]).decode("utf-8") for o, k in zip(key_off, key_len)]
    return keys, T.value, val_off


def timeSeriesRDDFromWire(index, data: bytes, device=None):
    """Records in the Python wire format -> TimeSeriesRDD (panel in HBM)."""
    from .timeseriesrdd import TimeSeriesRDD
    torch = _torch()
    dev = _device(device)
    keys, T, val_off = wire_scan(data)
    S = len(keys)
    panel = torch.empty((S, T), dtype=torch.float64, device=dev)
    if S * T:
        raw = torch.frombuffer(bytearray(data), dtype=torch.uint8).pin_memory().to(dev, non_blocking=True)
        off = torch.as_tensor(val_off, device=dev)
        check(_native.lib().sts_wire_decode(ptr(raw), ptr(off), S, T, ptr(panel), T, _stream(dev)), "wire_decode")
        torch.cuda.current_stream(dev).synchronize()
    return TimeSeriesRDD(index, keys, panel)


def toWire(rdd) -> bytes:
    """KeyAndSeriesToBytes for every record of the partition, in key order."""
    torch = _torch()
    p = Panel(rdd.data)
    keys = rdd.keys if rdd.keys is not None else [str(i) for i in range(p.S)]
    kb = [k.encode("utf-8") for k in keys]
    sizes = [8 + len(k) + 8 * p.T for k in kb]
    offs = np.zeros(p.S + 1, np.int64)
    np.cumsum(sizes, out=offs[1:])
    val_off = offs[:-1] + 8 + np.array([len(k) for k in kb], np.int64)
    out_dev = torch.empty(int(offs[-1]), dtype=torch.uint8, device=p.t.device)
    if p.S * p.T:
        off = torch.as_tensor(val_off, device=p.t.device)
        check(_native.lib().sts_wire_encode(ptr(p.t), p.S, p.T, p.ld, ptr(off), ptr(out_dev), p.stream), "wire_encode")
    out = bytearray(out_dev.cpu().numpy().tobytes())
    for o, k in zip(offs[:-1], kb):
        out[o: o + 4] = struct.pack(">i", len(k))
        out[o + 4: o + 4 + len(k)] = k
        out[o + 4 + len(k): o + 8 + len(k)] = struct.pack(">i", p.T)
    return bytes(out)


def java_string_hash(s: str) -> int:
    """java.lang.String.hashCode: h = 31 h + c over the UTF-16 code units, int32 wrap-around."""
    h = 0
    for cu in utf16_units(s):
        h = (31 * h + cu) & 0xFFFFFFFF
    return h - (1 << 32) if h >= (1 << 31) else h


def utf16_units(s: str):
    """The UTF-16 code units of s (java.lang.String's chars): String.compareTo orders by them."""
    b = s.encode("utf-16-be", "surrogatepass")
    return struct.unpack(">%dH" % (len(b) // 2), b)


def hash_partition(key: str, num_partitions: int) -> int:
    """Spark's HashPartitioner.getPartition for a String key: Utils.nonNegativeMod(
    key.hashCode, numPartitions) (Java's % truncates toward zero; a negative remainder is
    shifted up by numPartitions)."""
    h = java_string_hash(key)
    raw = abs(h) % num_partitions
    if h < 0:
        raw = -raw
    return raw + num_partitions if raw < 0 else raw


def observation_key_order(keys, num_partitions: int = 1):
    """The record order of timeSeriesRDDFromObservations (S/TimeSeriesRDD.scala:502-514): the
    observations are shuffled by HashPartitioner(numPartitions) on the key and sorted within
    each partition by (key, timestamp) with String.compareTo; one record per key, partition
    0's keys first.  Returns (ordered unique keys, partition of each)."""
    uniq = set(keys)
    part = {k: hash_partition(k, num_partitions) for k in uniq}
    ordered = sorted(uniq, key=lambda k: (part[k], utf16_units(k)))
    return ordered, [part[k] for k in ordered]


def timeSeriesRDDFromObservations(targetIndex, keys, timestamps, values, device=None, numPartitions=1):
    """S/TimeSeriesRDD.scala:493-542.  targetIndex: sorted instants (int64 / datetime64);
    keys: one string per observation; timestamps: one instant per observation; numPartitions:
    the input RDD's partition count (the reference shuffles into that many partitions).
    Series come out in the reference's record order: by hash partition of the key, then by
    String.compareTo within the partition (observation_key_order); timestamps not in the
    index are dropped (locAtDateTime == -1); among observations of one cell the last in input
    order wins.  The result's `partitions` lists each record's partition."""
    from .timeseriesrdd import TimeSeriesRDD
    torch = _torch()
    dev = _device(device)
    if numPartitions < 1:
        raise ValueError("numPartitions must be >= 1")
    idx = np.asarray(targetIndex)
    ts = np.asarray(timestamps)
    if idx.dtype.kind == "M":
        idx = idx.astype("datetime64[ns]").astype(np.int64)
    if ts.dtype.kind == "M":
        ts = ts.astype("datetime64[ns]").astype(np.int64)
    idx = idx.astype(np.int64)
    ts = ts.astype(np.int64)
    key_list = [str(k) for k in keys]
    order, parts = observation_key_order(key_list, numPartitions)
    rank = {k: i for i, k in enumerate(order)}
    sid = np.fromiter((rank[k] for k in key_list), dtype=np.int64, count=len(key_list))
    pos = np.searchsorted(idx, ts)
    pos_c = np.minimum(pos, max(len(idx) - 1, 0))
    loc = np.where((len(idx) > 0) & (idx[pos_c] == ts), pos_c, -1).astype(np.int64)
    S, T = len(order), len(idx)
    panel = torch.empty((S, T), dtype=torch.float64, device=dev)
    n = len(ts)
    sid_d = torch.as_tensor(sid.astype(np.int32), device=dev)
    loc_d = torch.as_tensor(loc, device=dev)
    val_d = torch.as_tensor(np.asarray(values, dtype=np.float64), device=dev)
    check(_native.lib().sts_observations_to_panel(ptr(sid_d), ptr(loc_d), ptr(val_d), n, ptr(panel), S, T, T,
                                                  _stream(dev)), "timeSeriesRDDFromObservations")
    rdd = TimeSeriesRDD(targetIndex, list(order), panel, partitions=parts)
    return rdd


def csv_parse(text: bytes):
    """`key,v1,...,vn` lines -> (keys, (S, T) float64 host array)."""
    buf = np.frombuffer(text, dtype=np.uint8)
    lib = _native.lib()
    n = ctypes.c_int64(0)
    T = ctypes.c_int64(0)
    st = lib.sts_csv_parse(buf.ctypes.data, buf.size, 0, ctypes.byref(n), ctypes.byref(T), None, None, None, 0)
    if st != 0 and n.value == 0:
        check(st, "csv_parse")
    S = n.value
    key_off = np.empty(max(S, 1), np.int64)
    key_len = np.empty(max(S, 1), np.int32)
    width = T.value
    vals = np.empty((S, width), np.float64)
    check(lib.sts_csv_parse(buf.ctypes.data, buf.size, S, ctypes.byref(n), ctypes.byref(T), key_off.ctypes.data,
                            key_len.ctypes.data, vals.ctypes.data, vals.size), "csv_parse")
    keys = [bytes(buf[o: o + k]).decode("utf-8") for o, k in zip(key_off[:S], key_len[:S])]
    return keys, vals


def timeSeriesRDDFromCsv(path: str, device=None):
    """S/TimeSeriesRDD.scala:547-561: every part file of `path` (lines `key,v1,...`) plus the
    `timeIndex` file (kept as its string; DateTimeIndex parsing is out of scope)."""
    from .timeseriesrdd import TimeSeriesRDD
    torch = _torch()
    dev = _device(device)
    names = sorted(f for f in os.listdir(path) if f != "timeIndex" and not f.startswith((".", "_")))
    text = b"".join(open(os.path.join(path, f), "rb").read() for f in names)
    keys, vals = csv_parse(text)
    index = None
    ti = os.path.join(path, "timeIndex")
    if os.path.exists(ti):
        index = open(ti).readline().rstrip("\n")
    panel = torch.as_tensor(vals, device=dev)
    return TimeSeriesRDD(index, keys, panel)


def java_double_to_string(v: float) -> str:
    """java.lang.Double.toString layout (NaN, Infinity, d.ddd, d.dddE±n outside [1e-3, 1e7))
    with shortest round-trip digits (JDK >= 19); values round-trip exactly either way."""
    if v != v:
        return "NaN"
    if v in (float("inf"), float("-inf")):
        return "Infinity" if v > 0 else "-Infinity"
    if v == 0.0:
        return "-0.0" if str(v).startswith("-") else "0.0"
    a = abs(v)
    sign = "-" if v < 0 else ""
    digits, exp = _shortest_digits(a)
    if 1e-3 <= a < 1e7:
        point = exp + 1
        if point <= 0:
            s = "0." + "0" * (-point) + digits
        elif point >= len(digits):
            s = digits + "0" * (point - len(digits)) + ".0"
        else:
            s = digits[:point] + "." + digits[point:]
        return sign + s
    mant = digits[0] + "." + (digits[1:] or "0")
    return sign + mant + "E" + str(exp)


def _shortest_digits(a: float):
    r = repr(a)          # shortest round-trip (Python), e.g. '1.5e-05', '123.0'
    if "e" in r:
        m, e = r.split("e")
        exp = int(e)
    else:
        m, exp = r, 0
    ip, _, fp = m.partition(".")
    digits = (ip + fp).lstrip("0")
    lead = len(ip.lstrip("0")) if ip.strip("0") else -(len(fp) - len(fp.lstrip("0")))
    exp = exp + (lead - 1 if ip.strip("0") else lead - 1)
    return digits.rstrip("0") or "0", exp


def saveAsCsv(rdd, path: str) -> None:
    """S/TimeSeriesRDD.scala:427-438: `key,v1,...` per series into path/part-00000 and the
    index string into path/timeIndex."""
    os.makedirs(path, exist_ok=True)
    d = rdd.data.cpu().numpy() if hasattr(rdd.data, "cpu") else np.asarray(rdd.data)
    keys = rdd.keys if rdd.keys is not None else [str(i) for i in range(d.shape[0])]
    with open(os.path.join(path, "part-00000"), "w") as f:
        for k, row in zip(keys, d):
            f.write(k + "," + ",".join(java_double_to_string(float(v)) for v in row) + "\n")
    with open(os.path.join(path, "timeIndex"), "w") as f:
        f.write(str(rdd.index) + "\n")
