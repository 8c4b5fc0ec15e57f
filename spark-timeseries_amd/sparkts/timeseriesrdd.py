"""Host mirror of com.cloudera.sparkts.TimeSeriesRDD's hot path (S/TimeSeriesRDD.scala:53-588).

A TimeSeriesRDD here is one PARTITION of keyed series resident in HBM: the (S, T)
panel of this rank's records (series-contiguous, exactly each record's
DenseVector.data), their keys, and the shared time index (metadata only -- the
hot path is position based).  Partitioning follows Spark's
`parallelize` slicing (contiguous key ranges per partition, `shard_range`); one
process per GPU owns one partition.  fill / mapSeries are narrow maps: no data
crosses ranks.  The only collective is `all_gather_results`, an all-gather (RCCL
over xGMI on ROCm) of small per-series results such as autocorrelations.
"""
from __future__ import annotations

from typing import Callable, Optional, Sequence

from . import UnivariateTimeSeries as uts
from . import _native
from ._panel import Panel, check, ptr


def shard_range(n_series: int, rank: int, world: int):
    """[start, end) of partition `rank` under ParallelCollectionRDD slicing:
    start = i*n/world, end = (i+1)*n/world (integer arithmetic)."""
    return (rank * n_series) // world, ((rank + 1) * n_series) // world


class TimeSeriesRDD:
    """A partition's panel: `data` (S, T), its `keys` (record order) and the shared `index`.
    `partitions` (optional, one int per record) is the Spark partition each record lives in --
    timeSeriesRDDFromObservations sets it (the reference's shuffle by key hash); every
    transformation below keeps keys, order and partitions."""

    def __init__(self, index, keys: Optional[Sequence[str]], data, partitions: Optional[Sequence[int]] = None):
        self.index = index
        self.data = data
        self.keys = list(keys) if keys is not None else None
        self.partitions = list(partitions) if partitions is not None else None

    def _derive(self, data, index=None) -> "TimeSeriesRDD":
        """A transformed panel with the same keys, record order and partitions."""
        return TimeSeriesRDD(self.index if index is None else index, self.keys, data, self.partitions)

    # --- S/TimeSeriesRDD.scala:180-182 ---
    def fill(self, method: str) -> "TimeSeriesRDD":
        """fill(method) == mapSeries(UnivariateTimeSeries.fillts(_, method))."""
        return self._derive(uts.fillts(self.data, method))

    # --- S/TimeSeriesRDD.scala:188-199 ---
    def mapSeries(self, f: Callable, index=None) -> "TimeSeriesRDD":
        """Apply f to every series; keys (and their order) are unchanged.  A closure marked
        `sparkts.pipelines.batched` (e.g. pipelines.ar_remove(p), the README.md:61 closure)
        runs ONCE on the whole (S, T) partition panel -- one kernel launch; any other
        closure runs per series as in the reference (correct for arbitrary code, one call
        per series)."""
        from .pipelines import apply_per_series, is_batched
        out = f(self.data) if is_batched(f) else apply_per_series(f, self.data)
        return self._derive(out, index)

    def autocorr(self, numLags: int):
        """rdd.mapValues(autocorr(_, numLags)) over the partition: (S, numLags)."""
        return uts.autocorr(self.data, numLags)

    def fillAndAutocorr(self, method: str, numLags: int):
        """fill(method) followed by autocorr of every filled series, fused into one pass
        over HBM.  Returns (filled TimeSeriesRDD, acf (S, K))."""
        p = Panel(self.data)
        code = uts.fill_method_code(method)
        lib = _native.lib()
        filled = p.empty()
        acf = p.empty(T=numLags)
        if not p.device:
            raise TypeError("fillAndAutocorr runs on device-resident partitions (torch GPU tensors)")
        check(lib.sts_fill_autocorr(ptr(p.t), ptr(filled), p.S, p.T, p.ld, p.T, code, numLags, ptr(acf), None,
                                    p.stream), "fill_autocorr")
        return self._derive(filled), acf

    # --- S/TimeSeriesRDD.scala:204-206 ---
    def seriesStats(self) -> "StatCounters":
        """map(kt => new StatCounter(kt._2.valuesIterator)) over the partition: one lane-per-
        series Welford pass on the device, in StatCounter.merge's order (bit-exact)."""
        p = Panel(self.data)
        if not p.device:
            raise TypeError("seriesStats runs on device-resident partitions (torch GPU tensors)")
        import torch
        st = torch.empty((p.S, 4), dtype=torch.float64, device=p.t.device)
        check(_native.lib().sts_series_stats(ptr(p.t), p.S, p.T, p.ld, ptr(st), p.stream), "seriesStats")
        return StatCounters(p.T, st)

    # --- S/TimeSeriesRDD.scala:131-152 ---
    def removeInstantsWithNaNs(self, group=None) -> "TimeSeriesRDD":
        """Drop every instant at which ANY series of the whole RDD is NaN.  The reference
        aggregates per-partition Boolean arrays with OR on the driver; here every rank
        flags its own partition on the device and the flags are combined with an
        all-reduce (MAX on uint8 = OR; RCCL over xGMI on the GPU box), then each partition
        is compacted locally.  Returns the new RDD; its index is self.index[active] when the
        index is indexable, else the kept positions."""
        import torch
        p = Panel(self.data)
        if not p.device:
            raise TypeError("removeInstantsWithNaNs runs on device-resident partitions (torch GPU tensors)")
        lib = _native.lib()
        flags = torch.zeros((p.T,), dtype=torch.uint8, device=p.t.device)
        check(lib.sts_nan_instants(ptr(p.t), p.S, p.T, p.ld, ptr(flags), p.stream), "removeInstantsWithNaNs")
        flags = all_reduce_nan_flags(flags, group)
        active = torch.empty((max(p.T, 1),), dtype=torch.int64, device=p.t.device)
        n_dev = torch.zeros((1,), dtype=torch.int64, device=p.t.device)
        check(lib.sts_active_instants(ptr(flags), p.T, ptr(active), ptr(n_dev), p.stream), "active_instants")
        n = int(n_dev.item())
        out = torch.empty((p.S, n), dtype=torch.float64, device=p.t.device)
        check(lib.sts_gather_instants(ptr(p.t), ptr(out), p.S, p.ld, n, ptr(active), n, p.stream), "gather_instants")
        kept = active[:n]
        index = self.index
        if index is not None:
            try:
                index = index[kept.cpu().numpy()]
            except (TypeError, IndexError, KeyError):
                index = kept.cpu().numpy()
        else:
            index = kept.cpu().numpy()
        return self._derive(p.out(out), index)

    # --- S/TimeSeriesRDD.scala:215-324 ---
    def toInstants(self, group=None):
        """One record per instant with every series' value, series in key (partition)
        order, instants in time order.  Locally a transpose kernel; across ranks the
        instants are re-partitioned by time with an all-to-all (RCCL over xGMI), so rank r
        returns instants [t0_r, t1_r) (shard_range over T) of ALL series -- Spark's
        toInstants shuffle.  Returns (index slice, (T_r, S_total) tensor)."""
        index, got, _ = self._instants(group)
        return index, got

    def _instants(self, group=None):
        import torch
        p = Panel(self.data)
        if not p.device:
            raise TypeError("toInstants runs on device-resident partitions (torch GPU tensors)")
        inst = torch.empty((p.T, p.S), dtype=torch.float64, device=p.t.device)
        check(_native.lib().sts_to_instants(ptr(p.t), ptr(inst), p.S, p.T, p.ld, p.S, p.stream), "toInstants")
        got, (t0, t1) = exchange_instants(inst, group)
        index = self.index
        if index is not None:
            try:
                index = index[t0:t1]
            except (TypeError, IndexError, KeyError):
                index = None
        return index, got, t0

    def toRowMatrix(self, group=None):
        """S/TimeSeriesRDD.scala:410-414: the toInstants rows without their instants (a
        RowMatrix's row order carries no meaning).  Returns this rank's (T_r, S_total) rows."""
        return self.toInstants(group)[1]

    def toIndexedRowMatrix(self, group=None):
        """S/TimeSeriesRDD.scala:385-400: toInstants rows indexed by frequency.difference(
        first, instant), i.e. the instant's position in a uniform index.  Non-uniform indices
        raise UnsupportedOperationException("only supported for uniform indices") as the
        reference does.  Returns (row indices int64 (T_r,), (T_r, S_total) rows)."""
        from .errors import UnsupportedOperationException
        if not _is_uniform(self.index):
            raise UnsupportedOperationException("only supported for uniform indices")
        import torch
        _, rows, t0 = self._instants(group)
        return torch.arange(t0, t0 + rows.shape[0], dtype=torch.int64, device=rows.device), rows

    def collectAsTimeSeries(self):
        """(index, keys, (T, S) column-major matrix) like S/TimeSeriesRDD.scala:62-74."""
        d = self.data.cpu().numpy() if hasattr(self.data, "cpu") else self.data
        return self.index, self.keys, d.T

    def count(self) -> int:
        return int(self.data.shape[0])


class StatCounters:
    """Per-series org.apache.spark.util.StatCounter values of a partition: count n (= T),
    mean, m2 from the device pass; the derived statistics follow StatCounter's own formulas."""

    def __init__(self, n: int, stats):
        self.n = n
        self.stats = stats   # (S, 4): mean, m2, max, min

    def count(self):
        return self.n

    def mean(self):
        return self.stats[:, 0]

    def sum(self):
        return self.n * self.stats[:, 0]

    def max(self):
        return self.stats[:, 2]

    def min(self):
        return self.stats[:, 3]

    def variance(self):
        return self.stats[:, 1] / self.n if self.n else self.stats[:, 1] * float("nan")

    def sampleVariance(self):
        return self.stats[:, 1] / (self.n - 1) if self.n > 1 else self.stats[:, 1] * float("nan")

    def stdev(self):
        return self.variance() ** 0.5

    def sampleStdev(self):
        return self.sampleVariance() ** 0.5


def all_reduce_nan_flags(flags, group=None):
    """OR the per-instant NaN flags (uint8) of every partition: all-reduce MAX (RCCL has
    no bitwise OR; MAX on 0/1 bytes is the same).  The reference's
    aggregate(zero)(merge, comb) (S/TimeSeriesRDD.scala:132-144)."""
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized():
        dist.all_reduce(flags, op=dist.ReduceOp.MAX, group=group)
    return flags


def exchange_instants(local, group=None):
    """Re-partition instant-major data by time: `local` is this rank's (T, S_r) block
    (every instant, this partition's series).  Returns ((T_r, S_total) for instants
    [t0, t1) = shard_range(T, rank, world), (t0, t1)); one all-to-all."""
    import torch
    import torch.distributed as dist
    T, S_r = int(local.shape[0]), int(local.shape[1])
    if not (dist.is_available() and dist.is_initialized()):
        return local, (0, T)
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    n = torch.tensor([S_r], device=local.device, dtype=torch.int64)
    sizes = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(sizes, n, group=group)
    s_all = [int(x.item()) for x in sizes]
    bounds = [shard_range(T, q, world) for q in range(world)]
    send = local.contiguous().reshape(-1)            # rows [t0_q, t1_q) are contiguous
    in_split = [(b - a) * S_r for a, b in bounds]
    t0, t1 = bounds[rank]
    out_split = [(t1 - t0) * s for s in s_all]
    recv = local.new_empty((sum(out_split),))
    dist.all_to_all_single(recv, send, out_split, in_split, group=group)
    blocks, off = [], 0
    for s, m in zip(s_all, out_split):
        blocks.append(recv[off: off + m].reshape(t1 - t0, s))
        off += m
    return torch.cat(blocks, dim=1), (t0, t1)


class ResultGather:
    """All-gather of per-series results (S_r, ...) of every partition into one (S, ...)
    tensor in partition order -- the build's only collective (RCCL over xGMI on ROCm).

    The partition sizes are static for a job, so they are exchanged ONCE here (one tiny
    all-gather + host sync at construction); every later call is a single
    all_gather_into_tensor into a buffer allocated once, with no size exchange and no
    host synchronisation.  Equal partitions return that buffer itself (valid until the
    next call; clone it to keep it); ragged ones are compacted with one precomputed
    index_select into a fresh tensor."""

    def __init__(self, n_local: int, row_shape=(), dtype=None, device=None, group=None):
        import torch
        import torch.distributed as dist
        self.group = group
        self.world = dist.get_world_size(group)
        n = torch.tensor([int(n_local)], device=device, dtype=torch.int64)
        sizes = [torch.zeros_like(n) for _ in range(self.world)]
        dist.all_gather(sizes, n, group=group)
        self.sizes = [int(x.item()) for x in sizes]
        self.n_local = int(n_local)
        self.m = max(self.sizes) if self.sizes else 0
        self.row_shape = tuple(row_shape)
        self.pad = torch.zeros((self.m,) + self.row_shape, dtype=dtype, device=device)
        self.buf = torch.empty((self.world * self.m,) + self.row_shape, dtype=dtype, device=device)
        self.uniform = all(s == self.m for s in self.sizes)
        self.keep = None
        if not self.uniform:
            idx = [q * self.m + i for q, s in enumerate(self.sizes) for i in range(s)]
            self.keep = torch.tensor(idx, dtype=torch.int64, device=device)

    def __call__(self, local):
        import torch.distributed as dist
        if int(local.shape[0]) != self.n_local or tuple(local.shape[1:]) != self.row_shape:
            raise ValueError("ResultGather: expected (%d,)+%s rows, got %s" % (self.n_local, self.row_shape,
                                                                              tuple(local.shape)))
        src = local
        if self.n_local != self.m or not local.is_contiguous():
            self.pad[: self.n_local] = local
            src = self.pad
        dist.all_gather_into_tensor(self.buf, src, group=self.group)
        return self.buf if self.uniform else self.buf.index_select(0, self.keep)


def all_gather_results(local, group=None, gather: Optional[ResultGather] = None):
    """All-gather per-series results of every partition (ragged S per rank allowed) into
    one tensor in partition order.  Pass a ResultGather built once per job to keep the
    size exchange out of a loop; without one, a one-shot gather is built for this call."""
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return local
    if gather is None:
        gather = ResultGather(local.shape[0], local.shape[1:], local.dtype, local.device, group)
    return gather(local)


def _is_uniform(index) -> bool:
    """A UniformDateTimeIndex analogue: None (positions), a range, or instants with one
    constant spacing (numpy datetime64 / numbers / ISO date strings)."""
    import numpy as np
    if index is None or isinstance(index, range):
        return True
    try:
        a = np.asarray(index)
        if a.dtype.kind in "US":
            a = a.astype("datetime64[ns]")
        if a.size < 3:
            return True
        d = np.diff(a)
        return bool((d == d[0]).all())
    except (TypeError, ValueError):
        return False
