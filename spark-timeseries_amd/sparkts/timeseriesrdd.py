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
    def __init__(self, index, keys: Optional[Sequence[str]], data):
        self.index = index
        self.data = data
        self.keys = list(keys) if keys is not None else None

    # --- S/TimeSeriesRDD.scala:180-182 ---
    def fill(self, method: str) -> "TimeSeriesRDD":
        """fill(method) == mapSeries(UnivariateTimeSeries.fillts(_, method))."""
        return TimeSeriesRDD(self.index, self.keys, uts.fillts(self.data, method))

    # --- S/TimeSeriesRDD.scala:188-199 ---
    def mapSeries(self, f: Callable, index=None) -> "TimeSeriesRDD":
        """Apply f to every series.  f receives the whole (S, T) partition panel and must
        be a batched operator (every function of UnivariateTimeSeries / models is), which
        is how a Spark task's per-record closure becomes one kernel launch."""
        out = f(self.data)
        return TimeSeriesRDD(self.index if index is None else index, self.keys, out)

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
        return TimeSeriesRDD(self.index, self.keys, filled), acf

    def collectAsTimeSeries(self):
        """(index, keys, (T, S) column-major matrix) like S/TimeSeriesRDD.scala:62-74."""
        d = self.data.cpu().numpy() if hasattr(self.data, "cpu") else self.data
        return self.index, self.keys, d.T

    def count(self) -> int:
        return int(self.data.shape[0])


def all_gather_results(local, group=None):
    """All-gather per-series results of every partition (ragged S per rank allowed) into
    one tensor in partition order -- the build's only collective (RCCL on ROCm)."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return local
    world = dist.get_world_size(group)
    n = torch.tensor([local.shape[0]], device=local.device, dtype=torch.int64)
    sizes = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(sizes, n, group=group)
    sizes = [int(x.item()) for x in sizes]
    m = max(sizes)
    pad = local.new_zeros((m,) + tuple(local.shape[1:]))
    pad[: local.shape[0]] = local
    bufs = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(bufs, pad, group=group)
    return torch.cat([b[:k] for b, k in zip(bufs, sizes)], dim=0)
