"""The N > 1 path on CPU: two gloo ranks on 127.0.0.1.

* shard_range reproduces Spark's ParallelCollectionRDD slicing (contiguous key ranges,
  the partitioning the reference's parallelize-built TimeSeriesRDDs use);
* all_gather_results (the build's only collective; RCCL on the GPU box) returns every
  rank's per-series results in partition order, ragged shards included.
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from sparkts.timeseriesrdd import all_gather_results, shard_range


def test_shard_range_covers_keys_in_order():
    for n in (0, 1, 7, 100, 12_500 * 8, 1_000_001):
        for world in (1, 2, 3, 4, 8):
            ranges = [shard_range(n, r, world) for r in range(world)]
            assert ranges[0][0] == 0 and ranges[-1][1] == n
            for (a, b), (c, d) in zip(ranges, ranges[1:]):
                assert b == c and a <= b
            sizes = [b - a for a, b in ranges]
            assert max(sizes) - min(sizes) <= 1


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, n, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    a, b = shard_range(n, rank, world)
    # per-series "results" = global series index, 3 values each (like an S x K ACF block)
    local = torch.arange(a, b, dtype=torch.float64)[:, None].repeat(1, 3)
    got = all_gather_results(local)
    q.put((rank, got.numpy().tolist()))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("n", [10, 7])
def test_all_gather_results_two_ranks(n):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, n, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = [[float(i)] * 3 for i in range(n)]
    assert res[0] == want and res[1] == want
