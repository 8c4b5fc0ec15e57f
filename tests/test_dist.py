"""The N > 1 path on CPU: two (and four) gloo ranks on 127.0.0.1.

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

from sparkts.timeseriesrdd import (ResultGather, all_gather_results, all_reduce_nan_flags, exchange_instants,
                                   shard_range)


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
    # the per-job gather (sizes exchanged once) reused over steps, as bench.py does
    gather = ResultGather(b - a, (3,), torch.float64, torch.device("cpu"))
    for step in range(3):
        again = all_gather_results(local + step, gather=gather)
        assert again.tolist() == (got + step).tolist()
    q.put((rank, got.numpy().tolist()))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("n,world", [(10, 2), (7, 2), (9, 4), (3, 4)])
def test_all_gather_results_ranks(n, world):
    # world 4 rehearses more ranks than the CPU pair (ragged shards, an empty one at n = 3)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = [[float(i)] * 3 for i in range(n)]
    assert all(res[r] == want for r in range(world))


def _worker_instants(rank, world, port, S, T, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    full = torch.arange(S * T, dtype=torch.float64).reshape(S, T)      # global panel, series-major
    a, b = shard_range(S, rank, world)
    # removeInstantsWithNaNs: rank r flags the instants its partition has NaN at
    flags = torch.zeros(T, dtype=torch.uint8)
    flags[(rank * 3) % T] = 1
    flags = all_reduce_nan_flags(flags)
    # toInstants: local transpose of the partition, then the all-to-all by time
    got, (t0, t1) = exchange_instants(full[a:b].t().contiguous())
    q.put((rank, flags.tolist(), (t0, t1), got.numpy().tolist()))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("S,T", [(5, 4), (7, 9), (3, 1)])
def test_instant_collectives_two_ranks(S, T):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_instants, args=(r, 2, port, S, T, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    for _ in procs:
        r, flags, rng, got = q.get(timeout=120)
        res[r] = (flags, rng, got)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want_flags = [0] * T
    for r in range(2):
        want_flags[(r * 3) % T] = 1
    full = torch.arange(S * T, dtype=torch.float64).reshape(S, T)
    for r in range(2):
        flags, (t0, t1), got = res[r]
        assert flags == want_flags
        assert (t0, t1) == shard_range(T, r, 2)
        assert got == full.t()[t0:t1].tolist()
