"""bench.py's N > 1 path, executed: two gloo ranks on 127.0.0.1 run the
same harness functions the driver's 8-GPU run uses -- fill_acf_step (the fused call, then the
ResultGather all-gather of the ACF block inside the timed loop), timed_region (warmup, barrier +
sync on both sides, max-over-ranks elapsed), result_line / emit (rank 0 prints the one JSON line)
-- with a CPU stand-in for the kernel call: the oracle's fill('linear') + autocorr over the rank's
partition (S/TimeSeriesRDD.scala:188-199 mapSeries per partition, :417-421 collect order).
"""
import contextlib
import io
import json
import os
import socket
import sys
import time

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
S_RANK, T, K, SEED = 6, 300, 20, 17


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world), RANK=str(rank),
                      LOCAL_RANK=str(rank))
    sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "spark-timeseries_amd")]
    import bench
    import oracle
    from sparkts.timeseriesrdd import ResultGather
    w, r, _ = bench.dist_env()
    assert (w, r) == (world, rank)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    cpu = torch.device("cpu")
    x = oracle.gen_panel(SEED, S_RANK, T, 0.05, s0=rank * S_RANK)    # this rank's key partition
    acf = torch.empty((S_RANK, K), dtype=torch.float64)
    calls = []

    def kernel():   # stand-in for sts_fill_autocorr on the rank's shard
        _, a, _ = oracle.panel_fill_autocorr(x, "linear", K)
        acf.copy_(torch.from_numpy(a) + len(calls))   # step-dependent values: the gather must be fresh
        calls.append(1)
        if rank == 1:
            time.sleep(0.05)                           # the slow rank sets the job's time

    gather = ResultGather(S_RANK, (K,), torch.float64, cpu)
    step = bench.fill_acf_step(kernel, acf, gather)
    steps, warmup = 3, 2
    wall, elapsed = bench.timed_region(step, steps, warmup, world, lambda: None, cpu)
    value = float(S_RANK) * T * world * steps / elapsed
    line = bench.result_line("c3", value, world, steps, warmup, elapsed / steps * 1e3, "gloo rehearsal", S_RANK, T,
                             K, 0.05, None, None)
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        bench.emit(line, rank)
    q.put((rank, wall, elapsed, len(calls), step.gathered.numpy().copy(), buf.getvalue()))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_bench_multi_rank_path(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in procs:
        r, wall, elapsed, ncalls, gathered, out = q.get(timeout=300)
        res[r] = (wall, elapsed, ncalls, gathered, out)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    sys.path[:0] = [os.path.join(ROOT, "oracle")]
    import oracle
    # every rank ran warmup + timed steps of the fused call, and the same max-over-ranks time
    assert all(res[r][2] == 5 for r in range(world))
    el = [res[r][1] for r in range(world)]
    assert len(set(el)) == 1 and el[0] == max(res[r][0] for r in range(world))
    assert el[0] >= 3 * 0.05                       # the slow rank's three timed steps
    # the gathered ACF block of the last timed step = every partition's block, in key order
    x = oracle.gen_panel(SEED, world * S_RANK, T, 0.05)
    _, want, _ = oracle.panel_fill_autocorr(x, "linear", K)
    for r in range(world):
        g = res[r][3]
        assert g.shape == (world * S_RANK, K)
        assert np.array_equal(g, want + 4.0, equal_nan=True), r   # the last step's values (step index 4)
    # rank 0 printed exactly one JSON line, the others nothing
    lines = res[0][4].strip().splitlines()
    assert len(lines) == 1 and all(res[r][4] == "" for r in range(1, world))
    line = json.loads(lines[0])
    assert line["n_gpus"] == world and line["scaling"] == "weak" and line["steps"] == 3
    assert line["value"] == pytest.approx(world * S_RANK * T * 3 / el[0])
