"""The multi-GPU path's collectives on RCCL, on one MI355X (world size 1).

The N > 1 bench and the sparkts collectives are covered with 2- and 4-rank gloo tests on CPU
(tests/test_dist.py, tests/test_bench_dist.py); 8-GPU runs belong to the driver.  What those
cannot show is the `nccl` (= RCCL) side itself: `init_process_group("nccl", device_id=...)` as
bench.py does it, and every collective the build issues -- ResultGather's all_gather /
all_gather_into_tensor, the NaN-flag all_reduce(MAX), exchange_instants' all_to_all_single,
timed_region's barrier and all_reduce(MAX) -- on device tensors.  A one-rank communicator
runs all of them through RCCL on the GPU here, in a child process (the process group must not
outlive the test), against the fused fill + ACF result of the product library."""
import os
import socket
import subprocess
import sys
import textwrap

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = textwrap.dedent("""
    import os, sys, json
    sys.path.insert(0, os.path.join({root!r}, "spark-timeseries_amd"))
    sys.path.insert(0, {root!r})
    import torch
    import torch.distributed as dist
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", init_method="tcp://127.0.0.1:{port}", rank=0, world_size=1, device_id=dev)
    from sparkts import TimeSeriesRDD
    from sparkts.timeseriesrdd import ResultGather, all_gather_results, all_reduce_nan_flags, exchange_instants
    import bench
    out = {{"backend": dist.get_backend()}}
    g = torch.Generator(device="cpu").manual_seed(7)
    x = torch.randn((6, 5000), generator=g, dtype=torch.float64)
    x[x.abs() < 0.05] = float("nan")
    x[:, 0] = 1.0
    x[:, -1] = 2.0
    filled, acf = TimeSeriesRDD(None, None, x.to(dev)).fillAndAutocorr("linear", 20)
    rg = ResultGather(6, (20,), torch.float64, dev)
    got = rg(acf)
    out["gather_equal"] = bool(torch.equal(got, acf))
    out["gather_again_equal"] = bool(torch.equal(rg(acf), acf))
    out["one_shot_equal"] = bool(torch.equal(all_gather_results(acf), acf))
    flags = torch.isnan(x.to(dev)).any(dim=0).to(torch.uint8)
    out["flags_equal"] = bool(torch.equal(all_reduce_nan_flags(flags.clone()), flags))
    inst = filled.data.t().contiguous()
    blk, (t0, t1) = exchange_instants(inst)
    out["instants_equal"] = bool(torch.equal(blk, inst)) and (t0, t1) == (0, 5000)
    calls = []
    wall, elapsed = bench.timed_region(lambda: calls.append(1), 3, 1, 2, lambda: torch.cuda.synchronize(dev), dev)
    out["timed_steps"] = len(calls)
    out["timed_max_equal"] = elapsed == wall
    dist.destroy_process_group()
    print("RESULT " + json.dumps(out))
""")


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.gpu
def test_rccl_collectives_one_rank_on_device():
    code = CHILD.format(root=ROOT, port=_free_port())
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    r = subprocess.run([sys.executable, "-u", "-c", code], capture_output=True, text=True, timeout=240, env=env,
                       cwd=ROOT)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("RESULT ")]
    assert r.returncode == 0 and lines, r.stdout[-3000:] + r.stderr[-3000:]
    import json
    res = json.loads(lines[-1][len("RESULT "):])
    assert res["backend"] == "nccl"
    assert res["gather_equal"] and res["gather_again_equal"] and res["one_shot_equal"], res
    assert res["flags_equal"] and res["instants_equal"], res
    # timed_region with world > 1 semantics: barrier + all_reduce(MAX) over the one rank
    assert res["timed_steps"] == 4 and res["timed_max_equal"], res
