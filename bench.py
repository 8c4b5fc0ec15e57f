#!/usr/bin/env python3
"""bench.py -- series-elements/s and % HBM roofline of the fused fill + ACF hot path.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload c3|c2|c4|c5|c1|ewma_fit]

Default workload (the BASELINE.json metric "fill+lag+ACF", config C3): every rank owns
a C3 shard of 12,500 series x 982,800 minute bars (fp64, 5 % NaN, Philox synthetic,
generated in HBM); one step = TimeSeriesRDD.fill("linear") + autocorr(numLags = 60)
of every series (fused: one pass over HBM) + the RCCL all-gather of the per-series
ACF results when N > 1.  Weak scaling: at N = 8 the job is exactly C3 (100k series,
786 GB).  Rank 0 prints ONE JSON line.

Multi-GPU: launched by the driver as torch.distributed.run (one process per GPU,
RANK / LOCAL_RANK / WORLD_SIZE from the env, backend "nccl" = RCCL).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "spark-timeseries_amd"))

HBM_PEAK_GBPS = 8000.0   # MI355X_MICROARCH.md: 8.0 TB/s spec

WORKLOADS = {
    # name: (series per GPU, steps per series, nan_p, seed, description)
    "c3": (12_500, 982_800, 0.05, 3,
           "C3 shard: fill('linear') + autocorr(60), 12,500 series x 982,800 steps per GPU "
           "(N=8 -> C3's 100k x 982,800, 786 GB)"),
    "c1": (10_000, 2_520, 0.05, 1, "C1: fill('linear') + autocorr(20), 10,000 series x 2,520 steps"),
    "c1_rule3": (10_000, 2_520, 0.05, 1,
                 "ACF rule-3 worst case at the C1 shape: every series the constant 100.1 with 5 % NaN (a suspended "
                 "instrument), fill('linear') + autocorr(20); every series flagged, every lag from the reference's "
                 "two-pass loop (sts_acf.hpp acf_exact_lag)"),
    "c3_rule3": (1_000, 982_800, 0.05, 3,
                 "ACF rule-3 worst case at the C3 length: 1,000 series of the constant 100.1 with 5 % NaN, "
                 "fill('linear') + autocorr(60); every series flagged (two-pass loop per lag)"),
    "c2": (1_000_000, 390, 0.05, 2,
           "C2: fillPrevious -> differencesAtLag(1) -> EWMA(0.2).add, 1,000,000 series x 390 steps"),
    "c4": (500_000, 2_520, 0.0, 4, "C4: AR(5) fit + removeTimeDependentEffects, 500,000 series x 2,520 steps"),
    "c4_levels": (500_000, 2_520, 0.0, 4,
                  "C4 shape on price levels (AR rule worst case): 1e4 + 0.01 x the C4 panel, every series flagged "
                  "and fitted with the reference's Householder-QR order (sts_ar_qr.hip), 500,000 series x 2,520 steps"),
    "stage_c2": (1_000_000, 390, 0.05, 2,
                 "C2 (fillPrevious -> differencesAtLag(1) -> EWMA(0.2).add, 1,000,000 series x 390 steps) from "
                 "HOST-resident panels through the _host entry points' pinned staging pipeline; value = the "
                 "HBM-resident rate, the host-resident rates are in 'staging'"),
    "ewma_fit": (1_000_000, 390, 0.0, 6,
                 "EWMA.fitModel (SURVEY.md 8(f) rank 1): commons-math3 NLCG + bracket + Brent per series, "
                 "1,000,000 series x 390 steps (the C2 shape)"),
    "garch_fit": (100_000, 2_520, 0.0, 11,
                  "GARCH.fitModel (SURVEY.md 8(f) rank 1): commons-math3 NLCG (3-D, goal-less) + bracket + Brent per "
                  "series, 100,000 series x 2,520 steps (x - x[:, 0] of the generated panel)"),
    "stats": (1_000_000, 390, 0.0, 7, "TimeSeriesRDD.seriesStats (Spark StatCounter per series), "
              "1,000,000 series x 390 steps (the C2 shape)"),
    "nan_instants": (1_000_000, 390, 0.0, 8,
                     "TimeSeriesRDD.removeInstantsWithNaNs, 1,000,000 series x 390 steps with NaNs at 39 "
                     "instants (flags + compaction + gather)"),
    "to_instants": (1_000_000, 390, 0.0, 9, "TimeSeriesRDD.toInstants local transpose, 1,000,000 series x 390 steps"),
    "wire_decode": (1_000_000, 390, 0.05, 10,
                    "Python wire format -> HBM panel (S/PythonConnector.scala:47-90): byte-swap decode of "
                    "1,000,000 records x 390 doubles already staged in HBM"),
    "spline": (1_000_000, 390, 0.05, 2,
               "fill('spline') (UnivariateTimeSeries.fillSpline, commons-math3 natural cubic spline, a1's fifth "
               "method), 1,000,000 series x 390 steps (the C2 shape), 5 % NaN"),
    "c5": (1_250, 10_000_000, 0.30, 5,
           "C5 shard: fill('nearest') + lag(10, false), 1,250 series x 10,000,000 steps per GPU (N=8 -> C5's "
           "10k x 10M); lag matrices written into a reused scratch slab, 10 series per call"),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="c3", choices=sorted(WORKLOADS))
    ap.add_argument("--series", type=int, default=0, help="override series per GPU (testing)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="budget of the CPU baseline sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--percall", action="store_true",
                    help="per-call latency of S = 1 (per-series) calls against the one-core CPU loop: the "
                         "crossover INTEGRATION.md's JVM facade uses (prints its own JSON line, not the metric)")
    return ap.parse_args()


def main():
    args = parse()
    if args.percall:
        return percall()
    import numpy as np
    import torch
    import torch.distributed as dist

    world, rank, local = dist_env()
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    from sparkts import _native
    from sparkts.errors import raise_for_status
    from sparkts.timeseriesrdd import ResultGather
    if os.environ.get("STS_HIP_LIB"):   # A/B runs of tools/variant.sh builds (tools/*.sh)
        _native.use_library(os.environ["STS_HIP_LIB"])
    _native.ensure_device(local)
    lib = _native.lib()
    global LIB_SHA16
    LIB_SHA16 = lib_sha16(lib._name)

    S, T, nan_p, seed, desc = WORKLOADS[args.workload]
    if args.series:
        S = args.series
    K, p_ar = 60, 5
    if args.workload in ("c1", "c1_rule3"):
        K = 20
    s0 = rank * S                      # this rank's partition of the keyed panel
    stream = torch.cuda.current_stream(dev)
    sp = stream.cuda_stream

    x = torch.empty((S, T), dtype=torch.float64, device=dev)
    out = torch.empty_like(x)
    acf = torch.empty((S, K), dtype=torch.float64, device=dev)
    err = torch.zeros(S, dtype=torch.int32, device=dev)
    if args.workload in ("stage_c2",):
        pass
    if args.workload in ("c4", "c4_levels"):
        cgen = torch.empty(S, dtype=torch.float64, device=dev)
        pgen = torch.empty((S, p_ar), dtype=torch.float64, device=dev)
        raise_for_status(lib.sts_gen_ar_panel(x.data_ptr(), cgen.data_ptr(), pgen.data_ptr(), s0, S, T, T, seed, p_ar,
                                              sp), "gen")
        if args.workload == "c4_levels":
            x.mul_(0.01).add_(1e4)
        c_fit = torch.empty(S, dtype=torch.float64, device=dev)
        coef_fit = torch.empty((S, p_ar), dtype=torch.float64, device=dev)
    else:
        raise_for_status(lib.sts_gen_panel(x.data_ptr(), s0, S, T, T, seed, nan_p, sp), "gen")
        if args.workload in ("c1_rule3", "c3_rule3"):
            x.masked_fill_(~torch.isnan(x), 100.1)
    smooth = torch.full((S,), 0.2, dtype=torch.float64, device=dev)
    if args.workload == "ewma_fit":
        smooth = torch.empty((S,), dtype=torch.float64, device=dev)
    if args.workload == "stats":
        stats = torch.empty((S, 4), dtype=torch.float64, device=dev)
    if args.workload == "garch_fit":
        x -= x[:, :1].clone()                      # return-like rows around 0 (exact, same on the CPU side)
        gpar = torch.empty((S, 3), dtype=torch.float64, device=dev)
    if args.workload == "nan_instants":
        x[::997, ::10] = float("nan")              # every 10th instant has a NaN somewhere
        flags = torch.zeros(T, dtype=torch.uint8, device=dev)
        active = torch.empty(T, dtype=torch.int64, device=dev)
        n_act = torch.zeros(1, dtype=torch.int64, device=dev)
        n_keep = T - len(range(0, T, 10))
    if args.workload == "to_instants":
        inst = torch.empty((T, S), dtype=torch.float64, device=dev)
    if args.workload == "wire_decode":   # records "k%07d": 16-B headers, 8-B aligned value blocks
        rec = 16 + 8 * T
        val_off = (torch.arange(S, dtype=torch.int64, device=dev) * rec + 16).contiguous()
        wire = torch.zeros(S * rec, dtype=torch.uint8, device=dev)
        raise_for_status(lib.sts_wire_encode(x.data_ptr(), S, T, T, val_off.data_ptr(), wire.data_ptr(), sp),
                         "wire_encode")
    if args.workload == "c5":
        P, LB = 10, 10            # lag(10, includeOriginal = false); series per call
        lagbuf = torch.empty((LB, P, T - P), dtype=torch.float64, device=dev)
        x[:, 1] = 1.0 + x[:, 1].nan_to_num(0.0)   # keep x[1] valid: fillNearest throws on an all-NaN tail

    # per-job result gathers: partition sizes exchanged once, outside the timed loop
    gather = None
    if world > 1 and args.workload in ("c3", "c1"):
        gather = ResultGather(S, (K,), torch.float64, dev)
    elif world > 1 and args.workload == "garch_fit":
        gather = ResultGather(S, (3,), torch.float64, dev)
    elif world > 1 and args.workload == "ewma_fit":
        gather = ResultGather(S, (1,), torch.float64, dev)
    elif world > 1 and args.workload in ("c4", "c4_levels"):
        gather = ResultGather(S, (1 + p_ar,), torch.float64, dev)

    # the headline step: one fused fill + ACF launch over the rank's shard, then the all-gather
    # of the ACF block (fill_acf_step, the same code the gloo test drives with a CPU stand-in)
    fill_acf = fill_acf_step(lambda: raise_for_status(
        lib.sts_fill_autocorr(x.data_ptr(), out.data_ptr(), S, T, T, T, 0, K, acf.data_ptr(), err.data_ptr(), sp),
        "fill_autocorr"), acf, gather)

    def step():
        if args.workload in ("c3", "c1", "c1_rule3", "c3_rule3"):
            fill_acf()
        elif args.workload in ("c2", "stage_c2"):
            raise_for_status(lib.sts_fill_diff_ewma(x.data_ptr(), out.data_ptr(), S, T, T, T, 3, 1, smooth.data_ptr(),
                                                    err.data_ptr(), sp), "fill_diff_ewma")
        elif args.workload == "spline":
            raise_for_status(lib.sts_fill(x.data_ptr(), out.data_ptr(), S, T, T, T, 4, err.data_ptr(), sp),
                             "fill(spline)")
        elif args.workload == "c5":
            for b0 in range(0, S, LB):
                nb = min(LB, S - b0)
                raise_for_status(lib.sts_fill_lag_matrix(x[b0].data_ptr(), out[b0].data_ptr(), lagbuf.data_ptr(), nb,
                                                         T, T, T, 1, P, 0, err[b0:].data_ptr(), sp),
                                 "fill_lag_matrix")
        elif args.workload == "stats":
            raise_for_status(lib.sts_series_stats(x.data_ptr(), S, T, T, stats.data_ptr(), sp), "seriesStats")
        elif args.workload == "nan_instants":
            flags.zero_()
            raise_for_status(lib.sts_nan_instants(x.data_ptr(), S, T, T, flags.data_ptr(), sp), "nan_instants")
            if world > 1:
                dist.all_reduce(flags, op=dist.ReduceOp.MAX)
            raise_for_status(lib.sts_active_instants(flags.data_ptr(), T, active.data_ptr(), n_act.data_ptr(), sp),
                             "active_instants")
            # the kept count is known to the driver after one sync; the bench reuses it
            raise_for_status(lib.sts_gather_instants(x.data_ptr(), out.data_ptr(), S, T, n_keep, active.data_ptr(),
                                                     n_keep, sp), "gather_instants")
        elif args.workload == "wire_decode":
            raise_for_status(lib.sts_wire_decode(wire.data_ptr(), val_off.data_ptr(), S, T, out.data_ptr(), T, sp),
                             "wire_decode")
        elif args.workload == "to_instants":
            raise_for_status(lib.sts_to_instants(x.data_ptr(), inst.data_ptr(), S, T, T, S, sp), "toInstants")
        elif args.workload == "garch_fit":
            raise_for_status(lib.sts_garch_fit(x.data_ptr(), S, T, T, gpar.data_ptr(), err.data_ptr(), sp),
                             "GARCH.fitModel")
            if world > 1:
                gather(gpar)
        elif args.workload == "ewma_fit":
            raise_for_status(lib.sts_ewma_fit(x.data_ptr(), S, T, T, smooth.data_ptr(), err.data_ptr(), sp),
                             "EWMA.fitModel")
            if world > 1:
                gather(smooth[:, None])
        elif args.workload in ("c4", "c4_levels"):
            raise_for_status(lib.sts_ar_fit_remove(x.data_ptr(), out.data_ptr(), S, T, T, T, p_ar, 0,
                                                   c_fit.data_ptr(), coef_fit.data_ptr(), err.data_ptr(), sp),
                             "ar_fit_remove")
            if world > 1:
                gather(torch.cat([c_fit[:, None], coef_fit], 1))

    kern_ms = np.zeros(1, dtype=np.float64)
    launches = np.zeros(1, dtype=np.int64)
    _, elapsed = timed_region(step, args.steps, args.warmup, world, lambda: torch.cuda.synchronize(dev), dev,
                              on_start=lib.sts_profile_begin,
                              on_stop=lambda: lib.sts_profile_end(kern_ms.ctypes.data, launches.ctypes.data))
    elems = float(S) * T * world * args.steps
    value = elems / elapsed
    ms_per_step = elapsed / args.steps * 1e3
    # dominant kernel (one launch per step, or one per lag-matrix batch for c5), timed with
    # HIP events the library records on the launch stream (sts_profile_begin/end)
    bytes_per_step = 16.0 * S * T        # 8 B read + 8 B written per element
    if args.workload == "c5":            # + the lag matrix: 8 * P bytes per row, (T - P) rows per series
        bytes_per_step += 8.0 * P * (T - P) * S
    if args.workload == "ewma_fit":      # the series read once + one parameter written (algorithmic)
        bytes_per_step = 8.0 * S * T + 8.0 * S
    if args.workload == "garch_fit":     # the series read once + three parameters written (algorithmic)
        bytes_per_step = 8.0 * S * T + 24.0 * S
    if args.workload == "stats":         # read once + 4 doubles per series
        bytes_per_step = 8.0 * S * T + 32.0 * S
    if args.workload == "nan_instants":  # flag pass reads everything; the gather reads + writes kept values
        bytes_per_step = 8.0 * S * T + 16.0 * S * n_keep
    kernel = {"c3": "sts::tile_kernel<4096,4,shifted> (fill linear + ACF partials, FP64 MFMA)",
              "c1_rule3": "sts::short_fill_acf_kernel<40,20> with rule 3 firing on every series (the reference's two-pass loop per lag, streamed through the LDS block: acf_exact_stream)",
              "c3_rule3": "sts::tile_kernel<4096,4,shifted> + acf_finalize_kernel with rule 3 firing on every series",
              "c1": "sts::short_fill_acf_kernel<40,20> (one wave per series in one-wave workgroups: series in by LDS-DMA, linear fill run by run in LDS, lag products as register FMAs, wave sums through LDS rows, fused ACF finalize; issue-bound, so trimmed to ~2 400 VALU per series)",
              "c5": "sts::tile_kernel<4096,0> (fill nearest + lag-matrix columns)",
              "spline": "sts::spline_lds_kernel (one lane per series: the natural spline's forward / backward "
                        "sweeps in the reference's order; rows, (mu, z) scratch and outputs moved through LDS tiles "
                        "as coalesced 16-B pieces, Horner evaluation)",
              "c2": "sts::recur_row_kernel<kFillDiffEwma,1,14,io,32> (fillPrevious -> differencesAtLag(1) -> EWMA add; whole rows through LDS, 32 lanes per series, bit-exact verified affine-scan EWMA)",
              "stage_c2": "sts::recur_row_kernel<kFillDiffEwma,1,14,io,32> (fillPrevious -> differencesAtLag(1) -> EWMA add; whole rows through LDS, 32 lanes per series)",
              "c4_levels": "sts::ar_fit_blk_kernel<5,40,4,dma> + sts::ar_qr_lane_kernel<5,true> (every series flagged: the reference's Householder-QR order, one series per lane, reflections replayed per row)",
              "c4": "sts::ar_fit_blk_kernel<5,40,4,dma> (AR(5): series in by LDS-DMA, lane-blocked register lag products, normal equations / Cholesky uniform in every lane + refinement, fused remove out through LDS)",
              "stats": "sts::stats_fast_kernel<64,16> (StatCounter.merge per lane, LDS-staged series block, division off the step chain)",
              "nan_instants": "sts::nan_instants16_kernel + sts::gather_instants_kernel (wave per row)",
              "to_instants": "sts::transpose16_kernel (64x64 LDS tiles, 16-B accesses)",
              "wire_decode": "sts::wire_decode_rows_kernel (big-endian value blocks -> panel, wave per record)",
              "garch_fit": "sts::garch_fit_kernel<64,64> (lane-per-series commons-math3 optimizer; one "
                           "logLikelihood+gradient pass over the wave's series block per optimizer request) + "
                           "sts::garch_tail_kernel<64> (wave per series past 64 passes)",
              "ewma_fit": "sts::ewma_fit_kernel<32,64> (lane-per-series commons-math3 optimizer; one sse+gradient "
                          "pass over the wave's series block per optimizer request)"}[args.workload]
    staging = staging_leg(args, lib, x, out, smooth, S, T) if args.workload == "stage_c2" and rank == 0 else None
    roofline = None
    if launches[0] > 0:
        avg_ms = kern_ms[0] / launches[0]
        bytes_per_launch = bytes_per_step * args.steps / launches[0]
        achieved = bytes_per_launch / (avg_ms * 1e-3) / 1e9
        roofline = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                    "frac": round(achieved / HBM_PEAK_GBPS, 4),
                    "traffic": measured_traffic(args.workload, S, T), "kernel": kernel, "lib_sha16": LIB_SHA16,
                    "avg_kernel_ms": round(avg_ms, 4), "bytes_per_launch": bytes_per_launch,
                    "kernel_launches_timed": int(launches[0])}
        fp = measured_fp64(args.workload, S, T, avg_ms)
        if fp is not None:
            roofline["fp64"] = fp

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline and args.workload != "stage_c2":   # the CPU leg is an N = 1 report
        cpu = cpu_baseline(args, S, T, K, seed, nan_p, out, acf, p_ar, smooth,
                           gpar if args.workload == "garch_fit" else None,
                           (c_fit, coef_fit) if args.workload in ("c4", "c4_levels") else None)

    line = result_line(args.workload, value, world, args.steps, args.warmup, ms_per_step, desc, S, T, K, nan_p,
                       roofline, cpu)
    if staging is not None:
        line["staging"] = staging
    emit(line, rank)
    if world > 1:
        dist.destroy_process_group()


# ---- the harness pieces every workload and the N > 1 gloo test (tests/test_bench_dist.py) share ----

def dist_env():
    """(world, rank, local rank) from torch.distributed.run's environment (1, 0, 0 without it)."""
    return (int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")),
            int(os.environ.get("LOCAL_RANK", "0")))


def fill_acf_step(kernel_call, acf, gather=None):
    """One C1 / C3 step: the fused fill + ACF call over the rank's shard, then (N > 1) the
    all-gather of its ACF block into every rank's (S_total, K) result -- the reference's
    rdd.mapSeries(...).collect of per-series results (S/TimeSeriesRDD.scala:188-199),
    partitions in key order."""
    def step():
        kernel_call()
        if gather is not None:
            step.gathered = gather(acf)
    step.gathered = None
    return step


def timed_region(step, steps, warmup, world, sync, reduce_device, on_start=None, on_stop=None):
    """W untimed warmup steps, then exactly K timed steps bracketed by a barrier and a device
    synchronize on both sides; returns (this rank's wall seconds, the MAX over ranks)."""
    import torch
    import torch.distributed as dist
    for _ in range(warmup):
        step()
    sync()
    if world > 1:
        dist.barrier()
    sync()
    if on_start is not None:
        on_start()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    sync()
    if world > 1:
        dist.barrier()
    sync()
    wall = time.perf_counter() - t0
    if on_stop is not None:
        on_stop()
    elapsed = wall
    if world > 1:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=reduce_device)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    return wall, elapsed


FILL_OF = {"spline": "spline", "c3": "linear", "c1": "linear", "c1_rule3": "linear", "c3_rule3": "linear", "c2": "previous", "stage_c2": "previous", "c4": None, "c4_levels": None,
           "c5": "nearest",
           "ewma_fit": None, "garch_fit": None, "stats": None, "nan_instants": None, "to_instants": None,
           "wire_decode": None}


def result_line(workload, value, world, steps, warmup, ms_per_step, desc, S, T, K, nan_p, roofline, cpu):
    """The ONE JSON line of the driver contract (value = whole-job series-elements/s)."""
    return {
        "metric": "series-elements/sec + % HBM roofline (fill+lag+ACF) at 1/2/4/8 MI355X",
        "value": value, "unit": "series-elements/s", "n_gpus": world, "steps": steps,
        "warmup": warmup, "ms_per_step": ms_per_step, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "f64",
        "data": "synthetic: Philox4x32-10 counter-based panel generated in HBM (SURVEY.md 8(d)), %g NaN" % nan_p,
        "config": {"workload": desc, "series_per_gpu": S, "steps_per_series": T,
                   "numLags": K if workload in ("c3", "c1", "c1_rule3", "c3_rule3") else None,
                   "fill": FILL_OF[workload],
                   "parallelism": "dp%d (series sharded by key, one process per GPU)" % world},
        "roofline": roofline,
        "cpu_baseline": cpu,
    }


def emit(line, rank):
    """Rank 0 prints the line; every other rank prints nothing."""
    if rank == 0:
        print(json.dumps(line), flush=True)


def staging_leg(args, lib, x, out, smooth, S, T):
    """Host-resident C2 through sts_fill_diff_ewma_host (csrc/sts_host.cpp): the panel and the
    result live in host memory -- pageable numpy arrays, and pinned buffers from
    sts_host_alloc -- and every call stages them through HBM in ~64 MB chunks on three
    overlapped streams.  Reports the end-to-end series-elements/s (wall time of the whole
    host-to-host call) and the PCIe transfer rates of the staging streams."""
    import ctypes
    import numpy as np
    import torch
    from sparkts.errors import raise_for_status
    torch.cuda.synchronize()
    host_x = x.cpu().numpy()
    want = out.cpu().numpy().view(np.uint64)      # the HBM-resident path's result
    sm = smooth.cpu().numpy()
    n = S * T * 8
    res = {}
    for kind in ("pageable", "pinned"):
        if kind == "pageable":
            hin, hout, keep = host_x, np.empty_like(host_x), None
        else:
            pin, pout = ctypes.c_void_p(), ctypes.c_void_p()
            raise_for_status(lib.sts_host_alloc(n, ctypes.byref(pin)), "sts_host_alloc")
            raise_for_status(lib.sts_host_alloc(n, ctypes.byref(pout)), "sts_host_alloc")
            hin = np.frombuffer((ctypes.c_char * n).from_address(pin.value), dtype=np.float64).reshape(S, T)
            hout = np.frombuffer((ctypes.c_char * n).from_address(pout.value), dtype=np.float64).reshape(S, T)
            hin[:] = host_x
            keep = (pin, pout)
        stats = np.zeros(8)
        walls = []
        for it in range(1 + max(1, min(args.steps, 3))):   # first call warms the staging buffers
            t0 = time.perf_counter()
            raise_for_status(lib.sts_fill_diff_ewma_host(hin.ctypes.data, hout.ctypes.data, S, T, T, 3, 1,
                                                         sm.ctypes.data, None), "fill_diff_ewma_host")
            if it:
                walls.append(time.perf_counter() - t0)
                lib.sts_staging_stats(stats.ctypes.data)
        wall = min(walls)
        wall_ms, h2d_ms, k_ms, d2h_ms, b_in, b_out, chunks, direct = stats
        res[kind] = {"series_elements_per_s": S * T / wall, "wall_ms": round(wall * 1e3, 2),
                     "h2d_GBps": round(b_in / (h2d_ms * 1e-3) / 1e9, 2) if h2d_ms > 0 else None,
                     "d2h_GBps": round(b_out / (d2h_ms * 1e-3) / 1e9, 2) if d2h_ms > 0 else None,
                     "pcie_both_ways_GBps": round((b_in + b_out) / wall / 1e9, 2),
                     "kernel_ms_sum": round(k_ms, 2), "chunks": int(chunks),
                     "direct_dma_fraction": round(direct, 4),
                     "bytes_h2d": b_in, "bytes_d2h": b_out}
        res[kind]["bit_exact_vs_hbm_path"] = bool(np.array_equal(hout.view(np.uint64), want))
        if kind == "pinned":
            del hin, hout
            for p in keep:
                lib.sts_host_free(p)
    lib.sts_staging_release()
    res["note"] = ("end-to-end = host panel in -> host panel out for one sts_fill_diff_ewma_host call; GB/s = "
                   "bytes / summed per-chunk DMA event time on the staging streams (transfers overlap the kernels "
                   "and each other, so they do not add up to the wall time)")
    return res


LIB_SHA16 = None   # sha256[:16] of the libsts_hip.so this process loaded (main)


def lib_sha16(path):
    import hashlib
    with open(path, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()[:16]


def measured_traffic(workload, S, T):
    """HBM bytes per launch of the dominant kernel from the committed rocprofv3 PMC passes
    (profiles/<round>_<workload>_traffic.json, written by tools/collect.py from separate
    FETCH_SIZE / WRITE_SIZE passes over this same workload at its default shape); None when no
    pass covers it, or when the newest pass was taken on a different build of libsts_hip.so
    (its lib_sha16 is not the loaded library's)."""
    import glob
    if workload not in WORKLOADS or (S, T) != WORKLOADS[workload][:2]:
        return None
    import re

    def version(path):   # r01_v11 after r01_v7: numeric, not lexical, order
        return tuple(int(n) for n in re.findall(r"\d+", os.path.basename(path)))

    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*_%s_traffic.json" % workload)), key=version)
    if not files:
        return None
    with open(files[-1]) as f:
        rec = json.load(f)
    if rec.get("lib_sha16") is None or rec.get("lib_sha16") != LIB_SHA16:
        return None
    return rec.get("traffic_bytes_per_launch")


FP64_PEAK_TFLOPS = 78.6   # MI355X_MICROARCH.md: dense FP64, vector and matrix alike


def measured_fp64(workload, S, T, avg_ms):
    """FP64 pipe use of the dominant kernel (north_star: "MFMA FP64 utilisation for AR
    fitting"): per-launch counters from the committed rocprofv3 pass over this same workload
    (profiles/<round>_<wl>_fp64.json, tools/collect.py), divided by THIS run's launch time."""
    import glob
    import re
    if workload not in ("c3", "c4") or (S, T) != WORKLOADS[workload][:2]:
        return None

    def version(path):
        return tuple(int(n) for n in re.findall(r"\d+", os.path.basename(path)))

    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*_%s_fp64.json" % workload)), key=version)
    if not files:
        return None
    with open(files[-1]) as f:
        rec = json.load(f)
    if rec.get("lib_sha16") is None or rec.get("lib_sha16") != LIB_SHA16:
        return None
    sec = avg_ms * 1e-3
    return {"source": os.path.basename(files[-1]),
            "tflops": round(rec["fp64_flops_per_launch"] / sec / 1e12, 2),
            "frac_of_fp64_peak": round(rec["fp64_flops_per_launch"] / sec / 1e12 / FP64_PEAK_TFLOPS, 4),
            "mfma_tflops": round(rec["mfma_fp64_flops_per_launch"] / sec / 1e12, 2),
            "valu_tflops": round(rec["valu_fp64_flops_per_launch"] / sec / 1e12, 2),
            "mfma_pipe_busy_frac": round(rec["mfma_busy_frac"], 4), "peak_tflops": FP64_PEAK_TFLOPS}


def cpu_threads():
    """Spark local[N] with N = the host cores this process may use: the CPU affinity set,
    capped by OMP_NUM_THREADS when the environment sets it (the GPU box grants each
    single-GPU job 16 of its cores and says so there, while nproc reports the whole machine)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    omp = os.environ.get("OMP_NUM_THREADS")
    if omp and omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    return max(1, n)


def cpu_baseline(args, S, T, K, seed, nan_p, out, acf, p_ar, smooth=None, gpar_ref=None, ar_model=None):
    """The oracle (CPU restatement of the reference loops, oracle/) on a bounded sample of
    the same workload, one series per thread like Spark local[N].  The sample series are
    the rank-0 series 0..n-1, so their GPU results are also checked here."""
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    threads = cpu_threads()
    per_round = threads
    if args.workload in ("stats", "nan_instants", "to_instants", "wire_decode"):
        threads, per_round = 1, 4096     # single-threaded restatements (one partition)
    done, elapsed, s_next = 0, 0.0, 0
    worst_rel, exact = 0.0, True
    ar_check = None
    while elapsed < args.cpu_seconds and s_next < S:
        n = min(per_round, S - s_next)
        if args.workload in ("c4", "c4_levels"):
            xs = oracle.gen_ar_panel(seed, n, T, p_ar, s0=s_next)
            if args.workload == "c4_levels":
                xs = xs * 0.01 + 1e4        # the same two roundings as the device's mul_ / add_
        else:
            xs = oracle.gen_panel(seed, n, T, nan_p, s0=s_next)
            if args.workload in ("c1_rule3", "c3_rule3"):
                xs[~np.isnan(xs)] = 100.1
        if args.workload == "wire_decode":
            wire_bytes = oracle.wire_records(["k%07d" % i for i in range(n)], xs)
        t0 = time.perf_counter()
        if args.workload in ("c3", "c1", "c1_rule3", "c3_rule3"):
            rf, racf, _ = oracle.panel_fill_autocorr(xs, "linear", K, threads=threads)
        elif args.workload == "c2":
            rf = oracle.panel_fill_diff_ewma(xs, 0.2, threads=threads)
        elif args.workload == "spline":
            rf, _ = oracle.panel_fill(xs, "spline", threads=threads)
        elif args.workload == "c5":
            xs[:, 1] = 1.0 + np.nan_to_num(xs[:, 1])
            rf, _ = oracle.panel_fill(xs, "nearest", threads=threads)
            for r in rf:
                oracle.lag(r, 10, False)
        elif args.workload == "ewma_fit":
            rf, _ = oracle.panel_ewma_fit(xs, threads=threads)
        elif args.workload == "garch_fit":
            xs = xs - xs[:, :1]
            rf, _ = oracle.panel_garch_fit(xs, threads=threads)
        elif args.workload in ("stats", "nan_instants", "to_instants", "wire_decode"):
            rf = None
            if args.workload == "stats":
                for r in xs:
                    oracle.stat_counter(r)
            elif args.workload == "nan_instants":
                oracle.remove_instants_with_nans(xs)
            elif args.workload == "to_instants":
                oracle.to_instants(xs)
            else:   # BytesToKeyAndSeries per record: header walk + big-endian doubles
                pos = 0
                for _ in range(n):
                    kl = int.from_bytes(wire_bytes[pos: pos + 4], "big")
                    vn = int.from_bytes(wire_bytes[pos + 4 + kl: pos + 8 + kl], "big")
                    np.frombuffer(wire_bytes, dtype=">f8", count=vn, offset=pos + 8 + kl).astype(np.float64)
                    pos += 8 + kl + 8 * vn
        else:
            rf, rc, rcoef = oracle.panel_ar_fit_remove(xs, p_ar, threads=threads)
        elapsed += time.perf_counter() - t0
        if s_next == 0 and rf is not None:
            g = {"ewma_fit": smooth, "garch_fit": gpar_ref}.get(args.workload, out)[:n].cpu().numpy()
            if args.workload not in ("c4", "c4_levels"):
                exact = bool(np.array_equal(np.isnan(g), np.isnan(rf)) and
                             np.array_equal(np.nan_to_num(g), np.nan_to_num(rf)))
            else:
                # the model: c, phi within 1e-10 elementwise of the reference (bit-identical where the AR
                # rule flags the series); the residuals bit-exact given the device's own model
                gc = ar_model[0][:n].cpu().numpy()
                gph = ar_model[1][:n].cpu().numpy()
                beta_d = np.column_stack([gc, gph])
                beta_r = np.column_stack([rc, rcoef])
                big = np.abs(beta_r) > 1e-6 * np.linalg.norm(beta_r, axis=1, keepdims=True)
                rel = np.where(big, np.abs(beta_d - beta_r) / np.where(big, np.abs(beta_r), 1.0), 0.0)
                worst_rel = float(rel.max())
                own = np.array([oracle.ar_remove(xs[i], gc[i], gph[i]) for i in range(min(n, 64))])
                exact = bool(np.array_equal(own.view(np.uint64), g[:own.shape[0]].view(np.uint64)))
                ar_check = {"model_max_rel_err_elementwise": worst_rel,
                            "model_bit_identical_series": int(np.sum(np.all(beta_d.view(np.uint64) ==
                                                                            beta_r.view(np.uint64), axis=1))),
                            "series_checked": int(n),
                            "residuals_bit_exact_given_device_model": exact}
            if args.workload in ("c3", "c1", "c1_rule3", "c3_rule3"):
                ga = acf[:n].cpu().numpy()
                fin = ~np.isnan(racf)
                if fin.any():
                    worst_rel = float((np.abs(ga[fin] - racf[fin]) / np.abs(racf[fin])).max())
        done += n
        s_next += n
    rate = done * T / elapsed if elapsed > 0 else None
    single = args.workload in ("stats", "nan_instants", "to_instants", "wire_decode")
    return {"value": rate, "unit": "series-elements/s", "cores": threads, "kind": "port",
            "host_nproc": os.cpu_count(),
            "cores_note": ("SINGLE-THREADED restatement (one partition, 1 core): a GPU / CPU ratio from this line "
                           "is per core, not against a local[N] executor" if single else
                           "threads = this process's CPU affinity capped by OMP_NUM_THREADS (the GPU box grants a "
                           "single-GPU job 16 of its nproc cores); Spark local[N] with N = cores"),
            "sample": "%d of the rank-0 series x %d steps (%.1f s of CPU work), oracle/sts_oracle.c restatement of "
                      "the reference loops, one series per thread (Spark local[%d] analogue); the JVM reference "
                      "cannot run here" % (done, T, elapsed, threads),
            "sample_check": ar_check if ar_check is not None else {"filled_bit_exact": exact, "acf_max_rel_err": worst_rel}}


def percall():
    """Per-call latency of the drop-in for ONE series (S = 1: UnivariateTimeSeries called from
    a per-record closure, ARIMA's differencing inside its optimizer, lbtest's autocorr) and for
    small partitions, against the same operation on one core (the oracle's C loop timed inside C
    -- a lower bound on the JIT-compiled Scala loop, so the crossover it gives is conservative).
    GPU legs: the `_host` entry point on pageable numpy memory (the JNI shim's form: arrays copied
    into pinned buffers, staged, results copied back), on pinned memory, and the device entry
    point on HBM-resident data (launch + stream synchronize).  Best of `reps` calls each."""
    import ctypes
    import numpy as np
    import torch
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    from sparkts import _native
    from sparkts.errors import raise_for_status
    _native.ensure_device(0)
    lib = _native.lib()
    reps = 40

    def best(fn, n=reps):
        fn()
        b = 1e300
        for _ in range(n):
            t0 = time.perf_counter()
            fn()
            b = min(b, time.perf_counter() - t0)
        return b * 1e6   # us

    def pinned(nbytes):
        p = ctypes.c_void_p()
        raise_for_status(lib.sts_host_alloc(max(nbytes, 16), ctypes.byref(p)), "sts_host_alloc")
        return p

    rows = []
    for T in (10, 100, 1000, 3000, 10_000, 30_000, 100_000):
        x = oracle.gen_panel(1, 1, T, 0.05)
        x[0, 0] = 1.0
        x[0, -1] = 2.0
        o = np.empty_like(x)
        K = min(20, T - 1)
        acf = np.empty(K)
        nb = 8 * T
        pin_in, pin_out = pinned(nb), pinned(nb)
        hin = np.frombuffer((ctypes.c_char * nb).from_address(pin_in.value), dtype=np.float64)
        hout = np.frombuffer((ctypes.c_char * nb).from_address(pin_out.value), dtype=np.float64)
        hin[:] = x[0]
        xd = torch.as_tensor(x, device="cuda:0")
        od = torch.empty_like(xd)
        ad = torch.empty(K, dtype=torch.float64, device="cuda:0")
        sp = torch.cuda.current_stream().cuda_stream
        row = {"T": T}
        for method, code in (("linear", 0), ("previous", 3), ("spline", 4)):
            row["fill_%s_host_pageable_us" % method] = best(
                lambda: raise_for_status(lib.sts_fill_host(x.ctypes.data, o.ctypes.data, 1, T, T, code, None), "f"))
            row["fill_%s_host_pinned_us" % method] = best(
                lambda: raise_for_status(lib.sts_fill_host(hin.ctypes.data, hout.ctypes.data, 1, T, T, code, None),
                                         "f"))

            def dev_call():
                raise_for_status(lib.sts_fill(xd.data_ptr(), od.data_ptr(), 1, T, T, T, code, None, sp), "f")
                torch.cuda.synchronize()
            row["fill_%s_device_us" % method] = best(dev_call)
            row["fill_%s_cpu_1core_us" % method] = oracle.time_fill_ns(x[0], method, reps) / 1e3
            assert np.array_equal(o.view(np.uint64), oracle.panel_fill(x, method)[0].view(np.uint64))
        row["autocorr%d_host_pageable_us" % K] = best(
            lambda: raise_for_status(lib.sts_autocorr_host(x.ctypes.data, 1, T, T, K, acf.ctypes.data), "a"))

        def dev_acf():
            raise_for_status(lib.sts_fill_autocorr(xd.data_ptr(), None, 1, T, T, T, -1, K, ad.data_ptr(), None, sp),
                             "a")
            torch.cuda.synchronize()
        row["autocorr%d_device_us" % K] = best(dev_acf)
        row["autocorr%d_cpu_1core_us" % K] = oracle.time_autocorr_ns(x[0], K, reps) / 1e3
        lib.sts_host_free(pin_in)
        lib.sts_host_free(pin_out)
        rows.append({k: (round(v, 2) if isinstance(v, float) else v) for k, v in row.items()})

    # partition-sized calls (the mapPartitions form): S series x 390 steps per call
    parts = []
    for S in (1, 16, 256, 4096, 65536):
        T = 390
        x = oracle.gen_panel(2, S, T, 0.05)
        o = np.empty_like(x)
        g = best(lambda: raise_for_status(lib.sts_fill_host(x.ctypes.data, o.ctypes.data, S, T, T, 3, None), "f"),
                 n=10)
        c = oracle.time_fill_ns(x[0], "previous", reps) / 1e3 * S
        parts.append({"S": S, "T": T, "fill_previous_host_pageable_us": round(g, 2),
                      "cpu_1core_us (S x one series)": round(c, 2)})
    lib.sts_staging_release()

    def crossover(op, gpu_key):
        for r in rows:
            cpu = r.get("%s_cpu_1core_us" % op)
            if cpu is not None and r.get(gpu_key) is not None and r[gpu_key] < cpu:
                return r["T"]
        return None
    K20 = "autocorr20"
    line = {"metric": "per-call latency, one series (S = 1) and small partitions, vs one CPU core",
            "unit": "us (best of %d calls)" % reps, "rows": rows, "partitions": parts,
            "crossover_T": {
                "fill_linear_host": crossover("fill_linear", "fill_linear_host_pageable_us"),
                "fill_previous_host": crossover("fill_previous", "fill_previous_host_pageable_us"),
                "fill_spline_host": crossover("fill_spline", "fill_spline_host_pageable_us"),
                "autocorr20_host": crossover(K20, "autocorr20_host_pageable_us"),
                "fill_linear_device": crossover("fill_linear", "fill_linear_device_us"),
                "autocorr20_device": crossover(K20, "autocorr20_device_us")},
            "note": "crossover_T = the smallest tested T at which ONE call through the GPU path beats the one-core "
                    "C loop (the oracle, timed inside C; the JVM's Breeze loop is not faster), None = never at "
                    "T <= 100000; the CPU leg runs on the GPU box's host",
            "lib_sha16": lib_sha16(lib._name)}
    print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
