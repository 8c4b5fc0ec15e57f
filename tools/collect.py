"""Collect one GPU session's evidence from gpurun_out/ into profiles/ (tracked).

    python tools/collect.py TAG [DIR]      (DIR: the session's output directory, default gpurun_out)

* gpurun_out/bench_<wl>.log          -> profiles/<TAG>_bench_<wl>.json   (the bench JSON line)
* gpurun_out/prof_<wl>/*kernel_stats.csv -> profiles/<TAG>_<wl>_kernel_stats.csv (rocprofv3 --stats
  of `python bench.py [--workload wl]`)
* gpurun_out/pmc_{fetch,write}_<wl>/ -> profiles/<TAG>_<wl>_traffic.json: HBM bytes per launch of
  the dominant kernel from separate FETCH_SIZE / WRITE_SIZE passes, corrected as
  MI355X_MICROARCH.md prescribes (FETCH_SIZE x 2 on gfx950; both in KiB).
"""
import csv
import glob
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "gpurun_out")
LIB_SHA = None   # sha256[:16] of the libsts_hip.so the session ran (DIR/libsha.txt, tools/r5_session.sh)
PROF = os.path.join(ROOT, "profiles")
KERNEL = "tile_kernel"


def pmc_values(d, counter, kernel=KERNEL):
    vals = []
    for f in glob.glob(os.path.join(OUT, d, "*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            if kernel in r["Kernel_Name"] and r["Counter_Name"] == counter:
                vals.append(float(r["Counter_Value"]))
    return vals


# FP64 pipe counters (tools/gpu_all.sh fp64_<wl>): one --pmc pass per workload
FP64_COUNTERS = ["SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_ADD_F64",
                 "SQ_INSTS_VALU_MFMA_MOPS_F64", "SQ_VALU_MFMA_BUSY_CYCLES", "GRBM_GUI_ACTIVE"]
FP64_KERNELS = {"c3": "tile_kernel", "c4": "ar_fit_blk_kernel", "ewma_fit": "ewma_fit_kernel",
                "garch_fit": "garch_fit_kernel"}
# dominant kernel per workload (the c3 passes are of the default `python bench.py` command;
# c3 directories keep their round-1 names pmc_fetch_c3 / pmc_write_c3 / prof_c3)
TRAFFIC_KERNELS = {"c3": "tile_kernel", "c1": "short_fill_acf_kernel", "c2": "recur_row_kernel", "c4": "ar_fit_blk_kernel",
                   "c5": "tile_kernel",
                   # the f rows; nan_instants: both of its kernels ("_instants" matches
                   # nan_instants16_kernel and gather_instants_kernel), per launch like bench.py's figure
                   "ewma_fit": "ewma_fit_kernel", "stats": "stats_fast_kernel", "nan_instants": "_instants",
                   "to_instants": "transpose16_kernel", "wire_decode": "wire_decode_rows_kernel",
                   "garch_fit": "garch_fit_kernel", "stage_c2": "recur_row_kernel",
                   "spline": "spline_fill_kernel"}


def collect_fp64(tag, wl):
    """Per-launch FP64 work of the dominant kernel: flops = (2 FMA + ADD + MUL) x 64 lanes +
    MFMA_MOPS x 512 (rocprofiler-sdk TOTAL_64_OPS), the MFMA pipe's busy cycles summed over
    the 1024 SIMDs, and GRBM_GUI_ACTIVE (summed over the 8 XCDs).  bench.py divides by its own
    launch time for the utilisation figures."""
    d = "pmc_fp64_%s" % wl
    vals = {c: pmc_values(d, c, FP64_KERNELS[wl]) for c in FP64_COUNTERS}
    if not all(vals.values()):
        return None
    per = {c: sum(v) / len(v) for c, v in vals.items()}
    flops = (2 * per["SQ_INSTS_VALU_FMA_F64"] + per["SQ_INSTS_VALU_ADD_F64"] + per["SQ_INSTS_VALU_MUL_F64"]) * 64 \
        + per["SQ_INSTS_VALU_MFMA_MOPS_F64"] * 512
    rec = {"kernel": FP64_KERNELS[wl], "workload": "%s (bench.py), --steps 2 --warmup 0" % wl,
           "launches": len(vals["GRBM_GUI_ACTIVE"]), "counters_per_launch": per,
           "fp64_flops_per_launch": flops,
           "valu_fp64_flops_per_launch": flops - per["SQ_INSTS_VALU_MFMA_MOPS_F64"] * 512,
           "mfma_fp64_flops_per_launch": per["SQ_INSTS_VALU_MFMA_MOPS_F64"] * 512,
           "mfma_busy_frac": per["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024.0 * per["GRBM_GUI_ACTIVE"] / 8.0),
           "effective_clock_note": "GRBM_GUI_ACTIVE / 8 = cycles per XCD over the launch",
           "formula": "TOTAL_64_OPS = (2 FMA_F64 + ADD_F64 + MUL_F64) x 64 + MFMA_MOPS_F64 x 512",
           "lib_sha16": LIB_SHA}
    with open(os.path.join(PROF, "%s_%s_fp64.json" % (tag, wl)), "w") as f:
        json.dump(rec, f, indent=1)
    print(json.dumps(rec))
    return rec


def main():
    global OUT, LIB_SHA
    tag = sys.argv[1]
    if len(sys.argv) > 2:
        OUT = os.path.abspath(sys.argv[2])
    sha = os.path.join(OUT, "libsha.txt")
    if os.path.exists(sha):
        LIB_SHA = open(sha).read().split()[0][:16]
    for log in glob.glob(os.path.join(OUT, "bench_*.log")):
        wl = os.path.basename(log)[len("bench_"):-len(".log")]
        lines = [ln for ln in open(log) if ln.startswith("{")]
        if lines:
            with open(os.path.join(PROF, "%s_bench_%s.json" % (tag, wl)), "w") as f:
                f.write(lines[-1])
    for wl in TRAFFIC_KERNELS:
        stats = glob.glob(os.path.join(OUT, "prof_%s" % wl, "*kernel_stats.csv"))
        if stats:
            shutil.copy(stats[0], os.path.join(PROF, "%s_%s_kernel_stats.csv" % (tag, wl)))
        kern = TRAFFIC_KERNELS[wl]
        fetch = pmc_values("pmc_fetch_%s" % wl, "FETCH_SIZE", kern)
        write = pmc_values("pmc_write_%s" % wl, "WRITE_SIZE", kern)
        if fetch and write:
            rd = 2.0 * 1024.0 * sum(fetch) / len(fetch)     # gfx950: FETCH_SIZE reports half the bytes
            wr = 1024.0 * sum(write) / len(write)
            rec = {"kernel": kern, "workload": "%s (bench.py), --steps 2 --warmup 0" % wl,
                   "launches": [len(fetch), len(write)],
                   "read_bytes_per_launch": rd, "write_bytes_per_launch": wr,
                   "traffic_bytes_per_launch": rd + wr,
                   "correction": "FETCH_SIZE (KiB) x 2 on gfx950, WRITE_SIZE (KiB) as is (MI355X_MICROARCH.md HBM)",
                   "lib_sha16": LIB_SHA}
            with open(os.path.join(PROF, "%s_%s_traffic.json" % (tag, wl)), "w") as f:
                json.dump(rec, f, indent=1)
            print(json.dumps(rec))
    for wl in FP64_KERNELS:
        collect_fp64(tag, wl)
    pc = os.path.join(OUT, "percall.log")   # bench.py --percall (tools/r5_session.sh percall)
    if os.path.exists(pc):
        lines = [ln for ln in open(pc) if ln.startswith("{")]
        if lines:
            with open(os.path.join(PROF, "%s_percall.json" % tag), "w") as f:
                f.write(lines[-1])


if __name__ == "__main__":
    main()
