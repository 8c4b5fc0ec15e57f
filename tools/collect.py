"""Collect one GPU session's evidence from gpurun_out/ into profiles/ (tracked).

    python tools/collect.py TAG

* gpurun_out/bench_<wl>.log          -> profiles/<TAG>_bench_<wl>.json   (the bench JSON line)
* gpurun_out/prof_c3/*kernel_stats.csv -> profiles/<TAG>_c3_kernel_stats.csv (rocprofv3 --stats
  of the default `python bench.py` command)
* gpurun_out/pmc_{fetch,write}_c3/   -> profiles/<TAG>_c3_traffic.json: HBM bytes per launch of
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
PROF = os.path.join(ROOT, "profiles")
KERNEL = "tile_kernel"


def pmc_values(d, counter):
    vals = []
    for f in glob.glob(os.path.join(OUT, d, "*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            if KERNEL in r["Kernel_Name"] and r["Counter_Name"] == counter:
                vals.append(float(r["Counter_Value"]))
    return vals


def main():
    tag = sys.argv[1]
    for log in glob.glob(os.path.join(OUT, "bench_*.log")):
        wl = os.path.basename(log)[len("bench_"):-len(".log")]
        lines = [ln for ln in open(log) if ln.startswith("{")]
        if lines:
            with open(os.path.join(PROF, "%s_bench_%s.json" % (tag, wl)), "w") as f:
                f.write(lines[-1])
    stats = glob.glob(os.path.join(OUT, "prof_c3", "*kernel_stats.csv"))
    if stats:
        shutil.copy(stats[0], os.path.join(PROF, "%s_c3_kernel_stats.csv" % tag))
    fetch = pmc_values("pmc_fetch_c3", "FETCH_SIZE")
    write = pmc_values("pmc_write_c3", "WRITE_SIZE")
    if fetch and write:
        rd = 2.0 * 1024.0 * sum(fetch) / len(fetch)     # gfx950: FETCH_SIZE reports half the bytes
        wr = 1024.0 * sum(write) / len(write)
        rec = {"kernel": KERNEL, "workload": "c3 (bench.py default shard), --steps 2 --warmup 0",
               "launches": [len(fetch), len(write)],
               "read_bytes_per_launch": rd, "write_bytes_per_launch": wr,
               "traffic_bytes_per_launch": rd + wr,
               "correction": "FETCH_SIZE (KiB) x 2 on gfx950, WRITE_SIZE (KiB) as is (MI355X_MICROARCH.md HBM)"}
        with open(os.path.join(PROF, "%s_c3_traffic.json" % tag), "w") as f:
            json.dump(rec, f, indent=1)
        print(json.dumps(rec))


if __name__ == "__main__":
    main()
