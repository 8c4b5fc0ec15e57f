"""Summarise the C5 process-to-process counter passes (tools/r5_session.sh c5diag):
per process, over the dominant tile_kernel dispatches: mean duration (kernel trace), effective
clock (GRBM_GUI_ACTIVE / 8 / duration), UTCL1 translation hit / miss per dispatch and the miss
rate.  Usage: python tools/c5diag_summary.py DIR [DIR ...] (each DIR = one process's
rocprofv3 output)."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def summary(d):
    cc = glob.glob(os.path.join(d, "*counter_collection.csv"))[0]
    per = defaultdict(dict)
    for r in csv.DictReader(open(cc)):
        if "tile_kernel" not in r["Kernel_Name"]:
            continue
        per[r["Dispatch_Id"]][r["Counter_Name"]] = float(r["Counter_Value"])
        per[r["Dispatch_Id"]]["dur"] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6
    rows = list(per.values())
    n = len(rows)
    mean = lambda k: sum(x[k] for x in rows) / n
    dur = mean("dur")
    hit, miss = mean("TCP_UTCL1_TRANSLATION_HIT_sum"), mean("TCP_UTCL1_TRANSLATION_MISS_sum")
    return {"dir": os.path.basename(d.rstrip("/")), "dispatches": n, "mean_ms": round(dur, 4),
            "eff_clock_GHz": round(mean("GRBM_GUI_ACTIVE") / 8 / (dur * 1e-3) / 1e9, 3),
            "utcl1_hit_per_dispatch": round(hit), "utcl1_miss_per_dispatch": round(miss),
            "utcl1_miss_rate": round(miss / (hit + miss), 5)}


if __name__ == "__main__":
    for d in sys.argv[1:]:
        print(json.dumps(summary(d)))
