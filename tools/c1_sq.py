"""SQ counters of the C1 short kernels per form (tools/sessions_r6.sh c1sq): per dispatch means,
per-series instruction counts and the wave-cycle split.

    python tools/c1_sq.py OUT.json [DIR]   (DIR default gpurun_out/r6; reads c1sq_<form>_<pass>/)

SQ_WAVE_CYCLES / SQ_WAIT_ANY / SQ_ACTIVE_INST_* / SQ_BUSY_CYCLES count quad-cycles
(MI355X_MICROARCH.md); per-SIMD VALU issue share = 4 SQ_ACTIVE_INST_VALU / (GRBM_GUI_ACTIVE x
SIMDs), since one SIMD issues at most one VALU instruction per cycle."""
import collections
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
S_C1 = 10_000
SIMDS = 256 * 4


def form_counters(d, form):
    v = collections.defaultdict(list)
    for f in sorted(glob.glob(os.path.join(d, "c1sq_%s_*" % form, "**", "*counter_collection.csv"), recursive=True)):
        per = collections.defaultdict(dict)
        for r in csv.DictReader(open(f)):
            if "short_" not in r["Kernel_Name"]:
                continue
            per[int(r["Dispatch_Id"])][r["Counter_Name"]] = per[int(r["Dispatch_Id"])].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        for c in per.values():
            for k, x in c.items():
                v[k].append(x)
    return {k: sum(x) / len(x) for k, x in v.items()}


def main():
    d = sys.argv[2] if len(sys.argv) > 2 else os.path.join(ROOT, "gpurun_out", "r6")
    res = {}
    for form in ("0", "1"):
        c = form_counters(d, form)
        if not c:
            continue
        g = c.get("GRBM_GUI_ACTIVE", 0)
        out = {"counters_per_dispatch": {k: round(x) for k, x in sorted(c.items())},
               "per_series": {k: round(c[k] / S_C1, 1) for k in sorted(c) if k.startswith("SQ_INSTS")}}
        if "SQ_WAVE_CYCLES" in c:
            out["wave_cycles_share"] = {
                "parked": round(c.get("SQ_WAIT_ANY", 0) / c["SQ_WAVE_CYCLES"], 3),
                "issuing": round(c.get("SQ_ACTIVE_INST_ANY", 0) / c["SQ_WAVE_CYCLES"], 3) if "SQ_ACTIVE_INST_ANY" in c else None}
        if g and "SQ_ACTIVE_INST_VALU" in c:
            out["valu_issue_share_per_simd"] = round(4 * c["SQ_ACTIVE_INST_VALU"] / (g * SIMDS), 3)
        if g and "SQ_BUSY_CYCLES" in c:
            out["sq_busy_share"] = round(4 * c["SQ_BUSY_CYCLES"] / (g * 32), 3)
        res["pair=" + form] = out
    json.dump({"what": "SQ counters of the C1 short kernel (10 000 x 2 520, fill linear + ACF 20), "
                       "one-series-per-block form (pair=0) and the two-wave ping-pong form (pair=1)",
               "forms": res}, open(sys.argv[1], "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
