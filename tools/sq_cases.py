"""Per wave-tile SQ instruction counts and wave-cycle split of tools/r3_sqcases.sh output.

    python tools/sq_cases.py OUT.json "what" [SUFFIX]   (reads gpurun_out/sqcases<SUFFIX>/ and .log)

Dispatches are matched to kbench cases in order (one warm-up + --reps calls per case; the
counters of one call are reported).  SQ_WAVE_CYCLES / SQ_WAIT_ANY / SQ_ACTIVE_INST_ANY count
quad-cycles (MI355X_MICROARCH.md); the shares are ratios of them."""
import collections
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "gpurun_out")


def main():
    suf = sys.argv[3] if len(sys.argv) > 3 else ""
    rows = list(csv.DictReader(open(os.path.join(OUT, "sqcases" + suf, "run_counter_collection.csv"))))
    d = collections.OrderedDict()
    for r in rows:
        if "tile_kernel" not in r["Kernel_Name"]:
            continue
        d.setdefault(int(r["Dispatch_Id"]), {})[r["Counter_Name"]] = float(r["Counter_Value"])
    cases = [json.loads(l) for l in open(os.path.join(OUT, "sqcases" + suf + ".log")) if l.startswith('{"case"')]
    disp = sorted(d)
    per = len(disp) // max(1, len(cases))
    res = []
    for i, c in enumerate(cases):
        v = d[disp[i * per]]
        S, T = c["S"], c["T"]
        wt = S * (-(-T // 4096)) * 4     # wave-tiles: 4 waves per 4096-step tile
        res.append({"case": c["case"], "ms": c["ms"], "GBps": c["GBps"],
                    "per_wave_tile": {k: round(v["SQ_INSTS_" + k] / wt, 1) for k in ("VALU", "SALU", "LDS", "MFMA")},
                    "wave_cycles_share": {"parked (s_waitcnt / barrier)": round(v["SQ_WAIT_ANY"] / v["SQ_WAVE_CYCLES"], 3),
                                          "issuing": round(v["SQ_ACTIVE_INST_ANY"] / v["SQ_WAVE_CYCLES"], 3),
                                          "issue-stalled": round(1 - (v["SQ_WAIT_ANY"] + v["SQ_ACTIVE_INST_ANY"]) / v["SQ_WAVE_CYCLES"], 3)},
                    "cycles_per_wave_tile": round(4 * v["SQ_WAVE_CYCLES"] / wt)})
    json.dump({"what": sys.argv[2], "cases": res}, open(sys.argv[1], "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
