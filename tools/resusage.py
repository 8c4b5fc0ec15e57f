"""Per-kernel register / scratch / occupancy table of one HIP source (gfx950), from hipcc's
-Rpass-analysis=kernel-resource-usage remarks.  Used to check that a change does not add
VGPRs or spills to a hot kernel before it goes to the GPU.

  python tools/resusage.py spark-timeseries_amd/csrc/sts_tile.hip [-DFOO ...] [--filter tile_kernel]
"""
import re
import subprocess
import sys

ROOT = __file__.rsplit("/tools/", 1)[0]


def usage(src, extra=(), incdir=None):
    inc = incdir or src.rsplit("/", 1)[0]
    cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-ffp-contract=off",
           "-I" + ROOT + "/include", "-I" + inc, "--cuda-device-only", "-c", src, "-o", "/dev/null",
           "-Rpass-analysis=kernel-resource-usage", *extra]
    out = subprocess.run(cmd, capture_output=True, text=True).stderr
    rows, cur = [], None
    for line in out.splitlines():
        m = re.search(r"remark: (.*) \[-Rpass-analysis", line)
        if not m:
            continue
        body = m.group(1).strip()
        if body.startswith("Function Name:"):
            cur = {"name": body.split(":", 1)[1].strip()}
            rows.append(cur)
        elif cur is not None and ":" in body:
            k, v = body.split(":", 1)
            cur[k.strip()] = v.strip()
    return rows


def demangle(names):
    try:
        r = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True,
                           text=True)
        return r.stdout.splitlines()
    except OSError:
        return names


if __name__ == "__main__":
    args = sys.argv[1:]
    filt = None
    if "--filter" in args:
        i = args.index("--filter")
        filt = args[i + 1]
        del args[i:i + 2]
    src, extra = args[0], args[1:]
    rows = usage(src, extra)
    names = demangle([r["name"] for r in rows])
    for r, n in zip(rows, names):
        if filt and filt not in n:
            continue
        n = n.replace("sts::(anonymous namespace)::", "").replace("sts::TileArgs", "TA")
        print("%-70s vgpr %4s agpr %3s sgpr %3s spillV %3s spillS %3s scratch %4s occ %s lds %s" % (
            n[:70], r.get("VGPRs"), r.get("AGPRs"), r.get("SGPRs"), r.get("VGPRs Spill"), r.get("SGPRs Spill"),
            r.get("ScratchSize [bytes/lane]"), r.get("Occupancy [waves/SIMD]"), r.get("LDS Size [bytes/block]")))
