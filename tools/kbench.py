"""Kernel-level A/B timing of the fill / fill + ACF paths on the C3 series length.

    python tools/kbench.py [--series N] [--T 982800] [--cases spec,...]

A case is  kernel:method:K  (kernel seg | tile, method linear | previous | next | nearest
| none, K = numLags, 0 = fill only), e.g. seg:linear:60,tile:linear:60,seg:linear:0.
Prints one JSON line per case: average ms per call (HIP events on the launch stream,
via sts_profile_*) and algorithmic GB/s (16 B per step; 8 B when nothing is written).
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "spark-timeseries_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from sparkts import _native  # noqa: E402
if os.environ.get("STS_HIP_LIB"):   # a tools/variant.sh build
    _native.use_library(os.environ["STS_HIP_LIB"])

METHODS = {"linear": 0, "nearest": 1, "next": 2, "previous": 3, "none": -1}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--series", type=int, default=2000)
    ap.add_argument("--T", type=int, default=982_800)
    ap.add_argument("--nan", type=float, default=0.05)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--cases", default="seg:linear:60,tile:linear:60,seg:linear:0,tile:linear:0,seg:none:60")
    args = ap.parse_args()
    _native.ensure_device(0)
    lib = _native.lib()
    S, T = args.series, args.T
    x = torch.empty((S, T), dtype=torch.float64, device="cuda")
    out = torch.empty_like(x)
    kmax = max(64, max(int(c.split(":")[2]) for c in args.cases.split(",")))
    acf = torch.empty((S, kmax), dtype=torch.float64, device="cuda")
    err = torch.zeros(S, dtype=torch.int32, device="cuda")
    sp = torch.cuda.current_stream().cuda_stream
    assert lib.sts_gen_panel(x.data_ptr(), 0, S, T, T, 3, args.nan, sp) == 0
    ref = {}
    for case in args.cases.split(","):
        kern, meth, K = case.split(":")
        K = int(K)
        code = METHODS[meth]
        os.environ["STS_TILE_KERNEL"] = kern     # "tile" (default path) or "seg" (opt-in)
        filled = out.data_ptr() if code >= 0 else None

        def call():
            if K > 0:
                st = lib.sts_fill_autocorr(x.data_ptr(), filled, S, T, T, T, code, K, acf.data_ptr(), err.data_ptr(), sp)
            else:
                st = lib.sts_fill(x.data_ptr(), out.data_ptr(), S, T, T, T, code, err.data_ptr(), sp)
            assert st == 0, case

        call()
        torch.cuda.synchronize()
        lib.sts_profile_begin()
        for _ in range(args.reps):
            call()
        torch.cuda.synchronize()
        kern_ms = np.zeros(1, dtype=np.float64)
        n = np.zeros(1, dtype=np.int64)
        lib.sts_profile_end(kern_ms.ctypes.data, n.ctypes.data)
        ms = kern_ms[0] / max(1, n[0])
        bpe = 16.0 if code >= 0 else 8.0
        key = (meth, K)
        sig = (float(out[:, :4096].double().nan_to_num(7.0).sum()) if code >= 0 else 0.0,
               float(acf[:, :K].nan_to_num(7.0).sum()) if K > 0 else 0.0)
        same = None
        if key in ref:
            same = bool(abs(sig[0] - ref[key][0]) <= 1e-9 * abs(ref[key][0]) + 1e-300 and
                        abs(sig[1] - ref[key][1]) <= 1e-9 * abs(ref[key][1]) + 1e-12)
        else:
            ref[key] = sig
        print(json.dumps({"case": case, "S": S, "T": T, "ms": round(ms, 4),
                          "GBps": round(bpe * S * T / (ms * 1e-3) / 1e9, 1),
                          "Gsteps": round(S * T / (ms * 1e-3) / 1e9, 2), "matches_first": same}), flush=True)


if __name__ == "__main__":
    main()
