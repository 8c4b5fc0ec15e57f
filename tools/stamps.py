"""Per-phase cycle shares of the tile kernel (diagnostic `make stamps` build only).

    STS_HIP_LIB=spark-timeseries_amd/build/libsts_hip_stamps.so python tools/stamps.py [S] [K] [method]

Shares, not absolute time: the stamps' own fences perturb the schedule
(cdna_hip_programming.md §7, In-kernel stamps).
"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "spark-timeseries_amd"))
os.environ.setdefault("STS_HIP_LIB", os.path.join(ROOT, "spark-timeseries_amd", "build", "libsts_hip_stamps.so"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from sparkts import _native  # noqa: E402
if os.environ.get("STS_HIP_LIB"):   # a tools/variant.sh build
    _native.use_library(os.environ["STS_HIP_LIB"])

NAMES = ["regs->LDS", "bar A", "ballots", "bar B", "scan+NaN list", "bar C", "NaN fill", "bar D",
         "store+y+prefetch", "bar E", "MFMA", "bar F"]


def main():
    S = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
    K = int(sys.argv[2]) if len(sys.argv) > 2 else 60
    method = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    T = 982_800
    _native.ensure_device(0)
    lib = _native.lib()
    lib.sts_debug_stamps.restype = ctypes.c_int
    lib.sts_debug_stamps.argtypes = [ctypes.c_void_p]
    x = torch.empty((S, T), dtype=torch.float64, device="cuda")
    out = torch.empty_like(x)
    acf = torch.empty((S, K), dtype=torch.float64, device="cuda")
    err = torch.zeros(S, dtype=torch.int32, device="cuda")
    sp = torch.cuda.current_stream().cuda_stream
    assert lib.sts_gen_panel(x.data_ptr(), 0, S, T, T, 3, 0.05, sp) == 0
    buf = np.zeros(16, dtype=np.uint64)
    for it in range(2):
        lib.sts_debug_stamps(buf.ctypes.data)
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev0.record()
        assert lib.sts_fill_autocorr(x.data_ptr(), out.data_ptr(), S, T, T, T, method, K, acf.data_ptr(),
                                     err.data_ptr(), sp) == 0
        ev1.record()
        torch.cuda.synchronize()
        ms = ev0.elapsed_time(ev1)
        lib.sts_debug_stamps(buf.ctypes.data)
    tot = float(buf[:12].sum())
    res = {"S": S, "K": K, "method": method, "ms": ms, "waves": int(buf[12]),
           "share": {n: round(float(buf[i]) / tot, 4) for i, n in enumerate(NAMES)}}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
