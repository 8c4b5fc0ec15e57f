"""Per-phase cycle shares of the register-resident AR fit kernel (diagnostic `make stamps`).

    STS_HIP_LIB=spark-timeseries_amd/build/libsts_hip_stamps.py python tools/ar_stamps.py [S]
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

NAMES = ["load+mean", "passA lag products", "reductions", "gram+chol+solve", "passB residual",
         "refine solve", "passC remove"]


def main():
    S = int(sys.argv[1]) if len(sys.argv) > 1 else 100000
    T, p = 2520, 5
    _native.ensure_device(0)
    lib = _native.lib()
    lib.sts_debug_ar_stamps.restype = ctypes.c_int
    lib.sts_debug_ar_stamps.argtypes = [ctypes.c_void_p]
    x = torch.empty((S, T), dtype=torch.float64, device="cuda")
    out = torch.empty_like(x)
    c = torch.empty(S, dtype=torch.float64, device="cuda")
    coef = torch.empty((S, p), dtype=torch.float64, device="cuda")
    err = torch.zeros(S, dtype=torch.int32, device="cuda")
    sp = torch.cuda.current_stream().cuda_stream
    assert lib.sts_gen_ar_panel(x.data_ptr(), c.data_ptr(), coef.data_ptr(), 0, S, T, T, 4, p, sp) == 0
    buf = np.zeros(16, dtype=np.uint64)
    for _ in range(2):
        lib.sts_debug_ar_stamps(buf.ctypes.data)
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev0.record()
        assert lib.sts_ar_fit_remove(x.data_ptr(), out.data_ptr(), S, T, T, T, p, 0, c.data_ptr(),
                                     coef.data_ptr(), err.data_ptr(), sp) == 0
        ev1.record()
        torch.cuda.synchronize()
        ms = ev0.elapsed_time(ev1)
        lib.sts_debug_ar_stamps(buf.ctypes.data)
    n = max(1, int(buf[15]))
    print(json.dumps({"S": S, "ms": ms, "waves": n,
                      "cycles_per_series": {NAMES[i]: round(float(buf[i]) / n) for i in range(7)}}))


if __name__ == "__main__":
    main()
