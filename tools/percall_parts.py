"""Where the ~40-50 us of a one-series call go (bench.py --percall): the device entry point with and
without a caller-provided err array, against a bare stream synchronize and a one-element torch
kernel + synchronize (the launch floor).  Best of N; prints one JSON line."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "spark-timeseries_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from sparkts import _native  # noqa: E402

_native.ensure_device(0)
lib = _native.lib()
T = 100
x = torch.randn((1, T), dtype=torch.float64, device="cuda:0")
o = torch.empty_like(x)
err = torch.zeros(1, dtype=torch.int32, device="cuda:0")
acf = torch.empty(20, dtype=torch.float64, device="cuda:0")
sp = torch.cuda.current_stream().cuda_stream
xh = x.cpu().numpy()
oh = np.empty_like(xh)


def best(fn, n=200):
    for _ in range(10):
        fn()
    b = 1e9
    for _ in range(n):
        t0 = time.perf_counter()
        fn()
        b = min(b, time.perf_counter() - t0)
    return round(b * 1e6, 2)


res = {
    "sync_only_us": best(lambda: torch.cuda.synchronize()),
    "torch_tiny_kernel_sync_us": best(lambda: (o[0, :1].copy_(x[0, :1]), torch.cuda.synchronize())),
    "fill_dev_err_given_us": best(lambda: (lib.sts_fill(x.data_ptr(), o.data_ptr(), 1, T, T, T, 0, err.data_ptr(), sp),
                                          torch.cuda.synchronize())),
    "fill_dev_err_null_us": best(lambda: (lib.sts_fill(x.data_ptr(), o.data_ptr(), 1, T, T, T, 0, None, sp),
                                         torch.cuda.synchronize())),
    "fill_host_us": best(lambda: lib.sts_fill_host(xh.ctypes.data, oh.ctypes.data, 1, T, T, 0, None)),
    "acf_dev_us": best(lambda: (lib.sts_fill_autocorr(x.data_ptr(), None, 1, T, T, T, -1, 20, acf.data_ptr(),
                                                      err.data_ptr(), sp), torch.cuda.synchronize())),
    "T": T,
}
print(json.dumps(res))
