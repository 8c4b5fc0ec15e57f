"""Diagnose a variant library's fill mismatch: run test_acf_robust's far-level rows through the
product and a variant build in one process and print the differing positions with their context.

    python tools/dbg_variant.py spark-timeseries_amd/build/var_NAME/libsts_hip.so [T] [K]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "spark-timeseries_amd"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import oracle  # noqa: E402
from sparkts import _native  # noqa: E402
from test_acf_robust import hard_rows, with_nans  # noqa: E402


def run(lib, x, K):
    S, T = x.shape
    xd = torch.as_tensor(np.ascontiguousarray(x), device="cuda:0")
    acf = torch.empty((S, K), dtype=torch.float64, device="cuda:0")
    filled = torch.empty_like(xd)
    assert lib.sts_fill_autocorr(xd.data_ptr(), filled.data_ptr(), S, T, T, T, 0, K, acf.data_ptr(), None, None) == 0
    torch.cuda.synchronize()
    return filled.cpu().numpy()


def main():
    var = _native.load_variant(sys.argv[1])
    T = int(sys.argv[2]) if len(sys.argv) > 2 else 16461
    K = int(sys.argv[3]) if len(sys.argv) > 3 else 20
    _native.ensure_device(0)
    var.sts_init(0)
    rng = np.random.default_rng(T * 7 + K)
    x = with_nans(hard_rows(T, T + K), rng)
    rf, _, _ = oracle.panel_fill_autocorr(x, "linear", K, threads=4)
    a = run(_native.lib(), x, K)
    b = run(var, x, K)
    print("product bit-exact:", np.array_equal(a.view(np.uint64), rf.view(np.uint64)))
    d = np.argwhere(b.view(np.uint64) != rf.view(np.uint64))
    print("variant mismatches:", len(d))
    for s, t in d[:40]:
        lo, hi = max(0, t - 3), min(T, t + 4)
        print(s, t, "tile", t // 4096, "pos", t % 4096, "x", x[s, lo:hi], "ref", rf[s, t], "got", b[s, t])


if __name__ == "__main__":
    main()
