"""pytest configuration: the `gpu` marker and import paths.

`-m "not gpu"` runs here (no GPU): the oracle against the reference's known-
answer tests and golden fixtures, host logic, and the C-ABI export check.
`-m gpu` runs on an MI355X: parity of the HIP path (through the C-ABI) with
the oracle.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "spark-timeseries_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device) and libsts_hip.so")
