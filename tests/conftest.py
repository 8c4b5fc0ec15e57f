"""pytest configuration: the `gpu` marker and import paths.

`-m "not gpu"` runs here (no GPU): the oracle against the reference's known-
answer tests and golden fixtures, host logic, and the C-ABI export check.
`-m gpu` runs on an MI355X: parity of the HIP path (through the C-ABI) with
the oracle.
"""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "spark-timeseries_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_addoption(parser):
    # tools/ab_variants.sh: the parity gate of an A/B variant library must run THAT library (the
    # package itself reads no environment variable, so the selection is an explicit option)
    parser.addoption("--sts-lib", default=None, help="run the tests against this build of libsts_hip.so")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device) and libsts_hip.so")
    path = config.getoption("--sts-lib")
    if path:
        if not os.path.exists(path):
            raise pytest.UsageError("--sts-lib %s: no such library" % path)
        # torch first: it loads the HIP runtime the library must bind to (a library loaded
        # before it pulls /opt/rocm's runtime in, and sts_init then sees no device)
        import torch  # noqa: F401
        from sparkts import _native
        _native.use_library(path)


@pytest.fixture
def ab_lib(monkeypatch):
    """Route the sparkts mirror through build/libsts_hip_ab.so (the -DSTS_AB build that reads
    the A/B experiment knobs) for one test; the product libsts_hip.so ignores the
    environment.  Yields a setter: ab_lib(NAME=value, ...) sets knobs for this test."""
    from sparkts import _native
    monkeypatch.setattr(_native, "_lib", _native.load_variant(_native.AB_LIB_PATH))

    def knobs(**kv):
        for k, v in kv.items():
            monkeypatch.setenv(k, str(v))
    return knobs
