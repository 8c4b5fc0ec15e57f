"""CPU-side checks of the C-ABI boundary (no GPU, no compute calls).

* libsts_hip.so builds for gfx950 and loads;
* every function declared in include/sts.h is exported and bound by the host mirror
  (sparkts/_native.py) with the same arity;
* pure host logic (method-name mapping, status -> exception mapping) behaves like the
  reference (S/UnivariateTimeSeries.scala:141-150).
"""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "sts.h")
LIB = os.path.join(ROOT, "spark-timeseries_amd", "build", "libsts_hip.so")


def declared():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    decls = {}
    for m in re.finditer(r"\b(int|const char\*)\s+(sts_\w+)\s*\(([^;]*?)\)\s*;", text, flags=re.S):
        args = m.group(3).strip()
        n = 0 if args in ("", "void") else args.count(",") + 1
        decls[m.group(2)] = n
    return decls


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(LIB):
        subprocess.check_call(["make", "-s", "-j8", "-C", os.path.join(ROOT, "spark-timeseries_amd")])
    from sparkts import _native
    return _native.load_library()


def test_header_declares_the_boundary():
    d = declared()
    for name in ("sts_fill", "sts_autocorr", "sts_fill_autocorr", "sts_diff_at_lag", "sts_lag_matrix",
                 "sts_ewma_add", "sts_ewma_remove", "sts_ar_fit", "sts_ar_remove", "sts_ar_add",
                 "sts_fill_diff_ewma", "sts_fill_lag_matrix", "sts_ar_fit_remove", "sts_last_error"):
        assert name in d, name


def test_library_exports_every_declared_symbol(lib):
    out = subprocess.check_output(["nm", "-D", "--defined-only", LIB]).decode()
    exported = set(re.findall(r" T (sts_\w+)", out))
    missing = set(declared()) - exported
    assert not missing, missing


def test_bindings_match_header_arity(lib):
    from sparkts import _native
    d = declared()
    assert set(d) == set(_native.SIGNATURES), set(d) ^ set(_native.SIGNATURES)
    for name, n in d.items():
        assert len(_native.SIGNATURES[name][1]) == n, name


def test_library_is_gfx950_code(lib):
    # the offload bundle inside the .so must target gfx950
    out = subprocess.check_output(["strings", LIB]).decode(errors="ignore")
    assert "gfx950" in out


def test_fill_method_names(lib):
    from sparkts import UnivariateTimeSeries as uts
    from sparkts.errors import UnsupportedOperationException
    assert uts.fill_method_code("linear") == 0
    assert uts.fill_method_code("nearest") == 1
    assert uts.fill_method_code("next") == 2
    assert uts.fill_method_code("previous") == 3
    assert uts.fill_method_code("spline") == 4
    with pytest.raises(UnsupportedOperationException):
        uts.fill_method_code("cubic")


def test_no_cpu_fallback_without_device(lib):
    # no GPU in this container: the product path must fail loudly, never compute on the CPU
    import numpy as np
    from sparkts import UnivariateTimeSeries as uts
    from sparkts.errors import DeviceError
    try:
        import torch
        if torch.cuda.is_available():
            pytest.skip("a GPU is visible")
    except ImportError:
        pass
    with pytest.raises(DeviceError):
        uts.fillLinear(np.array([1.0, np.nan, 3.0]))


def test_argument_errors_need_no_device(lib):
    # validation happens before any device call, with the reference's exception classes
    import numpy as np
    from sparkts import UnivariateTimeSeries as uts
    from sparkts.errors import IllegalArgumentException
    with pytest.raises(IllegalArgumentException, match="starting index cannot be less than lag"):
        uts.differencesAtLag(np.arange(5.0), 3, startIndex=1)


def test_indexed_row_matrix_needs_uniform_index():
    # S/TimeSeriesRDD.scala:386-388: UnsupportedOperationException for non-uniform indices,
    # raised before any device work
    import numpy as np
    from sparkts.errors import UnsupportedOperationException
    from sparkts.timeseriesrdd import TimeSeriesRDD, _is_uniform
    assert _is_uniform(None) and _is_uniform(np.array(["2015-04-09", "2015-04-10", "2015-04-11"]))
    irregular = np.array(["2015-04-09", "2015-04-10", "2015-04-12"])
    assert not _is_uniform(irregular)
    with pytest.raises(UnsupportedOperationException, match="only supported for uniform indices"):
        TimeSeriesRDD(irregular, None, np.zeros((2, 3))).toIndexedRowMatrix()


def test_sts_lib_option_runs_the_named_build(tmp_path):
    """tools/ab_variants.sh gates each variant library on the parity tests with --sts-lib (the
    package reads no environment variable): the option must load THAT build, and a missing
    build must stop the run instead of silently testing the product library."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    ab = os.path.join(root, "spark-timeseries_amd", "build", "libsts_hip_ab.so")
    probe = tmp_path / "test_probe.py"
    probe.write_text("def test_probe():\n    from sparkts import _native\n    print('LIB=' + _native.lib()._name)\n")
    conf = tmp_path / "conftest.py"
    conf.write_text(open(os.path.join(root, "tests", "conftest.py")).read().replace(
        "ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))", "ROOT = %r" % root))
    run = lambda lib: subprocess.run([sys.executable, "-m", "pytest", str(probe), "-q", "-s", "-p", "no:cacheprovider",
                                      "--sts-lib", lib], capture_output=True, text=True, cwd=str(tmp_path))
    r = run(ab)
    assert r.returncode == 0 and ("LIB=" + ab) in r.stdout, r.stdout + r.stderr
    r = run(str(tmp_path / "missing.so"))
    assert r.returncode != 0 and "no such library" in (r.stdout + r.stderr)
