"""bench.py's counter fields describe the kernel that was timed.

`roofline.traffic` and `roofline.fp64` come from committed rocprofv3 PMC records
(profiles/<round>_<workload>_{traffic,fp64}.json, tools/collect.py).  Each record carries the
`lib_sha16` of the libsts_hip.so it was taken on; bench.py uses the NEWEST record of the
workload (numeric version order) and only when that hash is the loaded library's -- else the
field is null.  CPU only: synthetic records in a temporary profiles/ tree."""
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

S3, T3 = bench.WORKLOADS["c3"][:2]


@pytest.fixture
def tree(tmp_path, monkeypatch):
    (tmp_path / "profiles").mkdir()
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    monkeypatch.setattr(bench, "LIB_SHA16", "aaaaaaaaaaaaaaaa")

    def put(name, rec):
        with open(tmp_path / "profiles" / name, "w") as f:
            json.dump(rec, f)
    return put


def test_traffic_used_only_for_the_loaded_library(tree):
    tree("r05_s9_c3_traffic.json", {"traffic_bytes_per_launch": 1.0e11, "lib_sha16": "aaaaaaaaaaaaaaaa"})
    assert bench.measured_traffic("c3", S3, T3) == 1.0e11
    # a newer record of another build hides the older matching one: null, not a stale figure
    tree("r05_s10_c3_traffic.json", {"traffic_bytes_per_launch": 2.0e11, "lib_sha16": "bbbbbbbbbbbbbbbb"})
    assert bench.measured_traffic("c3", S3, T3) is None


def test_traffic_without_a_hash_is_not_used(tree):
    tree("r04_v13_c3_traffic.json", {"traffic_bytes_per_launch": 1.0e11})
    assert bench.measured_traffic("c3", S3, T3) is None


def test_newest_record_by_numeric_version(tree):
    # r05_s10 is newer than r05_s9 (numeric, not lexical), r05 newer than r04_v13
    tree("r04_v13_c3_traffic.json", {"traffic_bytes_per_launch": 3.0e11, "lib_sha16": "aaaaaaaaaaaaaaaa"})
    tree("r05_s9_c3_traffic.json", {"traffic_bytes_per_launch": 4.0e11, "lib_sha16": "cccccccccccccccc"})
    tree("r05_s10_c3_traffic.json", {"traffic_bytes_per_launch": 5.0e11, "lib_sha16": "aaaaaaaaaaaaaaaa"})
    assert bench.measured_traffic("c3", S3, T3) == 5.0e11


def test_other_shapes_get_no_traffic(tree):
    tree("r05_s9_c3_traffic.json", {"traffic_bytes_per_launch": 1.0e11, "lib_sha16": "aaaaaaaaaaaaaaaa"})
    assert bench.measured_traffic("c3", S3 // 2, T3) is None


def test_fp64_used_only_for_the_loaded_library(tree):
    rec = {"fp64_flops_per_launch": 1.6e12, "mfma_fp64_flops_per_launch": 1.5e12,
           "valu_fp64_flops_per_launch": 1.0e11, "mfma_busy_frac": 0.58, "lib_sha16": "aaaaaaaaaaaaaaaa"}
    tree("r05_final_c3_fp64.json", rec)
    got = bench.measured_fp64("c3", S3, T3, 40.0)
    assert got is not None and got["tflops"] == round(1.6e12 / 0.040 / 1e12, 2)
    assert got["source"] == "r05_final_c3_fp64.json"
    tree("r05_final_c3_fp64.json", dict(rec, lib_sha16="dddddddddddddddd"))
    assert bench.measured_fp64("c3", S3, T3, 40.0) is None


def test_lib_sha16_is_the_library_file_hash(tmp_path):
    import hashlib
    p = tmp_path / "lib.so"
    p.write_bytes(b"\x7fELF-not-really")
    assert bench.lib_sha16(str(p)) == hashlib.sha256(b"\x7fELF-not-really").hexdigest()[:16]
