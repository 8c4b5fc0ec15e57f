"""The JNI shim (spark-timeseries_amd/jni/sts_jni.cpp) type-checks against include/sts.h.

No JDK exists in this image, so the shim is compiled with -fsyntax-only
against tests/native/jni_stub/jni.h, a stand-in declaring only the JNI C++ members the shim
uses with the JDK's signatures.  This catches drift between the shim and the C ABI (every
_host entry point it calls, their arity and pointer types); behaviour is exercised only on a
JVM host.  Also checks the shim's memory rules: no GetPrimitiveArrayCritical (no JVM array
is held across device work) and every native method validates array lengths.

Behaviour without a JVM: the shim is also LINKED against tests/native/jni_fake_env.cpp, an
in-memory stand-in for the JNIEnv members it uses plus a CPU backend of the C-ABI calls built
from the oracle's primitives, and run (under ASan/UBSan): the record-level natives
(fillRecords, fillDiffEwmaRecords, arFitRemoveRecords) must gather a partition's record
arrays, return a FRESH double[] per record (no two records share a backing array and none
aliases an input: each record owns its vector as in S/TimeSeriesRDD.scala:538, VERDICT r2
"What's missing" #4), keep record order and values, and throw the reference's exception
classes (unknown method, ragged records, nearest on [5, NaN], spline on fewer than 3 points), keep
"spline" a working method, and turn a partition
too large for any buffer into java.lang.OutOfMemoryError instead of aborting the JVM."""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SHIM = os.path.join(ROOT, "spark-timeseries_amd", "jni", "sts_jni.cpp")


@pytest.mark.skipif(shutil.which("g++") is None, reason="no g++")
def test_shim_type_checks_against_the_c_abi():
    r = subprocess.run(["g++", "-std=c++17", "-fsyntax-only", "-Wall", "-Werror",
                        "-I", os.path.join(ROOT, "tests", "native", "jni_stub"), "-I", os.path.join(ROOT, "include"),
                        SHIM], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


def test_shim_holds_no_critical_section_and_checks_lengths():
    src = open(SHIM).read()
    assert "GetPrimitiveArrayCritical" not in src
    methods = re.findall(r"Java_com_cloudera_sparkts_StsNative_(\w+)\(", src)
    assert len(methods) >= 15
    bodies = re.split(r"JNIEXPORT \w+ JNICALL Java_com_cloudera_sparkts_StsNative_", src)[1:]
    assert len(bodies) == len(methods)
    for b in bodies:
        # panel forms check every array's length; record forms check each record in gather_records
        assert "check_len(" in b or "gather_records(" in b, b.split("(")[0]


@pytest.mark.skipif(shutil.which("g++") is None or shutil.which("gcc") is None, reason="no compiler")
def test_shim_record_scatter_on_a_stand_in_jvm(tmp_path):
    oracle_dir = os.path.join(ROOT, "oracle")
    orc = str(tmp_path / "orc.o")
    subprocess.check_call(["gcc", "-std=c11", "-O1", "-ffp-contract=off", "-fopenmp", "-fPIC", "-I", oracle_dir,
                           "-c", os.path.join(oracle_dir, "sts_oracle.c"), "-o", orc])
    exe = str(tmp_path / "jni_fake")
    r = subprocess.run(["g++", "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
                        "-Wall", "-Werror", "-I", os.path.join(ROOT, "tests", "native", "jni_stub"),
                        "-I", os.path.join(ROOT, "include"), "-I", oracle_dir, SHIM,
                        os.path.join(ROOT, "tests", "native", "jni_fake_env.cpp"), orc, "-fopenmp", "-lm", "-o", exe],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-4000:]
    # pinned buffers available, and not (sts_host_alloc fails: every *Records / Region path falls
    # back to heap buffers instead of throwing -- ADVICE r3)
    for nopin in ("0", "1"):
        # allocator_may_return_null: the oversized-partition case must see a failed allocation
        # (std::bad_alloc / NULL), as on a real host, not ASan's own abort
        env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:allocator_may_return_null=1", JNI_FAKE_NO_PIN=nopin)
        r = subprocess.run([exe], capture_output=True, text=True, env=env, timeout=300)
        assert r.returncode == 0 and r.stdout.strip() == "ok", nopin + r.stdout[-3000:] + r.stderr[-3000:]
