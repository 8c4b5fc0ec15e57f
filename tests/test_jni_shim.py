"""The JNI shim (spark-timeseries_amd/jni/sts_jni.cpp) type-checks against include/sts.h.

No JDK exists in this image, so the shim is compiled with -fsyntax-only
against tests/native/jni_stub/jni.h, a stand-in declaring only the JNI C++ members the shim
uses with the JDK's signatures.  This catches drift between the shim and the C ABI (every
_host entry point it calls, their arity and pointer types); behaviour is exercised only on a
JVM host.  Also checks the shim's memory rules: no GetPrimitiveArrayCritical (no JVM array
is held across device work) and every native method validates array lengths."""
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
    assert len(methods) >= 12
    bodies = re.split(r"JNIEXPORT void JNICALL Java_com_cloudera_sparkts_StsNative_", src)[1:]
    for b in bodies:
        assert "check_len(" in b, b.split("(")[0]
