"""The JVM binding of the drop-in boundary: the JNI adapter
integration/jni/capf_jni.cpp covers every C-ABI entry point of
include/capf_gpu.h, type-checks against that header, and matches the @native
declarations of integration/scala/org/opencypher/gpu/Native.scala one to one.

No JDK exists in this image, so the adapter is compiled with g++ -fsyntax-only
against tests/jni_stub/jni.h (the JNI types and functions it uses, declared per
the JNI specification); a real build uses $JAVA_HOME/include/jni.h.
"""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SHIM = os.path.join(ROOT, "integration", "jni", "capf_jni.cpp")
NATIVE = os.path.join(ROOT, "integration", "scala", "org", "opencypher", "gpu", "Native.scala")
HEADER = os.path.join(ROOT, "include", "capf_gpu.h")


def header_functions():
    text = open(HEADER).read()
    return sorted(set(re.findall(r"^[a-z_0-9 ]+\*?\s*\*?(capf_[a-z0-9_]+)\(", text, re.M)))


def test_every_entry_point_is_bound():
    shim = open(SHIM).read()
    fns = header_functions()
    assert len(fns) >= 55, fns
    missing = [f for f in fns if f + "(" not in shim]
    assert not missing, f"C-ABI entry points without a JNI binding: {missing}"


def test_native_declarations_match_jni_symbols():
    shim = open(SHIM).read()
    jni = set(re.findall(r"^JNI\([^,]+,\s*(\w+)\)", shim, re.M))
    scala = set(re.findall(r"@native def (\w+)\(", open(NATIVE).read()))
    assert jni == scala, (sorted(jni - scala), sorted(scala - jni))


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not available")
def test_shim_type_checks_against_header():
    r = subprocess.run(["g++", "-std=c++17", "-fsyntax-only", "-Wall", "-Wextra", "-Werror",
                        "-Wno-unused-parameter", "-I", os.path.join(ROOT, "include"),
                        "-I", os.path.join(ROOT, "tests", "jni_stub"), SHIM],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
