"""The JNI glue (jni/deltareplay_jni.c) against the C ABI: type-checked with gcc (-Wall -Werror) on a
compile-check JNI header (tests/native/jni_min/jni.h; no JDK in this image), every native of the
Scala binding (jni/DeltaReplayNative.scala) defined with the JNI name of `object DeltaReplayNative`,
and every library function the glue calls exported by libdeltareplay.so's header."""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GLUE = os.path.join(ROOT, "jni", "deltareplay_jni.c")
SCALA = os.path.join(ROOT, "jni", "DeltaReplayNative.scala")
HEADER = os.path.join(ROOT, "include", "deltareplay.h")


@pytest.mark.skipif(shutil.which("gcc") is None, reason="no gcc")
def test_glue_type_checks_against_the_abi():
    r = subprocess.run(["gcc", "-std=c99", "-fsyntax-only", "-Wall", "-Wextra", "-Werror", "-Wno-unused-parameter",
                        "-I", os.path.join(ROOT, "tests", "native", "jni_min"), "-I", os.path.join(ROOT, "include"),
                        GLUE], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


def test_every_scala_native_has_its_jni_symbol():
    scala = open(SCALA).read()
    natives = set(re.findall(r"@native def (\w+)\(", scala))
    glue = open(GLUE).read()
    defined = set(re.findall(r"^NATIVE\(\w+, (\w+)\)\(", glue, re.M))
    assert natives and natives == defined, (natives - defined, defined - natives)


def test_glue_calls_only_declared_functions():
    header = open(HEADER).read()
    declared = set(re.findall(r"\b(dr_\w+)\s*\(", header))
    called = set(re.findall(r"\b(dr_\w+)\(", open(GLUE).read()))
    assert called <= declared, called - declared
