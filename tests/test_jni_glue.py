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


@pytest.mark.skipif(shutil.which("gcc") is None, reason="no gcc")
def test_glue_runs_against_a_mock_jni_env(tmp_path):
    """The glue on a mock JNIEnv (tests/native/jni_mock.c) over a stub library: an export column over
    2^31 - 1 bytes is refused with UnsupportedOperationException before any direct buffer is made; a
    buffer the JVM refuses stops the export; mismatched or null stage arrays raise
    IllegalArgumentException without reading past them or calling the library; UTF-8 text with a
    supplementary character crosses both ways unchanged and error messages are built from the exact
    UTF-8 bytes; exportRange hands back its range; no scenario makes a JNI call while an exception is
    pending."""
    glue_src = open(GLUE).read()
    stub_src = open(os.path.join(ROOT, "tests", "native", "jni_stub_lib.c")).read()
    defined = set(re.findall(r"^\S[^(\n]*\b(dr_\w+)\(", stub_src, re.M))
    called = set(re.findall(r"\b(dr_\w+)\(", glue_src))
    gen = tmp_path / "gen_stubs.c"
    gen.write_text("".join("int %s() { return 15; }\n" % f for f in sorted(called - defined)))
    exe = tmp_path / "jni_mock"
    inc = ["-I", os.path.join(ROOT, "tests", "native", "jni_min"), "-I", os.path.join(ROOT, "include")]
    r = subprocess.run(["gcc", "-std=gnu99", "-O1", "-g", "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
                        "-Wno-builtin-declaration-mismatch"] + inc +
                       [GLUE, os.path.join(ROOT, "tests", "native", "jni_mock.c"),
                        os.path.join(ROOT, "tests", "native", "jni_stub_lib.c"), str(gen), "-o", str(exe)],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]
    run = subprocess.run([str(exe)], capture_output=True, text=True, timeout=60,
                         env=dict(os.environ, ASAN_OPTIONS="detect_leaks=0"))
    lines = run.stdout.strip().splitlines()
    assert run.returncode == 0 and len(lines) == 9 and all(l.endswith(" ok") for l in lines), run.stdout + run.stderr


def test_scala_calls_resolve_to_the_binding():
    """Every DeltaReplayNative.<member> the Scala sources use (the binding itself and the partitioned
    state RDD, jni/DeltaReplayStateRDD.scala) is a native or a method / value of the binding."""
    scala = open(SCALA).read()
    members = (set(re.findall(r"(?:@native )?def (\w+)", scala)) | set(re.findall(r"\bval (\w+)", scala)) |
               set(re.findall(r"\bobject (\w+)", scala)))
    rdd = open(os.path.join(ROOT, "jni", "DeltaReplayStateRDD.scala")).read()
    used = set(re.findall(r"DeltaReplayNative\.(\w+)", scala + rdd))
    assert used and used <= members, used - members
