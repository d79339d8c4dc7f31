"""ISA properties of the K1 line walkers (hipcc -S for gfx950, CPU only): neither k_json_lines
instantiation has a private segment (no scratch) or a flat load/store. The staged walker reads its
LDS stage through the __shared__ array, so every stage read is a ds_read, which is bounds-checked
against the workgroup's LDS allocation; r03's one-walker build reached the stage through a generic
pointer that could also be global, so its reads became flat loads, and an out-of-allocation LDS
address through a flat load faults (HSA_STATUS_ERROR_MEMORY_APERTURE_VIOLATION)."""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "delta_amd", "csrc")
HIPCC = "/opt/rocm/bin/hipcc"


@pytest.fixture(scope="module")
def k_json_asm(tmp_path_factory):
    if not os.path.exists(HIPCC):
        pytest.skip("no hipcc")
    out = str(tmp_path_factory.mktemp("isa") / "k_json.s")
    r = subprocess.run([HIPCC, "-O3", "-std=c++17", "--offload-arch=gfx950", "--cuda-device-only", "-S",
                        "-I", CSRC, os.path.join(CSRC, "k_json.hip"), "-o", out],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    return open(out).read()


def _kernel(asm, mangled):
    i = asm.index(mangled + ":")
    body = asm[i:asm.index(".Lfunc_end", i)]
    md = asm[asm.index("amdhsa.kernels:"):]
    entry = next(e for e in re.split(r"\n  - \.", md) if re.search(r"name:\s+" + re.escape(mangled) + r"\n", e))
    private = int(re.search(r"private_segment_fixed_size:\s+(\d+)", entry).group(1))
    return body, private


@pytest.mark.parametrize("staged", [True, False])
def test_k_json_lines_has_no_scratch_and_no_flat_access(k_json_asm, staged):
    name = "_ZN2dr3dev12k_json_linesILb%dEEEvNS_13JsonParseArgsE" % int(staged)
    body, private = _kernel(k_json_asm, name)
    assert private == 0, "private segment of %d bytes" % private
    assert not re.search(r"\bscratch_(load|store)", body)
    flat = re.findall(r"^\s*flat_\w+.*$", body, re.M)
    assert not flat, flat[:5]
    if staged:
        assert re.search(r"\bds_read", body)  # the stage is read from LDS


def test_apply_commit_reads_its_stage_and_tapes_from_lds(k_json_asm):
    """k_apply_commit (a streamed commit's whole apply in one workgroup) walks wave-private tapes
    over an LDS stage like the staged walker: it has no flat access beyond those of k_apply_small,
    the same apply without the walk (byte reads through path pointers, which are global)."""
    name = ("_ZN2dr3dev14k_apply_commitENS_13JsonParseArgsENS_9CanonArgsENS_10AppendArgsENS_9IndexArgsE"
            "mNS_12ReadbackArgsE")  # (+ the fused expiry count and readback, r06)
    small = "_ZN2dr3dev13k_apply_smallENS_13JsonParseArgsENS_9CanonArgsENS_10AppendArgsENS_9IndexArgsE"
    body, _ = _kernel(k_json_asm, name)
    ref, _ = _kernel(k_json_asm, small)
    flat = len(re.findall(r"^\s*flat_\w+", body, re.M))
    assert flat <= len(re.findall(r"^\s*flat_\w+", ref, re.M)), flat
    assert re.search(r"\bds_read", body)
