"""The tape kernels' LDS index checks (k_json.hip built with -DDR_BOUNDS_CHECK:
delta_amd/libdeltareplay_bounds.so): every computed stage / tape index of build_tape, tape_lines,
k_apply_commit and the staged k_json_lines is compared with its array's extent before use, and a miss
prints "LDS-BOUNDS <site>". A ds_read outside the workgroup's allocation returns 0 instead of faulting,
so an over-read would only show as a wrong token (the r03 fault record's unisolated read, DESIGN.md
§4). The device walker's fuzz corpus and mutations (staged and not), the one-wave segments, the
writer-shaped waves and the random-commit applies run once on that library in a child process: all
pass and no index leaves its array."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_tape_kernels_stay_in_their_lds_arrays():
    lib = os.path.join(ROOT, "delta_amd", "libdeltareplay_bounds.so")
    assert os.path.exists(lib), "make builds libdeltareplay_bounds.so"
    sel = ["tests/test_gpu_edge_cases.py::test_device_walker_matches_fuzz_corpus",
           "tests/test_gpu_edge_cases.py::test_device_walker_mutations",
           "tests/test_gpu_edge_cases.py::test_device_walker_writer_shaped_waves",
           "tests/test_gpu_edge_cases.py::test_device_walker_one_wave_segments",
           "tests/test_gpu_parity.py::test_incremental_apply_random_commits",
           "tests/test_gpu_parity.py::test_incremental_apply_matches_full_replay"]
    env = dict(os.environ, DR_LIB="libdeltareplay_bounds.so")
    r = subprocess.run([sys.executable, "-u", "-m", "pytest", "-x", "-q", "-s", "-m", "gpu", "-p", "no:cacheprovider",
                        "--timeout", "600", "--timeout-method", "thread"] + sel,
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=1200)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert " passed" in out
    hits = [l for l in out.splitlines() if "LDS-BOUNDS" in l]
    assert not hits, hits[:20]
