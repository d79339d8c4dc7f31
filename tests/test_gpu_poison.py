"""The device allocator's debug mode (engine.hip dr_ctx::poisoned / release / check_quarantine):
with DR_POISON set, every block handed out is filled with 0xA5 (a kernel that reads memory it never
wrote sees the same garbage whatever ran before), and every released block is filled with 0xA5 and
held back until the API call ends, when it must still hold only 0xA5 -- a write after release is a
launch queued after its buffer was handed back. (That check found the deferred tail walk writing
its line count into a released block that the apply's index counters could reuse: a
history-dependent size_in_bytes error of the random-commit apply) The replay, apply,
walker, checkpoint-writer, export and filter suites run once (the sharded suite passed in this mode too, r05, and is left out for time) in that mode in a child process."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_suites_pass_with_poisoned_and_quarantined_blocks():
    sel = ["tests/test_gpu_parity.py",
           "tests/test_gpu_edge_cases.py::test_device_walker_matches_fuzz_corpus",
           "tests/test_gpu_edge_cases.py::test_device_walker_mutations",
           "tests/test_gpu_edge_cases.py::test_device_walker_one_wave_segments",
           "tests/test_gpu_edge_cases.py::test_snappy_long_literals_and_unstaged_blocks",
           "tests/test_gpu_checkpoint.py",
           "tests/test_gpu_export_range.py",
           "tests/test_gpu_filter.py"]
    env = dict(os.environ, DR_POISON="1", JL_GPU_FUZZ="20000")
    r = subprocess.run([sys.executable, "-u", "-m", "pytest", "-x", "-q", "-m", "gpu", "-p", "no:cacheprovider",
                        "--timeout", "600", "--timeout-method", "thread"] + sel,
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=1100)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert " passed" in out and "DR_POISON" not in out
