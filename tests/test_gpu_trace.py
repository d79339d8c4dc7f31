"""Stage tracing: with DR_ROCTX set, the library loads rocprofiler-sdk's roctx and
brackets each replay stage in a range (engine.hip StageRange: parse.json, decode.checkpoint,
canonicalize, hash.partition, reduce, compact, under delta.stateReconstruction; filter, export,
checkpoint.write, apply, exchange). DR_ROCTX=sync closes each range with a stream synchronize; the
replay's results are unchanged either way. (rocprofv3 --marker-trace shows the ranges; the round's
trace summary is under profiles/r05/.)"""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r'''
import os, sys, tempfile
sys.path.insert(0, %r)
from delta_amd.delta_log import Engine
from delta_amd.testing import synth as S
eng = Engine.get(0)
with tempfile.TemporaryDirectory() as d:
    exp = S.build_config(3, d, scale=0.002)
    staged = eng.stage_log(os.path.join(d, "_delta_log"))
    st = staged.replay(exp.min_file_retention_timestamp)
    assert st.counts["num_files"] == exp.num_files and st.counts["num_removes"] == exp.num_removes
    st.release()
    staged.release()
maps = open("/proc/self/maps").read()
print("ROCTX_LOADED", "roctx" in maps)
'''


@pytest.mark.parametrize("mode", ["1", "sync"])
def test_stage_ranges_load_roctx_and_keep_results(mode):
    env = dict(os.environ, DR_ROCTX=mode)
    r = subprocess.run([sys.executable, "-c", CHILD % ROOT], env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    assert "ROCTX_LOADED True" in r.stdout, r.stdout[-1000:]
