"""Parity at the benchmark's full size (config 3, scale 1.0: 16M actions, 10.8M survivors) by record
multisets: every survivor's full-record hash (dr_state_record_hashes, the definition of
oracle/delta_oracle.py:record_hash over every field of the record) sorted and compared element by
element with the CPU restatement's (oracle/_build/replay_oracle --record-hashes). Equal sorted lists
mean every record of both sides is equal up to a 64-bit collision of the record hash -- a stronger
statement than the order-free sums the bench compares, which compensating differences could cancel.
The oracle is the checker only (test infrastructure)."""
import os
import subprocess
import tempfile

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "oracle", "_build", "replay_oracle")


def test_full_size_record_multisets_equal_the_restatement(tmp_path):
    import json
    from delta_amd import _native as N
    from delta_amd.delta_log import Engine
    from delta_amd.testing import synth as S
    if not os.path.exists(EXE):
        pytest.skip("oracle/_build/replay_oracle is not built")
    table = os.path.join(tempfile.gettempdir(), "dr_fullsize_c3")
    if not os.path.exists(os.path.join(table, "expected.json")):
        subprocess.run([os.sys.executable, "-m", "delta_amd.testing.synth", "3", table, "1.0", "16"], cwd=ROOT,
                       check=True, stdout=subprocess.DEVNULL)
    exp = json.load(open(os.path.join(table, "expected.json")))
    cutoff = exp["min_file_retention_timestamp"]
    log = os.path.join(table, "_delta_log")
    eng = Engine.get(0)
    staged = eng.stage_log(log)
    st = staged.replay(cutoff)
    staged.release()
    try:
        assert st.counts["num_files"] == exp["num_files"] == 10_000_000
        gpu = {w: np.sort(st.record_hashes(w)) for w in (N.DR_LIVE, N.DR_TOMBSTONES)}
    finally:
        st.release()
    prefix = str(tmp_path / "rh")
    r = subprocess.run([EXE, log, str(cutoff), "--threads", "16", "--record-hashes", prefix], capture_output=True,
                       text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    cpu = {N.DR_LIVE: np.sort(np.fromfile(prefix + ".live", dtype=np.uint64)),
           N.DR_TOMBSTONES: np.sort(np.fromfile(prefix + ".tomb", dtype=np.uint64))}
    assert len(gpu[N.DR_LIVE]) == out["num_files"] and len(gpu[N.DR_TOMBSTONES]) == out["num_removes"]
    for w in (N.DR_LIVE, N.DR_TOMBSTONES):
        assert np.array_equal(gpu[w], cpu[w]), ("side", w, int(np.sum(gpu[w] != cpu[w])))
    # and the sums the bench compares are these lists' sums
    assert int(gpu[N.DR_LIVE].sum(dtype=np.uint64)) == out["live_record_sum"]
