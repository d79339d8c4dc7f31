"""Multi-GPU driver on CPU: the shard plan (host code of libdeltareplay) and a world_size-2 gloo
run of delta_amd/sharded.py with the oracle standing in for the device (tests/shard_fake.py),
compared with the single-process oracle replay."""
import json
import os
import socket
import subprocess
import sys

import pytest

from oracle import delta_oracle as O
from tests.conftest import GOLDEN, ROOT

REF = os.path.join(GOLDEN, "ref")


def _synthetic(tmp_path, rg=700):
    from delta_amd.testing import synth as S
    exp = S.build_table(str(tmp_path), S.config_spec(3, 0.0005), seed=11, row_group_size=rg)
    return os.path.join(str(tmp_path), "_delta_log"), exp


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_shard_plan_contiguous_and_complete(tmp_path, world):
    from delta_amd.sharded import shard_plan
    lp, exp = _synthetic(tmp_path)
    plan = shard_plan(lp, world)
    seg = O.get_log_segment(lp)
    # every checkpoint row group and every delta exactly once, in replay order
    import pyarrow.parquet as pq
    want = []
    for name in sorted(seg.checkpoint):
        for g in range(pq.ParquetFile(os.path.join(lp, name)).num_row_groups):
            want.append((name, g, g + 1))
    want += [(name, 0, -1) for name in seg.deltas]
    assert [(u["name"], u["rg_lo"], u["rg_hi"]) for u in plan] == want
    ranks = [u["rank"] for u in plan]
    assert ranks == sorted(ranks) and 0 <= ranks[0] and ranks[-1] < world
    # balance: no rank carries more than its share plus one unit
    tot = sum(u["weight"] for u in plan)
    biggest = max(u["weight"] for u in plan)
    for r in range(world):
        w = sum(u["weight"] for u in plan if u["rank"] == r)
        assert w <= tot / world + biggest


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def run_sharded(log_path, cutoff, out, nproc, backend, env=None):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(nproc),
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "tests", "workers", "sharded_worker.py"), log_path, str(cutoff), out, backend]
    e = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="1")
    e.update(env or {})
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=e, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-4000:]
    with open(out) as f:
        return json.load(f)


def _canon(rec):
    return repr(sorted((k, repr(v)) for k, v in rec.items()))


def _check(res, snap):
    c = res["counts"]
    assert c["num_files"] == snap.num_of_files
    assert c["size_in_bytes"] == snap.size_in_bytes
    assert c["num_removes"] == snap.num_of_removes
    assert c["num_protocol"] == snap.num_of_protocol
    assert c["num_metadata"] == snap.num_of_metadata
    assert c["num_set_transactions"] == snap.num_of_set_transactions
    assert sorted(r["path"] for r in res["live"]) == sorted(r["path"] for r in snap.all_files)
    assert sorted(r["path"] for r in res["tomb"]) == sorted(r["path"] for r in snap.tombstones)
    assert sorted(map(_canon, res["live"])) == sorted(map(_canon, snap.all_files))


@pytest.mark.parametrize("nproc", [2])
def test_sharded_gloo_synthetic(tmp_path, nproc):
    lp, exp = _synthetic(tmp_path / "t")
    res = run_sharded(lp, exp.min_file_retention_timestamp, str(tmp_path / "out.json"), nproc, "fake")
    snap = O.state_reconstruction(O.get_log_segment(lp), exp.min_file_retention_timestamp)
    assert res["counts"]["num_files"] == exp.num_files
    _check(res, snap)


def test_sharded_gloo_golden(tmp_path):
    lp = os.path.join(REF, "delta-0.2.0", "_delta_log")
    res = run_sharded(lp, 0, str(tmp_path / "out.json"), 2, "fake")
    _check(res, O.state_reconstruction(O.get_log_segment(lp), 0))
    assert [list(a)[0] for a in res["nonfile"]][:2] == ["protocol", "metaData"]


def test_sharded_checkpoint_mismatch_raises_on_every_rank(tmp_path):
    """A sharded checkpoint whose parts hold fewer add rows than numOfFiles: every rank raises the
    reference's error (D/Checkpoints.scala:325-328) -- none is left waiting in the final barrier, and
    no `_last_checkpoint` is written."""
    log = tmp_path / "_delta_log"
    log.mkdir()
    out = tmp_path / "out"
    out.mkdir()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "tests", "workers", "ckpt_mismatch_worker.py"), str(log), str(out)]
    e = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="1")
    r = subprocess.run(cmd, env=e, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    for rank in (0, 1):
        got = (out / ("%d.txt" % rank)).read_text()
        assert got.startswith("raised:") and "doesn't match" in got, got
    assert not (log / "_last_checkpoint").exists()
