"""GPU parity of the multi-GPU path (dr_stage_log_shard / dr_shard_*) on one MI355X: W ranks
emulated as threads of one process (each with its own context and stream) exchanging through
device tensors, and a 2-process gloo run of the real per-rank driver; compared with the oracle."""
import json
import os

import pytest

from oracle import delta_oracle as O
from tests.conftest import GOLDEN

pytestmark = pytest.mark.gpu

REF = os.path.join(GOLDEN, "ref")


def _canon(rec):
    return repr(sorted((k, repr(v)) for k, v in rec.items()))


def _sharded(lp, cutoff, world):
    from delta_amd.delta_log import Engine
    from delta_amd.sharded import replay_sharded, stage_shard
    from tests.thread_exchange import run_threads

    def rank_fn(r, ex):
        eng = Engine.get(0)  # thread-local context on device 0
        staged = stage_shard(eng, lp, world, r)
        try:
            st = replay_sharded(staged, cutoff, ex)
        finally:
            staged.release()
        out = (st.counts, st.nonfile, st.local.export(0), st.local.export(1))
        st.release()
        return out

    res = run_threads(world, rank_fn)
    counts, nonfile = res[0][0], res[0][1]
    for c, nf, _, _ in res:
        assert c == counts and nf == nonfile
    live = [x for r in res for x in r[2]]
    tomb = [x for r in res for x in r[3]]
    return counts, nonfile, live, tomb


def _check(counts, live, tomb, snap):
    assert O.record_sums(live, tomb) == O.record_sums(snap.all_files, snap.tombstones)
    assert counts["num_files"] == snap.num_of_files
    assert counts["size_in_bytes"] == snap.size_in_bytes
    assert counts["num_removes"] == snap.num_of_removes
    assert counts["num_protocol"] == snap.num_of_protocol
    assert counts["num_metadata"] == snap.num_of_metadata
    assert counts["num_set_transactions"] == snap.num_of_set_transactions
    assert sorted(map(_canon, live)) == sorted(map(_canon, snap.all_files))
    assert sorted(map(_canon, tomb)) == sorted(map(_canon, snap.tombstones))


@pytest.mark.parametrize("world", [1, 2, 3])
@pytest.mark.parametrize("name", ["delta-0.2.0", "dbr_8_1_generated_columns"])
def test_sharded_golden(name, world):
    lp = os.path.join(REF, name, "_delta_log")
    cutoff = 1564524298213
    counts, _, live, tomb = _sharded(lp, cutoff, world)
    _check(counts, live, tomb, O.state_reconstruction(O.get_log_segment(lp), cutoff))


@pytest.mark.parametrize("world", [1, 2, 4, 8])
def test_sharded_synthetic(tmp_path, world):
    from delta_amd.testing import synth as S
    exp = S.build_table(str(tmp_path), S.config_spec(3, 0.003), seed=5, row_group_size=4000)
    lp = os.path.join(str(tmp_path), "_delta_log")
    cutoff = exp.min_file_retention_timestamp
    counts, _, live, tomb = _sharded(lp, cutoff, world)
    assert (counts["num_files"], counts["num_removes"], counts["size_in_bytes"], counts["num_actions"],
            counts["num_file_actions"]) == (exp.num_files, exp.num_removes, exp.size_in_bytes,
                                            exp.num_actions, exp.num_file_actions)
    # the order-free key checksums equal the single-GPU replay's
    from delta_amd.delta_log import Engine
    staged = Engine.get(0).stage_log(lp)
    st = staged.replay(cutoff)
    staged.release()
    assert counts["live_key_sum"] == st.counts["live_key_sum"]
    assert counts["tomb_key_sum"] == st.counts["tomb_key_sum"]
    st.release()
    _check(counts, live, tomb, O.state_reconstruction(O.get_log_segment(lp), cutoff))


def test_sharded_two_processes_gloo(tmp_path):
    from delta_amd.testing import synth as S
    from tests.test_sharded_cpu import run_sharded
    exp = S.build_table(str(tmp_path / "t"), S.config_spec(2, 0.002), seed=9, row_group_size=500)
    lp = os.path.join(str(tmp_path / "t"), "_delta_log")
    res = run_sharded(lp, exp.min_file_retention_timestamp, str(tmp_path / "o.json"), 2, "gpu",
                      env={"DR_TEST_BACKEND": "gloo"})
    snap = O.state_reconstruction(O.get_log_segment(lp), exp.min_file_retention_timestamp)
    _check(res["counts"], res["live"], res["tomb"], snap)


# ---- the sharded replay inside the library (RCCL, dr_replay_sharded) ----------------------------------
@pytest.mark.parametrize("name", ["delta-0.2.0", "dbr_8_1_generated_columns"])
def test_rccl_library_single_rank(name):
    """dr_comm_create + dr_replay_sharded with one rank: the RCCL collectives (all-gather of counts
    and non-file winners, grouped send/recv to self, all-reduce of the counters) run for real and the
    state equals the oracle's."""
    from delta_amd.delta_log import Engine
    from delta_amd.sharded import stage_shard
    lp = os.path.join(REF, name, "_delta_log")
    cutoff = 1564524298213
    eng = Engine.get(0)
    comm = eng.comm(Engine.comm_unique_id(), 1, 0)
    try:
        staged = stage_shard(eng, lp, 1, 0)
        st = comm.replay_sharded(staged, cutoff)
        staged.release()
        try:
            _check(st.counts, st.export(0), st.export(1), O.state_reconstruction(O.get_log_segment(lp), cutoff))
        finally:
            st.release()
    finally:
        comm.release()


def _library_sharded(lp, cutoff, world, validate=True):
    """dr_comm_create + dr_replay_sharded with `world` ranks as threads of this process over the
    library's loopback transport (dr_comm_loopback_id): replay_sharded_rccl's own control flow --
    count-matrix all-gather, record / path / verdict all-to-alls, counter all-reduce, non-file
    all-gather -- at W > 1 on one GPU."""
    import threading
    from delta_amd.delta_log import Engine
    from delta_amd.sharded import stage_shard
    uid = Engine.comm_loopback_id()
    res, err = [None] * world, [None] * world

    def body(r):
        try:
            eng = Engine.get(0)  # thread-local context (own stream) on device 0
            comm = eng.comm(uid, world, r)
            try:
                staged = stage_shard(eng, lp, world, r)
                try:
                    st = comm.replay_sharded(staged, cutoff, validate)
                finally:
                    staged.release()
                try:
                    res[r] = (st.counts, st.nonfile, st.export(0), st.export(1), st.record_sums())
                finally:
                    st.release()
            finally:
                comm.release()
        except BaseException as e:  # noqa: BLE001
            err[r] = e

    th = [threading.Thread(target=body, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
    assert not any(t.is_alive() for t in th), "a loopback rank hung"
    for e in err:
        if e is not None:
            raise e
    counts, nonfile = res[0][0], res[0][1]
    for c, nf, _, _, _ in res:
        assert c == counts and nf == nonfile
    live, tomb = [x for r in res for x in r[2]], [x for r in res for x in r[3]]
    # the ranks' record checksums add up to the table's (each rank exports its own survivors)
    m = (1 << 64) - 1
    assert (sum(r[4][0] for r in res) & m, sum(r[4][1] for r in res) & m) == O.record_sums(live, tomb)
    return counts, nonfile, live, tomb


@pytest.mark.parametrize("world", [2, 3, 8])
@pytest.mark.parametrize("name", ["delta-0.2.0", "dbr_8_1_generated_columns"])
def test_library_sharded_loopback_golden(name, world):
    lp = os.path.join(REF, name, "_delta_log")
    cutoff = 1564524298213
    counts, _, live, tomb = _library_sharded(lp, cutoff, world)
    _check(counts, live, tomb, O.state_reconstruction(O.get_log_segment(lp), cutoff))


@pytest.mark.parametrize("world", [2, 4, 8])
def test_library_sharded_loopback_synthetic(tmp_path, world):
    """Config 3's shape (checkpoint + churned commits + retention cutoff) sharded over 2/4/8 ranks by
    the library driver: counters, key sums and both record sets equal the single-GPU replay and the
    oracle."""
    from delta_amd.delta_log import Engine
    from delta_amd.testing import synth as S
    exp = S.build_table(str(tmp_path), S.config_spec(3, 0.003), seed=5, row_group_size=4000)
    lp = os.path.join(str(tmp_path), "_delta_log")
    cutoff = exp.min_file_retention_timestamp
    counts, _, live, tomb = _library_sharded(lp, cutoff, world)
    assert (counts["num_files"], counts["num_removes"], counts["size_in_bytes"], counts["num_actions"],
            counts["num_file_actions"]) == (exp.num_files, exp.num_removes, exp.size_in_bytes,
                                            exp.num_actions, exp.num_file_actions)
    staged = Engine.get(0).stage_log(lp)
    st = staged.replay(cutoff)
    staged.release()
    for k in ("live_key_sum", "tomb_key_sum", "num_protocol", "num_metadata", "num_set_transactions"):
        assert counts[k] == st.counts[k], k
    st.release()
    _check(counts, live, tomb, O.state_reconstruction(O.get_log_segment(lp), cutoff))


def test_library_sharded_loopback_missing_metadata_fails_on_every_rank(tmp_path):
    """A collective error path: the table-wide validation (no metaData in any slice) fails on every
    rank with the reference's IllegalStateException text, and no rank hangs."""
    from delta_amd.delta_log import DeltaError
    lp = str(tmp_path / "_delta_log")
    os.makedirs(lp)
    with open(os.path.join(lp, "%020d.json" % 0), "w") as f:
        f.write('{"protocol":{"minReaderVersion":1,"minWriterVersion":2}}\n')
        f.write('{"add":{"path":"a","partitionValues":{},"size":1,"modificationTime":1,"dataChange":true}}\n')
    for v in (1, 2):
        with open(os.path.join(lp, "%020d.json" % v), "w") as f:
            f.write('{"add":{"path":"f%d","partitionValues":{},"size":1,"modificationTime":1,"dataChange":true}}\n' % v)
    with pytest.raises(DeltaError, match="metadata of your Delta table"):
        _library_sharded(lp, 0, 3)
    counts, _, live, _ = _library_sharded(lp, 0, 3, validate=False)
    assert counts["num_files"] == 3 and len(live) == 3 and counts["num_metadata"] == 0


def test_rccl_library_two_processes(tmp_path):
    """Two processes, one communicator, both on this box's one GPU. RCCL refuses two ranks on one
    device ("duplicate GPU"); then the test is skipped (the exchange logic is the one the thread and
    gloo tests cover; the RCCL calls themselves ran in the single-rank test)."""
    import subprocess
    import sys
    from delta_amd.testing import synth as S
    exp = S.build_table(str(tmp_path / "t"), S.config_spec(2, 0.002), seed=9, row_group_size=500)
    lp = os.path.join(str(tmp_path / "t"), "_delta_log")
    cutoff = exp.min_file_retention_timestamp
    script = os.path.join(os.path.dirname(os.path.abspath(__file__)), "rccl_rank.py")
    uid = str(tmp_path / "uid")
    outs = [str(tmp_path / ("r%d.json" % r)) for r in range(2)]
    procs = [subprocess.Popen([sys.executable, script, lp, str(cutoff), "2", str(r), uid, outs[r]],
                              stdout=subprocess.PIPE, stderr=subprocess.STDOUT, start_new_session=True)
             for r in range(2)]
    logs = []
    try:
        for p in procs:
            logs.append(p.communicate(timeout=120)[0].decode(errors="replace"))
    finally:
        for p in procs:
            if p.poll() is None:
                os.killpg(p.pid, 9)
    res = []
    for o, lg in zip(outs, logs):
        if not os.path.exists(o):
            pytest.skip("RCCL run did not complete on one device: " + lg[-400:])
        with open(o) as f:
            res.append(json.load(f))
    if any("error" in r for r in res):
        pytest.skip("RCCL refuses two ranks on one device: " + " | ".join(r.get("error", "") for r in res))
    snap = O.state_reconstruction(O.get_log_segment(lp), cutoff)
    assert res[0]["counts"] == res[1]["counts"] and res[0]["nonfile"] == res[1]["nonfile"]
    _check(res[0]["counts"], res[0]["live"] + res[1]["live"], res[0]["tomb"] + res[1]["tomb"], snap)


def test_sharded_one_process_rccl(tmp_path):
    """The torch.distributed driver over the "nccl" backend (RCCL) with one rank: every collective
    of replay_sharded (count / record / path / verdict all-to-alls, the counter all-reduce, the
    non-file all-gather) runs through RCCL on the device (the N-GPU bench's code path)."""
    from delta_amd.testing import synth as S
    from tests.test_sharded_cpu import run_sharded
    exp = S.build_table(str(tmp_path / "t"), S.config_spec(2, 0.002), seed=9, row_group_size=500)
    lp = os.path.join(str(tmp_path / "t"), "_delta_log")
    res = run_sharded(lp, exp.min_file_retention_timestamp, str(tmp_path / "o.json"), 1, "gpu",
                      env={"DR_TEST_BACKEND": "nccl"})
    _check(res["counts"], res["live"], res["tomb"], O.state_reconstruction(O.get_log_segment(lp),
                                                                          exp.min_file_retention_timestamp))


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_device_checkpoint_parts(tmp_path, world):
    """The multi-part checkpoint from the GPU shards: every emulated rank encodes
    its own part on the device (dr_state_write_checkpoint on its sharded state; part 1 also holds the
    table-wide protocol / metaData / txn set by dr_state_set_nonfile_json), rank 0 writes
    `_last_checkpoint`; a fresh replay then starts from the new parts and equals the oracle's state
    of the original log, as does the oracle's own replay of the rewritten log."""
    from delta_amd.delta_log import Engine
    from delta_amd.sharded import replay_sharded, stage_shard, write_checkpoint_sharded
    from delta_amd.testing import synth as S
    from tests.thread_exchange import run_threads
    table = str(tmp_path / "t")
    exp = S.build_config(2, table, scale=0.01)
    lp = os.path.join(table, "_delta_log")
    cutoff = exp.min_file_retention_timestamp
    snap = O.state_reconstruction(O.get_log_segment(lp), cutoff)

    def rank_fn(r, ex):
        eng = Engine.get(0)
        staged = stage_shard(eng, lp, world, r)
        try:
            st = replay_sharded(staged, cutoff, ex)
        finally:
            staged.release()
        try:
            return st.counts["version"], write_checkpoint_sharded(st, lp, st.counts["version"])
        finally:
            st.release()

    res = run_threads(world, rank_fn)
    version, total = res[0]
    assert all(x == res[0] for x in res)
    assert total == snap.num_of_files + snap.num_of_removes + snap.num_of_protocol + snap.num_of_metadata + \
        snap.num_of_set_transactions
    parts = sorted(f for f in os.listdir(lp) if f.startswith("%020d.checkpoint." % version))
    assert len(parts) == world, parts
    with open(os.path.join(lp, "_last_checkpoint")) as f:
        assert json.load(f) == {"version": version, "size": total, "parts": world}
    seg = O.get_log_segment(lp)
    assert len(seg.checkpoint) == world and seg.checkpoint_version == version
    again = O.state_reconstruction(seg, cutoff)
    _check(snap_counts(again), again.all_files, again.tombstones, snap)
    eng = Engine.get(0)
    staged = eng.stage_log(lp)
    try:
        st = staged.replay(cutoff)
    finally:
        staged.release()
    try:
        _check(st.counts, st.export(0), st.export(1), snap)
    finally:
        st.release()


def snap_counts(s):
    return {"num_files": s.num_of_files, "size_in_bytes": s.size_in_bytes, "num_removes": s.num_of_removes,
            "num_protocol": s.num_of_protocol, "num_metadata": s.num_of_metadata,
            "num_set_transactions": s.num_of_set_transactions}
