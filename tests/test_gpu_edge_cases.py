"""GPU parity on the reference's edge cases, through the C-ABI (dr_stage_log / dr_replay_staged /
dr_parse_commits), each against the oracle and the reference test it restates:

* path canonicalization and the URI replay key (T/DeltaLogSuite.scala:190-254, D/Snapshot.scala:301-328,
  D/actions/actions.scala:208-213): unqualified absolute adds vs `file:` / `file://` removes, special
  characters, JSON-escaped paths, absolute tombstones qualified as `file://...`, checkpoint rows;
* replay order: delete + re-add (T/DeltaLogSuite.scala:256-279), the same path twice in one commit;
* the replay's error branches: missing protocol / metadata from JSON and from a checkpoint
  (T/DeltaLogSuite.scala:306-400), corrupt `_last_checkpoint` (:162-188), truncated log, missing
  or incomplete checkpoint parts, zero-byte checkpoints, an empty log directory;
* K1's device walker (k_json_lines + k_json_hard) over the host fuzz corpus and its mutations
  (tests/test_json_lane.py), read back per line with dr_parse_commits;
* dr_state_apply with a retention cutoff that moved backwards (rebuild), and a replaced snapshot
  that stays usable.
"""
import json
import os
import random
import shutil

import pytest

from oracle import delta_oracle as O
from tests.conftest import GOLDEN
from tests.test_gpu_parity import _assert_same, _canon, _gpu_replay

pytestmark = pytest.mark.gpu

REF = os.path.join(GOLDEN, "ref")
PROTOCOL = {"protocol": {"minReaderVersion": 1, "minWriterVersion": 2}}
METADATA = {"metaData": {"id": "edge", "format": {"provider": "parquet", "options": {}},
                         "schemaString": '{"type":"struct","fields":[]}', "partitionColumns": [],
                         "configuration": {}, "createdTime": 1}}


@pytest.fixture(scope="module")
def engine():
    from delta_amd.delta_log import Engine
    return Engine.get(0)


def add(path, size=100, mtime=10, data_change=True):
    return {"add": {"path": path, "partitionValues": {}, "size": size, "modificationTime": mtime,
                    "dataChange": data_change}}


def remove(path, ts=200, data_change=False):
    return {"remove": {"path": path, "deletionTimestamp": ts, "dataChange": data_change}}


def write_commit(lp, version, actions, raw_lines=()):
    os.makedirs(lp, exist_ok=True)
    lines = [json.dumps(a, separators=(",", ":")) for a in actions] + list(raw_lines)
    with open(os.path.join(lp, "%020d.json" % version), "w") as f:
        f.write("\n".join(lines) + "\n")


def _same_as_oracle(engine, lp, cutoff=0, version=-1):
    snap = O.state_reconstruction(O.get_log_segment(lp, None if version < 0 else version), cutoff)
    st = _gpu_replay(engine, lp, cutoff, version=version)
    try:
        _assert_same(st, snap)
        return st.counts, st.export(0), st.export(1)
    finally:
        st.release()


def _error(engine, lp, cutoff=0, validate=True):
    from delta_amd.delta_log import DeltaError
    with pytest.raises(DeltaError) as ei:
        _gpu_replay(engine, lp, cutoff, validate=validate)
    return ei.value


# ---- canonicalization (T/DeltaLogSuite.scala:190-254) ---------------------------------------------
@pytest.mark.parametrize("scheme", ["file:", "file://"])
@pytest.mark.parametrize("path", ["/some/unqualified/absolute/path",
                                  "/some/unqualified/with%20space/p@%23h"])  # new Path(..).toUri.toString
def test_paths_are_canonicalized(engine, tmp_path, scheme, path):
    lp = str(tmp_path / "_delta_log")
    write_commit(lp, 0, [PROTOCOL, METADATA, add(path)])
    write_commit(lp, 1, [remove(scheme + path)])
    counts, live, tomb = _same_as_oracle(engine, lp)
    assert counts["num_files"] == 0 and counts["version"] == 1
    assert [t["path"] for t in tomb] == [scheme + path]  # a qualified path is kept as written


@pytest.mark.parametrize("add_path,rm_path,live", [
    ("file:/x/y.parquet", "/x/y.parquet", 0),          # the other direction
    ("file:///x/y.parquet", "file:/x/y.parquet", 0),   # URI equality: empty authority == none
    ("/x//y.parquet", "/x/y.parquet", 0),               # Hadoop Path normalisation of the absolute add
    ("file://host/x/y.parquet", "file:/x/y.parquet", 1),  # an authority is part of the key
    ("a/b.parquet", "/a/b.parquet", 1),                 # relative != absolute
])
def test_uri_replay_key(engine, tmp_path, add_path, rm_path, live):
    lp = str(tmp_path / "_delta_log")
    write_commit(lp, 0, [PROTOCOL, METADATA, add(add_path)])
    write_commit(lp, 1, [remove(rm_path)])
    counts, _, _ = _same_as_oracle(engine, lp)
    assert counts["num_files"] == live


@pytest.mark.parametrize("add_path,rm_path", [
    ("p%2fx.parquet", "p%2Fx.parquet"),        # percent-escape hex digits in another case
    ("file:/x/a.parquet", "FILE:/x/a.parquet"),  # scheme in another case
])
def test_uri_case_rules_parity_unpinned(engine, tmp_path, add_path, rm_path):
    """java.net.URI.equals ignores the case of the scheme and of escape hex digits, so the reference's
    per-partition HashMap would merge these two spellings -- but only when coalesce(add.path,
    remove.path)'s string hash puts both in one of its 50 shuffle partitions (D/Snapshot.scala:103-104),
    which differs per pair: the reference's own result is not fixed (parity unpinned).
    The device and the oracle key by bytes (besides file:/ = file:///): the two spellings stay two
    files, the add live and the remove a tombstone. This pins that behaviour."""
    lp = str(tmp_path / "_delta_log")
    write_commit(lp, 0, [PROTOCOL, METADATA, add(add_path)])
    write_commit(lp, 1, [remove(rm_path)])
    counts, live, tomb = _same_as_oracle(engine, lp)
    assert counts["num_files"] == 1 and [f["path"] for f in live] == [add_path]
    assert counts["num_removes"] == 1 and [t["path"] for t in tomb] == [rm_path]


def test_escaped_paths(engine, tmp_path):
    """JSON escapes in a path are decoded before canonicalization and keying: `\\/x\\/a` is `/x/a`,
    `a\\u0062c` is `abc`, `\\u00e9` is UTF-8 `é`."""
    lp = str(tmp_path / "_delta_log")
    write_commit(lp, 0, [PROTOCOL, METADATA, add("/x/a.parquet"), add("abc.parquet"), add("keep\u00e9.parquet")])
    write_commit(lp, 1, [], raw_lines=['{"remove":{"path":"file:\\/x\\/a.parquet","deletionTimestamp":5}}',
                                       '{"remove":{"path":"a\\u0062c.parquet","deletionTimestamp":6}}'])
    counts, live, tomb = _same_as_oracle(engine, lp)
    assert [f["path"] for f in live] == ["keep\u00e9.parquet"]
    assert sorted(t["path"] for t in tomb) == ["abc.parquet", "file:/x/a.parquet"]


def test_absolute_tombstone_is_qualified(engine, tmp_path):
    """"do not relativize paths in RemoveFiles": a tombstone of an absolute path is stored as
    file://<path> (T/DeltaLogSuite.scala:243-254)."""
    lp = str(tmp_path / "_delta_log")
    path = str(tmp_path / "a" / "b" / "c")
    write_commit(lp, 0, [PROTOCOL, METADATA, remove(path, ts=1700000000000, data_change=True)])
    _, live, tomb = _same_as_oracle(engine, lp)
    assert not live and [t["path"] for t in tomb] == ["file://" + path]
    assert tomb[0]["dataChange"] is False


def test_checkpoint_rows_with_absolute_paths(engine, tmp_path):
    """Canonicalization of checkpoint rows (k_ckpt_assemble flags them, k_canon rewrites them):
    a checkpoint with absolute and `file:` paths, removed by JSON commits in the other form."""
    from delta_amd.testing import synth as S
    lp = str(tmp_path / "_delta_log")
    os.makedirs(lp)
    adds = [{"path": p, "partitionValues": {}, "size": i + 1, "modificationTime": 5}
            for i, p in enumerate(["/abs/one.parquet", "file:/abs/two.parquet", "file:///abs/three.parquet",
                                   "rel/four.parquet"])]
    rms = [{"path": "/abs/gone.parquet", "deletionTimestamp": 50}]
    S.write_checkpoint_records(os.path.join(lp, "%020d.checkpoint.parquet" % 3), PROTOCOL["protocol"],
                               METADATA["metaData"], adds, rms)
    write_commit(lp, 4, [remove("file:///abs/one.parquet"), remove("/abs/two.parquet"),
                         add("file:/abs/gone.parquet")])
    counts, live, tomb = _same_as_oracle(engine, lp, cutoff=10)
    assert sorted(f["path"] for f in live) == sorted(["file:/abs/gone.parquet", "file:///abs/three.parquet",
                                                      "rel/four.parquet"])
    assert sorted(t["path"] for t in tomb) == ["file:///abs/one.parquet", "file:///abs/two.parquet"]


@pytest.mark.parametrize("hint", ["0", "16", "1000000"])
def test_canonicalisation_arena_hint(engine, tmp_path, request, hint):
    """A replay queues k_canon with an arena sized from the segment's last need (no read-back before
    K3); the context option DR_OPT_CANON_HINT stands in for that need on the first replay. An arena too small (no arena at
    all, 16 bytes) is detected after the replay and the replay redone at the exact size; an ample one
    is used as is. Every case, and a second replay of the same staged segment, equals the oracle."""
    lp = str(tmp_path / "_delta_log")
    write_commit(lp, 0, [PROTOCOL, METADATA, add("/abs/one.parquet"), add("file:/abs/two.parquet"),
                         add("rel/three.parquet")],
                 raw_lines=['{"add":{"path":"\\/abs\\/four.parquet","size":4,"modificationTime":1,"dataChange":true}}'])
    write_commit(lp, 1, [remove("file:///abs/one.parquet"), remove("/abs/two.parquet", ts=300)])
    engine.set_option("canon_hint", int(hint))
    request.addfinalizer(lambda: engine.set_option("canon_hint", -1))
    snap = O.state_reconstruction(O.get_log_segment(lp), 250)
    staged = engine.stage_log(lp)
    try:
        for _ in range(2):
            st = staged.replay(250)
            try:
                _assert_same(st, snap)
                assert st.counts["num_files"] == 2 and st.counts["num_removes"] == 1
            finally:
                st.release()
    finally:
        staged.release()


# ---- replay order -----------------------------------------------------------------------------------
def test_delete_and_readd_in_different_transactions(engine, tmp_path):
    """T/DeltaLogSuite.scala:256-279: add, remove, re-add -> live, dataChange=false."""
    lp = str(tmp_path / "_delta_log")
    write_commit(lp, 0, [PROTOCOL, METADATA, add("foo")])
    write_commit(lp, 1, [remove("foo", ts=10)])
    write_commit(lp, 2, [add("foo", size=7)])
    counts, live, tomb = _same_as_oracle(engine, lp)
    assert [(f["path"], f["size"], f["dataChange"]) for f in live] == [("foo", 7, False)] and not tomb


def test_same_path_twice_in_one_commit(engine, tmp_path):
    """PROTOCOL.md:209 forbids it; the reference's stable sort over a one-split commit makes the
    last line win (SURVEY.md §7 'Ordering')."""
    lp = str(tmp_path / "_delta_log")
    write_commit(lp, 0, [PROTOCOL, METADATA, add("a", size=1), add("a", size=2), add("b"), remove("b", ts=9),
                         remove("c", ts=9), add("c", size=3)])
    write_commit(lp, 1, [add("d", size=4), remove("d", ts=11), add("d", size=5), add("e", size=6),
                         add("e", size=7)])
    counts, live, tomb = _same_as_oracle(engine, lp)
    assert sorted((f["path"], f["size"]) for f in live) == [("a", 2), ("c", 3), ("d", 5), ("e", 7)]
    assert [t["path"] for t in tomb] == ["b"]


# ---- error branches -----------------------------------------------------------------------------------
@pytest.mark.parametrize("action", ["protocol", "metadata"])
def test_missing_action_in_json(engine, tmp_path, action):
    """T/DeltaLogSuite.scala:306-330."""
    lp = str(tmp_path / "_delta_log")
    write_commit(lp, 0, [PROTOCOL if action == "metadata" else METADATA, add("abc", 1, 1)])
    e = _error(engine, lp)
    assert e.kind == "IllegalStateException"
    assert str(e) == O.action_not_found(action, 0)
    with pytest.raises(O.DeltaError) as oe:
        O.state_reconstruction(O.get_log_segment(lp), 0)
    assert str(oe.value) == str(e)
    st = _gpu_replay(engine, lp, 0, validate=False)  # stateReconstructionValidation.enabled=false
    try:
        assert st.counts["version"] == 0 and st.counts["num_files"] == 1
    finally:
        st.release()


@pytest.mark.parametrize("action", ["protocol", "metadata"])
def test_missing_action_in_checkpoint(engine, tmp_path, action):
    """T/DeltaLogSuite.scala:332-400: the checkpoint at version 10 keeps the adds but lacks the action."""
    from delta_amd.testing import synth as S
    lp = str(tmp_path / "_delta_log")
    os.makedirs(lp)
    adds = [{"path": str(i), "partitionValues": {}, "size": 1, "modificationTime": 1} for i in range(11)]
    S.write_checkpoint_records(os.path.join(lp, "%020d.checkpoint.parquet" % 10),
                               None if action == "protocol" else PROTOCOL["protocol"],
                               None if action == "metadata" else METADATA["metaData"], adds)
    with open(os.path.join(lp, "_last_checkpoint"), "w") as f:
        f.write('{"version":10,"size":12}\n')
    for v in range(0, 11):
        write_commit(lp, v, [add(str(v), 1, 1)])
    e = _error(engine, lp)
    assert e.kind == "IllegalStateException" and str(e) == O.action_not_found(action, 10)
    st = _gpu_replay(engine, lp, 0, validate=False)
    try:
        assert st.counts["version"] == 10 and st.counts["num_files"] == 11
    finally:
        st.release()


def _checkpointed_table(tmp_path, parts=None, last=True):
    """v0..v7 with a complete checkpoint at v3 (single part) and one at v6 (`parts` parts)."""
    from delta_amd.testing import synth as S
    lp = str(tmp_path / "_delta_log")
    write_commit(lp, 0, [PROTOCOL, METADATA] + [add("f%d" % i) for i in range(4)])
    for v in range(1, 8):
        write_commit(lp, v, [remove("f%d" % (v - 1), ts=100 + v), add("g%d" % v, size=v)])

    def ckpt(version, nparts):
        snap = O.state_reconstruction(O.get_log_segment(lp, version), 0)
        adds, rms = snap.all_files, snap.tombstones
        if not nparts:
            S.write_checkpoint_records(os.path.join(lp, "%020d.checkpoint.parquet" % version), snap.protocol,
                                       snap.metadata, adds, rms)
            return
        for k in range(nparts):  # split the rows over the parts (protocol + metadata in part 1)
            sl = lambda xs: xs[k::nparts]
            S.write_checkpoint_records(
                os.path.join(lp, "%020d.checkpoint.%010d.%010d.parquet" % (version, k + 1, nparts)),
                snap.protocol if k == 0 else None, snap.metadata if k == 0 else None, sl(adds), sl(rms))

    ckpt(3, None)
    ckpt(6, parts)
    if last:
        with open(os.path.join(lp, "_last_checkpoint"), "w") as f:
            f.write(json.dumps({"version": 6, "size": 9, **({"parts": parts} if parts else {})}) + "\n")
    return lp


@pytest.mark.parametrize("content", [b"", b'{"version":', b"not json\n", b'{"version":"6"}'])
def test_corrupt_last_checkpoint_falls_back_to_listing(engine, tmp_path, content):
    """T/DeltaLogSuite.scala:162-188: a corrupted `_last_checkpoint` -> the latest complete
    checkpoint found by listing (D/Checkpoints.scala:166-173)."""
    lp = _checkpointed_table(tmp_path, parts=3)
    with open(os.path.join(lp, "_last_checkpoint"), "wb") as f:
        f.write(content)
    ver, files = engine.log_segment(lp)
    assert ver == 7 and {(k, v) for k, v, _, _ in files if k == 1} == {(1, 6)}
    counts, _, _ = _same_as_oracle(engine, lp)
    assert counts["version"] == 7


def test_missing_checkpoint_part(engine, tmp_path):
    """`_last_checkpoint` names a 3-part checkpoint one of whose parts is gone:
    missingPartFilesException (D/SnapshotManagement.scala:150-156, D/DeltaErrors.scala:543-546)."""
    lp = _checkpointed_table(tmp_path, parts=3)
    os.remove(os.path.join(lp, "%020d.checkpoint.%010d.%010d.parquet" % (6, 2, 3)))
    e = _error(engine, lp)
    assert e.kind == "IllegalStateException"
    assert str(e) == "Couldn't find all part files of the checkpoint version: 6"
    with pytest.raises(O.DeltaError) as oe:
        O.get_log_segment(lp)
    assert str(oe.value) == str(e)


@pytest.mark.parametrize("damage", ["part", "zero"])
def test_incomplete_or_empty_checkpoint_is_skipped(engine, tmp_path, damage):
    """Without `_last_checkpoint`, an incomplete multi-part checkpoint (a part missing) or a 0-byte
    checkpoint file is skipped for the previous complete one (D/Checkpoints.scala:210-218,
    D/SnapshotManagement.scala:90-92)."""
    lp = _checkpointed_table(tmp_path, parts=3 if damage == "part" else None, last=False)
    if damage == "part":
        os.remove(os.path.join(lp, "%020d.checkpoint.%010d.%010d.parquet" % (6, 3, 3)))
    else:
        open(os.path.join(lp, "%020d.checkpoint.parquet" % 6), "wb").close()
    ver, files = engine.log_segment(lp)
    assert ver == 7 and [v for k, v, _, _ in files if k == 1] == [3]
    assert [v for k, v, _, _ in files if k == 0] == [4, 5, 6, 7]
    _same_as_oracle(engine, lp)


def test_truncated_log(engine, tmp_path):
    """No checkpoint and no version 0: logFileNotFoundException (D/SnapshotManagement.scala:160-163)."""
    lp = str(tmp_path / "_delta_log")
    for v in (1, 2, 3):
        write_commit(lp, v, [add("x%d" % v)])
    e = _error(engine, lp)
    assert e.kind == "FileNotFoundException"
    assert str(e) == ("%s/%020d.json: Unable to reconstruct state at version 3 as the transaction log has been "
                      "truncated due to manual deletion or the log retention policy (delta.logRetentionDuration="
                      "30 days) and checkpoint retention policy (delta.checkpointRetentionDuration=2 days)" % (lp, 0))
    with pytest.raises(O.DeltaError) as oe:
        O.get_log_segment(lp)
    assert str(oe.value) == str(e)


def test_noncontiguous_and_empty(engine, tmp_path):
    lp = str(tmp_path / "_delta_log")
    write_commit(lp, 0, [PROTOCOL, METADATA])
    write_commit(lp, 2, [add("x")])
    e = _error(engine, lp)  # T/DeltaLogSuite.scala:281-304
    assert e.kind == "IllegalStateException" and str(e) == "Versions (Vector(0, 2)) are not contiguous."
    empty = str(tmp_path / "empty" / "_delta_log")
    os.makedirs(empty)
    e = _error(engine, empty)
    assert e.kind == "FileNotFoundException" and str(e) == "No file found in the directory: %s." % empty


# ---- K1 device walker fuzz ---------------------------------------------------------------------------------
def _walker_mode(engine, request, staged):
    """staged: every 64-line wave through the small-segment kernel (LDS stage, token tape, the
    wave-parallel tape walk; context option DR_OPT_JSON_STAGED) instead of the bulk per-lane walker."""
    engine.set_option("json_staged", 1 if staged else 0)
    request.addfinalizer(lambda: engine.set_option("json_staged", 0))


def _device_lines(engine, lines):
    body = b"".join(l + b"\n" for l in lines)
    staged = engine.stage_files([(0, 0, 0, body)])
    try:
        return staged.parse_lines()
    finally:
        staged.release()


def _device_view(rec):
    from tests.test_json_lane import K_ADD, K_REMOVE
    out = {"kind": rec["kind"]}
    if rec["kind"] in (K_ADD, K_REMOVE):
        raw = rec["path"]
        path = None if raw is None else (json.loads(b'"' + raw + b'"') if rec["escaped"] else raw.decode("utf-8"))
        out.update(path=path, size=rec["size"], delts=rec["deletionTimestamp"])
    return out


@pytest.mark.parametrize("staged", [False, True])
def test_device_walker_matches_fuzz_corpus(engine, request, staged):
    """Every corpus line (golden logs, synthetic formats, hand-written edge cases) at 16 byte
    alignments, through k_json_lines / k_json_hard on the GPU, against the PERMISSIVE-reader
    restatement that the host build of the walker is fuzzed against."""
    _walker_mode(engine, request, staged)
    from tests.test_json_lane import corpus, expected
    base = [l for l in corpus() if b"\n" not in l]
    lines = []
    for align in range(16):  # a prefix line of `align` bytes shifts every following line
        lines.append(b" " * align)
        lines.extend(base)
    got = _device_lines(engine, lines)
    assert len(got) == len(lines)
    for line, rec in zip(lines, got):
        assert rec["line"] == line
        assert _device_view(rec) == expected(line), line


@pytest.mark.parametrize("staged", [False, True])
def test_device_walker_mutations(engine, request, staged):
    _walker_mode(engine, request, staged)
    from tests.test_json_lane import K_ADD, K_ERROR, corpus, expected, mutate
    rng = random.Random(0xDE17B)
    base = corpus()
    lines = []
    while len(lines) < int(os.environ.get("JL_GPU_FUZZ", "60000")):
        line = mutate(rng, rng.choice(base))
        if b"\n" in line:
            continue
        try:
            line.decode("utf-8")
        except UnicodeDecodeError:
            continue
        lines.append(line)
    got = _device_lines(engine, lines)
    kinds = {}
    for line, rec in zip(lines, got):
        exp = expected(line)
        assert _device_view(rec) == exp, line
        kinds[exp["kind"]] = kinds.get(exp["kind"], 0) + 1
    assert kinds.get(K_ERROR, 0) > len(lines) // 10 and kinds.get(K_ADD, 0) > len(lines) // 20, kinds


def test_parse_commits_versions_and_golden_lines(engine):
    """dr_parse_commits over the reference's golden commits: versions per line, and the file
    actions equal Action.fromJson's (delta_amd/actions.py) path / size / deletionTimestamp."""
    from delta_amd.actions import from_json
    lp = os.path.join(REF, "delta-0.2.0", "_delta_log")
    files = []
    for v in range(4):
        with open(os.path.join(lp, "%020d.json" % v), "rb") as f:
            files.append((v, 0, 0, f.read()))
    staged = engine.stage_files(files)
    try:
        recs = staged.parse_lines()
    finally:
        staged.release()
    want = []
    for v, _, _, data in files:
        for line in data.decode().split("\n")[:-1] if data.endswith(b"\n") else data.decode().split("\n"):
            want.append((v, from_json(line)))
    assert [r["version"] for r in recs] == [v for v, _ in want]
    for r, (_, a) in zip(recs, want):
        kind = next(iter(a)) if a else None
        assert r["kind"] == {None: 0, "add": 1, "remove": 2, "metaData": 3, "txn": 4, "protocol": 5,
                             "cdc": 6, "commitInfo": 7}[kind]
        if kind in ("add", "remove"):
            assert r["path"].decode() == a[kind]["path"] and r["size"] == a[kind]["size"]
            if kind == "remove":
                assert r["deletionTimestamp"] == a[kind]["deletionTimestamp"]


# ---- incremental apply and snapshot lifetime -------------------------------------------------------------
def test_apply_with_earlier_cutoff_rebuilds(engine, tmp_path):
    """a tail commit that lengthens delta.deletedFileRetentionDuration moves the cutoff
    back; dr_state_apply refuses (DR_E_REBUILD) and DeltaLog.update(incremental=True) rebuilds, so
    the tombstones the base had dropped come back as the reference's full replay has them."""
    from delta_amd.delta_log import DeltaError, DeltaLog, ManualClock
    root = tmp_path / "t"
    lp = str(root / "_delta_log")
    write_commit(lp, 0, [PROTOCOL, METADATA] + [add("f%d" % i) for i in range(6)])
    write_commit(lp, 1, [remove("f%d" % i, ts=1000 + i * 1000) for i in range(6)])
    week = 7 * 86400000
    DeltaLog.clear_cache()
    log = DeltaLog.for_table(str(root), clock=ManualClock(week + 3500))  # cutoff 3500: 3 tombstones
    assert log.snapshot.num_of_removes == 3
    base = log.snapshot.state
    tail = engine.stage_files([(2, 0, 0, b'{"add":{"path":"z","size":1,"modificationTime":1,"dataChange":true}}\n')])
    try:
        with pytest.raises(DeltaError) as ei:
            base.apply(tail, 1500)
        assert ei.value.code == "DR_E_REBUILD"
    finally:
        tail.release()
    md = json.loads(json.dumps(METADATA))
    md["metaData"]["configuration"] = {"delta.deletedFileRetentionDuration": "interval 2 weeks"}
    write_commit(lp, 2, [md])
    # update() computes the new snapshot's cutoff from the current snapshot's metadata
    # (D/DeltaLog.scala:109-120, D/SnapshotManagement.scala:302): v2 still uses one week
    snap2 = log.update(incremental=True)
    assert snap2.version == 2 and snap2.min_file_retention_timestamp == 3500 and snap2.num_of_removes == 3
    write_commit(lp, 3, [add("z")])
    snap3 = log.update(incremental=True)  # two weeks now: the cutoff moves back -> rebuild
    assert snap3.version == 3 and snap3.min_file_retention_timestamp == week + 3500 - 2 * week
    ref = O.state_reconstruction(O.get_log_segment(lp), snap3.min_file_retention_timestamp)
    _assert_same(snap3.state, ref)
    assert snap3.num_of_removes == 6
    # the replaced snapshot stays usable (the reference only uncaches it)
    assert sorted(f["path"] for f in snap2.tombstones) == ["f3", "f4", "f5"]
    DeltaLog.clear_cache()


def test_incremental_update_falls_back_on_gap_or_newer_checkpoint(engine, tmp_path):
    """commits cleaned up behind a newer checkpoint -> DeltaLog.update(incremental=True)
    rebuilds from the new segment instead of failing on the gap."""
    from delta_amd.delta_log import DeltaLog, ManualClock
    root = tmp_path / "t"
    lp = _checkpointed_table(root, parts=None, last=False)
    hold = {}
    for v in range(4, 8):
        fn = os.path.join(lp, "%020d.json" % v)
        hold[v] = open(fn, "rb").read()
        os.remove(fn)
    os.rename(os.path.join(lp, "%020d.checkpoint.parquet" % 6), str(root / "ck6"))
    DeltaLog.clear_cache()
    log = DeltaLog.for_table(str(root), clock=ManualClock(0))
    assert log.snapshot.version == 3
    # v4, v5 were cleaned up after the checkpoint at v6
    for v in (6, 7):
        with open(os.path.join(lp, "%020d.json" % v), "wb") as f:
            f.write(hold[v])
    os.rename(str(root / "ck6"), os.path.join(lp, "%020d.checkpoint.parquet" % 6))
    snap = log.update(incremental=True)
    assert snap.version == 7
    _assert_same(snap.state, O.state_reconstruction(O.get_log_segment(lp), snap.min_file_retention_timestamp))
    DeltaLog.clear_cache()


# ---- assertLogBelongsToTable (D/Snapshot.scala:102,334-345) -----------------------------------------
def test_stage_named_files_must_belong_to_the_log(engine, tmp_path):
    """dr_stage_named: every named file must sit directly in the table's _delta_log (Hadoop Path
    equality: a bare path is file:, repeated and trailing slashes are normalised, file:/ and
    file:/// name the same path); a foreign file fails with the reference's AssertionError text; an
    unnamed input ("", as the reference's cached snapshots) passes; a name that contradicts its
    version fails."""
    from delta_amd import _native as N
    from delta_amd.delta_log import DeltaError
    lp = str(tmp_path / "t" / "_delta_log")
    other = str(tmp_path / "u" / "_delta_log")
    os.makedirs(lp)
    lines = ['{"protocol":{"minReaderVersion":1,"minWriterVersion":2}}',
             '{"metaData":{"id":"x","format":{"provider":"parquet","options":{}},"schemaString":"{}",'
             '"partitionColumns":[],"configuration":{}}}',
             '{"add":{"path":"a.parquet","size":3,"modificationTime":1,"dataChange":true}}']
    data = ("\n".join(lines) + "\n").encode()
    files = [(0, N.DR_FILE_JSON, 0, data)]
    name = "%020d.json" % 0
    for nm in (lp + "/" + name, "file:" + lp + "/" + name, "file://" + lp + "/" + name,
               lp.replace("/_delta_log", "//_delta_log") + "//" + name, ""):
        st = engine.stage_files(files, log_path=lp, names=[nm])
        try:
            s = st.replay(0)
            assert s.counts["num_files"] == 1
            s.release()
        finally:
            st.release()
    st = engine.stage_files(files, log_path=lp + "/", names=[lp + "/" + name])  # trailing slash on the log path
    st.release()
    bad = other + "/" + name
    with pytest.raises(DeltaError) as ei:
        engine.stage_files(files, log_path=lp, names=[bad])
    assert ei.value.kind == "AssertionError"
    assert str(ei.value).endswith("File (%s) doesn't belong in the transaction log at %s. Please contact "
                                  "Databricks Support." % (bad, lp))
    with pytest.raises(DeltaError) as ei:
        engine.stage_files(files, log_path=lp, names=[lp + "/%020d.json" % 4])
    assert "does not name a delta file of version 0" in str(ei.value)


def _writer_clean(line: bytes) -> bool:
    """Lines shaped like the Delta writer's (Jackson, no whitespace): no byte below 0x21, only
    \\" \\\\ \\/ \\b \\f \\n \\r \\t escapes, and no string left open at the line end."""
    if any(c < 0x21 for c in line) or len(line) > 400:
        return False
    i = quotes = 0
    while i < len(line):
        if line[i] == 0x5C:
            if i + 1 >= len(line) or line[i + 1] not in b'"\\/bfnrt':
                return False
            i += 2
        else:
            quotes += line[i] == 0x22
            i += 1
    return quotes % 2 == 0


@pytest.mark.parametrize("staged", [False, True])
def test_device_walker_writer_shaped_waves(engine, request, staged):
    """k_json_lines against the PERMISSIVE restatement on whole 64-line waves of writer-shaped
    lines (clean corpus lines and their clean mutations) at all 16 byte skews, with backslash runs
    and escaped quotes at every window offset, scalars of every length up to 19 digits, strings on
    both sides of the fast walker's 4096-byte single-token limit and nesting past its depth limit
    (the General walker's deferral), followed by unrestricted mutations. (The same test checked the
    r02 wave-cooperative tokenizer experiment)"""
    _walker_mode(engine, request, staged)
    from tests.test_json_lane import corpus, expected, mutate
    base = [l for l in corpus() if b"\n" not in l]
    rng = random.Random(0x7A9E)
    clean = [l for l in base if _writer_clean(l)]
    while len(clean) < 64 * 160:
        m = mutate(rng, rng.choice(base))
        try:
            m.decode("utf-8")
        except UnicodeDecodeError:
            continue
        if _writer_clean(m):
            clean.append(m)
    # backslash runs and escaped quotes at every offset of a 16-byte window, long scalars, strings
    # close to the 4096-byte limit (on both sides), deep nesting (the DFA's `hard` deferral)
    for k in range(40):
        bs = b"\\\\" * k
        clean.append(b'{"add":{"path":"a' + bs + b'\\"b","size":' + str(10 ** (k % 19)).encode() + b'}}')
        clean.append(b'{"remove":{"path":"' + b"x" * k + b'\\\\","deletionTimestamp":' + str(k).encode() + b'}}')
    clean.append(b'{"add":{"path":"' + b"p" * 4095 + b'","size":1}}')
    clean.append(b'{"add":{"path":"' + b"p" * 4096 + b'","size":1}}')
    clean.append(b"[" * 70 + b"]" * 70)
    lines = []
    for skew in range(16):
        lines.append(b"x" * skew)  # an error line that shifts everything after it
        lines.extend(clean[skew * 64:(skew + 8) * 64])
    lines.extend(clean)
    dirty = [mutate(rng, rng.choice(base)) for _ in range(3000)]
    dirty = [d for d in dirty if b"\n" not in d and not _writer_clean(d)]
    lines.extend(dirty)
    got = _device_lines(engine, lines)
    assert len(got) == len(lines)
    for line, rec in zip(lines, got):
        assert rec["line"] == line
        assert _device_view(rec) == expected(line), line


@pytest.mark.parametrize("clean", [True, False])
def test_device_walker_one_wave_segments(engine, clean):
    """Segments of at most 64 lines in one 16 KiB index block (a streamed commit): the parse kernel
    indexes the newlines itself -- from the token tape, or by a scan of the stage when the region
    is off the tape (whitespace, control bytes, long strings), every line then going to the General
    walker -- against the PERMISSIVE restatement, segment by segment."""
    from tests.test_json_lane import corpus, expected, mutate
    base = [l for l in corpus() if b"\n" not in l and len(l) < 2048]
    rng = random.Random(0x51AB + clean)
    for _ in range(120):
        want = rng.randint(1, 64)
        lines, size = [], 0
        while len(lines) < want:
            line = mutate(rng, rng.choice(base)) if rng.random() < 0.4 else rng.choice(base)
            if b"\n" in line or (clean and not _writer_clean(line)):
                continue
            try:
                line.decode("utf-8")
            except UnicodeDecodeError:
                continue
            if size + len(line) + 1 > 16384:
                break
            lines.append(line)
            size += len(line) + 1
        got = _device_lines(engine, lines)
        assert len(got) == len(lines)
        for line, rec in zip(lines, got):
            assert rec["line"] == line
            assert _device_view(rec) == expected(line), line


def test_device_walker_on_synthetic_commits(engine, tmp_path):
    """Writer-canonical commits (the benchmark's add / remove lines) read per line by
    dr_parse_commits equal Action.fromJson's path and size, and the replay equals the oracle's."""
    from delta_amd.testing import synth as S
    exp = S.build_config(1, str(tmp_path), scale=0.05)
    lp = os.path.join(str(tmp_path), "_delta_log")
    files = sorted(f for f in os.listdir(lp) if f.endswith(".json"))
    staged = engine.stage_files([(int(f[:20]), 0, 0, open(os.path.join(lp, f), "rb").read()) for f in files])
    try:
        recs = staged.parse_lines()
    finally:
        staged.release()
    from delta_amd.actions import from_json
    i = 0
    for f in files:
        for line in open(os.path.join(lp, f), "rb").read().split(b"\n")[:-1]:
            a = from_json(line.decode())
            r = recs[i]
            i += 1
            fa = a.get("add") or a.get("remove")
            if fa is not None:
                assert r["path"].decode() == fa["path"]
                assert r["size"] == fa.get("size", 0)
    assert i == len(recs)
    st = _gpu_replay(engine, lp, exp.min_file_retention_timestamp)
    try:
        _assert_same(st, O.state_reconstruction(O.get_log_segment(lp), exp.min_file_retention_timestamp))
    finally:
        st.release()


# ---- SNAPPY pages the compressor could not shrink -------------------------------------------------
def test_incompressible_snappy_pages(engine, tmp_path, capfd, monkeypatch):
    """Dictionary-encoded columns whose indices are random (add.size / remove.deletionTimestamp drawn
    from 60,000 random values) give SNAPPY data pages that are runs of literals, one per 64 KiB
    fragment; they are copied as they are (no serial fallback) and the replay and the export equal
    the oracle."""
    import random
    from delta_amd.testing import synth as S
    lp = str(tmp_path / "_delta_log")
    os.makedirs(lp)
    rng = random.Random(11)
    pool = [rng.randrange(1, 1 << 40) for _ in range(60000)]  # sizes sum within a Long
    adds = [{"path": "part-%06d.parquet" % i, "partitionValues": {}, "size": rng.choice(pool),
             "modificationTime": rng.choice(pool), "stats": "%x" % rng.getrandbits(120)} for i in range(120000)]
    rms = [{"path": "gone-%06d.parquet" % i, "deletionTimestamp": rng.choice(pool)} for i in range(60000)]
    S.write_checkpoint_records(os.path.join(lp, "%020d.checkpoint.parquet" % 0), PROTOCOL["protocol"],
                               METADATA["metaData"], adds, rms, use_dictionary=True)
    with open(os.path.join(lp, "_last_checkpoint"), "w") as f:
        f.write('{"version":0,"size":180002}\n')
    monkeypatch.setenv("DR_SNAP_DEBUG", "1")
    counts, live, tomb = _same_as_oracle(engine, lp, cutoff=1 << 39)
    assert counts["num_files"] == 120000
    err = capfd.readouterr().err
    assert "snappy bad page" not in err, err[-2000:]


def test_snappy_periodic_dictionary_pages(engine, tmp_path, capfd, monkeypatch):
    """Dictionary pages of consecutive int64 values compress to a period-4 element stream on which a
    mis-aligned speculative walk never meets the true chain; the entry resolver must carry on
    through every flagged chunk that starts no region of its own (these two pages -- the layouts of
    config 3's modificationTime dictionaries -- reproduced the r02 serial fallbacks; CPU restatement
    of the resolver in the commit that fixed it). Replay and export equal the oracle, no page
    falls back to the serial decoder."""
    from delta_amd.testing import synth as S
    lp = str(tmp_path / "_delta_log")
    os.makedirs(lp)
    t0 = 1_700_000_000_000
    adds = [{"path": "p%05d" % i, "partitionValues": {}, "size": t0 + 44 * 60000 + i,
             "modificationTime": t0 + 3 * 60000 + i} for i in range(60000)]
    rms = [{"path": "r%05d" % i, "deletionTimestamp": t0 + 3 * 60000 + i} for i in range(60000)]
    S.write_checkpoint_records(os.path.join(lp, "%020d.checkpoint.parquet" % 0), PROTOCOL["protocol"],
                               METADATA["metaData"], adds, rms, use_dictionary=True)
    with open(os.path.join(lp, "_last_checkpoint"), "w") as f:
        f.write('{"version":0,"size":120002}\n')
    monkeypatch.setenv("DR_SNAP_DEBUG", "1")
    counts, live, tomb = _same_as_oracle(engine, lp, cutoff=t0 + 3 * 60000 + 30000)
    assert counts["num_files"] == 60000 and len(tomb) == 29999
    err = capfd.readouterr().err
    assert "snappy bad page" not in err, err[-2000:]


@pytest.mark.parametrize("body,rows", [(100, 40000), (400, 12000)], ids=["long_literals", "unstaged_blocks"])
def test_snappy_long_literals_and_unstaged_blocks(engine, tmp_path, capfd, monkeypatch, body, rows):
    """k_snap_exec's rarer paths, parity against the oracle with no page sent to the serial decoder:
    paths whose random 100-character bodies are literals longer than the wave-copy threshold (64 B),
    more than the 256 queued per block, so the queue overflows into per-lane copies; and 400-character
    bodies drawn from 64 symbols, which leave only the row's length prefix + "d/" to copy, so a
    64 KiB output block takes more than 64 KiB of compressed input and its literals are read in
    place instead of from the LDS stage."""
    import random
    import string
    from delta_amd.testing import synth as S
    lp = str(tmp_path / "_delta_log")
    os.makedirs(lp)
    rng = random.Random(body)
    sym = string.ascii_letters + string.digits + "-_"
    adds = [{"path": "d/" + "".join(rng.choice(sym) for _ in range(body)), "partitionValues": {},
             "size": i + 1, "modificationTime": 1} for i in range(rows)]
    rms = [{"path": adds[i]["path"], "deletionTimestamp": 5} for i in range(0, rows, 97)]
    S.write_checkpoint_records(os.path.join(lp, "%020d.checkpoint.parquet" % 0), PROTOCOL["protocol"],
                               METADATA["metaData"], adds[: rows // 2], use_dictionary=False)
    with open(os.path.join(lp, "_last_checkpoint"), "w") as f:
        f.write('{"version":0,"size":%d}\n' % (rows // 2 + 2))
    line = lambda a: json.dumps(a, separators=(",", ":"))
    with open(os.path.join(lp, "%020d.json" % 1), "w") as f:
        f.write("\n".join(line({"add": a}) for a in adds[rows // 2:]) + "\n")
        f.write("\n".join(line({"remove": r}) for r in rms) + "\n")
    monkeypatch.setenv("DR_SNAP_DEBUG", "1")
    counts, live, tomb = _same_as_oracle(engine, lp, cutoff=0)
    assert counts["num_files"] == rows - len(rms)
    err = capfd.readouterr().err
    assert "snappy bad page" not in err, err[-2000:]
    assert "exec phases" in err  # the pages went through k_snap_exec


# ---- staging / scratch guards --------------------------------------------------------------------------
def test_check_lines_over_edge_corpus(engine, tmp_path, monkeypatch):
    """DR_CHECK_LINES=1 compares the staged newline count (which sizes the action arrays) with K1's
    device count, over commits without a trailing newline, with CRLF endings, empty and blank-line
    files, concatenated in one staging; the replay equals the oracle's."""
    monkeypatch.setenv("DR_CHECK_LINES", "1")
    lp = str(tmp_path / "_delta_log")
    os.makedirs(lp)
    line = lambda a: json.dumps(a, separators=(",", ":"))
    bodies = {
        0: "\r\n".join(line(a) for a in [PROTOCOL, METADATA, add("a"), add("b")]),  # CRLF, no final newline
        1: "",                                                                       # empty commit file
        2: "\n\n" + line(add("c")) + "\n\n" + line(remove("a", ts=5)) + "\n",        # blank lines
        3: line(add("d", size=7)),                                                   # one line, no newline
        4: "\r\n" + line(remove("b", ts=9)) + "\r\n",
    }
    for v, body in bodies.items():
        with open(os.path.join(lp, "%020d.json" % v), "w", newline="") as f:
            f.write(body)
    counts, live, tomb = _same_as_oracle(engine, lp, cutoff=0)
    assert sorted(f["path"] for f in live) == ["c", "d"] and sorted(t["path"] for t in tomb) == ["a", "b"]


def test_scan_scratch_capacity_is_checked(engine, tmp_path, monkeypatch):
    """A scan whose scratch is too small fails loudly (DR_E_INTERNAL) instead of writing past it --
    the failure mode of the 100M-row SNAPPY chunk scan fixed in round 2. DR_SCAN_SCRATCH_MAX forces a
    tiny scratch; without it the same replay succeeds."""
    from delta_amd.delta_log import DeltaError
    from delta_amd.testing import synth as S
    exp = S.build_config(2, str(tmp_path), scale=0.002)
    lp = os.path.join(str(tmp_path), "_delta_log")
    monkeypatch.setenv("DR_SCAN_SCRATCH_MAX", "8")  # below any scan's 16-byte minimum
    with pytest.raises(DeltaError) as ei:
        _gpu_replay(engine, lp, exp.min_file_retention_timestamp)
    assert ei.value.status == 15 and "scratch" in str(ei.value)
    monkeypatch.delenv("DR_SCAN_SCRATCH_MAX")
    st = _gpu_replay(engine, lp, exp.min_file_retention_timestamp)
    try:
        assert st.counts["num_files"] == exp.num_files
    finally:
        st.release()


def test_truncated_log_on_update_renders_table_retention(tmp_path):
    """On update() the reference renders the current snapshot's configured retention policies into
    logFileNotFoundException (D/SnapshotManagement.scala:161-163, D/DeltaErrors.scala:451-461)."""
    from delta_amd.delta_log import DeltaError, DeltaLog
    table = str(tmp_path / "t")
    lp = os.path.join(table, "_delta_log")
    md = json.loads(json.dumps(METADATA))
    md["metaData"]["configuration"] = {"delta.logRetentionDuration": "interval 1 week",
                                       "delta.checkpointRetentionDuration": "interval 36 hours"}
    write_commit(lp, 0, [PROTOCOL, md, add("a")])
    write_commit(lp, 1, [add("b")])
    log = DeltaLog(table)
    assert log.snapshot.num_of_files == 2
    os.remove(os.path.join(lp, "%020d.json" % 0))
    write_commit(lp, 2, [add("c")])
    with pytest.raises(DeltaError) as ei:
        log.update()
    assert ei.value.kind == "FileNotFoundException"
    assert str(ei.value).endswith("(delta.logRetentionDuration=7 days) and checkpoint retention policy "
                                  "(delta.checkpointRetentionDuration=36 hours)")
