"""Pins the CPU oracle (oracle/delta_oracle.py) to the reference's own golden fixtures.

The delta-0.2.0 checkpoint (`R/history/delta-0.2.0/_delta_log/...3.checkpoint.parquet`) was
written by the reference from its replay of JSON v0..v3, so replaying the JSON with the oracle
must reproduce it row for row (as a set). delta-0.1.0's checkpoint came from an older writer
(its adds keep dataChange=true) and its removes carry no deletionTimestamp (=0, expired).
The dbr_8_* `.crc` files pin the computedState aggregates (D/Checksum.scala:45-192).
"""
import os

import pytest

from oracle import delta_oracle as O
from tests.conftest import GOLDEN

REF = os.path.join(GOLDEN, "ref")


def _json_only_segment(name, version):
    lp = os.path.join(REF, name, "_delta_log")
    return O.LogSegment(lp, version, [O.delta_file(v) for v in range(version + 1)], [], None)


def _ckpt_rows(name, version):
    lp = os.path.join(REF, name, "_delta_log")
    return list(O.read_checkpoint_actions(os.path.join(lp, O.checkpoint_file_singular(version))))


def _file_set(rows, kind, drop=("dataChange",)):
    out = set()
    for r in rows:
        if r is None or r[0] != kind:
            continue
        d = {k: v for k, v in r[1].items() if k not in drop}
        out.add(repr(sorted((k, repr(v)) for k, v in d.items())))
    return out


def test_delta_020_json_replay_equals_reference_checkpoint():
    seg = _json_only_segment("delta-0.2.0", 3)
    r = O.InMemoryLogReplay(min_file_retention_timestamp=0)
    r.append(0, (a for _, a in O.load_actions(seg)))
    state = r.checkpoint()
    ckpt = _ckpt_rows("delta-0.2.0", 3)
    # adds: full records incl. dataChange=false (bit-for-bit current semantics)
    assert _file_set(state, O.ADD, drop=()) == _file_set(ckpt, O.ADD, drop=())
    # The checkpoint's remove struct only has (path, deletionTimestamp, dataChange): compare those.
    def rm(rows):
        return {(a["path"], a["deletionTimestamp"], a["dataChange"]) for k, a in
                (x for x in rows if x is not None) if k == O.REMOVE}
    assert rm(state) == rm(ckpt)
    assert len(rm(ckpt)) == 4 and all(dc is False for _, _, dc in rm(ckpt))
    prot = [a for k, a in state if k == O.PROTOCOL]
    assert prot == [{"minReaderVersion": 1, "minWriterVersion": 2}]
    txns = [a for k, a in state if k == O.TXN]
    assert [t["appId"] for t in txns] == ["e4a20b59-dd0e-4c50-b074-e8ae4786df30"]
    assert len(ckpt) == 10  # _last_checkpoint {"version":3,"size":10}


def test_delta_020_snapshot_from_checkpoint_matches_json_replay():
    lp = os.path.join(REF, "delta-0.2.0", "_delta_log")
    seg = O.get_log_segment(lp)
    assert seg.checkpoint_version == 3 and seg.deltas == []
    snap_ck = O.state_reconstruction(seg, 0)
    snap_js = O.state_reconstruction(_json_only_segment("delta-0.2.0", 3), 0)
    assert sorted(a["path"] for a in snap_ck.all_files) == sorted(a["path"] for a in snap_js.all_files)
    assert snap_ck.counts() == snap_js.counts()
    assert snap_ck.counts()["numOfFiles"] == 3 and snap_ck.counts()["numOfRemoves"] == 4
    # retention: cutoff at the deletion timestamps drops them (strict >)
    snap = O.state_reconstruction(seg, 1564524298214)
    assert snap.num_of_removes == 0
    snap = O.state_reconstruction(seg, 1564524298213)
    assert snap.num_of_removes == 3


def test_delta_010_json_replay_matches_checkpoint_modulo_datachange():
    seg = _json_only_segment("delta-0.1.0", 3)
    r = O.InMemoryLogReplay(min_file_retention_timestamp=0)
    r.append(0, (a for _, a in O.load_actions(seg)))
    state = r.checkpoint()
    ckpt = _ckpt_rows("delta-0.1.0", 3)
    assert _file_set(state, O.ADD) == _file_set(ckpt, O.ADD)
    # removes have no deletionTimestamp -> delTimestamp 0, not > 0 -> expired
    assert _file_set(state, O.REMOVE) == set() == _file_set(ckpt, O.REMOVE)
    assert len(ckpt) == 6  # _last_checkpoint {"version":3,"size":6}
    meta = [a for k, a in state if k == O.METADATA][0]
    assert meta["partitionColumns"] == ["id"]


@pytest.mark.parametrize("name", ["dbr_8_0_non_generated_columns", "dbr_8_1_generated_columns"])
def test_crc_aggregates(name):
    lp = os.path.join(REF, name, "_delta_log")
    snap = O.state_reconstruction(O.get_log_segment(lp), 0)
    crc = O.crc_counts(lp, 0)
    c = snap.counts()
    assert c["sizeInBytes"] == crc["tableSizeBytes"]
    assert c["numOfFiles"] == crc["numFiles"]
    assert c["numOfMetadata"] == crc["numMetadata"]
    assert c["numOfProtocol"] == crc["numProtocol"]
    assert c["numOfSetTransactions"] == crc["numTransactions"]


def test_unknown_action_ignored_and_null_partition_value(tmp_path):
    # T/EvolvabilitySuite.scala:43-96
    lp = tmp_path / "_delta_log"
    lp.mkdir()
    (lp / O.delta_file(0)).write_text(
        '{"protocol":{"minReaderVersion":1,"minWriterVersion":2}}\n'
        '{"metaData":{"id":"x","format":{"provider":"parquet","options":{}},"schemaString":'
        '"{\\"type\\":\\"struct\\",\\"fields\\":[{\\"name\\":\\"part\\",\\"type\\":\\"integer\\",'
        '\\"nullable\\":true,\\"metadata\\":{}}]}","partitionColumns":["part"],"configuration":{}}}\n'
        '{"some_new_feature":{"a":1}}\n'
        '{"add":{"path":"part=__HIVE_DEFAULT_PARTITION__/f1","partitionValues":{"part":null},'
        '"size":1,"modificationTime":1,"dataChange":true}}\n')
    snap = O.state_reconstruction(O.get_log_segment(str(lp)), 0)
    assert snap.num_of_files == 1
    assert snap.all_files[0]["partitionValues"] == {"part": None}
    sch = O.partition_schema(snap.metadata)
    assert O.filter_file_list(sch, snap.all_files, [("isnull", ("col", "part"))]) == snap.all_files
    assert O.filter_file_list(sch, snap.all_files, [("=", ("col", "part"), ("lit", "integer", 1))]) == []


def test_noncontiguous_versions_error(tmp_path):
    # T/DeltaLogSuite.scala:281-304
    lp = tmp_path / "_delta_log"
    lp.mkdir()
    for v in (0, 2):
        (lp / O.delta_file(v)).write_text('{"add":{"path":"foo","partitionValues":{},"size":1,'
                                          '"modificationTime":1,"dataChange":true}}\n')
    with pytest.raises(O.DeltaError) as e:
        O.get_log_segment(str(lp))
    assert str(e.value) == "Versions (Vector(0, 2)) are not contiguous."


def test_canonicalization_cases():
    # T/DeltaLogSuite.scala:190-254
    p = "/some/unqualified/absolute/path"
    assert O.canonicalize_path(p) == "file://" + p
    for scheme in ("file:", "file://"):
        assert O.replay_key(O.canonicalize_path(scheme + p)) == O.replay_key(O.canonicalize_path(p))
    assert O.canonicalize_path("a/b.parquet") == "a/b.parquet"


def test_file_names():
    # T/FileNamesSuite.scala:23-73
    assert O.is_checkpoint_file("00000000000000000010.checkpoint.parquet")
    assert O.is_checkpoint_file("00000000000000000010.checkpoint.0000000001.0000000002.parquet")
    assert not O.is_checkpoint_file("00000000000000000010.json")
    assert O.num_checkpoint_parts("00000000000000000010.checkpoint.0000000001.0000000002.parquet") == 2
    assert O.num_checkpoint_parts("00000000000000000010.checkpoint.parquet") is None
    assert O.checkpoint_file_with_parts(1, 2) == [
        "00000000000000000001.checkpoint.0000000001.0000000002.parquet",
        "00000000000000000001.checkpoint.0000000002.0000000002.parquet"]
    assert O.file_version("00000000000000000123.json") == 123
