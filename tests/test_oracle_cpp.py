"""The C++ restatement (oracle/replay_oracle.cpp: the CPU baseline and the full-size checker of the
GPU's key sums) against the Python oracle, which is pinned to the reference's golden logs: counts
and the order-free key sums on the golden logs, synthetic configs and canonicalization cases, at
several thread and partition counts (placement must not change the result)."""
import json
import os
import subprocess

import pytest
import xxhash

from oracle import delta_oracle as O
from tests.conftest import GOLDEN, ROOT

EXE = os.path.join(ROOT, "oracle", "_build", "replay_oracle")


@pytest.fixture(scope="module")
def exe():
    if not os.path.exists(EXE):
        subprocess.check_call(["make", "-C", os.path.join(ROOT, "oracle")])
    return EXE


def run(exe, lp, cutoff, threads=3, parts=7):
    r = subprocess.run([exe, lp, str(cutoff), "--threads", str(threads), "--partitions", str(parts), "--record-sums"],
                       capture_output=True, text=True, check=True)
    return json.loads(r.stdout.strip().splitlines()[-1])


def key_sum(records):
    return sum(xxhash.xxh64(O.replay_key(r["path"]).encode()).intdigest() >> 32 for r in records) % (1 << 64)


def check(res, snap):
    assert res["num_files"] == snap.num_of_files
    assert res["size_in_bytes"] == snap.size_in_bytes
    assert res["num_removes"] == snap.num_of_removes
    assert res["live_key_sum"] == key_sum(snap.all_files)
    assert res["tomb_key_sum"] == key_sum(snap.tombstones)
    # full records, not only paths: every field of every winner (BASELINE.md correctness gate)
    assert (res["live_record_sum"], res["tomb_record_sum"]) == O.record_sums(snap.all_files, snap.tombstones)


@pytest.mark.parametrize("name", ["delta-0.1.0", "delta-0.2.0", "dbr_8_0_non_generated_columns"])
@pytest.mark.parametrize("cutoff", [0, 1564524298213])
def test_golden(exe, name, cutoff):
    lp = os.path.join(GOLDEN, "ref", name, "_delta_log")
    check(run(exe, lp, cutoff), O.state_reconstruction(O.get_log_segment(lp), cutoff))


@pytest.mark.parametrize("config,scale", [(1, 0.2), (2, 0.002), (3, 0.0005)])
@pytest.mark.parametrize("threads,parts", [(1, 1), (4, 50)])
def test_synthetic(exe, tmp_path, config, scale, threads, parts):
    from delta_amd.testing import synth as S
    exp = S.build_config(config, str(tmp_path), scale=scale)
    lp = os.path.join(str(tmp_path), "_delta_log")
    res = run(exe, lp, exp.min_file_retention_timestamp, threads, parts)
    assert (res["num_actions"], res["num_file_actions"]) == (exp.num_actions, exp.num_file_actions)
    check(res, O.state_reconstruction(O.get_log_segment(lp), exp.min_file_retention_timestamp))


def test_canonical_keys_and_escapes(exe, tmp_path):
    lp = str(tmp_path / "_delta_log")
    os.makedirs(lp)
    lines0 = ['{"protocol":{"minReaderVersion":1,"minWriterVersion":2}}',
              '{"metaData":{"id":"x","format":{"provider":"parquet","options":{}},"schemaString":"{}",'
              '"partitionColumns":[],"configuration":{}}}']
    for p in ["/a//b.parquet", "file:///c.parquet", "rel.parquet", "keep/\\u00e9.parquet", "/d.parquet", "e"]:
        lines0.append(json.dumps({"add": {"path": p, "size": 3, "modificationTime": 1}}).replace("\\\\u", "\\u"))
    lines1 = ['{"remove":{"path":"file:/a/b.parquet","deletionTimestamp":9}}',
              '{"remove":{"path":"\\/c.parquet","deletionTimestamp":8}}',
              '{"add":{"path":"e","size":5}}', '{"add":{"path":"e","size":6}}', 'not json',
              '{"remove":{"path":"file:/d.parquet"}}']
    for v, lines in enumerate([lines0, lines1]):
        with open(os.path.join(lp, "%020d.json" % v), "w") as f:
            f.write("\n".join(lines) + "\n")
    for cutoff in (0, 8):
        check(run(exe, lp, cutoff), O.state_reconstruction(O.get_log_segment(lp), cutoff))


@pytest.mark.parametrize("cutoff", [0, 1_600_000_100_005])
@pytest.mark.parametrize("threads", [1, 3])
def test_record_corpus(exe, tmp_path, cutoff, threads):
    """The full-record checksum over a log that exercises every field (tests/record_corpus.py)."""
    from tests import record_corpus as R
    lp = R.build(str(tmp_path / "t"))
    check(run(exe, lp, cutoff, threads), O.state_reconstruction(O.get_log_segment(lp), cutoff))
