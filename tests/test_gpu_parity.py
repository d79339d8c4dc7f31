"""GPU parity: libdeltareplay (HIP, gfx950) vs the CPU oracle on the same inputs.

Bit-exact set equality of allFiles and tombstones (full records, dataChange=false) and equality
of every computedState counter, on the reference's golden logs and on seeded synthetic logs.
"""
import os

import pytest

from oracle import delta_oracle as O
from tests.conftest import GOLDEN

pytestmark = pytest.mark.gpu

REF = os.path.join(GOLDEN, "ref")


@pytest.fixture(scope="module")
def engine():
    from delta_amd.delta_log import Engine
    return Engine.get(0)


def _canon(rec):
    return repr(sorted((k, repr(v)) for k, v in rec.items()))


def _gpu_replay(engine, log_path, cutoff, version=-1, validate=True):
    staged = engine.stage_log(log_path, version)
    try:
        return staged.replay(cutoff, validate=validate)
    finally:
        staged.release()


def _assert_same(state, snap):
    c = state.counts
    assert c["num_files"] == snap.num_of_files
    assert c["size_in_bytes"] == snap.size_in_bytes
    assert c["num_removes"] == snap.num_of_removes
    assert c["num_metadata"] == snap.num_of_metadata
    assert c["num_protocol"] == snap.num_of_protocol
    assert c["num_set_transactions"] == snap.num_of_set_transactions
    live = state.export(0)
    tomb = state.export(1)
    assert sorted(map(_canon, live)) == sorted(map(_canon, snap.all_files))
    assert sorted(map(_canon, tomb)) == sorted(map(_canon, snap.tombstones))
    # the device's full-record checksums (the full-size parity gate of bench.py) agree with the oracle's
    assert state.record_sums() == O.record_sums(snap.all_files, snap.tombstones)
    prot = [a["protocol"] for a in state.nonfile if "protocol" in a]
    meta = [a["metaData"] for a in state.nonfile if "metaData" in a]
    assert prot == ([snap.protocol] if snap.protocol else [])
    if snap.metadata:
        assert meta[0]["id"] == snap.metadata["id"]
        assert meta[0]["partitionColumns"] == snap.metadata.get("partitionColumns", [])
        assert meta[0]["schemaString"] == snap.metadata["schemaString"]
    assert sorted(t["appId"] for t in (a["txn"] for a in state.nonfile if "txn" in a)) == \
        sorted(t["appId"] for t in snap.set_transactions)


@pytest.mark.parametrize("name", ["delta-0.1.0", "delta-0.2.0", "dbr_8_0_non_generated_columns",
                                  "dbr_8_1_generated_columns"])
@pytest.mark.parametrize("cutoff", [0, 1564524298213])
def test_golden_logs(engine, name, cutoff):
    lp = os.path.join(REF, name, "_delta_log")
    snap = O.state_reconstruction(O.get_log_segment(lp), cutoff)
    st = _gpu_replay(engine, lp, cutoff)
    try:
        _assert_same(st, snap)
    finally:
        st.release()


@pytest.mark.parametrize("name", ["delta-0.1.0", "delta-0.2.0"])
def test_golden_json_only_replay(engine, name):
    """Replay the JSON commits v0..v3 (skipping the checkpoint) and compare with the oracle."""
    lp = os.path.join(REF, name, "_delta_log")
    files = []
    for v in range(4):
        with open(os.path.join(lp, O.delta_file(v)), "rb") as f:
            files.append((v, 0, 0, f.read()))
    staged = engine.stage_files(files)
    st = staged.replay(0)
    staged.release()
    seg = O.LogSegment(lp, 3, [O.delta_file(v) for v in range(4)], [], None)
    try:
        _assert_same(st, O.state_reconstruction(seg, 0))
    finally:
        st.release()


@pytest.mark.parametrize("cutoff", [0, 1_600_000_100_005])
def test_record_sums_corpus(engine, tmp_path, cutoff):
    """dr_state_record_sums over a log that exercises every field of the record hash
    (tests/record_corpus.py): tags, null / empty maps, repeated members and keys, escapes, removes
    with and without deletionTimestamp, checkpoint and JSON survivors."""
    from tests import record_corpus as R
    lp = R.build(str(tmp_path / "t"))
    st = _gpu_replay(engine, lp, cutoff)
    try:
        _assert_same(st, O.state_reconstruction(O.get_log_segment(lp), cutoff))
    finally:
        st.release()


@pytest.mark.parametrize("config,scale", [(1, 1.0), (2, 0.01), (3, 0.005)])
def test_synthetic_configs(engine, tmp_path, config, scale):
    from delta_amd.testing import synth as S
    exp = S.build_config(config, str(tmp_path), scale=scale)
    lp = os.path.join(str(tmp_path), "_delta_log")
    st = _gpu_replay(engine, lp, exp.min_file_retention_timestamp)
    try:
        c = st.counts
        assert c["num_files"] == exp.num_files
        assert c["size_in_bytes"] == exp.size_in_bytes
        assert c["num_removes"] == exp.num_removes
        assert c["num_actions"] == exp.num_actions
        assert c["num_file_actions"] == exp.num_file_actions
        snap = O.state_reconstruction(O.get_log_segment(lp), exp.min_file_retention_timestamp)
        _assert_same(st, snap)
        # the device xxh64 (dev_common.h) against the published algorithm (python-xxhash): the
        # order-free key sums over the oracle's records (synthetic paths are their own keys)
        import xxhash
        for key, files in (("live_key_sum", snap.all_files), ("tomb_key_sum", snap.tombstones)):
            want = sum(xxhash.xxh64(f["path"].encode()).intdigest() >> 32 for f in files) % (1 << 64)
            assert c[key] == want, key
    finally:
        st.release()


@pytest.mark.parametrize("overlap", [0, 1])
def test_parse_streams_overlap_or_not(tmp_path, overlap):
    """K1 beside K2 on two streams (context option DR_OPT_OVERLAP = 1, for a segment with a
    checkpoint and a multi-block JSON part) and on one (the default): the same records as the oracle
    either way, on a fresh context set to each."""
    from delta_amd.delta_log import Engine
    from delta_amd.testing import synth as S
    eng = Engine(0)
    assert eng.get_option("overlap") == 0  # the default
    eng.set_option("overlap", overlap)
    exp = S.build_config(3, str(tmp_path), scale=0.02)
    lp = os.path.join(str(tmp_path), "_delta_log")
    st = _gpu_replay(eng, lp, exp.min_file_retention_timestamp)
    try:
        assert st.counts["num_files"] == exp.num_files and st.counts["num_removes"] == exp.num_removes
        _assert_same(st, O.state_reconstruction(O.get_log_segment(lp), exp.min_file_retention_timestamp))
    finally:
        st.release()


def test_newline_dense_blocks(engine, tmp_path):
    """The newline index keeps up to 512 positions per 16 KiB block and re-scans denser blocks:
    commits padded with runs of blank lines and `{}` rows (null actions, dropped by unwrap,
    D/actions/actions.scala:523-541) around real actions replay like the oracle."""
    from delta_amd.testing import synth as S
    exp = S.build_config(1, str(tmp_path), scale=0.2)
    lp = os.path.join(str(tmp_path), "_delta_log")
    for v in (1, 2, 5):
        fn = os.path.join(lp, S.delta_name(v))
        with open(fn) as f:
            lines = f.read().splitlines()
        out = []
        for i, ln in enumerate(lines):
            out.append(ln)
            out.extend(["", "{}", " ", "{}"] * (3000 if i == 1 else 5))
        with open(fn, "w") as f:
            f.write("\n".join(out) + "\n")
    st = _gpu_replay(engine, lp, exp.min_file_retention_timestamp)
    try:
        assert st.counts["num_files"] == exp.num_files
        _assert_same(st, O.state_reconstruction(O.get_log_segment(lp), exp.min_file_retention_timestamp))
    finally:
        st.release()


@pytest.mark.parametrize("reducer", ["reduce64", "exact"])
def test_fallback_reducers_agree(engine, tmp_path, reducer):
    """The collision fallbacks (k_bucket_reduce64 / k_bucket_exact, forced for every bucket) and the
    LDS rkey-table reducer give identical states; 160k actions span 64+ buckets."""
    from delta_amd.testing import synth as S
    exp = S.build_config(3, str(tmp_path), scale=0.01)
    lp = os.path.join(str(tmp_path), "_delta_log")
    staged = engine.stage_log(lp)
    try:
        a = staged.replay(exp.min_file_retention_timestamp)
        b = staged.replay(exp.min_file_retention_timestamp, reducer=reducer)
    finally:
        staged.release()
    try:
        for k in ("num_files", "size_in_bytes", "num_removes", "live_key_sum", "tomb_key_sum", "num_file_actions"):
            assert a.counts[k] == b.counts[k], k
        assert a.counts["num_files"] == exp.num_files and a.counts["num_removes"] == exp.num_removes
        assert sorted(r["path"] for r in a.export(0)) == sorted(r["path"] for r in b.export(0))
        assert sorted(r["path"] for r in a.export(1)) == sorted(r["path"] for r in b.export(1))
    finally:
        a.release()
        b.release()


@pytest.mark.parametrize("bits,split", [(3, 0), (5, 0), (3, 1), (5, 1), (1, 1)])
def test_reducer_subpasses_agree(engine, tmp_path, bits, split):
    """Buckets of more than 2048 records on average (config 4's 12K; forced here with 8 or 32
    buckets of ~20K / ~5K records): K3's refinement (k_bucket_split into 2^s sub-buckets by the next
    key bits, then one K4 pass per sub-bucket) and, with DR_OPT_SPLIT = 0, K4's own sub-pass path
    over the whole bucket give the one-pass reducer's state (DR_OPT_BUCKET_BITS forces the buckets;
    (1, 1) takes the refinement to its 6-bit cap, as 2^13 buckets do past ~2^29 actions)."""
    from delta_amd.testing import synth as S
    exp = S.build_config(3, str(tmp_path), scale=0.01)
    lp = os.path.join(str(tmp_path), "_delta_log")
    staged = engine.stage_log(lp)
    try:
        a = staged.replay(exp.min_file_retention_timestamp)
        with engine.options(bucket_bits=bits, split=split):
            b = staged.replay(exp.min_file_retention_timestamp)
    finally:
        staged.release()
    try:
        _same_state(a, b, (bits, split))
        assert b.counts["num_files"] == exp.num_files and b.counts["num_removes"] == exp.num_removes
    finally:
        a.release()
        b.release()


@pytest.mark.parametrize("page_size,compression,page_version,rg,dictionary", [
    (4096, "snappy", "1.0", 1 << 20, True),
    (64 << 10, "snappy", "1.0", 7000, True),
    (8 << 20, "snappy", "1.0", 1 << 20, True),
    (1 << 20, "none", "1.0", 1 << 20, True),
    (64 << 10, "snappy", "2.0", 1 << 20, True),
    (64 << 10, "none", "2.0", 1 << 20, True),
    (4096, "snappy", "1.0", 1 << 20, False),
    (1 << 20, "snappy", "1.0", 5000, False),
    (64 << 10, "snappy", "2.0", 1 << 20, False),
])
def test_checkpoint_page_layouts(engine, tmp_path, capfd, monkeypatch, page_size, compression, page_version, rg,
                                 dictionary):
    """K2 over page sizes (many tiny pages .. one 8 MiB page), several row groups, uncompressed
    pages and DATA_PAGE_V2: the replay must not depend on how the writer cut the column chunks, and
    no SNAPPY page falls back to the serial decoder (the fallback is exact too, so parity alone would
    not notice k_snap_exec refusing a page)."""
    from delta_amd.testing import synth as S
    monkeypatch.setenv("DR_SNAP_DEBUG", "1")
    exp = S.build_table(str(tmp_path), S.config_spec(3, 0.003), seed=77, data_page_size=page_size,
                        compression=compression, data_page_version=page_version, row_group_size=rg,
                        use_dictionary=dictionary)
    lp = os.path.join(str(tmp_path), "_delta_log")
    st = _gpu_replay(engine, lp, exp.min_file_retention_timestamp)
    try:
        c = st.counts
        assert (c["num_files"], c["num_removes"], c["size_in_bytes"]) == \
            (exp.num_files, exp.num_removes, exp.size_in_bytes)
        snap = O.state_reconstruction(O.get_log_segment(lp), exp.min_file_retention_timestamp)
        _assert_same(st, snap)
    finally:
        st.release()
    err = capfd.readouterr().err
    assert "snappy bad page" not in err, err[-2000:]


@pytest.mark.parametrize("fill", [b"\xff" * 256, b"\x01\x00" * 128], ids=["offset_past_start", "offset_zero"])
def test_corrupt_checkpoint_page_is_an_error(engine, tmp_path, fill):
    """A SNAPPY page body overwritten with copy elements reaching before the page start, or with
    copies of offset 0 (corrupt in SNAPPY's format; the host decoder rejects them too), cannot be
    decoded: the replay fails with DR_E_PARQUET (the reference's Parquet reader throws), it does not
    return a partial state."""
    import pyarrow.parquet as pq
    from delta_amd.delta_log import DeltaError
    from delta_amd.testing import synth as S
    S.build_table(str(tmp_path), S.config_spec(3, 0.001), seed=5, use_dictionary=False)
    lp = os.path.join(str(tmp_path), "_delta_log")
    cp = [f for f in os.listdir(lp) if f.endswith(".checkpoint.parquet")][0]
    fn = os.path.join(lp, cp)
    md = pq.ParquetFile(fn).metadata
    col = [md.row_group(0).column(i) for i in range(md.num_columns)
           if md.row_group(0).column(i).path_in_schema == "add.path"][0]
    assert col.compression == "SNAPPY" and col.total_compressed_size > 4096
    raw = bytearray(open(fn, "rb").read())
    at = col.data_page_offset + 512  # past the page header and the snappy length preamble
    raw[at:at + 256] = fill  # copy-4 elements with offset 0xffffffff / copy-1 elements with offset 0
    with open(fn, "wb") as f:
        f.write(bytes(raw))
    with pytest.raises(DeltaError) as ei:
        _gpu_replay(engine, lp, 0)
    assert ei.value.code == "DR_E_PARQUET"


def test_checkpoint_boundaries_found_in_parallel(engine, tmp_path, capfd, monkeypatch):
    """Every PLAIN BYTE_ARRAY page of a synthetic checkpoint is split by the parallel boundary
    kernels (k_ba_count/write: candidates, ranks and the chain check) and validated, so none falls back to the serial walker
    (the fallback is exact too, so parity alone would not notice)."""
    from delta_amd.testing import synth as S
    exp = S.build_config(3, str(tmp_path), scale=0.005)
    monkeypatch.setenv("DR_BA_DEBUG", "1")
    st = _gpu_replay(engine, os.path.join(str(tmp_path), "_delta_log"), exp.min_file_retention_timestamp)
    st.release()
    found = [l for l in capfd.readouterr().err.splitlines() if l.startswith("ba bounds:")]
    assert found
    for l in found:
        w = l.split()
        assert int(w[2]) == int(w[4]) > 0, l


def test_checkpoint_false_boundaries_are_refused(engine, tmp_path, capfd, monkeypatch):
    """Paths whose bytes hold fake length prefixes (NUL bytes: "\\x05\\0\\0\\0" + 5 bytes +
    "\\x03\\0\\0\\0" + 3 bytes) give the parallel boundary search kept candidates that are not
    value starts; the chain check (k_ba_count / k_ba_write) must refuse those pages -- they take the
    serial walker -- and the replay equals the oracle's."""
    import pyarrow as pa
    import pyarrow.parquet as pq
    from delta_amd.testing import synth as S
    exp = S.build_table(str(tmp_path), S.config_spec(3, 0.002), seed=9, use_dictionary=False)
    lp = os.path.join(str(tmp_path), "_delta_log")
    cp = os.path.join(lp, [f for f in os.listdir(lp) if f.endswith(".checkpoint.parquet")][0])
    t = pq.read_table(cp)
    add = t.column("add").combine_chunks()
    paths = add.field("path").to_pylist()
    fake = "x\x05\x00\x00\x00yyyyy\x03\x00\x00\x00zzz"
    bad = 0
    for i in range(0, len(paths), 97):
        if paths[i] is not None:
            paths[i] = paths[i][:20] + fake + paths[i][20:]
            bad += 1
    assert bad > 10
    fields = [pa.array(paths, type=add.type.field("path").type) if add.type.field(k).name == "path" else add.field(k)
              for k in range(add.type.num_fields)]
    new = pa.StructArray.from_arrays(fields, fields=list(add.type), mask=add.is_null())
    t = t.set_column(t.schema.get_field_index("add"), t.schema.field("add"), new)
    pq.write_table(t, cp, compression="snappy", use_dictionary=False)
    monkeypatch.setenv("DR_BA_DEBUG", "1")
    st = _gpu_replay(engine, lp, exp.min_file_retention_timestamp)
    try:
        _assert_same(st, O.state_reconstruction(O.get_log_segment(lp), exp.min_file_retention_timestamp))
    finally:
        st.release()
    found = [l.split() for l in capfd.readouterr().err.splitlines() if l.startswith("ba bounds:")]
    assert found and any(int(w[2]) < int(w[4]) for w in found), found


@pytest.mark.parametrize("table", ["dbr_8_0_non_generated_columns", "dbr_8_1_generated_columns"])
def test_checksum_validation(tmp_path, table):
    """ValidateChecksum (D/Checksum.scala:155-191) on the reference's own .crc files, then on
    tampered, extended, unparseable and missing copies."""
    import shutil
    from delta_amd.delta_log import DeltaError, DeltaLog, ManualClock
    root = tmp_path / table
    shutil.copytree(os.path.join(REF, table), root)
    crc = root / "_delta_log" / ("%020d.crc" % 0)
    good = crc.read_bytes().splitlines()[0]
    nf = json_field(good, "numFiles")
    cases = [
        (good, None),
        (b'{"numProtocol":1,"numMetadata":1,"tableSizeBytes":%d,"numTransactions":"0","numFiles":%d,'
         b'"histogramOpt":{"x":1}}' % (json_field(good, "tableSizeBytes"), json_field(good, "numFiles")), None),
        (good.replace(b'"numFiles":%d' % nf, b'"numFiles":%d' % (nf + 7)),
         "Number of files - Expected: %d Computed: %d" % (nf + 7, nf)),
        (b'{"tableSizeBytes":5,"numFiles":%d,"numMetadata":2,"numProtocol":1,"numTransactions":3}' % nf,
         "Table size (bytes) - Expected: 5 Computed: %d\nMetadata updates - Expected: 2 Computed: 1\n"
         "Transactions - Expected: 3 Computed: 0" % json_field(good, "tableSizeBytes")),
        (b"not json", None), (b"", None), (None, None),
    ]
    for content, mismatch in cases:
        if content is None:
            crc.unlink()
        else:
            crc.write_bytes(content + b"\n")
        DeltaLog.clear_cache()
        snap = DeltaLog.for_table(str(root), clock=ManualClock(0)).snapshot
        assert snap.validate_checksum(corruption_is_fatal=False) == mismatch, content
        if mismatch is None:
            snap.validate_checksum()
        else:
            with pytest.raises(DeltaError) as ei:
                snap.validate_checksum()
            assert ei.value.kind == "IllegalStateException"
            assert str(ei.value).endswith("Failed verification at version 0 of:\n" + mismatch)
    DeltaLog.clear_cache()


def json_field(line, name):
    import json
    return json.loads(line)[name]


def _commit_files(lp, lo, hi):
    from delta_amd import _native as N
    out = []
    for v in range(lo, hi + 1):
        with open(os.path.join(lp, "%020d.json" % v), "rb") as f:
            out.append((v, N.DR_FILE_JSON, 0, f.read()))
    return out


COUNT_KEYS = ("num_files", "size_in_bytes", "num_removes", "num_metadata", "num_protocol", "num_set_transactions",
              "num_actions", "num_file_actions", "malformed_lines", "live_key_sum", "tomb_key_sum", "version")


def _same_counts(a, b, tag):
    for k in COUNT_KEYS:
        assert a.counts[k] == b.counts[k], (tag, k, a.counts[k], b.counts[k])


def _same_state(a, b, tag):
    sides = []
    for which in (0, 1):
        ea, eb = a.export(which), b.export(which)
        ra, rb = sorted(map(_canon, ea)), sorted(map(_canon, eb))
        sa, sb = set(ra), set(rb)
        sides.append((ra, rb, sorted(sa - sb)[:8], sorted(sb - sa)[:8], sum(r.get("size") or 0 for r in ea)))
    try:
        _same_counts(a, b, tag)
    except AssertionError as e:  # name the rows that differ (and the live rows' size sum), not only the counter
        raise AssertionError("%s; only in a: %s; only in b: %s; live size sum %d" %
                             (e, [s[2] for s in sides], [s[3] for s in sides], sides[0][4]))
    for ra, rb, oa, ob, _ in sides:
        assert ra == rb, (tag, oa, ob)
    assert a.nonfile == b.nonfile, tag


def test_incremental_apply_matches_full_replay(engine, tmp_path):
    """dr_state_apply: a checkpointed base extended one commit at a time,
    then by a batch, equals the full replay of the segment at every version (records, counters,
    non-file winners) and the oracle; partition pruning runs over the multi-segment state."""
    from delta_amd.predicates import build_program, partition_schema
    from delta_amd.testing import synth as S
    from tests.filter_corpus import C, L
    spec = S.ChurnSpec(ckpt_files=4000, ckpt_version=3, n_deltas=6, removes_per_delta=500,
                       adds_per_delta=500, readd_frac=0.5, ncols=2)
    exp = S.build_table(str(tmp_path), spec, seed=11, row_group_size=1500)
    lp = os.path.join(str(tmp_path), "_delta_log")
    cutoff = exp.min_file_retention_timestamp
    last = spec.ckpt_version + spec.n_deltas
    st = _gpu_replay(engine, lp, cutoff, version=spec.ckpt_version + 1)
    states = [st]
    try:
        for v in range(spec.ckpt_version + 2, last + 1):
            tail = engine.stage_files(_commit_files(lp, v, v))
            nxt = states[-1].apply(tail, cutoff)
            tail.release()
            states.append(nxt)
            full = _gpu_replay(engine, lp, cutoff, version=v)
            try:
                _same_counts(nxt, full, v)
                assert sorted(map(_canon, nxt.export(0))) == sorted(map(_canon, full.export(0)))
                assert sorted(map(_canon, nxt.export(1))) == sorted(map(_canon, full.export(1)))
                assert nxt.nonfile == full.nonfile
            finally:
                full.release()
        snap = O.state_reconstruction(O.get_log_segment(lp), cutoff)
        _assert_same(states[-1], snap)
        # a batch tail, and pruning over the resulting four-segment state
        batch = engine.stage_files(_commit_files(lp, spec.ckpt_version + 2, last))
        b = states[0].apply(batch, cutoff)
        batch.release()
        states.append(b)
        _assert_same(b, snap)
        meta = next(a["metaData"] for a in b.nonfile if "metaData" in a)
        pred = [("in", C("p1"), [L("integer", v) for v in range(0, 400)])]
        for s in (b, states[-2]):
            live = s.export(0)
            got = sorted(live[i]["path"] for i in s.filter(build_program(partition_schema(meta), pred)))
            want = sorted(f["path"] for f in O.filter_file_list(O.partition_schema(snap.metadata), snap.all_files, pred))
            assert got == want and got
    finally:
        for s in states:
            s.release()


def test_incremental_index_chain(engine, tmp_path, monkeypatch):
    """The O(tail) path of dr_state_apply (k_index.hip): a chain of one-commit applies whose
    retention cutoff sweeps the deletion window (tombstones expire while the chain grows), checked
    against full replays; a forced key collision rolls the index back and takes the full reduction,
    after which the same head applies incrementally; older states of the chain materialise their
    survivors through the undo logs; a branch off an older state takes the full path and starts a
    new chain; the oracle agrees at the end."""
    from delta_amd.testing import synth as S
    spec = S.ChurnSpec(ckpt_files=3000, ckpt_version=2, n_deltas=24, removes_per_delta=40, adds_per_delta=30,
                       readd_frac=0.5, ncols=2)
    exp = S.build_table(str(tmp_path), spec, seed=5, row_group_size=1000)
    lp = os.path.join(str(tmp_path), "_delta_log")
    day = 86400000
    c0 = exp.min_file_retention_timestamp - 7 * day  # the deletion window's start: every tombstone kept
    step = 14 * day // spec.n_deltas
    b0 = spec.ckpt_version
    cut = lambda k: c0 + k * step
    states = [_gpu_replay(engine, lp, cut(0), version=b0)]
    extra = []
    try:
        for k in range(1, spec.n_deltas + 1):
            v = b0 + k
            tail = engine.stage_files(_commit_files(lp, v, v))
            if k == 8:
                monkeypatch.setenv("DR_IX_TEST_COLLIDE", "1")
                fb = states[-1].apply(tail, cut(k))
                monkeypatch.delenv("DR_IX_TEST_COLLIDE")
                extra.append(fb)
            nxt = states[-1].apply(tail, cut(k))
            tail.release()
            states.append(nxt)
            if k == 8:
                _same_state(nxt, fb, "rollback")
            if k % 5 == 0 or k in (1, 8, 9):
                full = _gpu_replay(engine, lp, cut(k), version=v)
                try:
                    _same_state(nxt, full, v)
                finally:
                    full.release()
        assert states[-1].counts["num_removes"] < states[12].counts["num_removes"]  # tombstones expired
        for k in (2, 11, 17):  # older states, materialised after later applies
            full = _gpu_replay(engine, lp, cut(k), version=b0 + k)
            try:
                _same_state(states[k], full, ("old", k))
            finally:
                full.release()
        tail = engine.stage_files(_commit_files(lp, b0 + 6, b0 + 9))
        br = states[5].apply(tail, cut(9))
        tail.release()
        extra.append(br)
        tail = engine.stage_files(_commit_files(lp, b0 + 10, b0 + 10))
        br2 = br.apply(tail, cut(10))
        tail.release()
        extra.append(br2)
        for s, k in ((br, 9), (br2, 10)):
            full = _gpu_replay(engine, lp, cut(k), version=b0 + k)
            try:
                _same_state(s, full, ("branch", k))
            finally:
                full.release()
        _assert_same(states[-1], O.state_reconstruction(O.get_log_segment(lp), cut(spec.n_deltas)))
    finally:
        for s in states + extra:
            s.release()


def test_incremental_apply_errors_and_delta_log_update(engine, tmp_path):
    import shutil
    from delta_amd.delta_log import DeltaError, DeltaLog, ManualClock
    root = tmp_path / "t"
    shutil.copytree(os.path.join(REF, "delta-0.2.0"), root)
    lp = str(root / "_delta_log")
    base = _gpu_replay(engine, lp, 0, version=1)
    try:
        gap = engine.stage_files(_commit_files(lp, 3, 3))
        with pytest.raises(DeltaError) as ei:
            base.apply(gap, 0)
        gap.release()
        assert ei.value.kind == "IllegalStateException" and "are not contiguous" in str(ei.value)
    finally:
        base.release()
    # DeltaLog.update(incremental=True) over a log that grows, against a rebuild
    for v in (2, 3):
        os.rename(os.path.join(lp, "%020d.json" % v), os.path.join(lp, "%020d.json.hold" % v))
    os.remove(os.path.join(lp, "_last_checkpoint"))
    os.remove(os.path.join(lp, "%020d.checkpoint.parquet" % 3))
    DeltaLog.clear_cache()
    log = DeltaLog.for_table(str(root), clock=ManualClock(1564524298213))
    assert log.snapshot.version == 1
    for v in (2, 3):
        os.rename(os.path.join(lp, "%020d.json.hold" % v), os.path.join(lp, "%020d.json" % v))
        snap = log.update(incremental=True)
        assert snap.version == v
        ref = O.state_reconstruction(O.get_log_segment(lp), log.min_file_retention_timestamp)
        _assert_same(snap.state, ref)
    assert log.update(incremental=True) is snap
    DeltaLog.clear_cache()


@pytest.mark.parametrize("parts", [1, 3])
def test_checkpoint_writer_round_trip(engine, tmp_path, parts):
    """writeCheckpoint (D/Checkpoints.scala:229-365) from the GPU state: the written checkpoint
    (single or multi-part, with _last_checkpoint) replays -- on the GPU and in the oracle, which
    reads it with pyarrow -- to the same state, and holds the reference's column layout."""
    import json
    import pyarrow.parquet as pq
    from delta_amd.checkpoint import write_checkpoint
    from delta_amd.delta_log import DeltaLog, ManualClock
    from delta_amd.testing import synth as S
    spec = S.ChurnSpec(ckpt_files=3000, ckpt_version=4, n_deltas=3, removes_per_delta=400,
                       adds_per_delta=400, readd_frac=0.5, ncols=2)
    exp = S.build_table(str(tmp_path), spec, seed=13, row_group_size=1000)
    lp = os.path.join(str(tmp_path), "_delta_log")
    DeltaLog.clear_cache()
    log = DeltaLog.for_table(str(tmp_path), clock=ManualClock(exp.min_file_retention_timestamp + 604800000))
    snap = log.snapshot
    cutoff = snap.min_file_retention_timestamp
    before = O.state_reconstruction(O.get_log_segment(lp), cutoff)
    meta = write_checkpoint(snap, parts=parts, row_group_size=1500)
    with open(os.path.join(lp, "_last_checkpoint")) as f:
        assert json.load(f) == meta
    assert meta["version"] == snap.version and meta["size"] == (2 + snap.num_of_files + snap.num_of_removes
                                                                + snap.num_of_set_transactions)
    names = sorted(n for n in os.listdir(lp) if n.startswith("%020d.checkpoint" % snap.version))
    assert len(names) == parts
    schema = pq.read_schema(os.path.join(lp, names[0]))
    assert schema.names == ["txn", "add", "remove", "metaData", "protocol"]
    # CheckpointV2 (checkpointV2.enabled default true, the table is partitioned): the partition
    # values cast to the partition schema follow stats (D/Checkpoints.scala:340-365,372-389)
    add_t = schema.field("add").type
    assert [f.name for f in add_t] == ["path", "partitionValues", "size", "modificationTime", "dataChange", "tags",
                                       "stats", "partitionValues_parsed"]
    parsed_t = add_t.field("partitionValues_parsed").type
    assert [(f.name, str(f.type)) for f in parsed_t] == [("p0", "date32[day]"), ("p1", "int32")]
    rows = pq.read_table(os.path.join(lp, names[0])).column("add").to_pylist()
    for r in rows:
        if r is not None:
            pv = dict(r["partitionValues"])
            assert r["partitionValues_parsed"]["p0"].isoformat() == pv["p0"]
            assert r["partitionValues_parsed"]["p1"] == int(pv["p1"])
    seg = O.get_log_segment(lp)
    assert seg.checkpoint_version == snap.version and not seg.deltas
    after = O.state_reconstruction(seg, cutoff)
    st = _gpu_replay(engine, lp, cutoff)
    try:
        _assert_same(st, before)
        _assert_same(st, after)
    finally:
        st.release()
    DeltaLog.clear_cache()


def test_checkpoint_writer_table_options(engine, tmp_path):
    """delta.checkpoint.writeStatsAsJson=false drops add.stats; writeStatsAsStruct=false drops
    partitionValues_parsed (D/Checkpoints.scala:340-352, D/DeltaConfig.scala:401-418)."""
    import json
    import pyarrow.parquet as pq
    from delta_amd.checkpoint import write_checkpoint
    from delta_amd.delta_log import DeltaLog, ManualClock
    from delta_amd.testing import synth as S
    spec = S.ChurnSpec(ckpt_files=500, ckpt_version=2, n_deltas=1, removes_per_delta=50, adds_per_delta=50,
                       readd_frac=0.0, ncols=2)
    S.build_table(str(tmp_path), spec, seed=21)
    lp = os.path.join(str(tmp_path), "_delta_log")
    md = S.metadata_dict(2, {"delta.checkpoint.writeStatsAsJson": "false",
                             "delta.checkpoint.writeStatsAsStruct": "false"})
    with open(os.path.join(lp, "%020d.json" % 4), "w") as f:
        f.write(json.dumps({"metaData": md}) + "\n")
    DeltaLog.clear_cache()
    snap = DeltaLog.for_table(str(tmp_path), clock=ManualClock(0)).snapshot
    write_checkpoint(snap)
    schema = pq.read_schema(os.path.join(lp, "%020d.checkpoint.parquet" % 4))
    assert [f.name for f in schema.field("add").type] == ["path", "partitionValues", "size", "modificationTime",
                                                         "dataChange", "tags"]
    st = _gpu_replay(engine, lp, snap.min_file_retention_timestamp)
    try:
        assert st.counts["num_files"] == snap.num_of_files
        assert st.counts["live_key_sum"] == snap.state.counts["live_key_sum"]
    finally:
        st.release()
    DeltaLog.clear_cache()


@pytest.mark.parametrize("compact", [False, True])
def test_incremental_apply_random_commits(engine, tmp_path, compact):
    """Property test of the O(tail) apply: 40 random commits -- new adds, re-adds, removes of live,
    removed and never-seen paths, the same path twice in one commit in either order, absolute /
    `file:` / escaped paths naming the same file, metaData and txn actions, malformed lines --
    applied one at a time (and some two at a time) with a cutoff that moves forward, checked
    against full replays and, at the end, the oracle. compact: the writer's separators (no
    whitespace), so a commit's lines take the token tape of k_apply_commit; spaced lines are off the
    tape and take its General walker."""
    import json
    import random
    from delta_amd import _native as N
    rng = random.Random(0xC0FFEE)
    lp = tmp_path / "_delta_log"
    lp.mkdir()
    head = ['{"protocol":{"minReaderVersion":1,"minWriterVersion":2}}',
            '{"metaData":{"id":"t","format":{"provider":"parquet","options":{}},"schemaString":"{}",'
            '"partitionColumns":[],"configuration":{}}}']
    pool = ["f%d.parquet" % i for i in range(400)]
    special = {"f7.parquet": ["/abs/f7.parquet", "file:/abs/f7.parquet", "file:///abs/f7.parquet"],
               "f9.parquet": ["dir/f\\u00e99.parquet", "dir/fé9.parquet"]}
    live = set()

    sep = (",", ":") if compact else (", ", ": ")

    def add(p, v, k):
        return json.dumps({"add": {"path": p, "size": 10 + k, "modificationTime": v, "dataChange": True}},
                          ensure_ascii=False, separators=sep).replace("\\\\u", "\\u")

    def rm(p, ts):
        return json.dumps({"remove": {"path": p, "deletionTimestamp": ts, "dataChange": True}},
                          ensure_ascii=False, separators=sep).replace("\\\\u", "\\u")

    def name(p):
        return rng.choice(special[p]) if p in special else p

    versions = []
    lines0 = head + [add(name(p), 0, i) for i, p in enumerate(pool[:150])]
    live.update(pool[:150])
    versions.append(lines0)
    for v in range(1, 41):
        lines = []
        for _ in range(rng.randint(1, 12)):
            r = rng.random()
            p = rng.choice(pool)
            if r < 0.35:
                lines.append(add(name(p), v, v))
                live.add(p)
            elif r < 0.7:
                lines.append(rm(name(p), 1000 * v + rng.randint(0, 999)))
                live.discard(p)
            elif r < 0.8:  # the same path twice in one commit
                a, b = add(name(p), v, 1), rm(name(p), 1000 * v)
                lines.extend([a, b] if rng.random() < 0.5 else [b, a])
            elif r < 0.87:
                lines.append('{"txn":{"appId":"app%d","version":%d,"lastUpdated":%d}}' % (rng.randint(0, 3), v, v))
            elif r < 0.92:
                lines.append('{"metaData":{"id":"t","format":{"provider":"parquet","options":{}},'
                             '"schemaString":"{}","partitionColumns":[],"configuration":{"v":"%d"}}}' % v)
            else:
                lines.append('{"add":{"path":"broken%d.parquet","size":1' % v)  # malformed: a null row
        versions.append(lines)
    for v, lines in enumerate(versions):
        (lp / ("%020d.json" % v)).write_text("\n".join(lines) + "\n")

    def commit(v):
        return (v, N.DR_FILE_JSON, 0, (lp / ("%020d.json" % v)).read_bytes())

    cut = lambda v: 1000 * v - 5000
    st = _gpu_replay(engine, str(lp), cut(0), version=0)
    states = [st]
    try:
        v = 0
        while v < 40:
            k = 2 if rng.random() < 0.2 and v + 2 <= 40 else 1
            tail = engine.stage_files([commit(x) for x in range(v + 1, v + k + 1)])
            nxt = states[-1].apply(tail, cut(v + k))
            tail.release()
            v += k
            states.append(nxt)
            live = nxt.export(0)  # every apply: the counters move with the rows
            got, want = (nxt.counts["num_files"], nxt.counts["size_in_bytes"]), (len(live), sum(r["size"] or 0 for r in live))
            if got != want:
                print("apply to v%d (%d commits): counters %s, rows %s\nbase %s\nnext %s\nbase rows %s" %
                      (v, k, got, want, states[-2].counts, nxt.counts,
                       sorted((r["path"], r["size"]) for r in states[-2].export(0))))
            assert got == want, (v, k)
            if v % 5 == 0 or v > 36:
                full = _gpu_replay(engine, str(lp), cut(v), version=v)
                try:
                    _same_state(nxt, full, v)
                finally:
                    full.release()
        _assert_same(states[-1], O.state_reconstruction(O.get_log_segment(str(lp)), cut(40)))
    finally:
        for s in states:
            s.release()
