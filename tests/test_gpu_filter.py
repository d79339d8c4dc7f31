"""GPU parity of K5 partition pruning (dr_filter) against the oracle's filterFileList restatement:
Spark non-ANSI casts of odd partition strings, three-valued logic, IN with NULL, null-safe
equality, JSON escapes in keys and values, values read from JSON commits and from the
checkpoint's add.partitionValues map column; the OptimisticTransactionSuite-style int-partition
predicates (T/OptimisticTransactionSuite.scala:117-450); the config-4 conjunction."""
import os

import pytest

from oracle import delta_oracle as O
from tests import filter_corpus as F

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def engine():
    from delta_amd.delta_log import Engine
    return Engine.get(0)


def _gpu_selected(engine, lp, preds_list, cutoff=0):
    from delta_amd.predicates import build_program, partition_schema
    staged = engine.stage_log(lp)
    st = staged.replay(cutoff)
    staged.release()
    try:
        live = st.export(0)
        meta = next(a["metaData"] for a in st.nonfile if "metaData" in a)
        schema = partition_schema(meta)
        out = []
        for preds in preds_list:
            sel = st.filter(build_program(schema, preds))
            assert sel == sorted(set(sel))
            out.append(sorted(live[i]["path"] for i in sel))
        return out
    finally:
        st.release()


def _oracle_selected(lp, preds_list, cutoff=0):
    snap = O.state_reconstruction(O.get_log_segment(lp), cutoff)
    schema = O.partition_schema(snap.metadata)
    return [sorted(f["path"] for f in O.filter_file_list(schema, snap.all_files, p)) for p in preds_list]


@pytest.mark.parametrize("checkpoint", [False, True])
@pytest.mark.parametrize("escaped_keys", [False, True])
@pytest.mark.parametrize("kernel", ["dict", "typed", "generic"])
def test_filter_cast_corpus(engine, tmp_path, checkpoint, escaped_keys, kernel):
    """The three K5 evaluators (context option DR_OPT_FILTER_EVAL): the leaf form over dictionary
    codes (k_dict_leaf + k_filter_dict, the default, 0), the leaf form over the typed cache
    (k_filter_leaf, 1) and the generic postfix interpreter k_filter_typed (2)."""
    lp = F.build(str(tmp_path), checkpoint=checkpoint, escaped_keys=escaped_keys)
    with engine.options(filter_eval={"dict": 0, "typed": 1, "generic": 2}[kernel]):
        got = _gpu_selected(engine, lp, F.PREDICATES)
    want = _oracle_selected(lp, F.PREDICATES)
    for p, g, w in zip(F.PREDICATES, got, want):
        assert g == w, p


def _int_table(tmp_path, cols, rows, checkpoint):
    """Small table partitioned by integer columns (OptimisticTransactionSuite's `part`, `a`/`b`)."""
    import json
    log = os.path.join(str(tmp_path), "_delta_log")
    os.makedirs(log)
    schema = {"type": "struct", "fields": [{"name": "x", "type": "long", "nullable": True, "metadata": {}}] +
              [{"name": c, "type": "integer", "nullable": True, "metadata": {}} for c in cols]}
    md = {"id": "ots", "format": {"provider": "parquet", "options": {}},
          "schemaString": json.dumps(schema), "partitionColumns": cols, "configuration": {}, "createdTime": 1}
    adds = [{"path": "/".join("%s=%s" % (c, v) for c, v in zip(cols, r)) + "/f%d" % k,
             "partitionValues": {c: str(v) for c, v in zip(cols, r)}, "size": 1, "modificationTime": 1,
             "dataChange": True} for k, r in enumerate(rows)]
    with open(os.path.join(log, "%020d.json" % 0), "w") as f:
        f.write(json.dumps({"protocol": {"minReaderVersion": 1, "minWriterVersion": 2}}) + "\n")
        f.write(json.dumps({"metaData": md}) + "\n")
        for a in adds:
            f.write(json.dumps({"add": a}) + "\n")
    if checkpoint:
        from delta_amd.testing import synth as S
        S.write_checkpoint_records(os.path.join(log, "%020d.checkpoint.parquet" % 0),
                                   {"minReaderVersion": 1, "minWriterVersion": 2}, md, adds)
    return log


C, L = F.C, F.L


@pytest.mark.parametrize("checkpoint", [False, True])
def test_filter_optimistic_txn_cases(engine, tmp_path, checkpoint):
    lp = _int_table(tmp_path / "one", ["part"], [(p,) for p in range(1, 6)] * 3, checkpoint)
    preds = [[("=", C("part"), L("integer", 3))], [("in", C("part"), [L("integer", 1)])],
             [(">=", C("part"), L("integer", 2))], [(">", C("part"), L("integer", 1)), ("<=", C("part"), L("integer", 3))],
             [(">", C("part"), L("integer", 3))], [("<=", C("part"), L("integer", 3))]]
    assert _gpu_selected(engine, lp, preds) == _oracle_selected(lp, preds)
    lp2 = _int_table(tmp_path / "two", ["a", "b"], [(a, b) for a in range(3) for b in range(3)], checkpoint)
    preds2 = [[("and", ("=", C("a"), L("integer", 1)), ("=", C("b"), L("integer", 1)))],
              [("=", C("a"), L("integer", 1))], [("or", (">=", C("a"), L("integer", 1)), (">", C("b"), L("integer", 1)))],
              [("=", C("a"), L("integer", 2))]]
    assert _gpu_selected(engine, lp2, preds2) == _oracle_selected(lp2, preds2)


def test_filter_dictionary_overflow_falls_back(engine, tmp_path):
    """A partition column with more distinct values than the u16 dictionary holds (70,000 > 65,534)
    takes the typed leaf kernel; a low-cardinality column beside it still selects exactly."""
    n = 70000
    lp = _int_table(tmp_path / "hi", ["part", "g"], [(k, k % 7) for k in range(n)], checkpoint=False)
    preds = [[(">=", C("part"), L("integer", 69990))], [("=", C("g"), L("integer", 3))],
             [("and", ("<", C("part"), L("integer", 20)), ("=", C("g"), L("integer", 5)))]]
    assert _gpu_selected(engine, lp, preds) == _oracle_selected(lp, preds)


@pytest.mark.parametrize("kernel", ["dict", "typed"])
def test_filter_config4_predicate(engine, tmp_path, kernel):
    """p0 >= DATE'2020-03-01' AND p0 < DATE'2020-06-01' AND p1 IN (1..100)
    AND p2 = 'w17' AND p3 = true, over a 4-column checkpoint + churn commits."""
    from delta_amd.testing import synth as S
    spec = S.ChurnSpec(ckpt_files=30000, ckpt_version=10, n_deltas=4, removes_per_delta=2000,
                       adds_per_delta=2000, readd_frac=0.5, ncols=4)
    exp = S.build_table(str(tmp_path), spec, seed=4, row_group_size=7000)
    lp = os.path.join(str(tmp_path), "_delta_log")
    word = S.WORDS[17]
    preds = [[(">=", C("p0"), L("date", "2020-03-01")), ("<", C("p0"), L("date", "2020-06-01")),
              ("in", C("p1"), [L("integer", v) for v in range(1, 101)]), ("=", C("p2"), L("string", word)),
              ("=", C("p3"), L("boolean", True))],
             [("isnull", C("p2"))],
             [("in", C("p1"), [L("integer", v) for v in range(1, 101)])]]
    with engine.options(filter_eval=1 if kernel == "typed" else 0):
        got = _gpu_selected(engine, lp, preds, exp.min_file_retention_timestamp)
    assert got == _oracle_selected(lp, preds, exp.min_file_retention_timestamp)
    assert len(got[0]) > 0 and len(got[1]) > 0


def test_delta_source_initial_files(tmp_path):
    """DeltaSourceSnapshot.initialFiles + iterator (D/files/DeltaSourceSnapshot.scala:53-95): the
    GPU state's allFiles in (modificationTime, path) order with their indices, partition-only
    filters applied whole on the GPU (a filter that also names a data column is not applied)."""
    from delta_amd.delta_log import DeltaLog, ManualClock
    from delta_amd.testing import synth as S
    spec = S.ChurnSpec(ckpt_files=3000, ckpt_version=5, n_deltas=3, removes_per_delta=400,
                       adds_per_delta=400, readd_frac=0.5, ncols=4)
    exp = S.build_table(str(tmp_path), spec, seed=7, row_group_size=1000)
    lp = os.path.join(str(tmp_path), "_delta_log")
    DeltaLog.clear_cache()
    clock = ManualClock(exp.min_file_retention_timestamp + 7 * 24 * 3600 * 1000)
    snap = DeltaLog.for_table(str(tmp_path), clock=clock).snapshot
    ref = O.state_reconstruction(O.get_log_segment(lp), snap.min_file_retention_timestamp)
    order = sorted(ref.all_files, key=lambda f: (f["modificationTime"], f["path"].encode("utf-8")))
    idx = {f["path"]: i for i, f in enumerate(order)}
    schema = O.partition_schema(ref.metadata)
    part = ("in", C("p1"), [L("integer", v) for v in range(0, 300)])
    mixed = ("and", ("=", C("p2"), L("string", S.WORDS[3])), ("=", C("value"), L("integer", 1)))
    for filters in ([], [part], [part, mixed]):
        got = snap.initial_files(filters)
        keep = O.filter_file_list(schema, order, [part]) if filters else order
        want = [(f["path"], idx[f["path"]]) for f in sorted(keep, key=lambda f: idx[f["path"]])]
        assert [(g["add"]["path"], g["index"]) for g in got] == want
        assert all(g["version"] == snap.version and g["remove"] is None and not g["isLast"] for g in got)
    assert 0 < len(snap.initial_files([part])) < len(order)
    DeltaLog.clear_cache()


def test_tahoe_list_files(tmp_path):
    """TahoeFileIndex.listFiles (D/files/TahoeFileIndex.scala:58-81): pruned files grouped by
    partitionValues, rows cast to the partition schema, sizes / mtimes / absolute paths."""
    import datetime as dt
    from delta_amd.delta_log import DeltaLog, ManualClock
    from delta_amd.testing import synth as S
    spec = S.ChurnSpec(ckpt_files=2000, ckpt_version=2, n_deltas=2, removes_per_delta=300,
                       adds_per_delta=300, readd_frac=0.5, ncols=4)
    exp = S.build_table(str(tmp_path), spec, seed=9, row_group_size=700)
    lp = os.path.join(str(tmp_path), "_delta_log")
    DeltaLog.clear_cache()
    snap = DeltaLog.for_table(str(tmp_path), clock=ManualClock(exp.min_file_retention_timestamp + 604800000)).snapshot
    ref = O.state_reconstruction(O.get_log_segment(lp), snap.min_file_retention_timestamp)
    schema = O.partition_schema(ref.metadata)
    pred = [("<", C("p1"), L("integer", 40))]
    kept = O.filter_file_list(schema, ref.all_files, pred)
    want = {}
    for f in kept:
        row = []
        for c, t in schema.items():
            v = O.cast_string(f["partitionValues"].get(c), t)
            row.append(dt.date(1970, 1, 1) + dt.timedelta(days=v) if t == "date" and v is not None
                       else (bool(v) if t == "boolean" and v is not None else v))
        want.setdefault(tuple(row), set()).add((f["size"], f["modificationTime"], os.path.join(str(tmp_path), f["path"])))
    got = {row: {(s["length"], s["modificationTime"], s["path"]) for s in stats} for row, stats in snap.list_files(pred)}
    assert got == want and len(got) > 1
    DeltaLog.clear_cache()


def test_config4_multipart_flow(engine, tmp_path):
    """Config 4 end to end at reduced scale (D/Checkpoints.scala:187-218,229-365,
    D/DeltaLog.scala:500-547): a 100-part checkpoint with 4 partition columns is reconstructed (parity
    with the oracle), pruned by the 4-column conjunction (twice: the second call reads the state's
    typed partition-value cache; the count equals the generator's), written back as a 4-part
    checkpoint, and the written parts replay to the same state."""
    import glob
    from delta_amd.delta_log import DeltaLog, ManualClock
    from delta_amd.predicates import build_program, partition_schema
    from delta_amd.testing import synth as S
    from tests.test_gpu_parity import _assert_same
    scale = 0.002
    exp = S.build_config(4, str(tmp_path), scale=scale, workers=4)
    lp = os.path.join(str(tmp_path), "_delta_log")
    assert len(glob.glob(os.path.join(lp, "*.checkpoint.*.0000000100.parquet"))) == 100
    DeltaLog.clear_cache()
    log = DeltaLog.for_table(str(tmp_path), clock=ManualClock(exp.min_file_retention_timestamp + 604800000))
    snap = log.snapshot
    cutoff = snap.min_file_retention_timestamp
    ref = O.state_reconstruction(O.get_log_segment(lp), cutoff)
    _assert_same(snap.state, ref)
    prog = build_program(partition_schema(snap.metadata), S.config4_predicate())
    live = snap.all_files
    first = snap.state.filter(prog)
    again = snap.state.filter(prog)
    assert first == again
    got = sorted(live[i]["path"] for i in first)
    want = sorted(f["path"] for f in O.filter_file_list(O.partition_schema(ref.metadata), ref.all_files,
                                                         S.config4_predicate()))
    assert got == want and len(got) == S.config4_selected(str(tmp_path), scale) > 0
    meta = log.checkpoint(parts=4)
    assert meta["parts"] == 4
    for f in glob.glob(os.path.join(lp, "*.checkpoint.*.0000000100.parquet")):
        os.remove(f)
    st = _gpu_replay_log(engine, lp, cutoff)
    try:
        _assert_same(st, ref)
    finally:
        st.release()
    DeltaLog.clear_cache()


def _gpu_replay_log(engine, lp, cutoff):
    staged = engine.stage_log(lp)
    try:
        return staged.replay(cutoff)
    finally:
        staged.release()


def test_scan_order_and_partition_groups_on_device(engine, tmp_path):
    """dr_state_scan_order / dr_state_partition_groups (the GPU side of DeltaSourceSnapshot's
    allFiles.sort("modificationTime", "path") and TahoeFileIndex.listFiles' groupBy(partitionValues))
    against the host export of the same state: checkpoint rows and JSON lines mixed, modificationTime
    ties broken by the path's UTF-8 bytes, canonicalised absolute and escaped paths, the JSON forms
    of modificationTime Jackson does not read as a long (missing, fraction, string, out of range:
    the primitive's 0), null / escaped / missing partition values, and an applied tail."""
    import json
    from delta_amd import _native as N
    from delta_amd.testing import synth as S
    spec = S.ChurnSpec(ckpt_files=600, ckpt_version=1, n_deltas=2, removes_per_delta=60, adds_per_delta=60,
                       readd_frac=0.5, ncols=2)
    S.build_table(str(tmp_path), spec, seed=21, row_group_size=250)
    lp = os.path.join(str(tmp_path), "_delta_log")
    mt = S.T0 + 5 * 60000  # ties with synthetic adds of version 5 (mtime T0 + version * 60000 + k)
    adds = [("/abs//x.parquet", '"p0":"2020-01-01","p1":"7"', str(mt)),
            ("b.parquet", '"p0":"2020-01-01","p1":"7"', str(mt)),
            ("a.parquet", '"p0":"2020-01-01","p1":null', str(mt)),
            ("\\u00e9.parquet", '"p0":"2020-01-01","p1":"7"', str(mt)),
            ("z\\u0301.parquet", '"p0":"2020-01-0\\u0031","p1":"7"', str(mt)),
            ("m1.parquet", '"p0":"2020-01-02"', None),
            ("m2.parquet", '"p0":"2020-01-02","p1":"8"', "1.5"),
            ("m3.parquet", '"p0":"2020-01-02","p1":"8"', '"12"'),
            ("m4.parquet", '"p0":"2020-01-02","p1":"8"', "99999999999999999999"),
            ("m5.parquet", '"p0":"2020-01-02","p1":"8"', "-3"),
            ("m6.parquet", '"p0":"2020-01-02","p1":"8"', "1e3")]
    lines = []
    for p, pv, m in adds:
        mt_s = ',"modificationTime":%s' % m if m is not None else ""
        lines.append('{"add":{"path":"%s","partitionValues":{%s},"size":1%s,"dataChange":true}}' % (p, pv, mt_s))
    lines.append('{"add":{"path":"k.parquet","partitionValues":{"p0":"2020-01-03","p1":"1"},"size":2,'
                 '"modificationTime":4,"modificationTime":%d,"dataChange":true}}' % mt)  # repeated member: the last
    v = spec.ckpt_version + spec.n_deltas + 1
    with open(os.path.join(lp, "%020d.json" % v), "w") as f:
        f.write("\n".join(lines) + "\n")

    def check(st):
        live = st.export(0)
        want = sorted(range(len(live)), key=lambda i: (live[i]["modificationTime"], live[i]["path"].encode("utf-8")))
        assert st.scan_order() == want
        for rows in (None, list(range(0, len(live), 3))):
            groups = st.partition_groups(rows)
            sel = list(range(len(live))) if rows is None else rows
            assert sorted(i for g in groups for i in g) == sorted(sel)
            keys = [tuple((live[i]["partitionValues"] or {}).get(c) for c in ("p0", "p1")) for i in sel]
            assert len(groups) == len(set(keys))
            for g in groups:
                assert g == sorted(g)
                assert len({tuple((live[i]["partitionValues"] or {}).get(c) for c in ("p0", "p1")) for i in g}) == 1
        return live

    staged = engine.stage_log(lp)
    st = staged.replay(0)
    staged.release()
    try:
        live = check(st)
        byp = {r["path"]: r for r in live}
        assert byp["m1.parquet"]["modificationTime"] == 0 and byp["m5.parquet"]["modificationTime"] == -3
        assert byp["m4.parquet"]["modificationTime"] == 0 and byp["k.parquet"]["modificationTime"] == mt
        # an applied tail (a chain state: JSON lines from two sources + checkpoint rows)
        with open(os.path.join(lp, "%020d.json" % (v + 1)), "w") as f:
            f.write('{"add":{"path":"t.parquet","partitionValues":{"p0":"2020-01-01","p1":"7"},"size":3,'
                    '"modificationTime":%d,"dataChange":true}}\n{"remove":{"path":"b.parquet","deletionTimestamp":1}}\n' % mt)
        with open(os.path.join(lp, "%020d.json" % (v + 1)), "rb") as f:
            tail = engine.stage_files([(v + 1, N.DR_FILE_JSON, 0, f.read())])
        st2 = st.apply(tail, 0)
        tail.release()
        try:
            check(st2)
        finally:
            st2.release()
    finally:
        st.release()
