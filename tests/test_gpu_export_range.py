"""Row-range export (ABI 3: dr_state_export_plan / dr_state_export_range): the drop-in's answer to
the JVM's 2^31 - 1-byte direct buffers and to the reference's partitioned state (Snapshot.state is a
partitioned cached RDD, D/Snapshot.scala:103-120, D/util/StateCache.scala:45-68). The planned ranges
tile the side, no column of a range exceeds the bound, and the ranges' columns -- offsets shifted
back -- are byte-for-byte dr_state_export's (every field of every record)."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def engine():
    from delta_amd.delta_log import Engine
    return Engine.get(0)


def _check_range(full, r, lo, hi, max_bytes):
    """r (rows [lo, hi), rebased) against the full export's columns."""
    def rows(name, a, b):
        np.testing.assert_array_equal(r[name], full[name][a:b], err_msg=name)

    def offs(name, a, b):  # an offset column: rebased slice
        want = full[name][a:b + 1] - full[name][a]
        np.testing.assert_array_equal(r[name], want, err_msg=name)
        return int(full[name][a]), int(full[name][b])

    for name in ("size", "modification_time", "deletion_timestamp", "deletion_timestamp_valid",
                 "extended_file_metadata", "stats_null", "pv_null", "tags_null"):
        rows(name, lo, hi)
    p0, p1 = offs("path_off", lo, hi)
    rows("path_bytes", p0, p1)
    s0, s1 = offs("stats_off", lo, hi)
    rows("stats_bytes", s0, s1)
    for side in ("pv", "tags"):
        e0, e1 = offs(side + "_entry_off", lo, hi)
        rows(side + "_val_null", e0, e1)
        for kv in ("key", "val"):
            b0, b1 = offs("%s_%s_off" % (side, kv), e0, e1)
            rows("%s_%s_bytes" % (side, kv), b0, b1)
    assert max(v.nbytes for v in r.values()) <= max_bytes


def _ranges_equal_full(st, which, max_rows, max_bytes):
    full = st.export_columns(which)
    n = len(full["path_off"]) - 1
    bounds = st.export_plan(which, max_rows, max_bytes)
    assert bounds[0] == 0 and bounds[-1] == n and all(a < b for a, b in zip(bounds, bounds[1:]))
    for lo, hi in zip(bounds, bounds[1:]):
        assert hi - lo <= max_rows
        _check_range(full, st.export_range(which, lo, hi), lo, hi, max_bytes)
    return bounds


@pytest.mark.parametrize("max_rows,max_bytes", [(1 << 30, 1 << 16), (5000, 1 << 30), (777, 4096)])
def test_ranges_tile_the_side(engine, tmp_path, max_rows, max_bytes):
    """Config 3's shape (checkpoint + JSON survivors, both sides): ranges bounded by bytes (row-level
    refinement of the 4096-row samples at 4 KiB), by rows, and by both."""
    from delta_amd.testing import synth as S
    exp = S.build_config(3, str(tmp_path), scale=0.005)
    staged = engine.stage_log(os.path.join(str(tmp_path), "_delta_log"))
    st = staged.replay(exp.min_file_retention_timestamp)
    staged.release()
    try:
        for which in (0, 1):
            b = _ranges_equal_full(st, which, max_rows, max_bytes)
            n = b[-1]
            assert len(b) - 1 >= -(-n // max_rows)
            if which == 0:
                assert len(b) > 2  # 50K live files: every bound here splits them
        # a small range (its copy; the range outliving its state and context is
        # test_range_outlives_its_state_and_context, at the C ABI)
        r = st.export_range(0, 3, 10)
        assert len(r["path_off"]) == 8 and r["path_off"][0] == 0
    finally:
        st.release()


def test_range_plan_refuses_a_row_over_the_bound(engine, tmp_path):
    from delta_amd.delta_log import DeltaError
    from delta_amd.testing import synth as S
    exp = S.build_config(1, str(tmp_path), scale=0.05)
    staged = engine.stage_log(os.path.join(str(tmp_path), "_delta_log"))
    st = staged.replay(exp.min_file_retention_timestamp)
    staged.release()
    try:
        with pytest.raises(DeltaError) as ei:
            st.export_plan(0, 1 << 20, 64)  # every stats string is longer than 64 bytes
        assert ei.value.code == "DR_E_UNSUPPORTED"
    finally:
        st.release()


def test_config4_through_range_exports(engine, tmp_path):
    """Config 4's 100-part checkpoint at scale 0.3 (30M live files): the plan under the JVM bound
    (2^31 - 1 bytes per direct buffer) needs several ranges -- the side's path bytes alone exceed
    it -- and ranges of at most 4M rows / 256 MiB per column reproduce the full export exactly."""
    from delta_amd.testing import synth as S
    exp = S.build_config(4, str(tmp_path), scale=0.3)
    staged = engine.stage_log(os.path.join(str(tmp_path), "_delta_log"))
    st = staged.replay(exp.min_file_retention_timestamp)
    staged.release()
    try:
        assert st.counts["num_files"] == exp.num_files
        jvm = st.export_plan(0, 1 << 62, (1 << 31) - 1)
        assert len(jvm) > 2, jvm
        b = _ranges_equal_full(st, 0, 4 << 20, 256 << 20)
        assert len(b) > 8
    finally:
        st.release()


def _native_range(st, which, lo, hi):
    import ctypes as C
    from delta_amd import _native as N
    e, h = N.dr_export(), C.c_void_p()
    st.eng.check(st.eng.lib.dr_state_export_range(st.h, which, int(lo), int(hi), C.byref(h), C.byref(e)))
    return h, e


def _check_native(full, e, lo, hi):
    from delta_amd.delta_log import State
    _check_range(full, {k: v.copy() for k, v in State._columns(e).items()}, lo, hi, 1 << 40)


def test_range_outlives_its_state_and_context(tmp_path):
    """The contract the JNI RDD relies on (include/deltareplay.h, ABI 4), at the C ABI: a range's host
    columns stay readable after dr_state_release and after dr_ctx_destroy, dr_range_release then
    unpins them (the destroyed context's cache is not touched), and a second release of the same
    range is refused instead of freeing twice."""
    from delta_amd import _native as N
    from delta_amd.delta_log import Engine
    from delta_amd.testing import synth as S
    exp = S.build_config(3, str(tmp_path), scale=0.003)
    eng = Engine(0)  # a context of its own: destroyed below
    staged = eng.stage_log(os.path.join(str(tmp_path), "_delta_log"))
    st = staged.replay(exp.min_file_retention_timestamp)
    staged.release()
    full = {k: v.copy() for k, v in st.export_columns(0).items()}
    tfull = {k: v.copy() for k, v in st.export_columns(1).items()}
    n, nt = len(full["path_off"]) - 1, len(tfull["path_off"]) - 1
    h1, e1 = _native_range(st, 0, 5, n // 2)
    h2, e2 = _native_range(st, 0, n // 2, n)
    h3, e3 = _native_range(st, 1, 0, nt)
    st.release()
    _check_native(full, e1, 5, n // 2)  # the state is gone
    assert eng.lib.dr_range_release(h1) == N.DR_OK
    assert eng.lib.dr_range_release(h1) == 1  # DR_E_INVALID_ARG: not a live range any more
    eng.lib.dr_ctx_destroy(eng.ctx)
    eng.ctx = None
    _check_native(full, e2, n // 2, n)  # the context is gone
    _check_native(tfull, e3, 0, nt)
    assert eng.lib.dr_range_release(h2) == N.DR_OK
    assert eng.lib.dr_range_release(h3) == N.DR_OK


def test_concurrent_range_exports_share_one_context(tmp_path):
    """Several host threads (a Spark executor's concurrent tasks) export ranges of one state through
    one context at once: the library serialises the calls (ABI 4), the first one materialises the
    side, and every range equals the full export's rows."""
    import threading
    from delta_amd import _native as N
    from delta_amd.delta_log import Engine
    from delta_amd.testing import synth as S
    exp = S.build_config(3, str(tmp_path), scale=0.003)
    eng = Engine(0)
    staged = eng.stage_log(os.path.join(str(tmp_path), "_delta_log"))
    st = staged.replay(exp.min_file_retention_timestamp)
    staged.release()
    try:
        # the ranges first, on a state whose export is not built yet (the threads race to build it)
        n = st.counts["num_files"]
        nt = st.counts["num_removes"]
        jobs = [(0, lo, min(n, lo + 997)) for lo in range(0, n, 997)] + [(1, 0, nt)]
        got, errs = {}, []
        go = threading.Barrier(8)

        def worker(k):
            try:
                go.wait()
                for j in range(k, len(jobs), 8):
                    which, lo, hi = jobs[j]
                    h, e = _native_range(st, which, lo, hi)  # no Python lock: straight into the library
                    from delta_amd.delta_log import State
                    got[j] = {c: v.copy() for c, v in State._columns(e).items()}
                    assert eng.lib.dr_range_release(h) == N.DR_OK
            except Exception as ex:  # noqa: BLE001 (reported below)
                errs.append(repr(ex))

        ts = [threading.Thread(target=worker, args=(k,)) for k in range(8)]
        for t in ts:
            t.start()
        for t in ts:
            t.join(120)
        assert not errs, errs
        full = {0: st.export_columns(0), 1: st.export_columns(1)}
        for j, (which, lo, hi) in enumerate(jobs):
            _check_range(full[which], got[j], lo, hi, 1 << 40)
    finally:
        st.release()
