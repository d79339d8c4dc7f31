"""The device checkpoint writer (dr_state_write_checkpoint; D/Checkpoints.scala:
229-365): its Parquet files read back with pyarrow equal the rows of the Arrow-encoded checkpoint of
the same state (every column: protocol / metaData / txn rows, adds with partitionValues, tags, stats,
partitionValues_parsed, tombstones with deletionTimestamp validity and extendedFileMetadata), in one
part or several, with small row groups; written into the log, the checkpoint replays on the GPU to
the oracle's state of the original log."""
import io
import os
import shutil

import pytest

from oracle import delta_oracle as O
from tests.conftest import GOLDEN

pytestmark = pytest.mark.gpu

REF = os.path.join(GOLDEN, "ref")


@pytest.fixture(scope="module")
def engine():
    import torch  # noqa: F401
    from delta_amd.delta_log import Engine
    return Engine.get(0)


def _rows(data):
    import pyarrow.parquet as pq
    return pq.read_table(io.BytesIO(data)).to_pylist()


def _norm(rows):
    # map columns come back as lists of (key, value) tuples: compare them as such
    return rows


def _check_state(engine, state, parts, rg, snappy=True):
    from delta_amd.checkpoint import checkpoint_options, checkpoint_table
    md = next((a["metaData"] for a in state.nonfile if "metaData" in a), None)
    stats, parsed = checkpoint_options(md)
    want = checkpoint_table(state)[0].to_pylist()
    got = []
    for k in range(parts):
        data, n = state.write_checkpoint_part(k + 1, parts, stats=stats, parsed=parsed is not None,
                                              row_group_rows=rg, snappy=snappy)
        rows = _rows(data)
        assert len(rows) == n
        got.extend(rows)
    assert len(got) == len(want)
    for i, (g, w) in enumerate(zip(got, want)):
        assert g == w, (i, g, w)


@pytest.mark.parametrize("name", ["delta-0.2.0", "delta-0.1.0", "dbr_8_1_generated_columns"])
def test_device_checkpoint_rows_golden(engine, name):
    lp = os.path.join(REF, name, "_delta_log")
    staged = engine.stage_log(lp)
    st = staged.replay(0)
    staged.release()
    try:
        _check_state(engine, st, 1, 0)
        _check_state(engine, st, 2, 2, snappy=False)
    finally:
        st.release()


def test_device_checkpoint_rows_synthetic(engine, tmp_path):
    from delta_amd.testing import synth as S
    spec = S.ChurnSpec(ckpt_files=3000, ckpt_version=2, n_deltas=3, removes_per_delta=400, adds_per_delta=400,
                       readd_frac=0.5, ncols=4)
    exp = S.build_table(str(tmp_path), spec, seed=3, row_group_size=900)
    lp = os.path.join(str(tmp_path), "_delta_log")
    staged = engine.stage_log(lp)
    st = staged.replay(exp.min_file_retention_timestamp)
    staged.release()
    try:
        _check_state(engine, st, 1, 0)
        _check_state(engine, st, 3, 1000, snappy=False)
        # the pages are SNAPPY: smaller than the uncompressed ones
        a, _ = st.write_checkpoint_part(1, 1, snappy=True)
        b, _ = st.write_checkpoint_part(1, 1, snappy=False)
        assert len(a) < 0.8 * len(b)
    finally:
        st.release()


@pytest.mark.parametrize("parts", [1, 3])
def test_device_checkpoint_round_trip(engine, tmp_path, parts):
    from delta_amd.delta_log import DeltaLog, ManualClock
    from delta_amd.testing import synth as S
    from tests.test_gpu_parity import _assert_same
    spec = S.ChurnSpec(ckpt_files=2000, ckpt_version=2, n_deltas=4, removes_per_delta=300, adds_per_delta=300,
                       readd_frac=0.5, ncols=2)
    root = str(tmp_path / "t")
    exp = S.build_table(root, spec, seed=13, row_group_size=700)
    lp = os.path.join(root, "_delta_log")
    cutoff = exp.min_file_retention_timestamp
    ref = O.state_reconstruction(O.get_log_segment(lp), cutoff)
    DeltaLog.clear_cache()
    log = DeltaLog.for_table(root, clock=ManualClock(cutoff + 7 * 86400000))
    meta = log.checkpoint(parts=parts)
    assert meta["version"] == exp.version and meta.get("parts", 1) == parts
    DeltaLog.clear_cache()
    # the new checkpoint is the segment's start now: replay it alone
    staged = engine.stage_log(lp)
    assert staged.plan()["checkpoint_rows"] > 0
    st = staged.replay(cutoff)
    staged.release()
    try:
        _assert_same(st, ref)
    finally:
        st.release()
    DeltaLog.clear_cache()
