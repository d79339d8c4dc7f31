"""A state's rows come out in action order: the order of each survivor's winning action in the log
segment (checkpoint rows, then every commit line by line), whatever order the reducer's atomics left
the survivor lists in (engine.hip:order_lists). The reference's state has no row order of its own
(Snapshot.state is repartitioned by path, D/Snapshot.scala:103-110); this one is fixed so that a row
range is a function of the log alone -- a partition of the GPU-backed RDD recomputed on another
executor replays the segment and exports the same rows. Expected orders come from
the oracle's own action stream (oracle/delta_oracle.py:load_actions), the checker only."""
import os

import pytest

from oracle import delta_oracle as O
from tests.test_gpu_parity import _commit_files, _gpu_replay

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def engine():
    from delta_amd.delta_log import Engine
    return Engine.get(0)


def _oracle_order(lp, cutoff, version=None):
    """(live paths, tombstone paths) ordered by the position of each path's last file action."""
    seg = O.get_log_segment(lp, version)
    last = {}
    for pos, (_, a) in enumerate(O.load_actions(seg)):
        if a is None or a[0] not in (O.ADD, O.REMOVE):
            continue
        p = O.canonicalize_path(a[1]["path"])
        last[O.replay_key(p)] = (pos, a[0], a[1], p)
    ordered = sorted(last.values(), key=lambda t: t[0])
    live = [p for _, k, _, p in ordered if k == O.ADD]
    tomb = [p for _, k, act, p in ordered if k == O.REMOVE and O.del_timestamp(act) > cutoff]
    return live, tomb


def _paths(st):
    return [r["path"] for r in st.export(0)], [r["path"] for r in st.export(1)]


@pytest.mark.parametrize("bits,split", [(None, None), (3, 1), (5, 0)])
def test_rows_in_winning_action_order(engine, tmp_path, bits, split):
    """Config 3's shape (checkpoint + commits, both sides non-empty) under the default buckets and
    under forced bucket counts (K3's refinement, K4's sub-passes): every replay lists the oracle's
    order, so replays with different internal orders export identical sequences."""
    from delta_amd.testing import synth as S
    exp = S.build_config(3, str(tmp_path), scale=0.005)
    lp = os.path.join(str(tmp_path), "_delta_log")
    cutoff = exp.min_file_retention_timestamp
    want = _oracle_order(lp, cutoff)
    assert want[0] and want[1]
    opts = {} if bits is None else {"bucket_bits": bits, "split": split}
    with engine.options(**opts):
        st = _gpu_replay(engine, lp, cutoff)
    try:
        assert _paths(st) == want
        # the row ranges tile that same sequence
        b = st.export_plan(0, 997, 1 << 30)
        cols = [st.export_range(0, lo, hi) for lo, hi in zip(b, b[1:])]
        got = []
        for c in cols:
            off, data = c["path_off"], c["path_bytes"].tobytes()
            got += [data[off[i]:off[i + 1]].decode() for i in range(len(off) - 1)]
        assert got == want[0]
    finally:
        st.release()


def test_applied_state_lists_the_full_replays_order(engine, tmp_path):
    """A state extended commit by commit (dr_state_apply: the path index's slot order underneath)
    lists its rows in the order of the full replay of the same segment, and of the oracle."""
    from delta_amd.testing import synth as S
    spec = S.ChurnSpec(ckpt_files=3000, ckpt_version=2, n_deltas=4, removes_per_delta=300,
                       adds_per_delta=300, readd_frac=0.5, ncols=1)
    exp = S.build_table(str(tmp_path), spec, seed=5, row_group_size=1000)
    lp = os.path.join(str(tmp_path), "_delta_log")
    cutoff = exp.min_file_retention_timestamp
    last = spec.ckpt_version + spec.n_deltas
    states = [_gpu_replay(engine, lp, cutoff, version=spec.ckpt_version + 1)]
    try:
        for v in range(spec.ckpt_version + 2, last + 1):
            tail = engine.stage_files(_commit_files(lp, v, v))
            states.append(states[-1].apply(tail, cutoff))
            tail.release()
        full = _gpu_replay(engine, lp, cutoff, version=last)
        try:
            assert _paths(states[-1]) == _paths(full) == _oracle_order(lp, cutoff, last)
        finally:
            full.release()
        # an older state of the chain (its later applies undone on a copy) keeps its own order
        mid = spec.ckpt_version + 2
        assert _paths(states[1]) == _oracle_order(lp, cutoff, mid)
    finally:
        for s in states:
            s.release()
