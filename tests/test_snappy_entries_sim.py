"""CPU restatement of the SNAPPY chunk-speculation entry rules (scripts/snappy_entries_sim.py,
following k_snappy.hip's k_snap_spec / assume / entries / regions / resolve): on the period-4
element streams of consecutive int64 dictionaries, the resolver leaves no chunk entry wrong, for
ascending and concurrent (interleaved) region walks. r02's stop rule fixed the interleaved case for the
window-by-window resolver (the device had fallen back to the serial decoder); r04's resolver follows
the breaks inside a window without leaving it, and still needs that stop rule."""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "scripts"))


@pytest.mark.parametrize("v,ch", [(3, 256), (44, 256), (57, 128)])
def test_resolver_stop_rule(v, ch):
    pa = pytest.importorskip("pyarrow")
    import snappy_entries_sim as sim
    data = (np.arange(60000, dtype=np.int64) + 1_700_000_000_000 + v * 60000).tobytes()
    raw = pa.compress(data, codec="snappy", asbytes=True)
    sim.FIX = True
    for order in (None, "interleave"):
        nreg, wrong = sim.resolve_all(raw, ch, order=order)
        assert nreg and not wrong, (order, wrong[:10])


def test_resolver_regions_of_a_page_in_order():
    """Pages of length-prefixed 102-byte random paths (the long-literal layout of
    tests/test_gpu_edge_cases.py::test_snappy_long_literals_and_unstaged_blocks): chunks spanned by
    long literals leave unflagged wrong entries that a region walk corrects on its way to the next
    region, so a later region walking concurrently from an entry not yet corrected leaves wrong
    entries (the interleaved schedule: the r04 one-wave-per-region k_snap_resolve, whose page then
    failed the size check). Walking a page's regions in ascending order (r05: one wave per page)
    leaves none."""
    import random
    import string
    import struct
    pa = pytest.importorskip("pyarrow")
    import snappy_entries_sim as sim
    rng = random.Random(100)
    sym = string.ascii_letters + string.digits + "-_"
    paths = ["d/" + "".join(rng.choice(sym) for _ in range(100)) for _ in range(10000)]
    data = b"".join(struct.pack("<I", len(p)) + p.encode() for p in paths)[: 1 << 20]
    raw = pa.compress(data, codec="snappy", asbytes=True)
    sim.FIX = True
    nreg, wrong = sim.resolve_all(raw, order=None)
    assert nreg > 1 and not wrong, wrong[:10]
    _, wrong_interleaved = sim.resolve_all(raw, order="interleave")
    assert wrong_interleaved  # the schedule the per-page walk rules out
