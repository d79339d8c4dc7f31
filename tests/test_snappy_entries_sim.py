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
