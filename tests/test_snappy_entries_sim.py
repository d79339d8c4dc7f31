"""CPU restatement of the SNAPPY chunk-speculation entry rules (scripts/snappy_entries_sim.py,
following k_snappy.hip's k_snap_spec / assume / entries / regions / resolve): on the period-4
element streams of consecutive int64 dictionaries, the resolver with the r02 stop rule leaves no
chunk entry wrong, for concurrent (interleaved) region walks; the earlier rule did (the device then
fell back to the serial decoder)."""
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
    try:
        sim.FIX = False
        _, wrong_before = sim.resolve_all(raw, ch, order="interleave")
        sim.FIX = True
        _, wrong_after = sim.resolve_all(raw, ch, order="interleave")
    finally:
        sim.FIX = True
    assert wrong_before and not wrong_after
