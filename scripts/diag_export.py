"""Diagnostic: SNAPPY fallbacks and time of the allFiles / tombstones export on a config table
(DR_SNAP_DEBUG=1 prints the exec phase clocks and per-page fallback codes of every decode)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["DR_SNAP_DEBUG"] = "1"
import ctypes as C  # noqa: E402
import bench  # noqa: E402
from delta_amd import _native as N  # noqa: E402
from delta_amd.delta_log import Engine  # noqa: E402

cfg, scale = int(sys.argv[1]), float(sys.argv[2])
table = "/tmp/dr_diag/c%d_s%g" % (cfg, scale)
exp = bench.build_table(table, cfg, scale)
eng = Engine.get(0)
staged = eng.stage_log(os.path.join(table, "_delta_log"))
st = staged.replay(exp["min_file_retention_timestamp"])
print(st.counts, flush=True)
ex = N.dr_export()
for which in (N.DR_LIVE, N.DR_TOMBSTONES):
    t = time.perf_counter()
    eng.check(eng.lib.dr_state_export(st.h, which, C.byref(ex)))
    print("export", which, "%.4f s" % (time.perf_counter() - t), flush=True)
st.release()
