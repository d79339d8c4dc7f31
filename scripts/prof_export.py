"""Profiling driver for the full-record state: stage a config table, replay, then materialise both
sides on the device (dr_state_materialize), and export them from a fresh replay (dr_state_export's
streamed path) -- for rocprofv3 --kernel-trace --stats."""
import ctypes as C
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from delta_amd import _native as N  # noqa: E402
from delta_amd.delta_log import Engine  # noqa: E402

cfg, scale = int(sys.argv[1]), float(sys.argv[2])
table = os.path.join(os.environ.get("TMPDIR", "/tmp"), "dr_bench", "c%d_s%g" % (cfg, scale))
exp = bench.build_table(table, cfg, scale)
eng = Engine.get(0)
staged = eng.stage_log(os.path.join(table, "_delta_log"))
for rep in range(2):
    st = staged.replay(exp["min_file_retention_timestamp"])
    t0 = time.perf_counter()
    ex = N.dr_export()
    for which in (N.DR_LIVE, N.DR_TOMBSTONES):  # streamed: extraction and copies overlapped
        eng.check(eng.lib.dr_state_export(st.h, which, C.byref(ex)))
    t1 = time.perf_counter()
    st.release()
    st = staged.replay(exp["min_file_retention_timestamp"])
    t2 = time.perf_counter()
    b = st.materialize()
    t3 = time.perf_counter()
    st.release()
    print("rep %d streamed export %.4f s; materialize %.4f s (%d bytes)" % (rep, t1 - t0, t3 - t2, b), flush=True)
