"""Diagnostic: SNAPPY page fallbacks on a config table (DR_SNAP_DEBUG=1 prints per-page codes)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["DR_SNAP_DEBUG"] = "1"
import bench  # noqa: E402
from delta_amd.delta_log import Engine  # noqa: E402

cfg, scale = int(sys.argv[1]), float(sys.argv[2])
table = "/tmp/dr_diag/c%d_s%g" % (cfg, scale)
exp = bench.build_table(table, cfg, scale)
eng = Engine.get(0)
staged = eng.stage_log(os.path.join(table, "_delta_log"))
print(staged.plan())
for i in range(int(sys.argv[3]) if len(sys.argv) > 3 else 1):
    print("replay", i, flush=True)
    st = staged.replay(exp["min_file_retention_timestamp"])
    print(st.counts, flush=True)
    st.release()
