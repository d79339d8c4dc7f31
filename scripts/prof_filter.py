"""Profiling driver for K5: stage config 4 at a scale, replay, then dr_filter with config 4's predicate
(the first call builds the typed cache) -- for rocprofv3 --kernel-trace --stats."""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from delta_amd.delta_log import Engine  # noqa: E402
from delta_amd.predicates import build_program, partition_schema  # noqa: E402
from delta_amd.testing import synth as S  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--scale", type=float, default=0.25)
ap.add_argument("--reps", type=int, default=10)
args = ap.parse_args()
table = os.path.join(os.environ.get("TMPDIR", "/tmp"), "dr_bench", "c4_s%g" % args.scale)
exp = bench.build_table(table, 4, args.scale)
eng = Engine.get(0)
staged = eng.stage_log(os.path.join(table, "_delta_log"))
st = staged.replay(exp["min_file_retention_timestamp"])
meta = next(a["metaData"] for a in st.nonfile if "metaData" in a)
prog = build_program(partition_schema(meta), S.config4_predicate())
sel = st.filter(prog)
t0 = time.perf_counter()
for _ in range(args.reps):
    st.filter(prog)
dt = (time.perf_counter() - t0) / args.reps
print("files %d selected %d call %.3f ms" % (st.counts["num_files"], len(sel), dt * 1e3), flush=True)
st.release()
