"""Diagnostics: per-field full-record sums of a config-4 table on the GPU and in the C++ restatement
(DR_RECORD_FIELDS masks the record-hash words: 1 path, 2 size, 3 modificationTime / deletionTimestamp,
5 stats, 6 partitionValues, 7 tags). Usage: python scripts/c4_fields.py SCALE"""
import json, os, sys, subprocess
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench
from delta_amd.delta_log import Engine

scale = float(sys.argv[1])
table = os.path.join("/tmp", "c4_s%g" % scale)
exp = bench.build_table(table, 4, scale)
log_path = os.path.join(table, "_delta_log")
cutoff = exp["min_file_retention_timestamp"]
eng = Engine.get(0)
st = eng.stage_log(log_path).replay(cutoff)
for name, mask in [("all", 0xff), ("path", 0x3), ("size", 0x5), ("mtime", 0x9), ("stats", 0x21), ("pv", 0x41), ("tags", 0x81)]:
    os.environ["DR_RECORD_FIELDS"] = str(mask)
    g = st.record_sums()
    c = bench.run_replay_oracle(log_path, cutoff, 16, record_sums=True)
    print(name, "gpu", g[0], "cpu", c["live_record_sum"], "MATCH" if g[0] == c["live_record_sum"] else "DIFF", flush=True)
