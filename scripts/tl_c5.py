"""Per-apply timeline from scripts/gpu_tl_c5.sh's rocprofv3 CSVs: for the applies of the untimed
pass, the median host time of each HIP API call kind between consecutive apply launches (k_apply_commit, or k_json_lines before it),
and the median device time of each kernel / copy and of the gaps between them."""
import csv
import statistics
import sys
from collections import defaultdict

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/tl_c5/t"
api = list(csv.DictReader(open(d + "/run_hip_api_trace.csv")))
ker = list(csv.DictReader(open(d + "/run_kernel_trace.csv")))
cpy = list(csv.DictReader(open(d + "/run_memory_copy_trace.csv")))
launch = {}  # correlation id -> api row
for a in api:
    launch[a["Correlation_Id"]] = a
dev = [(int(k["Start_Timestamp"]), int(k["End_Timestamp"]), k["Kernel_Name"].split("(")[0][:40], k["Correlation_Id"]) for k in ker]
dev += [(int(c["Start_Timestamp"]), int(c["End_Timestamp"]), "copy:" + c["Direction"][12:], c["Correlation_Id"]) for c in cpy]
dev.sort()
starts = [i for i, x in enumerate(dev) if "k_apply_commit" in x[2] or "k_json_lines" in x[2]]
# the last half of the applies (the untimed pass)
starts = starts[len(starts) // 2 + 2:-1]
per_api = defaultdict(list)
per_dev = defaultdict(list)
gaps = defaultdict(list)
span = []
apis = sorted((int(a["Start_Timestamp"]), int(a["End_Timestamp"]), a["Function"]) for a in api)
import bisect
ast = [x[0] for x in apis]
for s, e in zip(starts, starts[1:]):
    seq = dev[s:e]
    a0 = launch[seq[0][3]]
    t0 = int(a0["Start_Timestamp"])
    a1 = launch[dev[e][3]]
    t1 = int(a1["Start_Timestamp"])
    span.append((t1 - t0) / 1e3)
    cnt = defaultdict(float)
    for x in apis[bisect.bisect_left(ast, t0):bisect.bisect_left(ast, t1)]:
        cnt[x[2]] += (x[1] - x[0]) / 1e3
    for k, v in cnt.items():
        per_api[k].append(v)
    prev_end = None
    for j, x in enumerate(seq):
        per_dev["%d %s" % (j, x[2])].append((x[1] - x[0]) / 1e3)
        if prev_end is not None:
            gaps["%d before %s" % (j, x[2])].append((x[0] - prev_end) / 1e3)
        prev_end = x[1]
    la = launch[seq[0][3]]
    gaps["0 launch->start"].append((seq[0][0] - int(la["End_Timestamp"])) / 1e3)
print("applies", len(span), "median host span between applies (us) %.1f" % statistics.median(span))
print("-- host API time per apply (us, median)")
for k, v in sorted(per_api.items(), key=lambda kv: -statistics.median(kv[1])):
    print("  %-40s %7.2f  (n=%d)" % (k, statistics.median(v), len(v)))
print("-- device (us, median)")
for k, v in sorted(per_dev.items(), key=lambda kv: int(kv[0].split()[0])):
    print("  %-48s %7.2f" % (k, statistics.median(v)))
print("-- gaps (us, median)")
for k, v in sorted(gaps.items(), key=lambda kv: int(kv[0].split()[0])):
    print("  %-48s %7.2f" % (k, statistics.median(v)))
