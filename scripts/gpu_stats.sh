# Kernel-trace statistics of the profiling driver (config 3 at SCALE, default 0.25).
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
SCALE=${SCALE:-0.25}
mkdir -p $R/gpurun_out/stats
timeout -k 10 300 python $R/scripts/prof_replay.py --scale $SCALE --reps 1 > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/stats -o run --output-format csv -- python $R/scripts/prof_replay.py --scale $SCALE --reps 3 > $R/gpurun_out/stats/run.log 2>&1
f=$(find $R/gpurun_out/stats -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:30]:
    print("%-60s %4s %9.3f ms" % (r["Name"][:60], r["Calls"], float(r["AverageNs"]) / 1e6))
PY
