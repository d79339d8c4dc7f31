# k_json_lines on config 3: the lane-per-line walker against the staged (wave-ballot tape) walker for
# every segment (context option json_staged=1), rocprofv3 kernel stats of each.
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/jstaged
mkdir -p $O
SC=${SCALE:-1.0}
timeout -k 10 300 python $R/scripts/prof_replay.py --reps 1 --scale $SC > $O/gen.log 2>&1 || { tail -20 $O/gen.log; exit 1; }
for m in 0 1; do
  PROF_OPTS=json_staged=$m timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/m$m -o run --output-format csv -- python $R/scripts/prof_replay.py --reps 3 --scale $SC > $O/m$m.log 2>&1 || { echo "mode $m failed"; tail -5 $O/m$m.log; exit 1; }
  python - $O/m$m $m <<'PY'
import csv, sys, glob
rows = list(csv.DictReader(open(glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0])))
for r in rows:
    if "json" in r["Name"] or "tail" in r["Name"]:
        print("staged=" + sys.argv[2], r["Name"].split("(")[0][-60:], r["Calls"], "%.4f ms" % (float(r["AverageNs"]) / 1e6), flush=True)
PY
done
