# FETCH_SIZE calibration on k_snap_exec's own loads: per dispatch FETCH_SIZE,
# the 128-B and 32-B read requests to the fabric (TCC_EA0_RDREQ / _32B) and WRITE_SIZE, for config 3
# (scale 1.0) and config 4 (CONFIG4_SCALE), each in its own rocprofv3 pass; the staged plan's SNAPPY
# in / out bytes printed beside them (PROF_PLAN).
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/calib
mkdir -p $O
for cfg in "3 1.0" "4 ${CONFIG4_SCALE:-0.25}"; do
  set -- $cfg
  PROF_PLAN=1 timeout -k 10 600 python $R/scripts/prof_replay.py --config $1 --scale $2 --reps 1 > $O/c$1_plan.txt 2>&1 || { tail -5 $O/c$1_plan.txt; exit 1; }
  i=0
  for grp in "FETCH_SIZE" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum" "WRITE_SIZE"; do
    i=$((i+1))
    timeout -s KILL 300 rocprofv3 --pmc $grp --kernel-include-regex "k_snap_exec" -d $O/c$1_p$i -o pmc --output-format csv -- python $R/scripts/prof_replay.py --config $1 --scale $2 --reps 1 > $O/c$1_p$i.log 2>&1 || { tail -5 $O/c$1_p$i.log; exit 1; }
  done
  python - $O $1 <<'PY'
import csv, glob, sys, json, collections
o, c = sys.argv[1], sys.argv[2]
plan = [l for l in open("%s/c%s_plan.txt" % (o, c)) if l.startswith("{")]
acc = collections.defaultdict(list)
for f in glob.glob("%s/c%s_p*/**/*counter_collection.csv" % (o, c), recursive=True):
    for r in csv.DictReader(open(f)):
        acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
print("config", c, plan[0].strip() if plan else None, {k: sum(v) / len(v) for k, v in acc.items()}, flush=True)
PY
done
