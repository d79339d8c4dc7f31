# Kernel times (rocprofv3 stats over prof_replay.py) of the current library under two settings of an
# environment variable: ENVVAR=NAME VALUES="0 1" KRE=regex SCALE=s bash scripts/gpu_envcmp.sh
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/envcmp
timeout -k 10 300 python $R/scripts/prof_replay.py --reps 1 --scale ${SCALE:-0.25} > /dev/null || exit 1
for v in ${VALUES:-0 1}; do
  env $ENVVAR=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/envcmp/$v -o run --output-format csv -- python $R/scripts/prof_replay.py --reps 3 --scale ${SCALE:-0.25} > $R/gpurun_out/envcmp/$v.log 2>&1 || { echo "$v failed"; tail -5 $R/gpurun_out/envcmp/$v.log; exit 1; }
  f=$(find $R/gpurun_out/envcmp/$v -name "*kernel_stats.csv" | head -1)
  python - "$f" "$ENVVAR=$v" "${KRE:-k_snap_exec}" <<'PY'
import csv, re, sys
rows = list(csv.DictReader(open(sys.argv[1])))
pat = re.compile(sys.argv[3])
print(sys.argv[2], {r["Name"].split("(")[0].split("::")[-1]: round(float(r["AverageNs"]) / 1e6, 4) for r in rows if pat.search(r["Name"])})
PY
done
