# r04 probes: kernel variants (var_libs/) at config 3, export/materialise kernel trace, then the
# config-5 and config-4 bench lines
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/probe
SCALE=1.0 KRE="k_bucket_verify|k_snap_emit|k_snap_exec" timeout -k 10 600 bash $R/scripts/gpu_kvariants.sh || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/probe/exp -o run --output-format csv -- python $R/scripts/prof_export.py 3 1.0 > $R/gpurun_out/probe/exp.log 2>&1 || { tail -20 $R/gpurun_out/probe/exp.log; exit 1; }
grep rep $R/gpurun_out/probe/exp.log
python - $R/gpurun_out/probe/exp <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:25]:
    print("%-28s calls %5s total %8.3f ms avg %8.4f ms max %8.4f" % (r["Name"].split("(")[0].split("::")[-1][:28], r["Calls"], float(r["TotalDurationNs"]) / 1e6, float(r["AverageNs"]) / 1e6, float(r["MaxNs"]) / 1e6))
PY
C=5 K=5 timeout -k 10 600 bash $R/scripts/gpu_c4.sh || exit 1
python -c "
import json; d=json.load(open('$R/gpurun_out/c5.json')); print(d['stream']); print(d['kernels_per_commit_ms'])"
C=4 K=5 timeout -k 10 700 bash $R/scripts/gpu_c4.sh || exit 1
