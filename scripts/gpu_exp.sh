# r04 export probe: GPU suite, SNAPPY region diagnostics of the export decode (page dumps), then the
# materialise/export kernel trace at config 3
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/probe $R/gpurun_out/snapdump
bash $R/scripts/gpu_tests.sh || exit 1
cd /tmp && export TMPDIR=/tmp
DR_SNAP_DEBUG=1 DR_SNAP_DUMP=$R/gpurun_out/snapdump timeout -k 10 300 python $R/scripts/prof_export.py 3 1.0 > $R/gpurun_out/probe/snapdbg.log 2>&1 || { tail -20 $R/gpurun_out/probe/snapdbg.log; exit 1; }
grep -E "snappy|rep " $R/gpurun_out/probe/snapdbg.log | head -60
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/probe/exp2 -o run --output-format csv -- python $R/scripts/prof_export.py 3 1.0 > $R/gpurun_out/probe/exp2.log 2>&1 || { tail -20 $R/gpurun_out/probe/exp2.log; exit 1; }
grep rep $R/gpurun_out/probe/exp2.log
python - $R/gpurun_out/probe/exp2 <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:25]:
    print("%-28s calls %5s total %8.3f ms avg %8.4f ms max %8.4f" % (r["Name"].split("(")[0].split("::")[-1][:28], r["Calls"], float(r["TotalDurationNs"]) / 1e6, float(r["AverageNs"]) / 1e6, float(r["MaxNs"]) / 1e6))
PY
