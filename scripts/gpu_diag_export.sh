# export fallback diagnostic at a given scale
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 python $R/scripts/diag_export.py 3 ${SCALE:-1.0} > $R/gpurun_out/diag_export.log 2>&1 || { tail -20 $R/gpurun_out/diag_export.log; exit 1; }
grep -E "export|bad page|exec phases|snappy:" $R/gpurun_out/diag_export.log | head -30
