# exec iteration + export fallback diagnostic
set -e
R=$GRAFT_REPO_ROOT
bash $R/scripts/gpu_exec_iter.sh
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 python $R/scripts/diag_export.py 3 0.25 > $R/gpurun_out/diag_export.log 2>&1 || { tail -20 $R/gpurun_out/diag_export.log; exit 1; }
grep -E "export|bad page|exec phases" $R/gpurun_out/diag_export.log | head -20
