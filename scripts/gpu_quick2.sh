# selected GPU tests + export fallback diagnostic
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_edge_cases.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/quick.log 2>&1 || { tail -40 gpurun_out/quick.log; exit 1; }
tail -2 gpurun_out/quick.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 python $R/scripts/diag_export.py 3 0.25 > $R/gpurun_out/diag_export.log 2>&1 || { tail -20 $R/gpurun_out/diag_export.log; exit 1; }
grep -E "export|bad page|exec phases" $R/gpurun_out/diag_export.log | head -20
