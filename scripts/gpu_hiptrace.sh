cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/hiptrace
timeout -k 10 300 python $R/scripts/prof_replay.py --reps 1 --scale 0.25 > /dev/null || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace --memory-copy-trace -d $R/gpurun_out/hiptrace/t -o run --output-format csv -- python $R/scripts/prof_replay.py --reps 6 --scale 0.25 > $R/gpurun_out/hiptrace/log 2>&1 || { tail -20 $R/gpurun_out/hiptrace/log; exit 1; }
ls -la $R/gpurun_out/hiptrace/t
