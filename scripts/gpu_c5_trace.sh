# Config-5 bench line (with the CPU baseline), then a roctx marker trace of config-3 replays
# (DR_ROCTX=1: the library's stage ranges) with its kernel trace and stats.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/c5r $R/gpurun_out/trace
timeout -k 10 900 python -u $R/bench.py --config 5 > $R/gpurun_out/c5r/bench_config5.json 2> $R/gpurun_out/c5r/bench_config5.err || { tail -20 $R/gpurun_out/c5r/bench_config5.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/c5r/stats -o run --output-format csv -- python $R/bench.py --config 5 --no-cpu-baseline --steps 2 > $R/gpurun_out/c5r/stats.log 2>&1 || exit 1
DR_ROCTX=1 timeout -k 10 300 rocprofv3 --marker-trace --kernel-trace --stats -d $R/gpurun_out/trace -o trace --output-format csv -- python $R/scripts/prof_replay.py --reps 2 --scale 0.25 > $R/gpurun_out/trace/run.log 2>&1 || exit 1
ls -R $R/gpurun_out/trace | head -20
