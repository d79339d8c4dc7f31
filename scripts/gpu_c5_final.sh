# Config-5 evidence: the bench line with its CPU baseline, then a kernel-trace summary of the same run
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/c5final
cd /tmp && export TMPDIR=/tmp
timeout -k 10 900 python -u $R/bench.py --config 5 --steps 2 --warmup 1 > $R/gpurun_out/c5final/bench.json 2> $R/gpurun_out/c5final/bench.err || { tail -20 $R/gpurun_out/c5final/bench.err; exit 1; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/c5final/prof -o run --output-format csv -- python -u $R/bench.py --config 5 --steps 2 --warmup 1 --no-cpu-baseline > $R/gpurun_out/c5final/prof.json 2> $R/gpurun_out/c5final/prof.err || { tail -20 $R/gpurun_out/c5final/prof.err; exit 1; }
find $R/gpurun_out/c5final -name "*kernel_stats.csv" | head -1 | xargs head -12
