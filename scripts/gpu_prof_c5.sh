# rocprofv3 kernel trace of the streaming-tail bench (config 5) at reduced scale
set -e
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
O=$R/gpurun_out/prof_c5
rm -rf $O && mkdir -p $O
timeout -k 10 300 python $R/bench.py --config 5 --scale ${SCALE:-0.02} --no-cpu-baseline > $O/warm.json 2> $O/warm.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/stats -o run --output-format csv -- python $R/bench.py --config 5 --scale ${SCALE:-0.02} --no-cpu-baseline > $O/bench.json 2> $O/bench.err
head -30 $O/stats/run_kernel_stats.csv
