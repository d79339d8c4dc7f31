# Timeline of the streaming-tail apply (config 5, reduced scale): kernels, copies and HIP API calls
# (no counters), for scripts/tl_c5.py
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/tl_c5
rm -rf $O && mkdir -p $O
timeout -k 10 300 python $R/bench.py --config 5 --scale ${SCALE:-0.02} --no-cpu-baseline > $O/warm.json 2> $O/warm.err || { tail -20 $O/warm.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace --memory-copy-trace -d $O/t -o run --output-format csv -- python $R/bench.py --config 5 --scale ${SCALE:-0.02} --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
find $O/t -name "*.csv" | xargs ls -la
