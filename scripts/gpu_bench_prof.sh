# Round-end evidence: kernel-trace stats and HBM PMC passes of the default bench command, then the
# full bench line (with the CPU baseline) reading those PMC passes.
set -e
C=${C:-3}
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
KRE=${KRE:-"k_snap_exec|k_snap_spec|k_bucket_scatter|k_bucket_reduce|k_bucket_verify|k_json_lines|k_ckpt_assemble|k_pq_data"}
O=$R/gpurun_out/round
rm -rf $O && mkdir -p $O
timeout -k 10 400 python $R/bench.py --config $C --no-cpu-baseline > $O/warm.json 2> $O/warm.err
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/stats -o run --output-format csv -- python $R/bench.py --config $C --no-cpu-baseline > $O/stats.log 2>&1
timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$KRE" -d $O/pmc/fetch -o pmc --output-format csv -- python $R/bench.py --config $C --no-cpu-baseline > $O/fetch.log 2>&1
timeout -s KILL 400 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$KRE" -d $O/pmc/write -o pmc --output-format csv -- python $R/bench.py --config $C --no-cpu-baseline > $O/write.log 2>&1
timeout -k 10 600 python $R/bench.py --config $C --pmc-dir $O/pmc > $O/bench.json 2> $O/bench.err
cat $O/bench.json
