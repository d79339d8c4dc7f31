# Times one kernel (KRE) for each prebuilt library variant exp_<V>.so (experiments only).
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
KRE=${KRE:-k_json_lines}
timeout -k 10 300 python $R/scripts/prof_replay.py --scale 1.0 --reps 1 > /dev/null
for v in $VARIANTS; do
  cp $R/exp_$v.so $R/delta_amd/libdeltareplay.so
  rm -rf $R/gpurun_out/exp_$v
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/exp_$v -o run --output-format csv -- python $R/scripts/prof_replay.py --scale 1.0 --reps 3 > /dev/null 2>&1
  f=$(find $R/gpurun_out/exp_$v -name "*kernel_stats.csv" | head -1)
  echo "$v $(grep "$KRE" $f | head -1 | cut -d, -f1-6)"
done
