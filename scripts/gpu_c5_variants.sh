# Config-5 apply latency of the current library and of each variant in var_libs/ (bench.py --config 5
# at SCALE, default 0.1, no CPU baseline)
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/c5var
cp $R/delta_amd/libdeltareplay.so $R/gpurun_out/c5var/base.so
mkdir -p $R/var_libs/base && cp $R/gpurun_out/c5var/base.so $R/var_libs/base/libdeltareplay.so
for v in ${VARIANTS:-$(ls $R/var_libs)}; do
  cp $R/var_libs/$v/libdeltareplay.so $R/delta_amd/libdeltareplay.so
  timeout -k 10 300 python $R/bench.py --config 5 --scale ${SCALE:-0.1} --no-cpu-baseline > $R/gpurun_out/c5var/$v.json 2> $R/gpurun_out/c5var/$v.err || { echo "$v failed"; tail -5 $R/gpurun_out/c5var/$v.err; break; }
  python -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); s=d['stream']
print(sys.argv[2], 'apply', s['apply_ms'], 'k1', d['kernels_per_commit_ms'].get('k_json_lines'), 'match', s['matches_full_replay'])" $R/gpurun_out/c5var/$v.json $v
done
cp $R/gpurun_out/c5var/base.so $R/delta_amd/libdeltareplay.so
