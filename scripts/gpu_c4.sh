# config 4 bench line (100-part 100M-row checkpoint + 4-column predicate + checkpoint part write);
# C=5 for the streaming-tail line, CPU=1 to include the CPU baseline
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
CPUFLAG=--no-cpu-baseline; [ -n "$CPU" ] && CPUFLAG=
timeout -k 10 1100 python -u $R/bench.py --config ${C:-4} $CPUFLAG --steps ${K:-5} --warmup 2 > $R/gpurun_out/c${C:-4}.json 2> $R/gpurun_out/c${C:-4}.err || { tail -20 $R/gpurun_out/c${C:-4}.err; exit 1; }
python -c "
import json; d=json.load(open('$R/gpurun_out/c${C:-4}.json'))
print('ms/step', d['ms_per_step'], 'value', d['value'], 'roofline', d['roofline']['kernel'], d['roofline']['frac'])
print('k5', d.get('k5_filter')); print('ckpt', d.get('checkpoint_write'))
"
