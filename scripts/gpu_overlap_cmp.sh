cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/ovl
timeout -k 10 600 python -u $R/bench.py --no-cpu-baseline --steps 10 > $R/gpurun_out/ovl/base.json 2> $R/gpurun_out/ovl/base.err || { tail $R/gpurun_out/ovl/base.err; exit 1; }
DR_OVERLAP=1 timeout -k 10 600 python -u $R/bench.py --no-cpu-baseline --steps 10 > $R/gpurun_out/ovl/ovl.json 2> $R/gpurun_out/ovl/ovl.err || { tail $R/gpurun_out/ovl/ovl.err; exit 1; }
python -c "
import json
for n in ('base','ovl'):
    d=json.load(open('$R/gpurun_out/ovl/%s.json'%n)); print(n, d['ms_per_step'], d['value'], d.get('end_to_end',{}).get('replay_s'))
"
