# The default bench line (K1 on stream2 beside the checkpoint decode: DR_OVERLAP unset means on since
# r04) against DR_OVERLAP=0 (one stream), alternated twice on one box
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/ovl
for rep in 1 2; do
  DR_OVERLAP=0 timeout -k 10 600 python -u $R/bench.py --no-cpu-baseline --steps 20 > $R/gpurun_out/ovl/base$rep.json 2> $R/gpurun_out/ovl/base$rep.err || { tail $R/gpurun_out/ovl/base$rep.err; exit 1; }
  timeout -k 10 600 python -u $R/bench.py --no-cpu-baseline --steps 20 > $R/gpurun_out/ovl/ovl$rep.json 2> $R/gpurun_out/ovl/ovl$rep.err || { tail $R/gpurun_out/ovl/ovl$rep.err; exit 1; }
done
python -c "
import json
for n in ('base1','ovl1','base2','ovl2'):
    d=json.load(open('$R/gpurun_out/ovl/%s.json'%n)); print(n, d['ms_per_step'], d['value'])
"
