# SNAPPY exec iteration: parity tests of the checkpoint paths, exec phase clocks at config 3, bench.
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_checkpoint.py tests/test_gpu_edge_cases.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/par.log 2>&1 || { tail -40 gpurun_out/par.log; exit 1; }
tail -2 gpurun_out/par.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 python $R/scripts/diag_snappy.py 3 1.0 2 > $R/gpurun_out/diag.log 2>&1 || { tail -20 $R/gpurun_out/diag.log; exit 1; }
grep -E "exec phases|bad page" $R/gpurun_out/diag.log | head -8
timeout -k 10 400 python $R/bench.py --no-cpu-baseline > $R/gpurun_out/bench.json 2> $R/gpurun_out/bench.err || { tail -20 $R/gpurun_out/bench.err; exit 1; }
python -c "
import json; d=json.load(open('$R/gpurun_out/bench.json'))
print('ms/step', d['ms_per_step'], 'value', d['value'], 'roofline', d['roofline'].get('kernel'), d['roofline']['achieved'], d['roofline']['frac'])
for k,v in sorted(d.get('kernels',{}).items(), key=lambda x: -x[1].get('ms',0) if isinstance(x[1],dict) else 0)[:14]: print(k, v)
"
