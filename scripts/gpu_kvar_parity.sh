# Parity subset (replay + edge cases) on the current library, then rocprofv3 kernel times of it and of
# each var_libs/ variant at config 3 scale 1 (SCALE / KRE override), then a quick bench line.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_edge_cases.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/par.log 2>&1 || { tail -40 gpurun_out/par.log; exit 1; }
tail -2 gpurun_out/par.log
SCALE=${SCALE:-1.0} KRE=${KRE:-"k_bucket|k_sum_stats|k_survivor|k_compact2"} timeout -k 10 900 bash scripts/gpu_kvariants.sh || exit 1
if [ -n "$BENCH" ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 600 python $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/bench_quick.json 2> $GRAFT_REPO_ROOT/gpurun_out/bench_quick.err || { tail -30 $GRAFT_REPO_ROOT/gpurun_out/bench_quick.err; exit 1; }
  python - $GRAFT_REPO_ROOT/gpurun_out/bench_quick.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("ms_per_step", d["ms_per_step"], "value %.4g" % d["value"], "kernels_sum", d["roofline"]["kernels_sum_ms"])
print({k: (v["ms"], v["frac"]) for k, v in d["pipelines"].items() if v})
PY
fi
