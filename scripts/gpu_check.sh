# GPU tests (optionally a selection: scripts/gpu_check.sh <pytest args>), then a short bench line
# without the CPU baseline; outputs under gpurun_out/
set -o pipefail
mkdir -p gpurun_out
SEL=${@:-tests}
timeout -k 10 900 python -u -m pytest $SEL -m gpu -x -q -rs --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -60 gpurun_out/gpu_tests.log; exit 1; }
tail -4 gpurun_out/gpu_tests.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 python $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/bench_quick.json 2> $GRAFT_REPO_ROOT/gpurun_out/bench_quick.err || { tail -30 $GRAFT_REPO_ROOT/gpurun_out/bench_quick.err; exit 1; }
python - $GRAFT_REPO_ROOT/gpurun_out/bench_quick.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("ms_per_step", d["ms_per_step"], "value %.4g" % d["value"], "kernels_sum", d["roofline"]["kernels_sum_ms"],
      "e2e", d["end_to_end"])
print({k: v["ms"] for k, v in d["kernels"].items() if v["ms"] > 0.05})
print({k: (v["ms"], v["frac"]) for k, v in d["pipelines"].items() if v})
PY
