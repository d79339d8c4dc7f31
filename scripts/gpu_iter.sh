# One build-measure iteration: the selected GPU tests, then the bench without the CPU baseline.
# scripts/gpu_iter.sh "<pytest selection>"   (outputs under gpurun_out/iter/)
set -o pipefail
mkdir -p gpurun_out/iter
SEL=${1:-tests/test_gpu_edge_cases.py tests/test_gpu_parity.py}
timeout -k 10 600 python -u -m pytest $SEL -m gpu -x -v -rs --timeout 240 --timeout-method thread > gpurun_out/iter/tests.log 2>&1 || { tail -60 gpurun_out/iter/tests.log; exit 1; }
tail -3 gpurun_out/iter/tests.log
timeout -k 10 600 python bench.py --no-cpu-baseline > gpurun_out/iter/bench.json 2> gpurun_out/iter/bench.err || { tail -30 gpurun_out/iter/bench.err; exit 1; }
python - <<'PY'
import json
d = json.loads(open("gpurun_out/iter/bench.json").read().strip().splitlines()[-1])
k = d["kernels"]
print("ms/step", d["ms_per_step"], "value", d["value"], "roofline", d["roofline"]["kernel"], d["roofline"]["frac"])
print({n: round(v["ms"], 4) for n, v in sorted(k.items(), key=lambda kv: -kv[1]["ms"])[:14]})
PY
