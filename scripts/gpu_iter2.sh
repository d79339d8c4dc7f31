# GPU tests (selection), then the bench line, then the same bench with DR_OVERLAP=1 (K1 on a second stream)
set -o pipefail
mkdir -p gpurun_out/iter
SEL=${1:-tests/test_gpu_edge_cases.py tests/test_gpu_parity.py}
timeout -k 10 600 python -u -m pytest $SEL -m gpu -x -v -rs --timeout 240 --timeout-method thread > gpurun_out/iter/tests.log 2>&1 || { tail -60 gpurun_out/iter/tests.log; exit 1; }
tail -3 gpurun_out/iter/tests.log
summ() {
python - "$1" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d["kernels"]
print(sys.argv[1], "ms/step", d["ms_per_step"], "value", d["value"], "roofline", d["roofline"]["kernel"], d["roofline"]["frac"])
print({n: round(v["ms"], 4) for n, v in sorted(k.items(), key=lambda kv: -kv[1]["ms"])[:16]})
PY
}
timeout -k 10 600 python bench.py --no-cpu-baseline > gpurun_out/iter/bench.json 2> gpurun_out/iter/bench.err || { tail -30 gpurun_out/iter/bench.err; exit 1; }
summ gpurun_out/iter/bench.json
DR_OVERLAP=1 timeout -k 10 600 python bench.py --no-cpu-baseline > gpurun_out/iter/bench_ov.json 2> gpurun_out/iter/bench_ov.err || { tail -30 gpurun_out/iter/bench_ov.err; exit 1; }
summ gpurun_out/iter/bench_ov.json
