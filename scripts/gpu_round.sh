# Full GPU test suite, then the default bench line (with the CPU baseline), outputs under gpurun_out/
set -o pipefail
mkdir -p gpurun_out
bash scripts/gpu_tests.sh || exit 1
timeout -k 10 900 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -30 gpurun_out/bench.err; exit 1; }
tail -3 gpurun_out/bench.err
cat gpurun_out/bench.json
