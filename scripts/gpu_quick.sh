# GPU parity tests, then kernel-trace statistics of the profiling driver (no bench run).
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
SCALE=${SCALE:-1.0} bash scripts/gpu_stats.sh
