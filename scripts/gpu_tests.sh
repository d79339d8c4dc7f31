# GPU tests only: scripts/gpu_tests.sh [pytest selection ...] (default: every -m gpu test)
mkdir -p gpurun_out
SEL=${@:-tests}
timeout -k 10 900 python -u -m pytest $SEL -m gpu -x -v -rs --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -60 gpurun_out/gpu_tests.log; exit 1; }
tail -5 gpurun_out/gpu_tests.log
