# Config-4 full-record parity (GPU record sums vs the C++ restatement) at several scales (SCALES),
# the restatement on CPUT threads (default: all)
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/c4p
cd /tmp && export TMPDIR=/tmp
for sc in ${SCALES:-0.001 0.05 0.3}; do
  timeout -k 10 500 python -u $R/bench.py --config 4 --scale $sc --steps 1 --warmup 0 ${CPUT:+--cpu-threads $CPUT} > $R/gpurun_out/c4p/s$sc.json 2> $R/gpurun_out/c4p/s$sc.err || { echo "scale $sc failed"; tail -5 $R/gpurun_out/c4p/s$sc.err; exit 1; }
  grep -a "MISMATCH" $R/gpurun_out/c4p/s$sc.err || echo "scale $sc: records match"
done
