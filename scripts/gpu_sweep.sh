# Sweep prebuilt variants of libdeltareplay.so (var_libs/<name>/): parity tests + bench per variant.
mkdir -p gpurun_out/sweep
cp delta_amd/libdeltareplay.so gpurun_out/sweep/base.so
for v in ${VARIANTS:-$(ls var_libs)}; do
  cp var_libs/$v/libdeltareplay.so delta_amd/libdeltareplay.so
  timeout -k 10 300 python -u -m pytest ${SWEEP_TESTS:-tests/test_gpu_parity.py} -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/sweep/$v.tests.log 2>&1 || { echo "$v tests FAILED"; tail -30 gpurun_out/sweep/$v.tests.log; cp gpurun_out/sweep/base.so delta_amd/libdeltareplay.so; exit 1; }
  echo "$v: $(tail -1 gpurun_out/sweep/$v.tests.log)"
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 > gpurun_out/sweep/$v.json 2> gpurun_out/sweep/$v.err || { echo "$v bench FAILED"; tail -20 gpurun_out/sweep/$v.err; cp gpurun_out/sweep/base.so delta_amd/libdeltareplay.so; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/sweep/$v.json').read().strip().splitlines()[-1]);k=d['kernels'];print('$v', d['ms_per_step'], {n: k[n]['ms'] for n in ('${SWEEP_KERNELS:-k_json_lines}'.split(',')) if n in k})"
done
cp gpurun_out/sweep/base.so delta_amd/libdeltareplay.so
