# Kernel times of prebuilt library variants (var_libs/<name>/) without parity checks: rocprofv3
# kernel-trace stats over scripts/prof_replay.py per variant. KRE selects the kernels reported.
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/kvar
cp $R/delta_amd/libdeltareplay.so $R/gpurun_out/kvar/base.so
timeout -k 10 300 python $R/scripts/${DRIVER:-prof_replay.py} --reps 1 --scale ${SCALE:-0.25} > /dev/null || exit 1
mkdir -p $R/var_libs/base && cp $R/gpurun_out/kvar/base.so $R/var_libs/base/libdeltareplay.so
for v in ${VARIANTS:-$(ls $R/var_libs)}; do
  cp $R/var_libs/$v/libdeltareplay.so $R/delta_amd/libdeltareplay.so
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/kvar/$v -o run --output-format csv -- python $R/scripts/${DRIVER:-prof_replay.py} --reps 3 --scale ${SCALE:-0.25} > $R/gpurun_out/kvar/$v.log 2>&1 || { echo "$v failed"; tail -5 $R/gpurun_out/kvar/$v.log; break; }
  f=$(find $R/gpurun_out/kvar/$v -name "*kernel_stats.csv" | head -1)
  python - "$f" "$v" "${KRE:-k_json_lines}" <<'PY'
import csv, re, sys
rows = list(csv.DictReader(open(sys.argv[1])))
pat = re.compile(sys.argv[3])
print(sys.argv[2], {r["Name"].split("(")[0].split("::")[-1]: round(float(r["AverageNs"]) / 1e6, 4) for r in rows if pat.search(r["Name"])})
PY
done
cp $R/gpurun_out/kvar/base.so $R/delta_amd/libdeltareplay.so
