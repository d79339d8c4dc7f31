# k_snap_exec phase clocks (DR_SNAP_DEBUG=1) and kernel times (names matching KPAT, default k_snap)
# of the current library and of each var_libs/ variant (scripts/build_variant.sh), over
# scripts/prof_replay.py at SCALE (default 0.25)
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/snapvar
cp $R/delta_amd/libdeltareplay.so $R/gpurun_out/snapvar/base.so
timeout -k 10 300 python $R/scripts/prof_replay.py --reps 1 --scale ${SCALE:-0.25} > /dev/null || exit 1
mkdir -p $R/var_libs/base && cp $R/gpurun_out/snapvar/base.so $R/var_libs/base/libdeltareplay.so
for v in ${VARIANTS:-$(ls $R/var_libs)}; do
  cp $R/var_libs/$v/libdeltareplay.so $R/delta_amd/libdeltareplay.so
  DR_SNAP_DEBUG=1 timeout -k 10 300 python $R/scripts/prof_replay.py --reps 2 --scale ${SCALE:-0.25} > $R/gpurun_out/snapvar/$v.dbg 2>&1 || { echo "$v failed"; tail -5 $R/gpurun_out/snapvar/$v.dbg; break; }
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/snapvar/$v -o run --output-format csv -- python $R/scripts/prof_replay.py --reps 3 --scale ${SCALE:-0.25} > $R/gpurun_out/snapvar/$v.log 2>&1 || { echo "$v failed"; tail -5 $R/gpurun_out/snapvar/$v.log; break; }
  f=$(find $R/gpurun_out/snapvar/$v -name "*kernel_stats.csv" | head -1)
  echo "== $v: $(grep -m1 'exec phases' $R/gpurun_out/snapvar/$v.dbg) bad: $(grep -c 'bad page' $R/gpurun_out/snapvar/$v.dbg)"
  python - "$f" "${KPAT:-k_snap}" <<'PY'
import csv, re, sys
rows = list(csv.DictReader(open(sys.argv[1])))
print({r["Name"].split("(")[0].split("::")[-1]: round(float(r["AverageNs"]) / 1e6, 4) for r in rows if re.search(sys.argv[2], r["Name"])})
PY
done
cp $R/gpurun_out/snapvar/base.so $R/delta_amd/libdeltareplay.so
