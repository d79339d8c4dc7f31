# K3/K4 experiments: kernel times (rocprofv3 stats over prof_replay.py at SCALE) per bucket-bit
# setting (BITS list, the context option bucket_bits through PROF_OPTS) and per prebuilt variant (VARIANTS in var_libs/), plus
# WRITE_SIZE / FETCH_SIZE passes of the K3/K4 kernels at each bit setting.
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/k34
mkdir -p $O
SC=${SCALE:-1.0}
KRE=${KRE:-"k_bucket|k_compact2|k_survivor_scan|k_sum_stats"}
timeout -k 10 300 python $R/scripts/prof_replay.py --reps 1 --scale $SC > $O/gen.log 2>&1 || { tail -20 $O/gen.log; exit 1; }
summ() {
python - "$1" "$2" "$KRE" <<'PY'
import csv, re, sys, glob
fs = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)
rows = list(csv.DictReader(open(fs[0])))
pat = re.compile(sys.argv[3])
d = {r["Name"].split("(")[0].split("::")[-1].split("<")[0]: round(float(r["AverageNs"]) / 1e6, 4) for r in rows if pat.search(r["Name"])}
print(sys.argv[2], d, "sum=%.4f" % sum(d.values()), flush=True)
PY
}
pmc() {
python - "$1" "$2" <<'PY'
import csv, sys, glob, collections
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].split("::")[-1].split("<")[0]
        acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
print(sys.argv[2], {k: {c: "%.4g MB" % (sum(v) / len(v) / 1024) for c, v in d.items()} for k, d in acc.items()}, flush=True)
PY
}
for b in ${BITS:-13}; do
  [ "$b" = none ] && continue
  PROF_OPTS=bucket_bits=$b timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/bits$b -o run --output-format csv -- python $R/scripts/prof_replay.py --reps 3 --scale $SC > $O/bits$b.log 2>&1 || { echo "bits $b failed"; tail -5 $O/bits$b.log; exit 1; }
  summ $O/bits$b "bits=$b"
  if [ -n "$PMC" ]; then
    PROF_OPTS=bucket_bits=$b timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$KRE" -d $O/w$b -o pmc --output-format csv -- python $R/scripts/prof_replay.py --reps 1 --scale $SC > $O/w$b.log 2>&1 || { echo "pmc failed"; tail -5 $O/w$b.log; exit 1; }
    PROF_OPTS=bucket_bits=$b timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$KRE" -d $O/f$b -o pmc --output-format csv -- python $R/scripts/prof_replay.py --reps 1 --scale $SC > $O/f$b.log 2>&1 || { echo "pmc failed"; tail -5 $O/f$b.log; exit 1; }
    pmc $O/w$b "write bits=$b"
    pmc $O/f$b "fetch(x1) bits=$b"
  fi
done
if [ -n "$VARIANTS" ]; then
  cp $R/delta_amd/libdeltareplay.so $O/base.so
  for v in $VARIANTS; do
    cp $R/var_libs/$v/libdeltareplay.so $R/delta_amd/libdeltareplay.so
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/v_$v -o run --output-format csv -- python $R/scripts/prof_replay.py --reps 3 --scale $SC > $O/v_$v.log 2>&1 || { echo "$v failed"; tail -5 $O/v_$v.log; cp $O/base.so $R/delta_amd/libdeltareplay.so; exit 1; }
    summ $O/v_$v "variant=$v"
  done
  cp $O/base.so $R/delta_amd/libdeltareplay.so
fi
