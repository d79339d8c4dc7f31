# SQ counters of the big kernels (one --pmc pass, scale 0.25 replays), printed per kernel
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/sq
timeout -k 10 300 python $R/scripts/prof_replay.py --reps 1 --scale 0.25 > /dev/null || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY --kernel-include-regex "k_json_lines|k_snap_emit|k_snap_spec|k_snap_exec" -d $R/gpurun_out/sq/p1 -o pmc --output-format csv -- python $R/scripts/prof_replay.py --reps 1 --scale 0.25 > $R/gpurun_out/sq/p1.log 2>&1 || { tail -5 $R/gpurun_out/sq/p1.log; exit 1; }
f=$(find $R/gpurun_out/sq/p1 -name "*counter_collection.csv" | head -1)
python - "$f" <<'PY'
import csv, sys, collections
acc = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open(sys.argv[1])):
    k = r["Kernel_Name"].split("(")[0].split("::")[-1]
    acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, d in acc.items():
    print(k, {c: "%.3g" % v for c, v in sorted(d.items())})
PY
