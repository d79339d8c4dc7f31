cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/sq
timeout -k 10 300 python $R/scripts/prof_replay.py --reps 1 --scale 0.25 > /dev/null || exit 1
KRE=${KRE:-"k_json_lines|k_snap_spec|k_snap_exec|k_bucket_verify|k_bucket_scatter|k_pq_data|k_ckpt_assemble"}
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY" "SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_ANY" "SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_BUSY_CU_CYCLES"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-include-regex "$KRE" -d $R/gpurun_out/sq/p$i -o pmc --output-format csv -- python $R/scripts/prof_replay.py --reps 1 --scale 0.25 > $R/gpurun_out/sq/p$i.log 2>&1 || { tail -5 $R/gpurun_out/sq/p$i.log; exit 1; }
done
python - $R/gpurun_out/sq <<'PY'
import csv, sys, collections, glob
acc = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].split("::")[-1]
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, d in acc.items():
    print(k, {c: "%.4g" % v for c, v in sorted(d.items())})
PY
