# PMC passes over the profiling driver (one counter group per run).
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
KRE=${KRE:-k_json_lines}
OUT=${OUT:-prof}
mkdir -p $R/gpurun_out/$OUT
timeout -k 10 300 python $R/scripts/prof_replay.py --reps 1 > /dev/null
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_FLAT SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES" "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"; do
  n=$(echo $grp | cut -c1-12 | tr ' ' '_')
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-include-regex "$KRE" -d $R/gpurun_out/$OUT/$n -o pmc -- python $R/scripts/prof_replay.py --reps 1 > $R/gpurun_out/$OUT/$n.log 2>&1 || echo "pass $n failed"
done
find $R/gpurun_out/$OUT -name "*.csv" | head
