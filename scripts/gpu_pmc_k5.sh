# PMC passes of K5 (k_filter_leaf) at config 4 scale 0.25: instruction mix / waits, then FETCH_SIZE
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pmc_k5
rm -rf $O && mkdir -p $O
timeout -k 10 300 python $R/scripts/prof_filter.py --scale 0.25 --reps 2 > $O/warm.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY --kernel-include-regex "k_filter_leaf" -d $O/p1 -o pmc --output-format csv -- python $R/scripts/prof_filter.py --scale 0.25 --reps 2 > $O/p1.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_filter_leaf" -d $O/p2 -o pmc --output-format csv -- python $R/scripts/prof_filter.py --scale 0.25 --reps 2 > $O/p2.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_WAIT_ANY SQ_INSTS_SMEM --kernel-include-regex "k_filter_leaf" -d $O/p3 -o pmc --output-format csv -- python $R/scripts/prof_filter.py --scale 0.25 --reps 2 > $O/p3.log 2>&1 || exit 1
python $R/scripts/pmc_by_kernel.py $O
