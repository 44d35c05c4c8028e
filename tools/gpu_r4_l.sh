#!/bin/bash
# round-4 session L: PMC counters of three conv forward kernels (one counter pass per run, no traces)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --kernel-trace --output-format csv -d $OUT/pmcc_1 -o run -- python3 $R/tools/pmc_conv.py > $OUT/pmcc_1.log 2>&1 || { echo "pmc pass 1 failed"; tail -20 $OUT/pmcc_1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv -d $OUT/pmcc_2 -o run -- python3 $R/tools/pmc_conv.py > $OUT/pmcc_2.log 2>&1 || { echo "pmc pass 2 failed"; tail -20 $OUT/pmcc_2.log; exit 1; }
cd $R/tools
python3 pmc_conv.py --summary $(find $OUT/pmcc_1 $OUT/pmcc_2 -name "*counter_collection.csv") | tee $OUT/pmcc_summary.txt
