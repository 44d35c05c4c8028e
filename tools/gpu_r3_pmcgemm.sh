#!/bin/bash
# GPU session: PMC counters of the 256-row GEMM kernel on BERT-base FFN1 shapes (one counter pass per run).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --kernel-trace --output-format csv -d $OUT/pmcg_1 -o run -- python3 $R/tools/pmc_gemm.py > $OUT/pmcg_1.log 2>&1 || { echo "pmc pass 1 failed"; tail -20 $OUT/pmcg_1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $OUT/pmcg_2 -o run -- python3 $R/tools/pmc_gemm.py > $OUT/pmcg_2.log 2>&1 || { echo "pmc pass 2 failed"; tail -20 $OUT/pmcg_2.log; exit 1; }
cd $R
python3 tools/pmc_gemm.py --summary $(find $OUT/pmcg_1 $OUT/pmcg_2 -name "*counter_collection.csv") | tee $OUT/pmcg_summary.txt
