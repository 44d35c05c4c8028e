#!/bin/bash
# PMC passes (one counter set per run) over single ResNet-50 convs. Usage: CONVS="s3bX.c2:fwd s1bX.c2:wgrad"
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out/pmc; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for cv in ${CONVS}; do
  n=${cv%%:*}; k=${cv##*:}
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS --output-format csv -d $OUT/${n}_${k} -o p -- python3 $R/tools/conv_one.py $n $k 10 > $OUT/${n}_${k}.log 2>&1 || { echo "pmc $cv failed"; tail -5 $OUT/${n}_${k}.log; exit 1; }
  timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_BUSY_CYCLES --output-format csv -d $OUT/${n}_${k}_b -o p -- python3 $R/tools/conv_one.py $n $k 10 > $OUT/${n}_${k}_b.log 2>&1 || { echo "pmc2 $cv failed"; tail -5 $OUT/${n}_${k}_b.log; exit 1; }
done
echo ok
