#!/bin/bash
# GPU session: HBM traffic of the default ResNet-50 bench step (rocprofv3 PMC, one counter group per run).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for ctr in "FETCH_SIZE" "WRITE_SIZE" "GRBM_GUI_ACTIVE SQ_BUSY_CYCLES"; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d $OUT/pmc_$i -o run -- python3 $R/bench.py --steps 4 --warmup 3 > $OUT/pmc_$i.log 2>&1 || { echo "pmc [$ctr] failed"; tail -20 $OUT/pmc_$i.log; exit 1; }
  echo "[$ctr] done"
done
