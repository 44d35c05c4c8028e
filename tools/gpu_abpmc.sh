#!/bin/bash
# GPU session: optional test subset ($K), A/B benches ($AB as in gpu_ab.sh), then per-step HBM traffic (FETCH_SIZE,
# WRITE_SIZE) of the default bench into gpurun_out/pmc_{1,2} (skip with PMC=0).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
bash tools/gpu_ab.sh || exit 1
if [ "${PMC:-1}" = "1" ]; then
  cd /tmp && export TMPDIR=/tmp
  i=0
  for ctr in FETCH_SIZE WRITE_SIZE; do
    i=$((i+1))
    timeout -s KILL 300 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d $OUT/pmc_$i -o run -- python3 $R/bench.py --steps 4 --warmup 3 ${PMC_ARGS:-} > $OUT/pmc_$i.log 2>&1 || { echo "pmc [$ctr] failed"; tail -20 $OUT/pmc_$i.log; exit 1; }
  done
  python3 $R/tools/hbm_bytes.py $OUT/pmc_1/run_counter_collection.csv $OUT/pmc_2/run_counter_collection.csv
fi
