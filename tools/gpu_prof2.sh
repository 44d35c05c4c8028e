#!/bin/bash
# GPU session: rocprofv3 kernel traces of bench configs ($CFGS: ';'-separated bench arg lists) into gpurun_out/prof_<i>.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
IFS=';' read -ra CL <<< "${CFGS:-}"
i=0
for c in "${CL[@]}"; do
  i=$((i+1))
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$i -o run -- python3 $R/bench.py $c > $OUT/prof_$i.log 2>&1 || { echo "prof [$c] failed"; tail -20 $OUT/prof_$i.log; exit 1; }
  echo "[$c] $(tail -1 $OUT/prof_$i.log | cut -c1-200)"
  python3 $R/tools/timeline.py $OUT/prof_$i/run_kernel_trace.csv 3 8 || true
done
