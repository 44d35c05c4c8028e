#!/bin/bash
# One GPU session: smoke -> bench -> rocprofv3 kernel stats. Stops at the first failure.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed rc=$?"; tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 400 python bench.py --steps ${STEPS:-10} --warmup ${WARM:-3} ${BENCH_ARGS:-} > $OUT/bench.log 2>&1 || { echo "bench failed rc=$?"; tail -20 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log
if [ "${PROF:-1}" = "1" ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 $R/bench.py --steps 3 --warmup 2 ${BENCH_ARGS:-} > $OUT/prof.log 2>&1 || { echo "prof failed rc=$?"; tail -20 $OUT/prof.log; exit 1; }
  find $OUT/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} sh -c 'head -30 {}'
fi
