#!/bin/bash
# GPU session: rocprofv3 kernel-trace stats of a short bench run ($BENCH_ARGS), summary printed by tools/kstats.py.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
rm -rf $OUT/prof
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 $R/bench.py --steps ${STEPS:-5} --warmup ${WARM:-5} ${BENCH_ARGS:-} > $OUT/prof.log 2>&1 || { echo "prof failed rc=$?"; tail -20 $OUT/prof.log; exit 1; }
cd $R
f=$(find $OUT/prof -name "*kernel_stats.csv" | head -1)
python tools/kstats.py $f $(( ${STEPS:-5} + ${WARM:-5} )) 60 > $OUT/kstats.txt && head -40 $OUT/kstats.txt
