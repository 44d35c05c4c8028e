#!/bin/bash
# GPU session: full GPU test suite, default ResNet-50 bench, steady-state kernel profile of it.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
T="python -u -m pytest -q --timeout 300 --timeout-method thread"
timeout -k 10 900 $T tests -m gpu > $OUT/gputests.log 2>&1; rc=$?; echo "gpu suite rc=$rc"; grep -E "FAILED|ERROR|passed|failed" $OUT/gputests.log | tail -20
[ $rc -le 1 ] || exit 1
timeout -k 10 300 python bench.py > $OUT/bench_v.log 2>&1 || { echo "bench failed"; tail -20 $OUT/bench_v.log; exit 1; }
tail -1 $OUT/bench_v.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof_v -o run -- python3 $R/bench.py --steps 6 --warmup 3 > $OUT/prof_v.log 2>&1 || { echo "prof failed"; tail -20 $OUT/prof_v.log; exit 1; }
cd $R && python tools/steady_stats.py $(find $OUT/prof_v -name "*kernel_trace.csv" | head -1) > $OUT/stats_v.txt && head -3 $OUT/stats_v.txt
