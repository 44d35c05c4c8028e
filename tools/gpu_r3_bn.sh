#!/bin/bash
# GPU session: lazy-BN kernel tests, BatchNorm pass bandwidths (tools/bench_bn.py), default ResNet-50 bench and its
# steady-state kernel profile.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
T="python -u -m pytest -q --timeout 300 --timeout-method thread"
timeout -k 10 300 $T tests/test_lazy_bn_gpu.py > $OUT/t_lazy.log 2>&1; rc=$?; echo "lazy tests rc=$rc"; grep -E "FAILED|passed|failed|Error" $OUT/t_lazy.log | head -20
[ $rc -le 1 ] || exit 1
timeout -k 10 300 python tools/bench_bn.py > $OUT/bench_bn.log 2>&1 || { echo "bench_bn failed"; tail -20 $OUT/bench_bn.log; exit 1; }
cat $OUT/bench_bn.log
timeout -k 10 300 python bench.py > $OUT/bench_base.log 2>&1 || { echo "bench failed"; tail -20 $OUT/bench_base.log; exit 1; }
tail -1 $OUT/bench_base.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof_base -o run -- python3 $R/bench.py --steps 6 --warmup 3 > $OUT/prof_base.log 2>&1 || { echo "prof failed"; tail -20 $OUT/prof_base.log; exit 1; }
cd $R && python tools/steady_stats.py $(find $OUT/prof_base -name "*kernel_trace.csv" | head -1) > $OUT/stats_base.txt && head -4 $OUT/stats_base.txt
