#!/bin/bash
# GPU session: lazy BatchNorm outputs (gemm_core.h XF loaders) — kernel + bottleneck tests, the GPU suite, ResNet-50
# bench with lazy BN on / off, rocprofv3 kernel trace of the default bench (steady-state stats).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
T="python -u -m pytest -q --timeout 300 --timeout-method thread"
timeout -k 10 300 $T tests/test_lazy_bn_gpu.py > $OUT/t_lazy.log 2>&1; rc=$?; echo "lazy tests rc=$rc"; grep -E "FAILED|passed|failed|Error" $OUT/t_lazy.log | head -20
[ $rc -le 1 ] || exit 1
timeout -k 10 900 $T tests -m gpu > $OUT/gputests.log 2>&1; rc=$?; echo "gpu suite rc=$rc"; grep -E "FAILED|ERROR|passed|failed" $OUT/gputests.log | tail -20
[ $rc -le 1 ] || exit 1
timeout -k 10 300 python bench.py > $OUT/bench_lazy.log 2>&1 || { echo "bench failed"; tail -20 $OUT/bench_lazy.log; exit 1; }
tail -1 $OUT/bench_lazy.log
DTF_LAZY_BN=0 timeout -k 10 300 python bench.py > $OUT/bench_nolazy.log 2>&1 || { echo "bench nolazy failed"; tail -20 $OUT/bench_nolazy.log; exit 1; }
tail -1 $OUT/bench_nolazy.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof_lazy -o run -- python3 $R/bench.py --steps 6 --warmup 3 > $OUT/prof_lazy.log 2>&1 || { echo "prof failed"; tail -20 $OUT/prof_lazy.log; exit 1; }
cd $R && python tools/steady_stats.py $(find $OUT/prof_lazy -name "*kernel_trace.csv" | head -1) > $OUT/stats_lazy.txt && head -50 $OUT/stats_lazy.txt
