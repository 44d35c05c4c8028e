#!/bin/bash
# GPU session: steady-state kernel stats of one model's bench step ($MODEL), the full GPU suite, the default bench.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
M=${MODEL:-gpt2_medium_fp8}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof_chk -o run -- python3 $R/bench.py --model $M --steps 6 --warmup 3 > $OUT/prof_chk.log 2>&1 || { echo "prof failed"; tail -20 $OUT/prof_chk.log; exit 1; }
cd $R
F=$(find $OUT/prof_chk -name "*kernel_trace.csv" | head -1)
MK=optim_kernel; [ "$M" = resnet50 ] || MK=softmax_ce_fwd_kernel; python tools/steady_stats.py $F --marker $MK > $OUT/stats_chk.txt 2>&1; head -45 $OUT/stats_chk.txt
rm -rf $OUT/prof_chk
timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread tests -m gpu > $OUT/gputests.log 2>&1; rc=$?; echo "gpu suite rc=$rc"; grep -E "FAILED|ERROR|passed|failed" $OUT/gputests.log | tail -20
[ $rc -le 1 ] || exit 1
timeout -k 10 300 python bench.py > $OUT/bench_chk.log 2>&1 || { echo "bench failed"; tail -20 $OUT/bench_chk.log; exit 1; }
tail -1 $OUT/bench_chk.log
