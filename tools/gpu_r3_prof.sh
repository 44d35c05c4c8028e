#!/bin/bash
# GPU session: steady-state kernel stats of one model's bench step ($MODEL, extra env passed through).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
M=${MODEL:-gpt2_medium_fp8}; TAG=${TAG:-p}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof_$TAG -o run -- python3 $R/bench.py --model $M --steps 6 --warmup 3 > $OUT/prof_$TAG.log 2>&1 || { echo "prof failed"; tail -20 $OUT/prof_$TAG.log; exit 1; }
cd $R
F=$(find $OUT/prof_$TAG -name "*kernel_trace.csv" | head -1)
MK=optim_kernel; [ "$M" = resnet50 ] || MK=softmax_ce_fwd_kernel
python tools/steady_stats.py $F --marker $MK > $OUT/stats_$TAG.txt 2>&1; head -${HEAD:-60} $OUT/stats_$TAG.txt
[ "${KEEP:-0}" = "1" ] || rm -rf $OUT/prof_$TAG
