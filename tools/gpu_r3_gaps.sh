#!/bin/bash
# GPU session: rocprofv3 kernel trace of the default ResNet-50 bench -> step timeline (GPU-idle gaps by the kernel
# that precedes them) and steady-state kernel stats.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
M=${MODEL:-resnet50}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof_gaps -o run -- python3 $R/bench.py --model $M --steps 6 --warmup 3 ${BARGS:-} > $OUT/prof_gaps.log 2>&1 || { echo "prof failed"; tail -20 $OUT/prof_gaps.log; exit 1; }
tail -1 $OUT/prof_gaps.log
cd $R
F=$(find $OUT/prof_gaps -name "*kernel_trace.csv" | head -1)
python tools/timeline.py $F 3 25 > $OUT/timeline_gaps.txt 2>&1; head -120 $OUT/timeline_gaps.txt
python tools/steady_stats.py $F > $OUT/stats_gaps.txt 2>&1
