#!/bin/bash
# GPU session: steady-state kernel profiles of GPT-2-medium fp8 and bf16 (rocprofv3 kernel trace + tools/steady_stats.py)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p $OUT; cd /tmp && export TMPDIR=/tmp
for m in gpt2_medium_fp8 gpt2_medium; do
  timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof_$m -o run -- python3 $R/bench.py --model $m --steps 5 --warmup 3 > $OUT/prof_$m.log 2>&1 || { echo "prof $m failed"; tail -20 $OUT/prof_$m.log; exit 1; }
  (cd $R && python tools/steady_stats.py $(find $OUT/prof_$m -name "*kernel_trace.csv" | head -1) > $OUT/stats_$m.txt) && head -3 $OUT/stats_$m.txt
done
