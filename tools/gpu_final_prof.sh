#!/bin/bash
# GPU session: default benches of every BASELINE config, then rocprofv3 kernel stats + per-stream split of each.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
for m in resnet50 bert_base gpt2_medium gpt2_medium_fp8; do
  timeout -k 10 300 python bench.py --model $m > $OUT/final_bench_$m.log 2>&1 || { echo "bench $m failed"; tail -20 $OUT/final_bench_$m.log; exit 1; }
  tail -1 $OUT/final_bench_$m.log | cut -c1-160
done
cd /tmp && export TMPDIR=/tmp
for m in resnet50 bert_base gpt2_medium gpt2_medium_fp8; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/fprof_$m -o run -- python3 $R/bench.py --model $m --steps 4 --warmup 3 > $OUT/fprof_$m.log 2>&1 || { echo "prof $m failed"; tail -20 $OUT/fprof_$m.log; exit 1; }
done
echo profiled
