#!/bin/bash
# GPU session: BERT-base / GPT-2-medium bf16 / fp8 benches, then rocprofv3 kernel stats of the GPT-2 configs.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
for m in ${MODELS:-bert_base gpt2_medium gpt2_medium_fp8}; do
  timeout -k 10 300 python bench.py --model $m --steps 10 --warmup 3 > $OUT/bench_$m.log 2>&1 || { echo "bench $m failed"; tail -20 $OUT/bench_$m.log; exit 1; }
  tail -1 $OUT/bench_$m.log
done
cd /tmp && export TMPDIR=/tmp
for m in ${PMODELS:-gpt2_medium gpt2_medium_fp8}; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$m -o run -- python3 $R/bench.py --model $m --steps 4 --warmup 3 > $OUT/prof_$m.log 2>&1 || { echo "prof $m failed"; tail -20 $OUT/prof_$m.log; exit 1; }
  python3 $R/tools/kstats.py $OUT/prof_$m/run_kernel_stats.csv 7 40 > $OUT/kstats_$m.txt
done
