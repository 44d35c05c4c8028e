#!/bin/bash
# rocprofv3 kernel stats for the transformer configs (BERT-base, GPT-2-medium fp8).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for m in ${MODELS:-bert_base gpt2_medium_fp8}; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$m -o run -- python3 $R/bench.py --model $m --steps 3 --warmup 2 ${BENCH_ARGS:-} > $OUT/prof_$m.log 2>&1 || { echo "prof $m failed rc=$?"; tail -20 $OUT/prof_$m.log; exit 1; }
  tail -1 $OUT/prof_$m.log
done
