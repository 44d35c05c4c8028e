#!/bin/bash
# Transformer configs on one GPU (each step bounded by its own timeout; stop at first failure).
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
timeout -k 10 400 python bench.py --model bert_base --steps ${STEPS:-5} --warmup 2 > $OUT/bench_bert.log 2>&1 || { echo "bert failed"; tail -20 $OUT/bench_bert.log; exit 1; }
tail -1 $OUT/bench_bert.log
timeout -k 10 400 python bench.py --model gpt2_medium_fp8 --steps ${STEPS:-5} --warmup 2 > $OUT/bench_gpt2.log 2>&1 || { echo "gpt2 failed"; tail -20 $OUT/bench_gpt2.log; exit 1; }
tail -1 $OUT/bench_gpt2.log
timeout -k 10 400 python bench.py --model gpt2_medium --steps ${STEPS:-5} --warmup 2 > $OUT/bench_gpt2bf16.log 2>&1 || { echo "gpt2 bf16 failed"; tail -20 $OUT/bench_gpt2bf16.log; exit 1; }
tail -1 $OUT/bench_gpt2bf16.log
