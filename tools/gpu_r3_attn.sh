#!/bin/bash
# GPU session: attention tests, attention microbenchmark with the keep-bits backward on / off, BERT-base and
# GPT-2-medium bench A/B (DTF_ATTN_DBITS).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_attention.py > $OUT/t_attn.log 2>&1 || { echo "attention tests failed"; tail -30 $OUT/t_attn.log; exit 1; }
tail -1 $OUT/t_attn.log
for d in 0 1; do
  DTF_ATTN_DBITS=$d timeout -k 10 200 python tools/bench_attention.py > $OUT/attn_b$d.log 2>&1 || { echo "attn bench failed"; tail -5 $OUT/attn_b$d.log; exit 1; }
  echo "== DTF_ATTN_DBITS=$d"; cat $OUT/attn_b$d.log
done
for m in bert_base gpt2_medium; do
  for d in 0 1 0 1; do
    DTF_ATTN_DBITS=$d timeout -k 10 300 python bench.py --model $m --steps 10 --warmup 3 > $OUT/ab_$m$d.log 2>&1 || { echo "bench failed"; tail -5 $OUT/ab_$m$d.log; exit 1; }
    echo "$m DTF_ATTN_DBITS=$d $(tail -1 $OUT/ab_$m$d.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"].get("final_loss"))')"
  done
done
