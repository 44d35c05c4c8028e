#!/bin/bash
# GPU session: attention microbenchmark, BERT-base and GPT-2-medium (bf16, fp8) benches.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
timeout -k 10 200 python tools/bench_attention.py > $OUT/attn_b.log 2>&1 || { echo "attn bench failed"; tail -5 $OUT/attn_b.log; exit 1; }
grep -v amdgpu.ids $OUT/attn_b.log
for m in ${MODELS:-bert_base gpt2_medium gpt2_medium_fp8}; do
  env ${XENV:-} timeout -k 10 300 python bench.py --model $m --steps 10 --warmup 3 > $OUT/x_$m.log 2>&1 || { echo "bench failed"; tail -5 $OUT/x_$m.log; exit 1; }
  echo "$m $(tail -1 $OUT/x_$m.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"].get("final_loss"))')"
done
