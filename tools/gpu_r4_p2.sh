# round 4 session P2: GPT-2 / BERT knobs after the hipBLASLt routes: LN backward rows per block, attention dS path
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
n=0
for i in 1 2; do
  for e in "gpt2_medium X=1" "gpt2_medium DTF_LN_BWD_ROWS=16" "gpt2_medium DTF_LN_BWD_ROWS=8" "gpt2_medium DTF_ATTN_DS=0" "bert_base X=1" "bert_base DTF_LN_BWD_ROWS=16" "bert_base DTF_ATTN_DS=1"; do
    n=$((n+1)); set -- $e
    env $2 timeout -k 10 300 python bench.py --model $1 --steps 10 --warmup 3 > gpurun_out/r4p2_$n.log 2>&1 || exit 1
    grep '^{"metric"' gpurun_out/r4p2_$n.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(sys.argv[1], d["value"], d["ms_per_step"])' "$e"
  done
done
