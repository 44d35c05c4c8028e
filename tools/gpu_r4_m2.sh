# round 4 session M2: per-bucket overlapped optimizer update A/B on the transformer benches (after the hipBLASLt routes)
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
n=0
for i in 1 2; do
  for e in "gpt2_medium X=1" "gpt2_medium DTF_OVERLAP_UPDATE=1" "bert_base X=1" "bert_base DTF_OVERLAP_UPDATE=1" "gpt2_medium_fp8 X=1" "gpt2_medium_fp8 DTF_OVERLAP_UPDATE=0"; do
    n=$((n+1)); set -- $e
    env $2 timeout -k 10 300 python bench.py --model $1 --steps 10 --warmup 3 > gpurun_out/r4m2_$n.log 2>&1 || exit 1
    grep '^{"metric"' gpurun_out/r4m2_$n.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(sys.argv[1], d["value"], d["ms_per_step"], d.get("host_issue_ms_single_step"))' "$e"
  done
done
