set -o pipefail
mkdir -p gpurun_out
tag=${1:-r5s}
for i in 1 2; do
  for v in 0 1; do
    for m in bert_base gpt2_medium; do
      DTF_SPLIT_MODEL=$v timeout -k 10 300 python -u bench.py --model $m --steps 10 --warmup 5 > gpurun_out/${tag}_${m}_${v}_$i.log 2>&1 || { tail -20 gpurun_out/${tag}_${m}_${v}_$i.log; exit 1; }
      echo "$m DTF_SPLIT_MODEL=$v run $i $(tail -n 1 gpurun_out/${tag}_${m}_${v}_$i.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
    done
  done
done
