set -o pipefail
mkdir -p gpurun_out
tag=${1:-r5cm}
for i in 1 2; do
  for k in 0 8 16; do
    for m in bert_base resnet50; do
      DTF_SIDE_CU_SKIP=$k timeout -k 10 300 python -u bench.py --model $m --steps 10 --warmup 5 > gpurun_out/${tag}_${m}_${k}_$i.log 2>&1 || { tail -20 gpurun_out/${tag}_${m}_${k}_$i.log; exit 1; }
      echo "$m skip=$k run $i $(tail -n 1 gpurun_out/${tag}_${m}_${k}_$i.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
    done
  done
done
