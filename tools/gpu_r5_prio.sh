set -o pipefail
mkdir -p gpurun_out
tag=${1:-r5p}
for i in 1 2; do
  for p in 0 1; do
    for m in bert_base gpt2_medium resnet50; do
      timeout -k 10 300 python -u bench.py --model $m --steps 10 --warmup 5 --hiprio $p > gpurun_out/${tag}_${m}_${p}_$i.log 2>&1 || { tail -20 gpurun_out/${tag}_${m}_${p}_$i.log; exit 1; }
      echo "$m hiprio=$p run $i $(tail -n 1 gpurun_out/${tag}_${m}_${p}_$i.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"].get("hipgraph"))')"
    done
  done
done
