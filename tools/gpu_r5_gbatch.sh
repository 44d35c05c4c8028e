set -o pipefail
mkdir -p gpurun_out
tag=${1:-r5g}
for m in gpt2_medium_fp8 gpt2_medium; do
  for b in 8 16 32; do
    timeout -k 10 300 python -u bench.py --model $m --batch $b --steps 15 --warmup 5 > gpurun_out/${tag}_${m}_b$b.log 2>&1 || { tail -20 gpurun_out/${tag}_${m}_b$b.log; exit 1; }
    echo "$m batch $b $(tail -n 1 gpurun_out/${tag}_${m}_b$b.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"].get("hipgraph"))')"
  done
done
