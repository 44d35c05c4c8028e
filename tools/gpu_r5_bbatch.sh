set -o pipefail
mkdir -p gpurun_out
tag=${1:-r5h}
for b in 32 64 128; do
  timeout -k 10 300 python -u bench.py --model bert_base --batch $b --steps 15 --warmup 5 > gpurun_out/${tag}_bert_b$b.log 2>&1 || { tail -20 gpurun_out/${tag}_bert_b$b.log; exit 1; }
  echo "bert batch $b $(tail -n 1 gpurun_out/${tag}_bert_b$b.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"].get("hipgraph"))')"
done
for g in 0 1; do
  timeout -k 10 300 python -u bench.py --model gpt2_medium --batch 32 --graph $g --steps 15 --warmup 5 > gpurun_out/${tag}_gpt2_b32_g$g.log 2>&1 || { tail -20 gpurun_out/${tag}_gpt2_b32_g$g.log; exit 1; }
  echo "gpt2 b32 graph $g $(tail -n 1 gpurun_out/${tag}_gpt2_b32_g$g.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"].get("hipgraph"))')"
done
timeout -k 10 300 python -u bench.py --model gpt2_medium_fp8 --batch 32 --graph 0 --steps 15 --warmup 5 > gpurun_out/${tag}_f8_b32_g0.log 2>&1 || exit 1
echo "fp8 b32 graph 0 $(tail -n 1 gpurun_out/${tag}_f8_b32_g0.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"].get("hipgraph"))')"
