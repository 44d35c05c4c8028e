set -o pipefail
mkdir -p gpurun_out
tag=${1:-r5c}
for b in 512 768 1024; do
  timeout -k 10 300 python -u bench.py --model resnet50 --batch $b --steps 20 --warmup 5 > gpurun_out/${tag}_b${b}.log 2>&1 || { tail -20 gpurun_out/${tag}_b${b}.log; exit 1; }
  echo "batch $b $(tail -n 1 gpurun_out/${tag}_b${b}.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"].get("hipgraph"))')"
done
for s in 4 8; do
  DTF_FP8_WGRAD_SPLIT_MAX=$s timeout -k 10 300 python -u bench.py --model gpt2_medium_fp8 --steps 30 --warmup 5 > gpurun_out/${tag}_f8s$s.log 2>&1 || { tail -20 gpurun_out/${tag}_f8s$s.log; exit 1; }
  echo "fp8 split $s $(tail -n 1 gpurun_out/${tag}_f8s$s.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
