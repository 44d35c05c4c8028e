# ResNet-50 per-GPU batch sweep on the default (graph) step, interleaved: bash tools/gpu_r5_batch.sh <tag>
set -o pipefail
mkdir -p gpurun_out
tag=${1:-r5b}
for i in 1 2; do
  for b in 256 384 512; do
    timeout -k 10 300 python -u bench.py --model resnet50 --batch $b --steps 20 --warmup 5 > gpurun_out/${tag}_b${b}_$i.log 2>&1 || { tail -20 gpurun_out/${tag}_b${b}_$i.log; exit 1; }
    echo "batch $b run $i $(tail -n 1 gpurun_out/${tag}_b${b}_$i.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"].get("hipgraph"))')"
  done
done
