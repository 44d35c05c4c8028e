# interleaved eager vs per-stream hipGraph A/B on one model: bash tools/gpu_r5_graphab.sh <tag> <model> [reps]
set -o pipefail
mkdir -p gpurun_out
tag=${1:-r5ga}; m=${2:-resnet50}; reps=${3:-3}
for i in $(seq 1 $reps); do
  for g in 0 1; do
    timeout -k 10 300 python -u bench.py --model $m --steps 30 --warmup 5 --graph $g > gpurun_out/${tag}_${m}_g${g}_$i.log 2>&1 || { tail -20 gpurun_out/${tag}_${m}_g${g}_$i.log; exit 1; }
    echo "$m graph=$g run $i $(tail -n 1 gpurun_out/${tag}_${m}_g${g}_$i.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
