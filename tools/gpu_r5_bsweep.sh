# ResNet-50 per-GPU batch sweep above the default (bench.py --batch), interleaved: bash tools/gpu_r5_bsweep.sh <tag>
set -o pipefail
mkdir -p gpurun_out
tag=${1:-r5bs}
for b in 1024 1536 1280 1024 1536 1280; do
  timeout -k 10 300 python -u bench.py --model resnet50 --batch $b --steps 20 --warmup 5 > gpurun_out/${tag}_$b.log 2>&1 || { tail -20 gpurun_out/${tag}_$b.log; exit 1; }
  echo "b=$b $(tail -n 1 gpurun_out/${tag}_$b.log | grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|peak[^,]*' | tr '\n' ' ')"
done
