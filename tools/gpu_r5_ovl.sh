# Overlapped per-bucket optimizer update A/B (DTF_OVERLAP_UPDATE 0 / 1), interleaved, default batches.
# bash tools/gpu_r5_ovl.sh <tag> [models]
set -o pipefail
mkdir -p gpurun_out
tag=${1:-r5ov}; models=${2:-gpt2_medium_fp8 bert_base gpt2_medium resnet50}
for rnd in 1 2; do
  for m in $models; do
    for v in 0 1; do
      DTF_OVERLAP_UPDATE=$v timeout -k 10 300 python -u bench.py --model $m --steps 15 --warmup 5 > gpurun_out/${tag}_${m}_${v}_${rnd}.log 2>&1 || { tail -20 gpurun_out/${tag}_${m}_${v}_${rnd}.log; exit 1; }
      echo "$m ovl=$v round $rnd: $(tail -n 1 gpurun_out/${tag}_${m}_${v}_${rnd}.log | cut -c1-150 | grep -o '"value": [0-9.]*')"
    done
  done
done
