# hipGraph replay vs eager on the four bench configs: bash tools/gpu_r5_graph.sh <tag> [models...]
set -o pipefail
mkdir -p gpurun_out
tag=${1:-r5g}; shift
models=${@:-resnet50 bert_base gpt2_medium gpt2_medium_fp8}
for m in $models; do
  for g in 0 1; do
    timeout -k 10 300 python -u bench.py --model $m --steps 20 --warmup 5 --graph $g > gpurun_out/${tag}_${m}_g$g.log 2>&1 || { tail -20 gpurun_out/${tag}_${m}_g$g.log; exit 1; }
    echo "$m graph=$g $(tail -n 1 gpurun_out/${tag}_${m}_g$g.log | cut -c1-160)"
  done
done
