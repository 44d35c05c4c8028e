# split-K fixup threshold A/B (GPT-2-medium, eager): bash tools/gpu_r5_fix2.sh <tag>
set -o pipefail
mkdir -p gpurun_out
tag=${1:-r5fy}
for fx in 5 0 5 0 16; do
  timeout -k 10 300 python -u tools/bench_with.py native:dtf_set_split_fixup=$fx -- --model gpt2_medium --steps 20 --warmup 5 > gpurun_out/${tag}_$fx.log 2>&1 || { tail -20 gpurun_out/${tag}_$fx.log; exit 1; }
  echo "fix=$fx $(tail -n 1 gpurun_out/${tag}_$fx.log | cut -c1-110)"
done
