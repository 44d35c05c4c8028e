# transformer per-GPU batch sweep above the defaults (bench.py --batch), interleaved: bash tools/gpu_r5_tsweep.sh <tag>
set -o pipefail
mkdir -p gpurun_out
tag=${1:-r5ts}
for mb in gpt2_medium:32 gpt2_medium:64 gpt2_medium:48 gpt2_medium:32 gpt2_medium:64 bert_base:128 bert_base:256 bert_base:128 bert_base:256; do
  m=${mb%%:*}; b=${mb##*:}
  timeout -k 10 300 python -u bench.py --model $m --batch $b --steps 12 --warmup 4 > gpurun_out/${tag}_${m}_$b.log 2>&1 || { tail -20 gpurun_out/${tag}_${m}_$b.log; exit 1; }
  echo "$m b=$b $(tail -n 1 gpurun_out/${tag}_${m}_$b.log | grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' | tr '\n' ' ')"
done
