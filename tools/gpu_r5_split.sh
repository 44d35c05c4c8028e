# split-K penalty of the dense weight-gradient plan (gemm.hip plan_w4_split, native:dtf_set_split_penalty), interleaved
# bash tools/gpu_r5_split.sh <tag>
set -o pipefail
mkdir -p gpurun_out
tag=${1:-r5sp}
for m in gpt2_medium bert_base; do
  for pen in ${PENS:-30 80 200 30 80 200}; do
    timeout -k 10 300 python -u tools/bench_with.py native:dtf_set_split_penalty=$pen -- --model $m --steps 20 --warmup 5 > gpurun_out/${tag}_${m}_$pen.log 2>&1 || { tail -20 gpurun_out/${tag}_${m}_$pen.log; exit 1; }
    echo "$m pen=$pen $(tail -n 1 gpurun_out/${tag}_${m}_$pen.log | cut -c1-110)"
  done
done
