# GPT-2-medium fp8 (graph replay): overlapped per-bucket update and weight-gradient split-K, interleaved
set -o pipefail
mkdir -p gpurun_out
tag=${1:-r5k}
for i in 1 2; do
  for cfg in "base" "ovl DTF_OVERLAP_UPDATE=1" "split2 DTF_FP8_WGRAD_SPLIT_MAX=2" "split4 DTF_FP8_WGRAD_SPLIT_MAX=4"; do
    set -- $cfg; name=$1; shift
    env "$@" timeout -k 10 300 python -u bench.py --model gpt2_medium_fp8 --steps 30 --warmup 5 > gpurun_out/${tag}_${name}_$i.log 2>&1 || { tail -20 gpurun_out/${tag}_${name}_$i.log; exit 1; }
    echo "$name run $i $(tail -n 1 gpurun_out/${tag}_${name}_$i.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"].get("hipgraph"))')"
  done
done
