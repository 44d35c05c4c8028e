# GPT-2-medium fp8 with the 4-wave fp8 kernel vs the 8-wave one, and the bf16 run, eager and per-stream graph:
# bash tools/gpu_r5_fp8ab.sh <tag>
set -o pipefail
mkdir -p gpurun_out
tag=${1:-r5f}
run() {  # name, env..., -- bench args
  local name=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 $BARGS > gpurun_out/${tag}_$name.log 2>&1 || { tail -20 gpurun_out/${tag}_$name.log; exit 1; }
  echo "$name $(tail -n 1 gpurun_out/${tag}_$name.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"].get("hipgraph"))')"
}
for g in 0 1; do
  BARGS="--model gpt2_medium_fp8 --graph $g" run fp8w4_g$g DTF_FP8_W4=1
  BARGS="--model gpt2_medium_fp8 --graph $g" run fp8old_g$g DTF_FP8_W4=0
  BARGS="--model gpt2_medium --graph $g" run bf16_g$g DTF_FP8_W4=1
done
