# Attention dropout path A/B: attention GPU tests, tools/bench_attention.py and the transformer benches.
# bash tools/gpu_r5_attn.sh <tag>
set -o pipefail
mkdir -p gpurun_out
tag=${1:-r5at}
timeout -k 10 300 python -u -m pytest -x -q -m gpu tests/test_attention.py --timeout 120 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1 || { tail -30 gpurun_out/${tag}_tests.log; exit 1; }
tail -n 2 gpurun_out/${tag}_tests.log
timeout -k 10 200 python -u tools/bench_attention.py > gpurun_out/${tag}_attn.log 2>&1 || { tail -20 gpurun_out/${tag}_attn.log; exit 1; }
cat gpurun_out/${tag}_attn.log
for m in bert_base gpt2_medium; do
  timeout -k 10 300 python -u bench.py --model $m --steps 20 --warmup 5 > gpurun_out/${tag}_bench_$m.log 2>&1 || { tail -20 gpurun_out/${tag}_bench_$m.log; exit 1; }
  tail -n 1 gpurun_out/${tag}_bench_$m.log | cut -c1-200
done
