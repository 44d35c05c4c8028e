# Full GPU validation on one MI355X: the GPU test suite, smoke(), the default bench (ResNet-50) and the transformer
# benches. Each step under its own time limit; stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
tag=${1:-r6}
timeout -k 10 900 python -u -m pytest tests/ -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/${tag}_gputests.log 2>&1 || { tail -40 gpurun_out/${tag}_gputests.log; exit 1; }
tail -n 3 gpurun_out/${tag}_gputests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${tag}_smoke.log 2>&1 || { tail -20 gpurun_out/${tag}_smoke.log; exit 1; }
tail -n 1 gpurun_out/${tag}_smoke.log
for m in resnet50 bert_base gpt2_medium gpt2_medium_fp8; do
  timeout -k 10 300 python -u bench.py --model $m --steps 20 --warmup 5 > gpurun_out/${tag}_bench_$m.log 2>&1 || { tail -20 gpurun_out/${tag}_bench_$m.log; exit 1; }
  tail -n 1 gpurun_out/${tag}_bench_$m.log | cut -c1-220
done
