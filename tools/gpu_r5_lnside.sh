# LayerNorm [dgamma | dbeta] reduction on the side stream: transformer / graph GPU tests and the transformer benches.
# bash tools/gpu_r5_lnside.sh <tag>
set -o pipefail
mkdir -p gpurun_out
tag=${1:-r5ln}
timeout -k 10 600 python -u -m pytest -x -q -m gpu tests/test_graphs.py tests/test_model_training_gpu.py tests/test_kernel_paths_gpu.py tests/test_kernels_gpu.py --timeout 200 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1 || { tail -30 gpurun_out/${tag}_tests.log; exit 1; }
tail -n 2 gpurun_out/${tag}_tests.log
for m in bert_base gpt2_medium gpt2_medium_fp8; do
  timeout -k 10 300 python -u bench.py --model $m --steps 20 --warmup 5 > gpurun_out/${tag}_bench_$m.log 2>&1 || { tail -20 gpurun_out/${tag}_bench_$m.log; exit 1; }
  tail -n 1 gpurun_out/${tag}_bench_$m.log | cut -c1-200
done
