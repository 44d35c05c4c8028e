# Epilogue store fast paths (w4 / fp8 w4 / generic): GEMM/conv GPU tests, the w4 K sweep and
# the three end-to-end benches. bash tools/gpu_r5_epi2.sh <tag>
set -o pipefail
mkdir -p gpurun_out
tag=${1:-r5e2}
timeout -k 10 400 python -u -m pytest -x -q -m gpu tests/test_kernels_gpu.py tests/test_fp8_fused_gpu.py --timeout 120 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1 || { tail -30 gpurun_out/${tag}_tests.log; exit 1; }
tail -n 2 gpurun_out/${tag}_tests.log
timeout -k 10 200 python -u tools/bench_gemm_w4.py --sweepk 16384x3072 > gpurun_out/${tag}_sweepk.log 2>&1 || exit 1
for m in bert_base gpt2_medium resnet50; do
  timeout -k 10 300 python -u bench.py --model $m --steps 20 --warmup 5 > gpurun_out/${tag}_bench_$m.log 2>&1 || { tail -20 gpurun_out/${tag}_bench_$m.log; exit 1; }
  tail -n 1 gpurun_out/${tag}_bench_$m.log | cut -c1-200
done
