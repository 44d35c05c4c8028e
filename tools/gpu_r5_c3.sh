# 3x3 convolution forward on the 4-wave implicit-GEMM kernel: conv / ResNet GPU tests and the ResNet-50 bench.
# bash tools/gpu_r5_c3.sh <tag>
set -o pipefail
mkdir -p gpurun_out
tag=${1:-r5c3}
timeout -k 10 400 python -u -m pytest -x -q -m gpu tests/test_kernels_gpu.py tests/test_resnet_gpu.py tests/test_pwconv_gpu.py tests/test_kernel_paths_gpu.py --timeout 200 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1 || { tail -30 gpurun_out/${tag}_tests.log; exit 1; }
tail -n 2 gpurun_out/${tag}_tests.log
for rnd in 1 2 3; do
  timeout -k 10 300 python -u bench.py --model resnet50 --steps 20 --warmup 5 > gpurun_out/${tag}_bench_${rnd}.log 2>&1 || { tail -20 gpurun_out/${tag}_bench_${rnd}.log; exit 1; }
  tail -n 1 gpurun_out/${tag}_bench_${rnd}.log | cut -c1-200
done
