# 3x3 data gradients on the 4-wave gather kernel: conv / ResNet GPU tests, per-layer dgrad timing at batch 1024 and
# the ResNet-50 bench. bash tools/gpu_r5_dg.sh <tag>
set -o pipefail
mkdir -p gpurun_out
tag=${1:-r5dg}
timeout -k 10 400 python -u -m pytest -x -q -m gpu tests/test_kernels_gpu.py tests/test_resnet_gpu.py tests/test_kernel_paths_gpu.py --timeout 200 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1 || { tail -30 gpurun_out/${tag}_tests.log; exit 1; }
tail -n 2 gpurun_out/${tag}_tests.log
timeout -k 10 500 python -u tools/conv_roofline.py --batch 1024 --only dgrad --match c2 --tiles --tile-list 8,12 > gpurun_out/${tag}_dgrad.log 2>&1 || { tail -20 gpurun_out/${tag}_dgrad.log; exit 1; }
grep -v amdgpu gpurun_out/${tag}_dgrad.log
for rnd in 1 2; do
  timeout -k 10 300 python -u bench.py --model resnet50 --steps 20 --warmup 5 > gpurun_out/${tag}_bench_${rnd}.log 2>&1 || { tail -20 gpurun_out/${tag}_bench_${rnd}.log; exit 1; }
  tail -n 1 gpurun_out/${tag}_bench_${rnd}.log | cut -c1-200
done
