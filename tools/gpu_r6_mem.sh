# HBM bytes per step of the ResNet-50 bench, then eager (uncaptured) steps on a created stream and on the default stream
set -o pipefail
mkdir -p gpurun_out
bash tools/gpu_hbm.sh r6_hbm || exit 1
timeout -k 10 200 python -u tools/eager_mem_probe.py 1024 5 stream > gpurun_out/eager_1024s.log 2>&1; rc=$?; grep step gpurun_out/eager_1024s.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 200 python -u tools/eager_mem_probe.py 1024 5 > gpurun_out/eager_1024.log 2>&1; rc=$?; grep step gpurun_out/eager_1024.log; [ $rc -eq 0 ] || exit 1
