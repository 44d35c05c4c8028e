#!/bin/bash
# GPU session: PS data-plane tests, then 1-GPU ResNet-50 ParameterServerStrategy rehearsals (shm/IPC transport).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
timeout -k 10 400 python -u -m pytest tests/test_ps_gpu.py -x -v --timeout 200 --timeout-method thread > $OUT/ps_tests.log 2>&1 || { echo "ps tests failed"; tail -40 $OUT/ps_tests.log; exit 1; }
tail -3 $OUT/ps_tests.log
timeout -k 10 400 python tools/bench_ps.py --gpus 1 --ps 1 --trainers 3 --steps 10 --warmup 3 --batch 128 --timeout 350 > $OUT/bench_ps_gpu.log 2>&1 || { echo "bench_ps gpu failed"; tail -30 $OUT/bench_ps_gpu.log; exit 1; }
grep '"metric"' $OUT/bench_ps_gpu.log
timeout -k 10 400 python tools/bench_ps.py --gpus 1 --ps_cpu --trainers 2 --steps 5 --warmup 2 --batch 128 --timeout 350 > $OUT/bench_ps_cpu.log 2>&1 || { echo "bench_ps cpu-ps failed"; tail -30 $OUT/bench_ps_cpu.log; exit 1; }
grep '"metric"' $OUT/bench_ps_cpu.log
