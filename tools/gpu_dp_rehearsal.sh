#!/bin/bash
# 2-rank rehearsal of the multi-GPU data path on one GPU (gloo between ranks sharing cuda:0),
# then the bench.py --gpus 2 relaunch path the driver uses for N>1.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_dp_gpu.py > $OUT/dp_tests.log 2>&1 || { echo "dp tests failed"; tail -40 $OUT/dp_tests.log; exit 1; }
tail -3 $OUT/dp_tests.log
DTF_COLLECTIVE_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --steps 3 --warmup 2 --batch 64 > $OUT/bench_dp2.log 2>&1 || { echo "bench dp2 failed"; tail -30 $OUT/bench_dp2.log; exit 1; }
tail -1 $OUT/bench_dp2.log
