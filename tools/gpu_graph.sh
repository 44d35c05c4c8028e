#!/bin/bash
# GPU session: GPU tests, then ResNet-50 bench eager vs hipGraph-captured.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
timeout -k 10 500 python -m pytest tests -m gpu -x -q > $OUT/gputests.log 2>&1 || { echo "gpu tests failed rc=$?"; tail -30 $OUT/gputests.log; exit 1; }
tail -2 $OUT/gputests.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/bench_eager.log 2>&1 || { echo "bench eager failed"; tail -20 $OUT/bench_eager.log; exit 1; }
tail -1 $OUT/bench_eager.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --graph 1 > $OUT/bench_graph.log 2>&1 || { echo "bench graph failed"; tail -20 $OUT/bench_graph.log; exit 1; }
tail -1 $OUT/bench_graph.log
