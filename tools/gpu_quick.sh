#!/bin/bash
# GPU session: kernel tests (optionally filtered by $K), then one bench config ($BENCH_ARGS).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
timeout -k 10 600 python -m pytest tests -m gpu -x -q ${K:+-k "$K"} > $OUT/gputests.log 2>&1 || { echo "gpu tests failed rc=$?"; tail -40 $OUT/gputests.log; exit 1; }
tail -2 $OUT/gputests.log
if [ -n "${BENCH_ARGS:-}" ]; then
  timeout -k 10 400 python bench.py $BENCH_ARGS > $OUT/bench_q.log 2>&1 || { echo "bench failed"; tail -20 $OUT/bench_q.log; exit 1; }
  tail -1 $OUT/bench_q.log
fi
