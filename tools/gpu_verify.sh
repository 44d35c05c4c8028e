#!/bin/bash
# Round-end rehearsal: GPU test suite, smoke(), default bench; stop at the first failure.
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/gputests.log 2>&1 || { echo "gpu tests failed"; tail -40 $OUT/gputests.log; exit 1; }
tail -3 $OUT/gputests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 400 python bench.py ${BENCH_ARGS:-} > $OUT/bench_default.log 2>&1 || { echo "bench failed"; tail -20 $OUT/bench_default.log; exit 1; }
tail -1 $OUT/bench_default.log
