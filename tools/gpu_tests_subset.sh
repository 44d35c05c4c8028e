#!/bin/bash
# GPU session: a subset of the GPU tests (pytest -k "$K"), then optional bench runs ($BENCHES: ';'-separated arg lists).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
timeout -k 10 ${TT:-500} python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ${K:+-k "$K"} > $OUT/gputests.log 2>&1 || { echo "gpu tests failed"; grep -E "PASS|FAIL|ERROR|Error|assert" $OUT/gputests.log | tail -40; exit 1; }
grep -cE "PASSED" $OUT/gputests.log; tail -2 $OUT/gputests.log
IFS=';' read -ra BL <<< "${BENCHES:-}"
i=0
for b in "${BL[@]}"; do
  i=$((i+1))
  timeout -k 10 300 python bench.py $b > $OUT/bench_$i.log 2>&1 || { echo "bench $b failed"; tail -20 $OUT/bench_$i.log; exit 1; }
  echo "[$b]"; tail -1 $OUT/bench_$i.log
done
