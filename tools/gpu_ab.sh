#!/bin/bash
# GPU session: optional test subset ($K), then A/B benches: each ';'-separated entry of $AB is "ENV=.. ENV2=..|bench args".
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
if [ -n "${K:-}" ]; then
  timeout -k 10 ${TT:-500} python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "$K" > $OUT/ab_tests.log 2>&1 || { echo "gpu tests failed"; grep -E "FAIL|Error|assert" $OUT/ab_tests.log | head -30; tail -5 $OUT/ab_tests.log; exit 1; }
  grep -c PASSED $OUT/ab_tests.log; tail -1 $OUT/ab_tests.log
fi
IFS=';' read -ra BL <<< "${AB:-}"
i=0
for e in "${BL[@]}"; do
  i=$((i+1)); envs="${e%%|*}"; args="${e#*|}"
  env $envs timeout -k 10 300 python bench.py $args > $OUT/ab_$i.log 2>&1 || { echo "bench [$e] failed"; tail -20 $OUT/ab_$i.log; exit 1; }
  echo "[$e] $(tail -1 $OUT/ab_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"].get("final_loss"))')"
done
