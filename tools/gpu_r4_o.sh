#!/bin/bash
# round-4 session O: apply-by-recompute with the residual prefetched a tile ahead; staged C_in 128 pointwise
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
R=$GRAFT_REPO_ROOT
step() {
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $R/gpurun_out/r4o_$n.log 2>&1; local rc=$?
  echo "$n rc=$rc"
  if [ $rc -ge 124 ]; then echo "stopping after $n"; exit $rc; fi
}
step pwtest 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_pwconv_gpu.py
step bw 200 python tools/bw_probe.py
step b1 300 python bench.py
DTF_PW_APPLY=0 step b0 300 python bench.py
step b1b 300 python bench.py
DTF_PW_APPLY=0 step b0b 300 python bench.py
tail -2 gpurun_out/r4o_pwtest.log; grep "^s" gpurun_out/r4o_bw.log | cut -c1-120
for f in b1 b0 b1b b0b; do grep '^{"metric"' gpurun_out/r4o_$f.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("'$f'", d["value"], d["ms_per_step"], d["config"]["final_loss"])'; done
