#!/bin/bash
# round-4 session J2: graph tests + bench A/B of the side-stream projection
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
R=$GRAFT_REPO_ROOT
step() {
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $R/gpurun_out/r4j_$n.log 2>&1; local rc=$?
  echo "$n rc=$rc"
  if [ $rc -ge 124 ]; then echo "stopping after $n"; exit $rc; fi
}
step gtests 300 python -u -m pytest tests/test_graphs.py tests/test_resnet_gpu.py tests/test_dp_gpu.py -x -v --timeout 150 --timeout-method thread
step bench1 300 python bench.py
DTF_PROJ_SIDE=0 step bench0 300 python bench.py
step bench1b 300 python bench.py
grep -E "FAIL|passed|failed" gpurun_out/r4j_gtests.log | tail -8
for f in bench1 bench0 bench1b; do tail -1 gpurun_out/r4j_$f.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"]["final_loss"])'; done
