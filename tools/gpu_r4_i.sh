#!/bin/bash
# round-4 session I: full GPU suite, bench, steady-state kernel stats
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
R=$GRAFT_REPO_ROOT
step() {
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $R/gpurun_out/r4i_$n.log 2>&1; local rc=$?
  echo "$n rc=$rc"
  if [ $rc -ge 124 ]; then echo "stopping after $n"; exit $rc; fi
}
step bench 300 python bench.py
cd /tmp && export TMPDIR=/tmp
step prof 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r4i_prof -o run -- python3 $R/bench.py --steps 10 --warmup 5
cd $R
step tests 900 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread
tail -1 gpurun_out/r4i_bench.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["host_issue_ms_single_step"])'
grep -E "FAIL|passed|failed" gpurun_out/r4i_tests.log | tail -8
