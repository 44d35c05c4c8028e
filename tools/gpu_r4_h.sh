#!/bin/bash
# round-4 session H: deeper pwconv pipeline (tests + probe), graphs tests, bench, steady-state kernel stats
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
R=$GRAFT_REPO_ROOT
step() {
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $R/gpurun_out/r4h_$n.log 2>&1; local rc=$?
  echo "$n rc=$rc"
  if [ $rc -ge 124 ]; then echo "stopping after $n"; exit $rc; fi
}
step pwtest 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_pwconv_gpu.py tests/test_graphs.py
step bw 200 python tools/bw_probe.py
step roof 300 python tools/conv_roofline.py --only fwd
step bench 300 python bench.py
cd /tmp && export TMPDIR=/tmp
step prof 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r4h_prof -o run -- python3 $R/bench.py --steps 10 --warmup 5
cd $R
tail -3 gpurun_out/r4h_pwtest.log; grep "^s" gpurun_out/r4h_bw.log | cut -c1-140; grep -E "c2|c3|TOTAL" gpurun_out/r4h_roof.log
tail -1 gpurun_out/r4h_bench.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["host_issue_ms_single_step"])'
