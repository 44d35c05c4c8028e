#!/bin/bash
# round-4 session D: P2P race fix check, per-step weight diff of the captured overlapped update, host issue time
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
R=$GRAFT_REPO_ROOT
step() {  # step <name> <timeout> <cmd...>: python failures (rc 1) continue, timeouts/crashes stop
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $R/gpurun_out/r4d_$n.log 2>&1; local rc=$?
  echo "$n rc=$rc"
  if [ $rc -ge 124 ]; then echo "stopping after $n"; exit $rc; fi
}
step pwtest 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_pwconv_gpu.py
step bw 300 python tools/bw_probe.py
step p2p 300 python tools/debug_r4.py p2p
step capture 300 python tools/debug_r4.py capture base upd_main
step bench 300 python bench.py
step bench_graph 300 python bench.py --graph 1
grep -E "PASS|FAIL|Error|assert" gpurun_out/r4d_pwtest.log | head -20; cat gpurun_out/r4d_bw.log | grep -v amdgpu; grep -v "amdgpu\|Gloo\|socket.cpp" gpurun_out/r4d_p2p.log gpurun_out/r4d_capture.log | tail -50
for f in bench bench_graph; do tail -1 gpurun_out/r4d_$f.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["host_issue_ms_per_step"], d["host_issue_ms_single_step"], d["config"]["hipgraph"])'; done
