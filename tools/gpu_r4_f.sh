#!/bin/bash
# round-4 session F: side-hold fix vs P2P mismatch and captured overlapped update; pointwise blocks-per-CU A/B
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
R=$GRAFT_REPO_ROOT
step() {
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $R/gpurun_out/r4f_$n.log 2>&1; local rc=$?
  echo "$n rc=$rc"
  if [ $rc -ge 124 ]; then echo "stopping after $n"; exit $rc; fi
}
step p2p 300 python tools/debug_r4.py p2p gloo p2p
step capture 300 python tools/debug_r4.py capture base
step pwtest 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_pwconv_gpu.py
DTF_PW_BPC=2 step bw2 200 python tools/bw_probe.py
DTF_PW_BPC=3 step bw3 200 python tools/bw_probe.py
step dptests 400 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_dp_gpu.py tests/test_graphs.py tests/test_p2p_allreduce_gpu.py
grep -v "amdgpu\|Gloo\|socket.cpp" gpurun_out/r4f_p2p.log gpurun_out/r4f_capture.log | tail -30
tail -2 gpurun_out/r4f_pwtest.log; grep "^s1\|^s2" gpurun_out/r4f_bw2.log gpurun_out/r4f_bw3.log | cut -c1-200
grep -E "PASS|FAIL" gpurun_out/r4f_dptests.log | tail -30
