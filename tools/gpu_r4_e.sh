#!/bin/bash
# round-4 session E: which stream interaction breaks the P2P bucket sums in training
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
R=$GRAFT_REPO_ROOT
step() {
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $R/gpurun_out/r4e_$n.log 2>&1; local rc=$?
  echo "$n rc=$rc"
  if [ $rc -ge 124 ]; then echo "stopping after $n"; exit $rc; fi
}
step p2p 400 python tools/debug_r4.py p2p gloo p2p p2p_before p2p_barrier p2p_mainwait p2p_main
grep -v "amdgpu\|Gloo\|socket.cpp" gpurun_out/r4e_p2p.log | tail -80
