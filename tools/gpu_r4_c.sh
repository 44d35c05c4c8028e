#!/bin/bash
# round-4 session C: bisect the captured overlapped update and the 2-rank P2P mismatch; store-bound 1x1 probe;
# kernel stats with the in-launch BN finalize off/on. A step that times out / crashes ends the script.
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
R=$GRAFT_REPO_ROOT
step() {  # step <name> <timeout> <cmd...>: python failures (rc 1) continue, timeouts/crashes stop
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $R/gpurun_out/r4c_$n.log 2>&1; local rc=$?
  echo "$n rc=$rc"
  if [ $rc -ge 124 ]; then echo "stopping after $n"; exit $rc; fi
}
step capture 300 python tools/debug_r4.py capture base upd_main
DTF_WGRAD_STREAM=0 step capture_noside 200 python tools/debug_r4.py capture base
step p2p 300 python tools/debug_r4.py p2p
step bw 300 python tools/bw_probe.py
cd /tmp && export TMPDIR=/tmp
step prof_base 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r4c_prof_base -o base -- python3 $R/bench.py --steps 10 --warmup 5
DTF_BN_FIN_FUSED=1 step prof_fin 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r4c_prof_fin -o fin -- python3 $R/bench.py --steps 10 --warmup 5
cd $R
cat gpurun_out/r4c_capture.log gpurun_out/r4c_capture_noside.log gpurun_out/r4c_p2p.log gpurun_out/r4c_bw.log | grep -v amdgpu | tail -60
