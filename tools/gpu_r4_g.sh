#!/bin/bash
# round-4 session G: captured overlapped update variants, each in a fresh process
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
R=$GRAFT_REPO_ROOT
step() {
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $R/gpurun_out/r4g_$n.log 2>&1; local rc=$?
  echo "$n rc=$rc"
  if [ $rc -ge 124 ]; then echo "stopping after $n"; exit $rc; fi
}
step upd_main 200 python tools/debug_r4.py capture upd_main
step defer 200 python tools/debug_r4.py capture defer
step sync_upd 200 python tools/debug_r4.py capture sync_upd
DTF_WGRAD_STREAM=0 step noside 200 python tools/debug_r4.py capture base
DTF_STEM_KERNEL=0 step nostem 200 python tools/debug_r4.py capture base
for f in upd_main defer sync_upd noside nostem; do echo "== $f"; grep -v amdgpu gpurun_out/r4g_$f.log | grep -v "after step [56]" | cut -c1-250; done
