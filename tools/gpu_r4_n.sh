#!/bin/bash
# round-4 session N: staged pwconv epilogue (tests + probe A/B), then forced-collective vs single, then PMC
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
R=$GRAFT_REPO_ROOT
step() {
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $R/gpurun_out/r4n_$n.log 2>&1; local rc=$?
  echo "$n rc=$rc"
  if [ $rc -ge 124 ]; then echo "stopping after $n"; exit $rc; fi
}
step pwtest 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_pwconv_gpu.py
step bench 300 python bench.py
DTF_PW_APPLY=0 step bench_noapply 300 python bench.py
step bw1 200 python tools/bw_probe.py
DTF_PW_STAGE=0 step bw0 200 python tools/bw_probe.py
tail -2 gpurun_out/r4n_pwtest.log; for f in bench bench_noapply; do tail -1 gpurun_out/r4n_$f.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"]["final_loss"])'; done; grep "^s" gpurun_out/r4n_bw1.log | cut -c1-120; grep "^s" gpurun_out/r4n_bw0.log | cut -c1-120
step stem 300 python tools/stem_wgrad_probe.py
cat gpurun_out/r4n_stem.log | grep -v amdgpu
bash tools/gpu_r4_kl.sh
