#!/bin/bash
# round-4 session P: pwconv apply/stage + BN finalize (rows summed in the finalize kernel) — tests and bench A/Bs
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
R=$GRAFT_REPO_ROOT
step() {
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $R/gpurun_out/r4p_$n.log 2>&1; local rc=$?
  echo "$n rc=$rc"
  if [ $rc -ge 124 ]; then echo "stopping after $n"; exit $rc; fi
}
step tests 600 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_pwconv_gpu.py tests/test_resnet_gpu.py tests/test_bn_fin_gpu.py tests/test_kernels_gpu.py tests/test_model_training_gpu.py
step bw 200 python tools/bw_probe.py
step b1 300 python bench.py
DTF_PW_APPLY=0 step b0 300 python bench.py
DTF_BN_GROUP_TARGET=32 step bg 300 python bench.py
step b1b 300 python bench.py
DTF_PW_APPLY=0 step b0b 300 python bench.py
DTF_BN_GROUP_TARGET=32 step bgb 300 python bench.py
tail -2 gpurun_out/r4p_tests.log; grep "^s" gpurun_out/r4p_bw.log | cut -c1-120
for f in b1 b0 bg b1b b0b bgb; do grep '^{"metric"' gpurun_out/r4p_$f.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("'$f'", d["value"], d["ms_per_step"], d["config"]["final_loss"])'; done
