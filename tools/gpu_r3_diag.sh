#!/bin/bash
# GPU session: fused-BN-finalize diagnosis (residual-link test with the fused finalize off/on), whole GPU suite
# without -x, ResNet-50 bench with the finalize fused and not.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
T="python -u -m pytest -q --timeout 300 --timeout-method thread"
DTF_BN_FIN_FUSED=0 timeout -k 10 300 $T tests/test_resnet_gpu.py > $OUT/t_res_nofin.log 2>&1; echo "res nofin rc=$?"; tail -3 $OUT/t_res_nofin.log
timeout -k 10 900 $T tests -m gpu > $OUT/gputests.log 2>&1; echo "gpu suite rc=$?"; grep -E "FAILED|ERROR|passed|failed" $OUT/gputests.log | tail -20
timeout -k 10 300 python bench.py > $OUT/bench_base.log 2>&1 || { echo "bench failed"; tail -20 $OUT/bench_base.log; exit 1; }
tail -1 $OUT/bench_base.log
DTF_BN_FIN_FUSED=0 timeout -k 10 300 python bench.py > $OUT/bench_nofin.log 2>&1 || { echo "bench nofin failed"; tail -20 $OUT/bench_nofin.log; exit 1; }
tail -1 $OUT/bench_nofin.log
