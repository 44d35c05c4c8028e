#!/bin/bash
# GPU session: fused-BN-finalize tests, full GPU test suite, ResNet-50 bench A/B (fused finalize on/off, forced
# single-rank collective path), rocprofv3 kernel trace of the default bench.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 300 $T tests/test_bn_fin_gpu.py > $OUT/t_binfin.log 2>&1 || { echo "binfin tests failed"; tail -40 $OUT/t_binfin.log; exit 1; }
tail -1 $OUT/t_binfin.log
timeout -k 10 900 $T tests -m gpu > $OUT/gputests.log 2>&1 || { echo "gpu tests failed rc=$?"; tail -40 $OUT/gputests.log; exit 1; }
tail -1 $OUT/gputests.log
timeout -k 10 300 python bench.py > $OUT/bench_base.log 2>&1 || { echo "bench failed"; tail -20 $OUT/bench_base.log; exit 1; }
tail -1 $OUT/bench_base.log
DTF_BN_FIN_FUSED=0 timeout -k 10 300 python bench.py > $OUT/bench_nofin.log 2>&1 || { echo "bench nofin failed"; tail -20 $OUT/bench_nofin.log; exit 1; }
tail -1 $OUT/bench_nofin.log
DTF_FORCE_COLLECTIVE=1 MASTER_ADDR=127.0.0.1 timeout -k 10 300 python bench.py > $OUT/bench_forcecoll.log 2>&1 || { echo "bench forced collective failed"; tail -20 $OUT/bench_forcecoll.log; exit 1; }
tail -1 $OUT/bench_forcecoll.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_base -o run -- python3 $R/bench.py --steps 6 --warmup 3 > $OUT/prof_base.log 2>&1 || { echo "prof failed"; tail -20 $OUT/prof_base.log; exit 1; }
echo profiled
