#!/bin/bash
# GPU session: PS data plane (tests + 1-GPU 1 PS x 3 trainer rehearsal with the common-window aggregate), the forced
# single-rank collective path (hook / bucket / RCCL cost vs the single-replica bench), hipGraph-captured step bench +
# rocprofv3 trace of its replays.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
timeout -k 10 400 python -u -m pytest tests/test_ps_gpu.py -q --timeout 200 --timeout-method thread > $OUT/ps_tests.log 2>&1; rc=$?; echo "ps tests rc=$rc"; tail -3 $OUT/ps_tests.log
[ $rc -le 1 ] || exit 1
timeout -k 10 400 python tools/bench_ps.py --gpus 1 --ps 1 --trainers 3 --steps 10 --warmup 3 --batch 128 --timeout 350 > $OUT/bench_ps_gpu.log 2>&1 || { echo "bench_ps gpu failed"; tail -30 $OUT/bench_ps_gpu.log; exit 1; }
grep '"metric"' $OUT/bench_ps_gpu.log
DTF_FORCE_COLLECTIVE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29531 timeout -k 10 300 python bench.py > $OUT/bench_forcecoll.log 2>&1 || { echo "bench forced collective failed"; tail -20 $OUT/bench_forcecoll.log; exit 1; }
tail -1 $OUT/bench_forcecoll.log
timeout -k 10 300 python bench.py --graph 1 > $OUT/bench_graph.log 2>&1 || { echo "graph bench failed"; tail -20 $OUT/bench_graph.log; exit 1; }
tail -1 $OUT/bench_graph.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof_graph -o run -- python3 $R/bench.py --graph 1 --steps 6 --warmup 3 > $OUT/prof_graph.log 2>&1 || { echo "graph prof failed"; tail -20 $OUT/prof_graph.log; exit 1; }
echo profiled
