set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/ -m gpu > gpurun_out/t_all.log 2>&1 || { echo TESTFAIL; tail -40 gpurun_out/t_all.log; exit 1; }
tail -n 2 gpurun_out/t_all.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1 || { echo BENCHFAIL; tail -20 gpurun_out/bench.log; exit 1; }
tail -n 1 gpurun_out/bench.log
DTF_LAZY_RES=0 timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench0.log 2>&1 || { echo BENCHFAIL; tail -20 gpurun_out/bench0.log; exit 1; }
tail -n 1 gpurun_out/bench0.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof -o run -- python3 $R/bench.py --steps 3 --warmup 2 > $R/gpurun_out/prof.log 2>&1 || { echo PROFFAIL; tail -5 $R/gpurun_out/prof.log; exit 1; }
echo profiled
