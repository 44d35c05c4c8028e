set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
DTF_FUSE_BN_BWD=0 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/prof0 -o run -- python3 $R/bench.py --steps 3 --warmup 2 > $R/gpurun_out/prof0.log 2>&1 || { echo PROFFAIL; tail -5 $R/gpurun_out/prof0.log; exit 1; }
echo ok
