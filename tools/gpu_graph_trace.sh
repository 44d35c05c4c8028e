#!/bin/bash
# GPU session: hipGraph-captured ResNet-50 step (bench.py --graph 1) vs eager, benches + a rocprofv3 kernel trace of
# the captured replays (which queue / stream each kernel of the replayed graph ran on).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
timeout -k 10 300 python bench.py --graph 1 > $OUT/bench_graph.log 2>&1 || { echo "graph bench failed"; tail -20 $OUT/bench_graph.log; exit 1; }
tail -1 $OUT/bench_graph.log
# HIP runtime graph-execution knobs: packet capture (all kernel nodes batched onto one queue) vs per-branch streams
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -k 10 300 python bench.py --graph 1 > $OUT/bench_graph_nopc.log 2>&1 || { echo "graph nopc bench failed"; tail -20 $OUT/bench_graph_nopc.log; exit 1; }
tail -1 $OUT/bench_graph_nopc.log
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 DEBUG_HIP_FORCE_GRAPH_QUEUES=2 timeout -k 10 300 python bench.py --graph 1 > $OUT/bench_graph_q2.log 2>&1 || { echo "graph q2 bench failed"; tail -20 $OUT/bench_graph_q2.log; exit 1; }
tail -1 $OUT/bench_graph_q2.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof_graph -o run -- python3 $R/bench.py --graph 1 --steps 6 --warmup 3 > $OUT/prof_graph.log 2>&1 || { echo "graph prof failed"; tail -20 $OUT/prof_graph.log; exit 1; }
echo profiled
