#!/bin/bash
# GPU session: attribute per-step runtime copies/at::native work, then eager vs hipGraph ResNet-50 bench.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
timeout -k 10 300 python tools/attribute_step_ops.py > $OUT/attrib.log 2>&1 || { echo "attrib failed"; tail -30 $OUT/attrib.log; exit 1; }
head -60 $OUT/attrib.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/bench_eager.log 2>&1 || { echo "bench eager failed"; tail -20 $OUT/bench_eager.log; exit 1; }
tail -1 $OUT/bench_eager.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --graph 1 > $OUT/bench_graph.log 2>&1 || { echo "bench graph failed"; tail -20 $OUT/bench_graph.log; exit 1; }
tail -1 $OUT/bench_graph.log
