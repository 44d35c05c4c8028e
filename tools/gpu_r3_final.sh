#!/bin/bash
# GPU session: full GPU suite, default ResNet-50 bench (JSON to gpurun_out/bench_final.json), steady-state ResNet-50
# kernel stats, GPT-2-medium fp8 vs bf16 50-step loss curves (fused fp8 path).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread tests -m gpu > $OUT/gputests.log 2>&1; rc=$?; echo "gpu suite rc=$rc"; grep -E "FAILED|ERROR|passed|failed" $OUT/gputests.log | tail -20
[ $rc -le 1 ] || exit 1
timeout -k 10 300 python bench.py > $OUT/bench_final.log 2>&1 || { echo "bench failed"; tail -20 $OUT/bench_final.log; exit 1; }
tail -1 $OUT/bench_final.log | tee $OUT/bench_final.json
MODEL=resnet50 TAG=final HEAD=3 bash tools/gpu_r3_prof.sh || exit 1
timeout -k 10 600 python tools/fp8_loss_curve.py 50 8 > $OUT/fp8_curve.log 2>&1 || { echo "curve failed"; tail -5 $OUT/fp8_curve.log; exit 1; }
tail -3 $OUT/fp8_curve.log
