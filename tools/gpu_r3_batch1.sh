#!/bin/bash
# GPU session: BN grouping-target sweep (ResNet-50 bench), fp8 GEMM staging sweep (tools/bench_fp8_gemms.py with
# DTF_FP8_PIPE 2/3/4), whole-model gradient calibration (tools/calib_resnet_grad.py).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
bash tools/gpu_r3_grp.sh || exit 1
for p in 2 3 4; do
  DTF_FP8_PIPE=$p timeout -k 10 300 python tools/bench_fp8_gemms.py > $OUT/fp8g_p$p.log 2>&1 || { echo "fp8 gemm bench pipe $p failed"; tail -5 $OUT/fp8g_p$p.log; exit 1; }
  echo "pipe $p: $(tail -1 $OUT/fp8g_p$p.log)"
done
timeout -k 10 400 python tools/calib_resnet_grad.py > $OUT/calib.log 2>&1 || { echo "calib failed"; tail -20 $OUT/calib.log; exit 1; }
tail -6 $OUT/calib.log
for k in fwd dgrad; do
  timeout -k 10 400 python tools/conv_roofline.py --tiles --tile-list 8,9,15,16 --only $k > $OUT/roof_$k.log 2>&1 || { echo "roofline $k failed"; tail -5 $OUT/roof_$k.log; exit 1; }
  tail -1 $OUT/roof_$k.log
done
