#!/bin/bash
# GPU session: GPT-2-medium fp8 vs bf16 50-step loss curves under fp8 path variants ($VARIANTS: ';'-separated env sets)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
IFS=';' read -ra VL <<< "${VARIANTS:-DTF_FP8_FUSE=0 DTF_FP8_TILES=0;DTF_FP8_FUSE=0}"
i=0
for v in "${VL[@]}"; do
  i=$((i+1))
  env $v timeout -k 10 600 python tools/fp8_loss_curve.py 50 8 > $OUT/curve_$i.log 2>&1 || { echo "curve [$v] failed"; tail -5 $OUT/curve_$i.log; exit 1; }
  echo "[$v] $(tail -1 $OUT/curve_$i.log)"
done
