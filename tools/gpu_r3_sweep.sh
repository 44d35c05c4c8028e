#!/bin/bash
# GPU session: per-layer conv tile sweep (forward, data gradient) and the BERT-base steady-state kernel profile.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
for k in fwd dgrad; do
  timeout -k 10 500 python tools/conv_roofline.py --tiles --only $k --tile-list 0,1,2,3,4,5,6,7,8,9,10,15,16 > $OUT/roof_${k}_tiles.txt 2>&1 || { echo "sweep $k failed"; tail -5 $OUT/roof_${k}_tiles.txt; exit 1; }
  tail -1 $OUT/roof_${k}_tiles.txt
done
MODEL=bert_base TAG=bert HEAD=40 bash tools/gpu_r3_prof.sh
