#!/bin/bash
# GPU session: interleaved A/B of one env knob on the ResNet-50 bench: gpu_r3_ab.sh "A env" "B env" [rounds]
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
A=$1; B=$2; N=${3:-2}; BARGS=${BARGS:-}
for i in $(seq 1 $N); do
  for tag in A B; do
    if [ $tag = A ]; then E=$A; else E=$B; fi
    env $E timeout -k 10 300 python bench.py $BARGS > $OUT/ab_$tag$i.log 2>&1 || { echo "$tag$i failed"; tail -5 $OUT/ab_$tag$i.log; exit 1; }
    echo "$tag$i ($E) $(grep '"metric"' $OUT/ab_$tag$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
