#!/bin/bash
# GPU session: ResNet-50 bench with the BN statistics grouping pass at 32 / 64 / 128 / 256 leader rows.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
run() { local tag=$1; shift; env "$@" timeout -k 10 300 python bench.py $BARGS > $OUT/g_$tag.log 2>&1 || { echo "$tag failed"; tail -5 $OUT/g_$tag.log; exit 1; }; echo "$tag $(grep '"metric"' $OUT/g_$tag.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"; }
BARGS=""
run t32 DTF_BN_GROUP_TARGET=32
run t64 DTF_BN_GROUP_TARGET=64
run t128 DTF_BN_GROUP_TARGET=128
run t256 DTF_BN_GROUP_TARGET=256
run t32b DTF_BN_GROUP_TARGET=32
