#!/bin/bash
# GPU session: whole-model tests (frozen-BN gradient check), GPT-2-medium fp8 bench with the LDS-DMA fp8 tiles.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
timeout -k 10 600 python -u -m pytest -q --timeout 500 --timeout-method thread tests/test_model_training_gpu.py tests/test_resnet_gpu.py > $OUT/t_model.log 2>&1; rc=$?; echo "model tests rc=$rc"; grep -E "FAILED|passed|failed|assert|Error" $OUT/t_model.log | head -20
[ $rc -le 1 ] || exit 1
timeout -k 10 300 python bench.py --model gpt2_medium_fp8 --steps 10 --warmup 3 > $OUT/f_fp8p3.log 2>&1 || { echo "fp8 bench failed"; tail -5 $OUT/f_fp8p3.log; exit 1; }
grep '"metric"' $OUT/f_fp8p3.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("fp8 pipe3", d["value"], d["ms_per_step"])'
