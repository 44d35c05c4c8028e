#!/bin/bash
# GPU session: GPT-2-medium fp8 vs bf16 benches and fp8 GEMM tiling A/B (256-row pipelined kernel for more shapes).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
run() { local tag=$1; shift; env "$@" timeout -k 10 300 python bench.py $BARGS > $OUT/f_$tag.log 2>&1 || { echo "$tag failed"; tail -5 $OUT/f_$tag.log; exit 1; }; echo "$tag $(grep '"metric"' $OUT/f_$tag.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"; }
BARGS="--model gpt2_medium_fp8 --steps 10 --warmup 3"
run fp8 X=1
run fp8_narrow DTF_G256_NARROW=1
run fp8_min64 DTF_G256_MIN=64
BARGS="--model gpt2_medium --steps 10 --warmup 3"
run bf16 X=1
run bf16_narrow DTF_G256_NARROW=1
