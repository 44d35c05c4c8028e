#!/bin/bash
# GPU session: forward Dense GEMM timing under GEMM dispatch knobs ($VARIANTS, ';'-separated env sets)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
IFS=';' read -ra VL <<< "${VARIANTS:-X=0}"
for v in "${VL[@]}"; do
  echo "== $v"
  env $v timeout -k 10 120 python tools/bench_dense_fwd.py 2>&1 | grep -v amdgpu.ids || exit 1
done
