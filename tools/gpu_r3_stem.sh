#!/bin/bash
# GPU session: stem kernel tests, stem microbench (dedicated kernel vs implicit-GEMM tiles), ResNet-50 A/B.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_stem_gpu.py tests/test_resnet_gpu.py tests/test_model_training_gpu.py -m gpu 2>&1 | tail -5 || exit 1
timeout -k 10 200 python -u tools/bench_stem.py 2>&1 | grep -v amdgpu.ids || exit 1
for v in 1 0 1 0; do
  DTF_STEM_KERNEL=$v timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $OUT/stem_ab_$v.json 2>$OUT/stem_ab.err || { tail -5 $OUT/stem_ab.err; exit 1; }
  python -c "import json,sys; d=json.loads(open('$OUT/stem_ab_$v.json').read().strip().splitlines()[-1]); print('DTF_STEM_KERNEL=$v', d['value'], d['ms_per_step'], d['config'].get('final_loss'))"
done
