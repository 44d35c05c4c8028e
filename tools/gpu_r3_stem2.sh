#!/bin/bash
# GPU session: stem kernel store variants (microbench), then the full GPU suite.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
timeout -k 10 120 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_stem_gpu.py -m gpu 2>&1 | tail -2 || exit 1
for v in 1 0 1 0; do
  DTF_STEM_STORE=$v timeout -k 10 200 python -u tools/bench_stem.py 2>&1 | grep "s2d   fwd" | cut -c1-40 | sed "s/^/store=$v /" || exit 1
done
for cfg in "DTF_STEM_STORE=0" "DTF_STEM_STORE=1" "DTF_POOLBN_RED_GRID=2048" "DTF_STEM_STORE=0" "DTF_STEM_STORE=1" "DTF_POOLBN_RED_GRID=2048"; do
  env $cfg timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $OUT/stem_st.json 2>$OUT/stem_st.err || { tail -5 $OUT/stem_st.err; exit 1; }
  python -c "import json; d=json.loads(open('$OUT/stem_st.json').read().strip().splitlines()[-1]); print('$cfg', d['value'], d['ms_per_step'], d['config'].get('final_loss'))"
done
if [ "${SUITE:-1}" = 1 ]; then
  timeout -k 10 600 python -u -m pytest -q --timeout 120 --timeout-method thread tests -m gpu > $OUT/suite_full.log 2>&1
  grep -E '^FAILED' $OUT/suite_full.log | head -20; tail -1 $OUT/suite_full.log
fi
