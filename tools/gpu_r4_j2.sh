# round 4 session J2: full GPU suite after the capture guard; bf16 transformer hipGraph replay
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
R=$GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread > gpurun_out/r4j2_tests.log 2>&1; rc=$?; echo "tests rc=$rc"
grep -E "FAILED|passed|failed" gpurun_out/r4j2_tests.log | tail -6
[ $rc -lt 124 ] || exit $rc
for m in gpt2_medium bert_base; do
  timeout -k 10 300 python bench.py --model $m --steps 10 --warmup 3 --graph 1 > gpurun_out/r4j2_g$m.log 2>&1 || { echo "$m graph failed"; tail -3 gpurun_out/r4j2_g$m.log; continue; }
  grep '^{"metric"' gpurun_out/r4j2_g$m.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("graph '$m'", d["value"], d["ms_per_step"], d["config"].get("hipgraph"))'
done
