# round 4 session I2: full GPU suite + smoke + ResNet-50 bench under the final defaults
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
R=$GRAFT_REPO_ROOT
step() {
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $R/gpurun_out/r4i2_$n.log 2>&1; local rc=$?
  echo "$n rc=$rc"
  if [ $rc -ge 124 ]; then echo "stopping after $n"; exit $rc; fi
}
step tests 900 python -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread
grep -E "FAILED|passed|failed" gpurun_out/r4i2_tests.log | tail -6
step smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
tail -1 gpurun_out/r4i2_smoke.log
step b1 300 python bench.py
step b2 300 python bench.py
for f in b1 b2; do grep '^{"metric"' gpurun_out/r4i2_$f.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("'$f'", d["value"], d["ms_per_step"], d.get("host_issue_ms_single_step"))'; done
