# round 4 session J2: full GPU suite, smoke and the default bench on the final tree
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
R=$GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread > gpurun_out/r4j2_tests.log 2>&1; rc=$?; echo "tests rc=$rc"
grep -E "FAILED|passed|failed" gpurun_out/r4j2_tests.log | tail -6
[ $rc -lt 124 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r4j2_smoke.log 2>&1; echo "smoke rc=$?"
timeout -k 10 300 python bench.py > gpurun_out/r4j2_bench.log 2>&1 || exit 1
grep '^{"metric"' gpurun_out/r4j2_bench.log
