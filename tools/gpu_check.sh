# GPU session: a pytest subset ($1, a -k expression or test paths in $T), then optional profiles.
#   T="tests/test_x.py ..." bash tools/gpu_check.sh [tag]
set -o pipefail
mkdir -p gpurun_out
tag=${1:-check}
timeout -k 10 ${TT:-900} python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu ${T:-tests} > gpurun_out/${tag}_tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|SKIPPED" gpurun_out/${tag}_tests.log | cut -c1-150 | tail -60
tail -3 gpurun_out/${tag}_tests.log
exit $rc
