# round 4 session G2: raw current-stream accessor, cached fp8 state views (host issue time): tests that use side streams / capture, benches
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu tests/test_graphs.py tests/test_dp_gpu.py tests/test_model_training_gpu.py tests/test_resnet_gpu.py tests/test_p2p_allreduce_gpu.py tests/test_fp8_fused_gpu.py tests/test_fp8_large.py > gpurun_out/r4g2_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r4g2_tests.log; [ $rc -eq 0 ] || exit 1
for m in resnet50 gpt2_medium gpt2_medium_fp8 bert_base; do
  a=""; [ $m = resnet50 ] || a="--model $m --steps 10 --warmup 3"
  timeout -k 10 300 python bench.py $a > gpurun_out/r4g2_$m.log 2>&1 || exit 1
  grep '^{"metric"' gpurun_out/r4g2_$m.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("'$m'", d["value"], d["ms_per_step"], "host_issue", d.get("host_issue_ms_per_step"), d.get("host_issue_ms_single_step"))'
done
