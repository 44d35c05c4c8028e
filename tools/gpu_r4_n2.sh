# round 4 session N2: tests touching GPT-2 training / DP / capture after the overlap-update flip; final transformer benches
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu tests/test_dp_gpu.py tests/test_model_training_gpu.py tests/test_graphs.py tests/test_fp8_fused_gpu.py tests/test_direct_grads.py > gpurun_out/r4n2_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r4n2_tests.log; [ $rc -eq 0 ] || exit 1
for m in gpt2_medium gpt2_medium_fp8 bert_base gpt2_medium gpt2_medium_fp8 bert_base; do
  timeout -k 10 300 python bench.py --model $m --steps 10 --warmup 3 > gpurun_out/r4n2_$m.log 2>&1 || exit 1
  grep '^{"metric"' gpurun_out/r4n2_$m.log | tee -a gpurun_out/r4n2_$m.jsonl | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("'$m'", d["value"], d["ms_per_step"], d.get("host_issue_ms_single_step"))'
done
timeout -k 10 300 python -u tools/bench_gemm256.py > gpurun_out/r4n2_gemm.log 2>&1; echo "gemm rc=$?"
grep -c TF gpurun_out/r4n2_gemm.log
