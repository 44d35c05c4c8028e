# round 4 session E2: tests under the new defaults; A/B: fused activation backward under plain BLAS, fp8 with / without
# plain BLAS (3 repeats)
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu tests/test_fp8_fused_gpu.py tests/test_model_training_gpu.py tests/test_kernels_gpu.py tests/test_direct_grads.py tests/test_dp_gpu.py tests/test_graphs.py > gpurun_out/r4e2_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r4e2_tests.log; [ $rc -eq 0 ] || exit 1
js() { grep '^{"metric"' $1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(sys.argv[1], d["value"], d["ms_per_step"], d["config"].get("final_loss"))' "$2"; }
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --model gpt2_medium --steps 10 --warmup 3 > gpurun_out/r4e2_g0$i.log 2>&1 || exit 1; js gpurun_out/r4e2_g0$i.log gpt2_default
  DTF_PLAIN_DACT=1 timeout -k 10 300 python bench.py --model gpt2_medium --steps 10 --warmup 3 > gpurun_out/r4e2_g1$i.log 2>&1 || exit 1; js gpurun_out/r4e2_g1$i.log gpt2_plain_dact
  timeout -k 10 300 python bench.py --model gpt2_medium_fp8 --steps 10 --warmup 3 > gpurun_out/r4e2_f0$i.log 2>&1 || exit 1; js gpurun_out/r4e2_f0$i.log fp8_default
  DTF_PLAIN_BLAS=0 timeout -k 10 300 python bench.py --model gpt2_medium_fp8 --steps 10 --warmup 3 > gpurun_out/r4e2_f1$i.log 2>&1 || exit 1; js gpurun_out/r4e2_f1$i.log fp8_noplain
done
timeout -k 10 300 python bench.py --model bert_base --steps 10 --warmup 3 > gpurun_out/r4e2_b.log 2>&1 || exit 1; js gpurun_out/r4e2_b.log bert_default
