# round 4 session D2: new defaults (bf16 forward projections + fp8 weight gradients on hipBLASLt): tests, A/B of the
# backward plain GEMMs on hipBLASLt and of the forward size threshold
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu tests/test_fp8_fused_gpu.py tests/test_model_training_gpu.py tests/test_kernels_gpu.py tests/test_direct_grads.py tests/test_dp_gpu.py > gpurun_out/r4d2_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r4d2_tests.log; [ $rc -eq 0 ] || exit 1
js() { grep '^{"metric"' $1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("'$2'", d["value"], d["ms_per_step"], d["config"].get("final_loss"))'; }
n=0
for i in 1 2; do
  for e in "X=1" "DTF_PLAIN_BLAS=1" "DTF_BLAS_FWD_MIN=4000000000"; do
    n=$((n+1))
    for m in gpt2_medium bert_base gpt2_medium_fp8; do
      env $e timeout -k 10 300 python bench.py --model $m --steps 10 --warmup 3 > gpurun_out/r4d2_$m$n.log 2>&1 || { tail -20 gpurun_out/r4d2_$m$n.log; exit 1; }
      js gpurun_out/r4d2_$m$n.log "$m [$e]"
    done
  done
done
