# round 4 session S: resnet/training GPU tests, diag L2, GPT-2 benches with the causal dS attention backward
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ $rc -lt 124 ] || exit $rc; return 0; }
step diag timeout -k 10 120 python -u tools/diag_resnet_link.py > gpurun_out/r4s_diag.log 2>&1
grep "^x " gpurun_out/r4s_diag.log
step tests timeout -k 10 600 python -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu tests/test_resnet_gpu.py tests/test_model_training_gpu.py tests/test_attention.py > gpurun_out/r4s_tests.log 2>&1
tail -2 gpurun_out/r4s_tests.log
js() { grep '^{"metric"' $1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("'$2'", d["value"], d["ms_per_step"], d["config"].get("final_loss"))'; }
step g1 timeout -k 10 300 python bench.py --model gpt2_medium --steps 10 --warmup 3 > gpurun_out/r4s_g1.log 2>&1
DTF_ATTN_DS=0 step g0 timeout -k 10 300 python bench.py --model gpt2_medium --steps 10 --warmup 3 > gpurun_out/r4s_g0.log 2>&1
step f1 timeout -k 10 300 python bench.py --model gpt2_medium_fp8 --steps 10 --warmup 3 > gpurun_out/r4s_f1.log 2>&1
DTF_ATTN_DS=0 step f0 timeout -k 10 300 python bench.py --model gpt2_medium_fp8 --steps 10 --warmup 3 > gpurun_out/r4s_f0.log 2>&1
step r timeout -k 10 300 python bench.py > gpurun_out/r4s_r.log 2>&1
js gpurun_out/r4s_g1.log gpt2_ds; js gpurun_out/r4s_g0.log gpt2_nods; js gpurun_out/r4s_f1.log fp8_ds; js gpurun_out/r4s_f0.log fp8_nods; js gpurun_out/r4s_r.log resnet
