# round 4 session Q: diagnose test_residual_grad_link_matches_reference (finalize row groups), the rest of P's tests,
# LDS-DMA 3-deep ring tiles (17/18) per conv layer and end to end
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ $rc -lt 124 ] || exit $rc; return 0; }
step att timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_attention.py > gpurun_out/r4q_att.log 2>&1
tail -2 gpurun_out/r4q_att.log
step ab0 timeout -k 10 200 python -u tools/bench_attention.py > gpurun_out/r4q_ab0.log 2>&1
DTF_ATTN_DS=1 step ab1 timeout -k 10 200 python -u tools/bench_attention.py > gpurun_out/r4q_ab1.log 2>&1
grep -v Warn gpurun_out/r4q_ab0.log gpurun_out/r4q_ab1.log
step diag timeout -k 10 240 python -u tools/diag_resnet_link.py > gpurun_out/r4q_diag.log 2>&1
DTF_BN_GROUP_TARGET=32 step diag32 timeout -k 10 240 python -u tools/diag_resnet_link.py > gpurun_out/r4q_diag32.log 2>&1
step tests timeout -k 10 600 python -u -m pytest -x -v --timeout 150 --timeout-method thread -m gpu tests/test_resnet_gpu.py tests/test_bn_fin_gpu.py tests/test_kernels_gpu.py tests/test_model_training_gpu.py > gpurun_out/r4q_tests.log 2>&1
cat gpurun_out/r4q_diag.log gpurun_out/r4q_diag32.log | grep -v Warning
tail -3 gpurun_out/r4q_tests.log
step roof timeout -k 10 400 python -u tools/conv_roofline.py --tiles --tile-list 8,9,17,18 > gpurun_out/r4q_roof.log 2>&1
grep TOTAL gpurun_out/r4q_roof.log
step b0 timeout -k 10 300 python bench.py > gpurun_out/r4q_b0.log 2>&1
DTF_GLDS_RING=1 step br timeout -k 10 300 python bench.py > gpurun_out/r4q_br.log 2>&1
step b0b timeout -k 10 300 python bench.py > gpurun_out/r4q_b0b.log 2>&1
DTF_GLDS_RING=1 step brb timeout -k 10 300 python bench.py > gpurun_out/r4q_brb.log 2>&1
for f in b0 br b0b brb; do grep '^{"metric"' gpurun_out/r4q_$f.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("'$f'", d["value"], d["ms_per_step"], d["config"]["final_loss"])'; done
