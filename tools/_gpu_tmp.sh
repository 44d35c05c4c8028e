set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "conv" > gpurun_out/t_conv.log 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/t_conv.log; exit 1; }
tail -n 2 gpurun_out/t_conv.log
timeout -k 10 400 python tools/conv_roofline.py --only wgrad --tiles > gpurun_out/rf_wg1.log 2>&1
DTF_WGRAD_ROWMAP=0 timeout -k 10 300 python tools/conv_roofline.py --only wgrad > gpurun_out/rf_wg0.log 2>&1
tail -n 1 gpurun_out/rf_wg0.log gpurun_out/rf_wg1.log
