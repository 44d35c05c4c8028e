set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
DTF_GLDS_WGRAD=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "conv" > gpurun_out/t_conv.log 2>&1 || { echo TESTFAIL; tail -40 gpurun_out/t_conv.log; exit 1; }
tail -n 1 gpurun_out/t_conv.log
DTF_GLDS_WGRAD=1 timeout -k 10 500 python tools/conv_roofline.py --tiles --tile-list 0,2,3,4,7,8,9,10 --only wgrad > gpurun_out/rf_w.log 2>&1
tail -n 1 gpurun_out/rf_w.log
