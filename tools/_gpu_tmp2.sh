set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
timeout -k 10 500 python tools/conv_roofline.py --tiles --tile-list 0,2,7,8,9,10 --only dgrad > gpurun_out/rf_d.log 2>&1
tail -n 1 gpurun_out/rf_d.log
