# round 4 session R2: per-layer 128x64 LDS-DMA tiles synchronous (t8) vs double-buffered (t10), and 256-row (t11-14)
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u tools/conv_roofline.py --tiles --tile-list 8,10,9 --only fwd > gpurun_out/r4r2_fwd.log 2>&1; echo "fwd rc=$?"
timeout -k 10 400 python -u tools/conv_roofline.py --tiles --tile-list 8,10,9 --only dgrad > gpurun_out/r4r2_dgrad.log 2>&1; echo "dgrad rc=$?"
grep TOTAL gpurun_out/r4r2_fwd.log gpurun_out/r4r2_dgrad.log
