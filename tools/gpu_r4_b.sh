#!/bin/bash
# round-4 GPU session B: P2P all-reduce test, 8-phase GEMM (BN 256/128) vs gemm256/hipBLASLt, per-layer conv times
# with the 8-phase tiles forced (20 = 256x256, 21 = 256x128).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
timeout -k 10 300 python -u -m pytest tests/test_p2p_allreduce_gpu.py -x -q --timeout 200 --timeout-method thread > $OUT/r4b_p2p.log 2>&1
echo "p2p_rc=$?"; tail -3 $OUT/r4b_p2p.log
timeout -k 10 300 python -u -m pytest tests/test_graphs.py -q --timeout 200 --timeout-method thread > $OUT/r4b_graphs.log 2>&1
echo "graphs_rc=$?"; tail -15 $OUT/r4b_graphs.log
timeout -k 10 300 python tools/bench_gemm8p.py --rounds 2 > $OUT/r4b_gemm8p.log 2>&1; rc=$?; echo "gemm8p_rc=$rc"; grep -v amdgpu.ids $OUT/r4b_gemm8p.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 400 python tools/conv_roofline.py --tiles --tile-list 20,21 --only fwd > $OUT/r4b_roof_fwd.log 2>&1; echo "roof_fwd_rc=$?"; grep -v amdgpu.ids $OUT/r4b_roof_fwd.log | tail -60
timeout -k 10 400 python tools/conv_roofline.py --tiles --tile-list 20,21 --only dgrad > $OUT/r4b_roof_dgrad.log 2>&1; echo "roof_dgrad_rc=$?"; grep -v amdgpu.ids $OUT/r4b_roof_dgrad.log | tail -60
