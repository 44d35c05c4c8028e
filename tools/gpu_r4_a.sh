#!/bin/bash
# round-4 GPU session A: default bench, bench with the in-launch BN finalize, the 8-phase GEMM (BN 256/128) vs
# gemm256/hipBLASLt, the full GPU suite, per-layer conv times with the 8-phase tiles forced (20: 256x256, 21: 256x128).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
timeout -k 10 200 python bench.py > $OUT/r4a_bench.log 2>&1 || { echo "bench failed"; tail -20 $OUT/r4a_bench.log; exit 1; }
tail -1 $OUT/r4a_bench.log | cut -c1-200
DTF_BN_FIN_FUSED=1 timeout -k 10 200 python bench.py > $OUT/r4a_bench_fin.log 2>&1 || { echo "fin bench failed"; tail -20 $OUT/r4a_bench_fin.log; exit 1; }
tail -1 $OUT/r4a_bench_fin.log | cut -c1-200
timeout -k 10 300 python tools/bench_gemm8p.py --rounds 2 > $OUT/r4a_gemm8p.log 2>&1; rc=$?; echo "gemm8p_rc=$rc"; grep -v amdgpu.ids $OUT/r4a_gemm8p.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > $OUT/r4a_tests.log 2>&1
echo "tests_rc=$?"; grep -E "passed|failed|FAILED|Error" $OUT/r4a_tests.log | tail -15
timeout -k 10 400 python tools/conv_roofline.py --tiles --tile-list 20,21 --only fwd > $OUT/r4a_roof_fwd.log 2>&1; echo "roof_fwd_rc=$?"; grep -v amdgpu.ids $OUT/r4a_roof_fwd.log | tail -40
