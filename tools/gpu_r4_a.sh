#!/bin/bash
# round-4 GPU session A: full GPU suite, default bench, bench with the in-launch BN finalize, the new 8-phase GEMM.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/r4a_tests.log 2>&1
echo "tests_rc=$?"; tail -3 $OUT/r4a_tests.log
timeout -k 10 200 python bench.py > $OUT/r4a_bench.log 2>&1 || { echo "bench failed"; tail -20 $OUT/r4a_bench.log; exit 1; }
tail -1 $OUT/r4a_bench.log | cut -c1-220
DTF_BN_FIN_FUSED=1 timeout -k 10 200 python bench.py > $OUT/r4a_bench_fin.log 2>&1 || { echo "fin bench failed"; tail -20 $OUT/r4a_bench_fin.log; exit 1; }
tail -1 $OUT/r4a_bench_fin.log | cut -c1-220
timeout -k 10 240 python tools/bench_gemm8p.py --rounds 2 > $OUT/r4a_gemm8p.log 2>&1; echo "gemm8p_rc=$?"; cat $OUT/r4a_gemm8p.log | grep -v amdgpu.ids
