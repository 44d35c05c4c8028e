#!/bin/bash
# GPU session: transformer benches (BERT-base, GPT-2-medium bf16 / fp8, each with hipBLASLt on and off for the
# plain backward GEMMs), the attention and plain-GEMM microbenchmarks, and a kernel profile of BERT-base.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
AB="${AB:-|--model bert_base --steps 10 --warmup 3;DTF_PLAIN_BLAS=0|--model bert_base --steps 10 --warmup 3;|--model gpt2_medium --steps 10 --warmup 3;DTF_PLAIN_BLAS=0|--model gpt2_medium --steps 10 --warmup 3;|--model gpt2_medium_fp8 --steps 10 --warmup 3;DTF_PLAIN_BLAS=0|--model gpt2_medium_fp8 --steps 10 --warmup 3}" bash tools/gpu_ab.sh || exit 1
if [ "${MICRO:-1}" = "1" ]; then
  timeout -k 10 300 python tools/bench_attention.py > $OUT/attn.log 2>&1 || { echo "attn bench failed"; tail $OUT/attn.log; exit 1; }
  cat $OUT/attn.log
  timeout -k 10 300 python tools/bench_blas_plain.py > $OUT/blas.log 2>&1 || { echo "blas bench failed"; tail $OUT/blas.log; exit 1; }
  cat $OUT/blas.log
fi
if [ "${PROF:-1}" = "1" ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/xprof -o run -- python3 $R/bench.py --model ${PMODEL:-bert_base} --steps 4 --warmup 3 > $OUT/xprof.log 2>&1 || { echo "prof failed"; tail -20 $OUT/xprof.log; exit 1; }
  python3 $R/tools/kstats.py $OUT/xprof/run_kernel_stats.csv 7 30
fi
