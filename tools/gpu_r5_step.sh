set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/r5i_kt.log 2>&1; echo "kernel tests rc=$?" >> gpurun_out/r5i_kt.log
timeout -k 10 200 python -u bench.py --model bert_base --steps 10 --warmup 3 > gpurun_out/r5i_bert.log 2>&1 || exit 1
timeout -k 10 200 python -u bench.py --model gpt2_medium --steps 10 --warmup 3 > gpurun_out/r5i_gpt2.log 2>&1 || exit 1
timeout -k 10 200 python -u bench.py --model gpt2_medium_fp8 --steps 10 --warmup 3 > gpurun_out/r5i_fp8.log 2>&1 || exit 1
timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 > gpurun_out/r5i_rn50.log 2>&1 || exit 1
tail -n 3 gpurun_out/r5i_kt.log; for f in bert gpt2 fp8 rn50; do tail -n 1 gpurun_out/r5i_$f.log | cut -c1-200; done
