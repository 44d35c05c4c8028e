# split-K fixup inside the 4-wave GEMM (native:dtf_set_split_fixup): kernel tests, then interleaved A/B benches
# bash tools/gpu_r5_fix.sh <tag>
set -o pipefail
mkdir -p gpurun_out
tag=${1:-r5fx}
timeout -k 10 300 python -u -m pytest -x -v -m gpu tests/test_kernels_gpu.py -k "splitk_fixup or wgrad" --timeout 120 --timeout-method thread > gpurun_out/${tag}_k.log 2>&1 || { tail -40 gpurun_out/${tag}_k.log; exit 1; }
grep -E "PASS|FAIL" gpurun_out/${tag}_k.log | cut -c1-150
timeout -k 10 600 python -u -m pytest -x -q -m gpu tests/test_graphs.py tests/test_model_training_gpu.py tests/test_kernel_paths_gpu.py tests/test_dp_gpu.py --timeout 200 --timeout-method thread > gpurun_out/${tag}_t.log 2>&1 || { tail -30 gpurun_out/${tag}_t.log; exit 1; }
tail -n 1 gpurun_out/${tag}_t.log
for m in gpt2_medium bert_base; do
  for fx in 16 0 16 0; do
    timeout -k 10 300 python -u tools/bench_with.py native:dtf_set_split_fixup=$fx -- --model $m --steps 20 --warmup 5 > gpurun_out/${tag}_${m}_$fx.log 2>&1 || { tail -20 gpurun_out/${tag}_${m}_$fx.log; exit 1; }
    echo "$m fix=$fx $(tail -n 1 gpurun_out/${tag}_${m}_$fx.log | cut -c1-110)"
  done
done
