# add_dropout + LayerNorm forward fusion (ops.nn._FUSE_ADD_LN): transformer GPU tests, then interleaved A/B benches.
# bash tools/gpu_r5_addln.sh <tag>
set -o pipefail
mkdir -p gpurun_out
tag=${1:-r5al}
timeout -k 10 600 python -u -m pytest -x -q -m gpu tests/test_graphs.py tests/test_model_training_gpu.py tests/test_attention.py --timeout 200 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1 || { tail -30 gpurun_out/${tag}_tests.log; exit 1; }
tail -n 2 gpurun_out/${tag}_tests.log
for m in bert_base gpt2_medium; do
  for on in True False True False; do
    timeout -k 10 300 python -u tools/bench_with.py distributed_tensorflow_amd.ops.nn:_FUSE_ADD_LN=$on -- --model $m --steps 20 --warmup 5 > gpurun_out/${tag}_bench_${m}_$on.log 2>&1 || { tail -20 gpurun_out/${tag}_bench_${m}_$on.log; exit 1; }
    echo "$m fuse=$on $(tail -n 1 gpurun_out/${tag}_bench_${m}_$on.log | cut -c1-120)"
  done
done
