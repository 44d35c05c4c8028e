# small-table embedding backward (register accumulators): kernel test, model tests, BERT bench and kernel trace
# bash tools/gpu_r5_emb.sh <tag>
set -o pipefail
mkdir -p gpurun_out
tag=${1:-r5em}
timeout -k 10 300 python -u -m pytest -x -q -m gpu tests/test_kernels_gpu.py -k "embed" tests/test_model_training_gpu.py tests/test_graphs.py --timeout 120 --timeout-method thread > gpurun_out/${tag}_t.log 2>&1 || { tail -30 gpurun_out/${tag}_t.log; exit 1; }
tail -n 1 gpurun_out/${tag}_t.log
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --model bert_base --steps 20 --warmup 5 > gpurun_out/${tag}_bert_$i.log 2>&1 || { tail -20 gpurun_out/${tag}_bert_$i.log; exit 1; }
  echo "bert $(tail -n 1 gpurun_out/${tag}_bert_$i.log | cut -c1-110)"
done
MARKER=embed_fwd_kernel bash tools/gpu_r5_prof.sh bert_base ${tag}_prof > /dev/null && grep -E "embed|total kernel|wall" gpurun_out/prof_${tag}_prof/steady.txt | head -8 | cut -c1-150
