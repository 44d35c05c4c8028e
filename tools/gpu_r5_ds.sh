# BERT-base attention backward: recompute dQ kernel (default for non-causal) vs the dS^T scratch path, interleaved.
set -o pipefail
mkdir -p gpurun_out
tag=${1:-r5ds}
for rnd in 1 2; do
  for v in None True; do
    timeout -k 10 300 python -u tools/bench_with.py distributed_tensorflow_amd.ops.mha:_ATTN_DS=$v -- --model bert_base --steps 20 --warmup 5 > gpurun_out/${tag}_${v}_${rnd}.log 2>&1 || { tail -20 gpurun_out/${tag}_${v}_${rnd}.log; exit 1; }
    echo "ATTN_DS=$v round $rnd: $(tail -n 1 gpurun_out/${tag}_${v}_${rnd}.log | grep -o '"value": [0-9.]*')"
  done
done
