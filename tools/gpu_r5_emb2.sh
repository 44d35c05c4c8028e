# small-table embedding gradient, all table sizes on the register kernel: bash tools/gpu_r5_emb2.sh <tag>
set -o pipefail
mkdir -p gpurun_out
tag=${1:-r5e2}
timeout -k 10 400 python -u -m pytest -x -q -m gpu tests/test_kernels_gpu.py tests/test_model_training_gpu.py tests/test_graphs.py --timeout 120 --timeout-method thread > gpurun_out/${tag}_t.log 2>&1 || { tail -30 gpurun_out/${tag}_t.log; exit 1; }
tail -n 1 gpurun_out/${tag}_t.log
timeout -k 10 300 python -u bench.py --model bert_base --steps 20 --warmup 5 > gpurun_out/${tag}_bert.log 2>&1 || { tail -20 gpurun_out/${tag}_bert.log; exit 1; }
echo "bert $(tail -n 1 gpurun_out/${tag}_bert.log | cut -c1-110)"
