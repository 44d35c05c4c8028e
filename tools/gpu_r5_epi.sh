set -o pipefail
mkdir -p gpurun_out
tag=${1:-r5e}
timeout -k 10 200 python -u tools/bench_gemm_w4.py --sweepk 16384x3072 > gpurun_out/${tag}_sweep.log 2>&1 || { tail -20 gpurun_out/${tag}_sweep.log; exit 1; }
cat gpurun_out/${tag}_sweep.log | grep -v amdgpu.ids
DTF_W4_EPI=2 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "gemm or dense or beta or dact" > gpurun_out/${tag}_t.log 2>&1 || { tail -20 gpurun_out/${tag}_t.log; exit 1; }
tail -n 1 gpurun_out/${tag}_t.log
for i in 1 2; do
  for v in 0 2; do
    for m in bert_base gpt2_medium; do
      DTF_W4_EPI=$v timeout -k 10 300 python -u bench.py --model $m --steps 10 --warmup 5 > gpurun_out/${tag}_${m}_${v}_$i.log 2>&1 || { tail -20 gpurun_out/${tag}_${m}_${v}_$i.log; exit 1; }
      echo "$m DTF_W4_EPI=$v run $i $(tail -n 1 gpurun_out/${tag}_${m}_${v}_$i.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
    done
  done
done
