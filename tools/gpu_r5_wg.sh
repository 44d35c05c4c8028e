set -o pipefail
mkdir -p gpurun_out
tag=${1:-r5w}
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "conv or wgrad" > gpurun_out/${tag}_t.log 2>&1 || { tail -20 gpurun_out/${tag}_t.log; exit 1; }
tail -n 1 gpurun_out/${tag}_t.log
timeout -k 10 300 python -u tools/conv_roofline.py --only wgrad > gpurun_out/${tag}_roof.txt 2>&1 || exit 1
grep -E "c1 |c3 |proj|TOTAL wgrad" gpurun_out/${tag}_roof.txt | cut -c1-100
for i in 1 2; do
  for v in 1 0; do
    DTF_WGRAD_W4=$v timeout -k 10 300 python -u bench.py --model resnet50 --steps 20 --warmup 5 > gpurun_out/${tag}_rn_${v}_$i.log 2>&1 || { tail -20 gpurun_out/${tag}_rn_${v}_$i.log; exit 1; }
    echo "DTF_WGRAD_W4=$v b1024 run $i $(tail -n 1 gpurun_out/${tag}_rn_${v}_$i.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
