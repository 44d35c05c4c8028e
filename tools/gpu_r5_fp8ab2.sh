# interleaved A/B of the q8 (producer-quantizing) GEMMs on the 4-wave kernel (DTF_FP8_W4=1) vs gemm256 (=2)
set -o pipefail
mkdir -p gpurun_out
tag=${1:-r5q}
for i in 1 2; do
  for v in 1 2; do
    DTF_FP8_W4=$v timeout -k 10 300 python -u bench.py --model gpt2_medium_fp8 --steps 30 --warmup 5 > gpurun_out/${tag}_${v}_$i.log 2>&1 || { tail -20 gpurun_out/${tag}_${v}_$i.log; exit 1; }
    echo "DTF_FP8_W4=$v run $i $(tail -n 1 gpurun_out/${tag}_${v}_$i.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
