# round 4 session L2: ResNet-50 knob sweep on the final code (BN pass rows per trip, finalize grouping), interleaved
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
n=0
for i in 1 2; do
  for e in "X=1" "DTF_EW_APPLY_NU=4" "DTF_EW_VARIANT=0" "DTF_BN_GROUP_TARGET=128" "DTF_NARROW_ROWS=0"; do
    n=$((n+1))
    env $e timeout -k 10 300 python bench.py > gpurun_out/r4l2_$n.log 2>&1 || exit 1
    grep '^{"metric"' gpurun_out/r4l2_$n.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(sys.argv[1], d["value"], d["ms_per_step"])' "$e"
  done
done
