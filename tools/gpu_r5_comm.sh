# Forced-collective (RCCL world 1) bench: the native C++ communicator vs torch's process group, interleaved.
set -o pipefail
mkdir -p gpurun_out
tag=${1:-r5c}; m=${2:-resnet50}
for i in 1 2; do
  for c in native torch; do
    DTF_FORCE_COLLECTIVE=1 DTF_COMM=$c timeout -k 10 300 python -u bench.py --model $m --steps 20 --warmup 5 > gpurun_out/${tag}_${m}_${c}_$i.log 2>&1 || { tail -20 gpurun_out/${tag}_${m}_${c}_$i.log; exit 1; }
    echo "$m $c $i $(tail -n 1 gpurun_out/${tag}_${m}_${c}_$i.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"].get("allreduce_paths"), d.get("exposed_comm_ms_per_step", d["config"].get("exposed_comm_ms_per_step")))')"
  done
done
