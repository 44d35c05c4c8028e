# round 4 session O2: ResNet-50 hipGraph replay under the HIP runtime's graph execution knobs (vs eager)
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
n=0
for e in "X=1|" "X=1|--graph 1" "DEBUG_HIP_FORCE_GRAPH_QUEUES=4|--graph 1" "DEBUG_HIP_FORCE_GRAPH_QUEUES=2|--graph 1" "DEBUG_CLR_GRAPH_PACKET_CAPTURE=0|--graph 1" "DEBUG_CLR_GRAPH_PACKET_CAPTURE=1|--graph 1"; do
  n=$((n+1)); envs="${e%%|*}"; args="${e#*|}"
  env $envs timeout -k 10 300 python bench.py $args > gpurun_out/r4o2_$n.log 2>&1; rc=$?
  if [ $rc -ne 0 ]; then echo "[$e] rc=$rc"; tail -3 gpurun_out/r4o2_$n.log; [ $rc -lt 124 ] || exit $rc; continue; fi
  grep '^{"metric"' gpurun_out/r4o2_$n.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(sys.argv[1], d["value"], d["ms_per_step"], d["config"].get("hipgraph"))' "$e"
done
