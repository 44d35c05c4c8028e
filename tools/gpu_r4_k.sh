#!/bin/bash
# round-4 session K: forced-collective path (RCCL world 1, bucketed all-reduce from the hooks) vs single replica at the
# box's default 4 HW queues; stream -> queue map of the forced path
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
R=$GRAFT_REPO_ROOT
step() {
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $R/gpurun_out/r4k_$n.log 2>&1; local rc=$?
  echo "$n rc=$rc"
  if [ $rc -ge 124 ]; then echo "stopping after $n"; exit $rc; fi
}
step single 300 python bench.py
DTF_FORCE_COLLECTIVE=1 step forced 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1
step single2 300 python bench.py
DTF_FORCE_COLLECTIVE=1 step forced2 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 1
cd /tmp && export TMPDIR=/tmp
DTF_FORCE_COLLECTIVE=1 RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29535 step prof 300 rocprofv3 --kernel-trace -d $R/gpurun_out/r4k_prof -o run -- python3 $R/bench.py --steps 6 --warmup 3
cd $R
for f in single forced single2 forced2; do tail -1 gpurun_out/r4k_$f.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"].get("allreduce_paths"), d["config"].get("forced_collective"), d["process_group_backend"])'; done
python tools/queue_map.py gpurun_out/r4k_prof/run_results.db
