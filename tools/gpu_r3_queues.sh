#!/bin/bash
# GPU session: HW-queue sharing of the N>1 path — forced single-rank collective with GPU_MAX_HW_QUEUES 4 vs 8, without
# the weight-gradient side stream, and hipGraph replays with more queues / without packet capture; rocprof trace of the
# forced-collective step (which queue each stream's kernels ran on).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
B="timeout -k 10 300 python bench.py"
run() { local tag=$1; shift; env "$@" $B > $OUT/q_$tag.log 2>&1 || { echo "$tag failed"; tail -5 $OUT/q_$tag.log; exit 1; }; echo "$tag $(tail -1 $OUT/q_$tag.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"; }
run fc_q8 DTF_FORCE_COLLECTIVE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29532 GPU_MAX_HW_QUEUES=8
run fc_noside DTF_FORCE_COLLECTIVE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29533 DTF_WGRAD_STREAM=0
run base_q8 GPU_MAX_HW_QUEUES=8
run noside DTF_WGRAD_STREAM=0
run fc_q4 DTF_FORCE_COLLECTIVE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29534
B="timeout -k 10 300 python bench.py --graph 1"
run graph_q8 GPU_MAX_HW_QUEUES=8
run graph_nopc DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
run graph_noside DTF_WGRAD_STREAM=0
cd /tmp && export TMPDIR=/tmp
DTF_FORCE_COLLECTIVE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29535 timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof_fc -o run -- python3 $R/bench.py --steps 6 --warmup 3 > $OUT/prof_fc.log 2>&1 || { echo "fc prof failed"; tail -20 $OUT/prof_fc.log; exit 1; }
echo profiled
