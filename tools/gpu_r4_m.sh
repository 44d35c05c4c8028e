#!/bin/bash
# round-4 session M: why the forced-collective (torchrun, RCCL world 1) bench hangs: stack dump after 90 s
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
R=$GRAFT_REPO_ROOT
DTF_BENCH_WATCHDOG=90 DTF_FORCE_COLLECTIVE=1 timeout -k 10 150 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --steps 3 --warmup 2 > gpurun_out/r4m_forced.log 2>&1; echo "forced rc=$?"
grep -v "amdgpu.ids\|socket.cpp" gpurun_out/r4m_forced.log | tail -60
